"""Host-side rates around the kernel path, one JSON line each:

  host_feed  decoded FASTQ bytes in host memory -> fr_feed (pinned ring, PCIe copies
             overlapped with the tally kernel) -> end_file -> finalize -> classify
  gz_scan    the whole `scan` command (frender_amd.scan.frender_scan) over .fastq.gz
             files: inflate thread + fr_feed + classify + CSV, like the reference's CLI

usage: python scripts/e2e.py [reads] [gz_reads]
"""
import json
import os
import sys
import tempfile
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from frender_amd import _lib, synth  # noqa: E402
from frender_amd.host import reverse_complement  # noqa: E402
from frender_amd.scan import _sheet_names, frender_scan  # noqa: E402


def host_feed(n, R=8, piece=64 << 20):
    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, R)
    ctx = _lib.Context(device=0, chunk_bytes=256 << 20, table_slots=1 << 22)
    dev = ctx.device_alloc(n * reclen + 64)
    ctx.synth_device(dev, 0, n, R, 1, sheet.idx1, sheet.idx2)
    data = ctx.copy_to_host(dev, n * reclen)
    ctx.device_free(dev)
    names, nid = _sheet_names(sheet.ids)
    idx2rc = [reverse_complement(x) for x in sheet.idx2]
    mv = memoryview(data)

    def run():
        ctx.reset()
        ctx.begin_file(None)
        for off in range(0, len(data), piece):
            ctx.feed(mv[off:off + piece])
        st = ctx.end_file()
        assert st.records == n
        ctx.finalize()
        ctx.set_sheet(sheet.idx1, sheet.idx2, idx2rc, nid, len(names))
        ctx.classify(1, False, to_host=False)
        ctx.sync()

    run()
    t0 = time.perf_counter()
    for _ in range(3):
        run()
    dt = (time.perf_counter() - t0) / 3
    ctx.close()
    return {"path": "host_feed", "reads": n, "bytes_per_record": reclen, "s": round(dt, 4),
            "M_reads_per_s": round(n / dt / 1e6, 1), "GB_per_s": round(n * reclen / dt / 1e9, 2)}


def gz_scan(n, files=4):
    sheet = synth.make_sheet(96, 8, 8)
    with tempfile.TemporaryDirectory() as d:
        paths = synth.make_dataset(d, sheet, n, n_files=files, R=8, seed=1, level=1)
        sheet_csv = os.path.join(d, "sheet.csv")
        with open(sheet_csv, "w") as f:
            f.write("Sample_ID,index,index2\n")
            for name, a, b in zip(sheet.ids, sheet.idx1, sheet.idx2):
                f.write(f"{name},{a},{b}\n")
        args = types.SimpleNamespace(files=paths, b=sheet_csv, n=1, c=files, s=None, rc=False, o=None, p=None)
        cwd = os.getcwd()
        os.chdir(d)
        try:
            t0 = time.perf_counter()
            frender_scan(args)
            dt = time.perf_counter() - t0
        finally:
            os.chdir(cwd)
    return {"path": "gz_scan", "reads": n, "files": files, "s": round(dt, 3),
            "M_reads_per_s": round(n / dt / 1e6, 3)}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    gzn = int(sys.argv[2]) if len(sys.argv) > 2 else 8_000_000
    if n:
        print(json.dumps(host_feed(n)), flush=True)
    print(json.dumps(gz_scan(gzn)), flush=True)
