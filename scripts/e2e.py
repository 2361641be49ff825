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


def _bgzf(data: bytes, block: int = 65280, level: int = 1) -> bytes:
    import struct
    import zlib
    out = []
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = c.compress(chunk) + c.flush()
        bsize = 18 + len(body) + 8
        out.append(b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<HBBHH", 6, 66, 67, 2, bsize - 1)
                   + body + struct.pack("<II", zlib.crc32(chunk), len(chunk)))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def gz_scan(n, files=4, cores=None, bgzf=False):
    sheet = synth.make_sheet(96, 8, 8)
    with tempfile.TemporaryDirectory() as d:
        if bgzf:  # BGZF members: the native inflate splits each file across threads
            paths = []
            for f in range(files):
                p = os.path.join(d, f"syn_L{f + 1:03d}_R1_001.fastq.gz")
                with open(p, "wb") as fh:
                    fh.write(_bgzf(synth.generate_bytes(sheet, f * (n // files), n // files, R=8, seed=1)))
                paths.append(p)
        else:
            paths = synth.make_dataset(d, sheet, n, n_files=files, R=8, seed=1, level=1)
        sheet_csv = os.path.join(d, "sheet.csv")
        with open(sheet_csv, "w") as f:
            f.write("Sample_ID,index,index2\n")
            for name, a, b in zip(sheet.ids, sheet.idx1, sheet.idx2):
                f.write(f"{name},{a},{b}\n")
        cores = cores or files
        args = types.SimpleNamespace(files=paths, b=sheet_csv, n=1, c=cores, s=None, rc=False, o=None, p=None)
        cwd = os.getcwd()
        os.chdir(d)
        try:
            t0 = time.perf_counter()
            frender_scan(args)
            dt = time.perf_counter() - t0
        finally:
            os.chdir(cwd)
    return {"path": "gz_scan" + ("_bgzf" if bgzf else ""), "reads": n, "files": files, "inflate_threads": cores,
            "s": round(dt, 3), "M_reads_per_s": round(n / dt / 1e6, 3)}


def gz_demux(n, files=2, level=9):
    """The whole `demux` command over `files` R1/R2 .fastq.gz pairs of n/files pairs each."""
    import csv

    import numpy as np

    from frender_amd.demux import frender_demux

    sheet = synth.make_sheet(96, 8, 8)
    with tempfile.TemporaryDirectory() as d:
        per = n // files
        codes_total = {}
        for f in range(files):
            t1 = synth.generate_bytes(sheet, f * per, per, R=150, seed=1)
            t2 = t1.replace(b" 1:N:0:", b" 2:N:0:")
            synth.write_fastq_gz(os.path.join(d, f"syn_L{f + 1:03d}_R1_001.fastq.gz"), t1, level=1)
            synth.write_fastq_gz(os.path.join(d, f"syn_L{f + 1:03d}_R2_001.fastq.gz"), t2, level=1)
            ctx = _lib.Context(device=0, chunk_bytes=256 << 20, table_slots=1 << 20)
            ctx.reset()
            ctx.begin_file(None)
            ctx.feed(t1)
            ctx.end_file()
            ctx.finalize()
            keys, counts, _ = ctx.unique()
            names, nid = _sheet_names(sheet.ids)
            ctx.set_sheet(sheet.idx1, sheet.idx2, [reverse_complement(x) for x in sheet.idx2], nid, len(names))
            c = ctx.classify(1, False)
            ctx.close()
            kinds = ("undetermined", "index_hop", "demuxable", "ambiguous")
            for code, cls, row in zip(_lib.decode_keys(keys), c["cls"].tolist(), c["row"].tolist()):
                codes_total[code] = (kinds[cls], sheet.ids[row] if cls == 2 else "")
        res = os.path.join(d, "results.csv")
        with open(res, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["idx1", "idx2", "reads", "matched_idx1", "matched_idx2", "read_type", "sample_name", "demux_ok"])
            for code, (t, sid) in codes_total.items():
                a, b = code.split("+")[0:2]
                w.writerow([a, b, 1, "", "", t, sid, True])
        ins = sorted(os.path.join(d, x) for x in os.listdir(d) if x.endswith(".gz"))
        args = types.SimpleNamespace(r=res, d=os.path.join(d, "out"), o=None, no_index_hop=False, no_ambiguous=False,
                                     no_undeter=False, no_samples=False, files=ins, gz_level=level)
        t0 = time.perf_counter()
        frender_demux(args)
        dt = time.perf_counter() - t0
        out_bytes = sum(os.path.getsize(os.path.join(args.d, x)) for x in os.listdir(args.d))
    return {"path": "gz_demux", "read_pairs": per * files, "files": files, "gz_level": level, "s": round(dt, 3),
            "M_pairs_per_s": round(per * files / dt / 1e6, 3), "out_gz_bytes": out_bytes}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    gzn = int(sys.argv[2]) if len(sys.argv) > 2 else 8_000_000
    if n:
        print(json.dumps(host_feed(n)), flush=True)
    if gzn:
        print(json.dumps(gz_scan(gzn)), flush=True)
        print(json.dumps(gz_scan(2 * gzn, files=8)), flush=True)
        print(json.dumps(gz_scan(gzn, files=16)), flush=True)
        print(json.dumps(gz_scan(gzn, files=4, bgzf=True)), flush=True)
        print(json.dumps(gz_scan(2 * gzn, files=1, cores=16, bgzf=True)), flush=True)
    dmn = int(sys.argv[3]) if len(sys.argv) > 3 else 2_000_000
    if dmn:
        for lvl in (9, 1):
            print(json.dumps(gz_demux(dmn, level=lvl)), flush=True)
