"""Host-side time of each library call in the bench step (config 2 by default): where the host
blocks (a call that waits on the GPU) and where it falls behind the GPU (gaps in the kernel
trace).  Usage on the GPU box: python scripts/host_timeline.py [--reads N] [--steps K]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from frender_amd import _lib, synth  # noqa: E402
from frender_amd.host import reverse_complement  # noqa: E402
from frender_amd.scan import _sheet_names  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, 8)
    nbytes = a.reads * reclen
    ctx = _lib.Context(device=0, chunk_bytes=(4 << 30) - (1 << 20), table_slots=1 << 22)
    buf = ctx.device_alloc(nbytes + 64)
    ctx.synth_device(buf, 0, a.reads, 8, 1, sheet.idx1, sheet.idx2)
    names, nid = _sheet_names(sheet.ids)
    idx2rc = [reverse_complement(x) for x in sheet.idx2]
    acc = {}

    def timed(name, fn, *args, **kw):
        t = time.perf_counter()
        r = fn(*args, **kw)
        acc.setdefault(name, []).append(time.perf_counter() - t)
        return r

    def step():
        timed("reset", ctx.reset)
        timed("begin_file", ctx.begin_file, None, file_index=0, byte_base=0)
        timed("feed_device", ctx.feed_device, buf, nbytes)
        timed("end_file", ctx.end_file)
        timed("timing", ctx.timing)
        timed("finalize", ctx.finalize)
        timed("set_sheet", ctx.set_sheet, sheet.idx1, sheet.idx2, idx2rc, nid, len(names))
        timed("classify", ctx.classify, 1, False, to_host=False)
        timed("sync", ctx.sync)

    for _ in range(3):
        step()
    acc.clear()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    dt = (time.perf_counter() - t0) / a.steps
    for k, v in acc.items():
        print(f"{k:12s} {1e6 * sum(v) / len(v):9.1f} us")
    print(f"{'step':12s} {1e6 * dt:9.1f} us")


if __name__ == "__main__":
    main()
