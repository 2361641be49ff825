"""Demux row (f-1) on one MI355X with both mates resident in HBM (BASELINE config 5 shape:
96 samples, 8+8 bp, n=1, paired-end; --reads pairs per GPU).  One step = index R1 + index R2
(record starts, R2 code -> destination) + route (stable partition by destination and the
destination-major gather of both mates).  Prints one JSON line; the gzip of the outputs is the
host's part and is not in the timed region.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from frender_amd import _lib, synth  # noqa: E402
from frender_amd.host import reverse_complement  # noqa: E402
from frender_amd.scan import _sheet_names  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, a.read_len)
    n, nbytes = a.reads, a.reads * reclen
    ctx = _lib.Context(device=0, chunk_bytes=1 << 30, table_slots=1 << 22)
    r1 = ctx.device_alloc(nbytes + 64)
    r2 = ctx.device_alloc(nbytes + 64)
    ctx.synth_device(r1, 0, n, a.read_len, 1, sheet.idx1, sheet.idx2)
    ctx.synth_device(r2, 0, n, a.read_len, 1, sheet.idx1, sheet.idx2)  # mate with the same headers
    # the scan results of these records -> destination per code (samples, then und, hop, amb)
    ctx.reset()
    ctx.begin_file(None)
    ctx.feed_device(r1, nbytes)
    ctx.end_file()
    ctx.finalize()
    keys, _, _ = ctx.unique()
    names, nid = _sheet_names(sheet.ids)
    ctx.set_sheet(sheet.idx1, sheet.idx2, [reverse_complement(x) for x in sheet.idx2], nid, len(names))
    c = ctx.classify(1, False)
    S = len(sheet.ids)
    dest = np.where(c["cls"] == 2, c["row"].astype(np.int32),
                    np.where(c["cls"] == 1, S + 1, np.where(c["cls"] == 3, S + 2, S))).astype(np.int32)
    dmx = _lib.Demux(0)
    dmx.set_table(keys, dest)
    n_dest = S + 3

    def step():
        n1 = dmx.load_device(0, r1, nbytes)
        n2 = dmx.load_device(1, r2, nbytes)
        fe, _, b1, b2 = dmx.route(n_dest, min(n1, n2))
        assert fe < 0 and n1 == n2 == n and int(b1.sum()) == nbytes
        return b1

    for _ in range(a.warmup):
        step()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        b1 = step()
    dt = (time.perf_counter() - t0) / a.steps
    moved = 2 * nbytes  # both mates
    print(json.dumps({"metric": "M read pairs/sec demultiplexed (96 samples, 8+8bp, n=1, PE)",
                      "value": round(n / dt / 1e6, 2), "unit": "M read pairs/s", "ms_per_step": round(dt * 1e3, 3),
                      "reads": n, "bytes_per_record": reclen, "decoded_GB_per_s": round(moved / dt / 1e9, 1),
                      "dest_nonempty": int((b1 > 0).sum()), "data": "synthetic SYN-v1 pairs in HBM"}), flush=True)
    dmx.close()
    ctx.device_free(r1)
    ctx.device_free(r2)
    ctx.close()


if __name__ == "__main__":
    main()
