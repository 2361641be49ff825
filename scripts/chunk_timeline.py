"""Timeline of the tally launches (diagnostic): where a launch's time goes beyond the steady walk.

Needs the FR_STAMPS=3 build (scripts/build_exp.sh tl "-DFR_STAMPS=3"), which records per chunk
{workgroup, XCD, tiles, ticket time, walked time, committed time} and per workgroup {entry, exit}
with s_memrealtime (100 MHz).  Runs the bench workload (config 2: 100M SYN-v1 reads in HBM, two
3.7-GB launches), one warm step, then one traced step, and prints per launch:
  span        first workgroup entry -> last exit
  ramp-in     entry -> first ticket, per workgroup (launch start skew)
  tail        each workgroup's exit -> the launch's last exit (idle at the end)
  busy        sum over chunks of ticket -> committed, / (span x workgroups)
  by chunk size: walk and commit time per tile for ramp and full chunks
usage: FRENDER_HIP_LIB=frender_amd/libfrender_hip_exp_tl.so python scripts/chunk_timeline.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TRACE_CHUNKS, TRACE_WGS = 1 << 14, 4096


def main():
    from frender_amd import _lib, synth
    n = int(os.environ.get("READS", "100000000"))
    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, 8)
    ctx = _lib.Context(device=0, chunk_bytes=(4 << 30) - (1 << 20), table_slots=1 << 22)
    buf = ctx.device_alloc(n * reclen + 64)
    ctx.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
    L = _lib.lib
    L.fr_trace_read.argtypes = [C.c_void_p, C.c_void_p]
    chunks = np.zeros(2 * TRACE_CHUNKS * 4, dtype=np.uint64)
    wgs = np.zeros(2 * TRACE_WGS * 2, dtype=np.uint64)
    out = {}
    for rep in range(3):
        if rep == 2:
            assert L.fr_trace_clear() == 0
        ctx.reset()
        ctx.begin_file(None, file_index=0, byte_base=0)
        ctx.feed_device(buf, n * reclen)
        st = ctx.end_file()
        assert st.records == n
        ctx.sync()
    assert L.fr_trace_read(chunks.ctypes.data, wgs.ctypes.data) == 0
    ch = chunks.reshape(2, TRACE_CHUNKS, 4)
    wg = wgs.reshape(2, TRACE_WGS, 2)
    for par in range(2):
        w = wg[par]
        w = w[w[:, 0] != 0].astype(np.int64)
        c = ch[par]
        c = c[c[:, 3] != 0]
        if not len(w):
            continue
        t0 = int(w[:, 0].min())
        info = c[:, 0].astype(np.int64)
        wid, xcc, tiles = info & 0xFFFF, (info >> 16) & 0xFFFF, info >> 32
        tk, tw, tc = (c[:, k].astype(np.int64) - t0 for k in (1, 2, 3))
        ent, ext = w[:, 0] - t0, w[:, 1] - t0
        span = int(ext.max())
        first_ticket = np.full(len(w), -1)
        for i in range(len(w)):
            m = wid == i
            if m.any():
                first_ticket[i] = int(tk[m].min())
        busy = float((tc - tk).sum())
        full = tiles == tiles.max()
        d = {
            "chunks": int(len(c)), "workgroups": int(len(w)), "span_us": span / 100.0,
            "entry_skew_us": [float(np.percentile(ent, q)) / 100 for q in (0, 50, 90, 100)],
            "first_ticket_us": [float(np.percentile(first_ticket, q)) / 100 for q in (0, 50, 90, 100)],
            "exit_us": [float(np.percentile(ext, q)) / 100 for q in (0, 10, 50, 90, 100)],
            "tail_idle_frac": float((span - ext).sum()) / (span * len(w)),
            "head_idle_frac": float(first_ticket.sum()) / (span * len(w)),
            "busy_frac": busy / (span * len(w)),
            "walk_ns_per_tile_full": float(((tw - tk)[full] * 10).sum() / tiles[full].sum()),
            "commit_us_full": float(np.median((tc - tw)[full])) / 100,
            "walk_ns_per_tile_small": float(((tw - tk)[~full] * 10).sum() / max(1, tiles[~full].sum())),
            "commit_us_small": float(np.median((tc - tw)[~full])) / 100 if (~full).any() else None,
            "tiles_small_frac": float(tiles[~full].sum() / tiles.sum()),
            "by_xcc_walk_ns_per_tile": {int(x): round(float(((tw - tk)[xcc == x] * 10).sum() / tiles[xcc == x].sum()), 1)
                                        for x in np.unique(xcc)},
        }
        # idle after each workgroup's last chunk, and the last chunks' sizes
        order = np.argsort(tc)
        d["last_16_chunks"] = [[int(tiles[i]), round(float(tc[i] - tk[i]) / 100, 1), int(xcc[i])]
                               for i in order[-16:]]
        out[f"launch{par}"] = d
    print(json.dumps(out, indent=1))
    ctx.device_free(buf)
    ctx.close()


if __name__ == "__main__":
    main()
