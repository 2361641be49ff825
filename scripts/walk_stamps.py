"""Where a wave's time goes in the tally's walk (diagnostic; FR_STAMPS=4 build: scripts/build_exp.sh ws
"-DFR_STAMPS=4").  Per wave, walk_wave adds s_memtime cycles of: 0 the wait for the tile's VMEM loads, 1 the
LDS copy + classify (its LDS read-back included), 2 the rare-event drain + bitmap stores + LDS fence, 3 the
header parse; 4 counts walk steps, 5 sums whole-kernel wave cycles, 6 counts walk calls.  The stamps cost
time themselves (their s_memtime waits on lgkmcnt): read the shares, not the absolute kernel time.
usage: FRENDER_HIP_LIB=frender_amd/libfrender_hip_exp_ws.so python scripts/walk_stamps.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from frender_amd import _lib, synth
    n = int(os.environ.get("READS", "100000000"))
    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, 8)
    ctx = _lib.Context(device=0, chunk_bytes=(16 << 30) - (1 << 20), table_slots=1 << 22)
    buf = ctx.device_alloc(n * reclen + 64)
    ctx.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
    for rep in range(3):  # the last feed is one launch (the first is cut into ranges <= 4 GiB)
        ctx.reset()
        ctx.begin_file(None, file_index=0, byte_base=0)
        ctx.feed_device(buf, n * reclen)
        ctx.end_file()
        ctx.sync()
        if rep == 1:
            d0 = ctx.diag().get("stamps", {})
    d1 = ctx.diag().get("stamps", {})
    v = [b - a for a, b in zip(d0.values(), d1.values())] if d0 else list(d1.values())
    if any(x < 0 for x in v):  # fr_reset zeroed the stamps between the feeds: the last feed's own
        v = list(d1.values())
    names = ("vmem_wait", "copy_classify", "drain_bitmaps", "parse")
    walk = sum(v[:4])
    out = {"raw_last_feed": v, "walk_steps": v[4], "walk_calls": v[6], "kernel_wave_cycles": v[5],
           "walk_share_of_kernel": round(walk / v[5], 4) if v[5] else None,
           "walk_phase_frac": {k: round(x / walk, 4) for k, x in zip(names, v[:4])} if walk else None,
           "cycles_per_step": {k: round(x / v[4], 1) for k, x in zip(names, v[:4])} if v[4] else None}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)
    ctx.device_free(buf)
    ctx.close()


if __name__ == "__main__":
    main()
