"""The commit's phases at the bench workload (diagnostic; FR_STAMPS=2 build: scripts/build_exp.sh cs
"-DFR_STAMPS=2").  Per wave, commit_buffers adds s_memtime cycles of: the entry barrier, the LDS slots'
resolve, the cold batch's resolve, the applies + exotic + note, the LDS barrier, the LDS reset; and the
live LDS slots and cold entries.  Printed per commit (4 waves per commit) in microseconds at the clock
given by CLOCK_GHZ (the kernel's s_memtime rate, profiles/r04c_ubench_valu.txt: ~2.37).
usage: FRENDER_HIP_LIB=frender_amd/libfrender_hip_exp_cs.so python scripts/commit_stamps.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from frender_amd import _lib, synth
    n = int(os.environ.get("READS", "100000000"))
    ghz = float(os.environ.get("CLOCK_GHZ", "2.37"))
    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, 8)
    ctx = _lib.Context(device=0, chunk_bytes=(4 << 30) - (1 << 20), table_slots=1 << 22)
    buf = ctx.device_alloc(n * reclen + 64)
    ctx.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
    for rep in range(2):
        ctx.reset()
        ctx.begin_file(None, file_index=0, byte_base=0)
        ctx.feed_device(buf, n * reclen)
        ctx.end_file()
        ctx.sync()
    d = ctx.diag()
    st = d.get("stamps", {})
    v = list(st.values())
    t = ctx.timing()
    commits = t.scan_launches  # placeholder for the per-launch count below
    names = ("entry_barrier", "resolve_lds", "resolve_cold", "apply_exo_note", "lds_barrier", "reset")
    # stamps 6, 7: live LDS slots and cold entries summed by lane 0 of every wave (4 per commit)
    waves = None
    out = {"raw": st}
    if len(v) == 8 and v[6]:
        nl_sum, nc_sum = v[6], v[7]
        out["per_wave_us"] = {}
        # commits = waves / 4; the per-commit means need the commit count: the LDS-slot mean is known per
        # commit from the FR_STAMPS=2 build only through the sums, so report per-wave totals and ratios
        tot = sum(v[:6])
        out["phase_frac"] = {k: round(x / tot, 4) for k, x in zip(names, v[:6])}
        out["total_commit_wave_us"] = round(tot / ghz / 1e3, 1)
        out["lds_slots_sum_x4"] = nl_sum
        out["cold_sum_x4"] = nc_sum
    out["scan_ms"] = t.scan_ms
    print(json.dumps(out, indent=1))
    ctx.device_free(buf)
    ctx.close()


if __name__ == "__main__":
    main()
