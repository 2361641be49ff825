"""Collect the tally kernel's rocprofv3 outputs into profiles/ (run here, after gpu_profile.sh).

Reads gpurun_out/prof_trace (kernel-trace --stats) and gpurun_out/prof_fetch / prof_write
(--pmc FETCH_SIZE / --pmc WRITE_SIZE, separate runs), writes
  profiles/<tag>_kernel_stats.csv       the --stats summary
  profiles/<tag>_pmc_<kernel>.csv       per-dispatch FETCH_SIZE / WRITE_SIZE rows of the kernel
  profiles/$TRAFFIC_JSON                HBM bytes per launch, corrected per MI355X_MICROARCH.md:
                                        FETCH_SIZE counts 1/2 of 16-B/lane streaming reads on
                                        gfx950 (x2), both counters in KiB; stamped with the
                                        library's source tree hash (bench.py refuses another tree's)
                                        and, when gpurun_out/prof_fetch_stream exists (a FETCH pass of
                                        the stream-only ablation FR_ABLATE=1), the calibration of the
                                        x2 rule on this kernel's own 16-B/lane tile loads.
usage: python scripts/make_traffic.py <tag> [reads] [read_len] [launches_per_step]
env:   SAMPLES / INDEX_LEN / COMBINATORIAL (the bench shape), RECLEN, PROF_DIR, TRAFFIC_JSON
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "fr::chunk_kernel"
VALU_PEAK_G = 600.0  # 4-cycle VALU class at 4 waves/SIMD, steady state (profiles/r06_ubench_valu.txt, scripts/ubench_valu.hip)


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(ROOT, pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def per_dispatch(rs, counter):
    """Per-dispatch sums of `counter` for the tally kernel.  Only the full-size launches count: a device
    feed's first launches can be smaller (bench.py: the first feed is cut into ranges <= 4 GiB, later
    feeds are one launch), so dispatches under 70 % of the largest FETCH/WRITE/VALU value are dropped."""
    acc = {}
    for r in rs:
        if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]:
            acc[int(r["Dispatch_Id"])] = acc.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    if acc:
        top = max(acc.values())
        acc = {d: v for d, v in acc.items() if v >= 0.7 * top}
    keep = set(acc)
    return acc, [r for r in rs if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]
                 and int(r["Dispatch_Id"]) in keep]


def main():
    tag = sys.argv[1]
    reads = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
    read_len = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    launches = int(sys.argv[4]) if len(sys.argv) > 4 else 7
    reclen = int(os.environ.get("RECLEN", 36 + 8 + 1 + 8 + 1 + 2 * read_len + 4))  # RECLEN: other index lengths
    prof = os.path.join(ROOT, "profiles")
    src = os.environ.get("PROF_DIR", "gpurun_out")
    stats = glob.glob(os.path.join(ROOT, src, "prof_trace/**/*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch, frows = per_dispatch(rows(src + "/prof_fetch/**/*counter_collection.csv"), "FETCH_SIZE")
    write, wrows = per_dispatch(rows(src + "/prof_write/**/*counter_collection.csv"), "WRITE_SIZE")
    with open(os.path.join(prof, f"{tag}_pmc_chunk_kernel.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(frows[0].keys()))
        w.writeheader()
        for r in frows + wrows:
            w.writerow(r)
    sys.path.insert(0, ROOT)
    from frender_amd._lib import source_tree_hash
    fkb = sum(fetch.values()) / len(fetch)
    wkb = sum(write.values()) / len(write)
    alg = reads * reclen / launches
    stream, _ = per_dispatch(rows(src + "/prof_fetch_stream/**/*counter_collection.csv"), "FETCH_SIZE")
    calib = None
    if stream:  # stream-only ablation: every byte read once by 16-B/lane tile loads, nothing else
        skb = sum(stream.values()) / len(stream)
        calib = {"fetch_size_kb_avg": skb, "hbm_bytes_x2": int(2 * skb * 1024),
                 "x2_over_algorithmic": round(2 * skb * 1024 / alg, 4)}
    valu, _ = per_dispatch(rows(src + "/prof_valu/**/*counter_collection.csv"), "SQ_INSTS_VALU")
    vact, _ = per_dispatch(rows(src + "/prof_valu/**/*counter_collection.csv"), "SQ_ACTIVE_INST_VALU")
    valu_d = None
    if valu:  # VALU issue: wave64 instructions against the measured chip ceiling
        vi = sum(valu.values()) / len(valu)
        valu_d = {"insts_per_launch": int(vi), "insts_per_record": round(vi / (reads / launches), 3),
                  "active_quad_cycles_per_launch": int(sum(vact.values()) / len(vact)) if vact else None,
                  "peak_g_insts_per_s": VALU_PEAK_G,
                  "peak_note": "steady state (deadline mode) at 4 waves/SIMD, 2.35-2.38 GHz: v_perm, v_dot4, DPP, v_ffbl, "
                                "64-bit shifts, v_alignbit, v_or3, v_lshl_or, v_bcnt, v_min issue every 4 cycles "
                                "(600 G/s); v_and, v_add, v_lshrrev every ~2 (profiles/r06_ubench_valu.txt)",
                  "mix_ceiling_g_insts_per_s": 666.2}
    # A lower reading of the same counters: the table probes beyond the stream (random 32-B slot reads)
    # are one 64-B FETCH unit each (profiles/r04h_table_pmc/summary.json); x2 assumes each is a 128-B
    # line tallied at 64 B like the streaming loads, x1 that it is a 64-B fill.  Needs the stream-only pass.
    lower = None
    if calib:
        extra_kb = max(fkb - calib["fetch_size_kb_avg"], 0.0)
        lb = 2 * calib["fetch_size_kb_avg"] * 1024 + extra_kb * 1024 + wkb * 1024
        lower = {"hbm_bytes_per_launch": int(lb), "traffic_over_algorithmic": round(lb / alg, 4),
                 "note": "stream fetch x2 (16-B/lane loads, calibrated) + the rest of FETCH_SIZE x1 (table probes "
                         "counted at one 64-B unit each, profiles/r04h_table_pmc) + WRITE_SIZE"}
    # the full-size launches' rocprof duration (the kernel trace of the same command): the --stats average
    # also counts the first feed's smaller launches
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for r in rows(src + "/prof_trace/**/*kernel_trace.csv") if KERNEL in r["Kernel_Name"]]
    full = [d for d in durs if durs and d >= 0.7 * max(durs)]
    out = {
        "round": int(os.environ.get("ROUND", "6")),
        "rocprof_full_launch_ms": round(sum(full) / len(full), 4) if full else None,
        "rocprof_full_launches": len(full),
        "tree_hash": source_tree_hash(),
        "samples": int(os.environ.get("SAMPLES", "96")),
        "index_len": int(os.environ.get("INDEX_LEN", "8")),
        "combinatorial": os.environ.get("COMBINATORIAL", "0") == "1",
        "kernel": KERNEL,
        "reads": reads,
        "read_len": read_len,
        "launches_per_step": launches,
        "algorithmic_bytes_per_launch": alg,
        "fetch_size_kb_avg": fkb,
        "write_size_kb_avg": wkb,
        "correction": "MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE reads 1/2 of a 16-B/lane streaming read "
                      "-> x2; WRITE_SIZE taken as is; units KiB",
        "hbm_bytes_per_launch": int(2 * fkb * 1024 + wkb * 1024),
        "traffic_over_algorithmic": round((2 * fkb * 1024 + wkb * 1024) / alg, 4),
        "fetch_over_algorithmic": round(2 * fkb * 1024 / alg, 4),
        "stream_only_calibration": calib,
        "lower_reading": lower,
        "valu": valu_d,
        "source": f"profiles/{tag}_pmc_chunk_kernel.csv (rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, "
                  f"separate runs of bench.py {os.environ.get('PROF_ARGS', '--steps 5 --warmup 1 --no-cpu')})",
    }
    with open(os.path.join(prof, os.environ.get("TRAFFIC_JSON", "traffic_r06.json")), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
