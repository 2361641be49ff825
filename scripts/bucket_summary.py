"""Summarise scripts/gpu_buckets.sh's SQ counter passes for fr::chunk_kernel.

usage: python scripts/bucket_summary.py <dir under gpurun_out> [records_per_launch] [bytes_per_launch] [out.json]

Per counter: the mean over the kernel's full-size dispatches (>= 70 % of the largest SQ_WAVE_CYCLES /
counter value: a device feed's first launches can be smaller).  The wave-cycle buckets
(MI355X_MICROARCH.md "rocprofv3 PMC slots"): SQ_WAIT_ANY (wave parked on s_waitcnt / barrier),
SQ_WAIT_INST_ANY (issue stall: dependency / pipe busy), SQ_ACTIVE_INST_ANY (issuing), disjoint, summing to
about SQ_WAVE_CYCLES.  SQ_*CYCLES counters are in quad-cycles (the guide's cycle-constants table)."""
import csv
import glob
import json
import os
import sys

KERNEL = "fr::chunk_kernel"


def load(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if KERNEL not in r["Kernel_Name"]:
                    continue
                key = (os.path.dirname(f), int(r["Dispatch_Id"]))
                per.setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
                per[r["Counter_Name"]][key] += float(r["Counter_Value"])
    out = {}
    for c, acc in per.items():
        top = max(acc.values())
        vals = [v for v in acc.values() if v >= 0.7 * top] if top > 0 else list(acc.values())
        out[c] = sum(vals) / len(vals)
    return out


def main():
    d = sys.argv[1]
    recs = float(sys.argv[2]) if len(sys.argv) > 2 else 1e8
    nbytes = float(sys.argv[3]) if len(sys.argv) > 3 else 7.4e9
    m = load(d)
    for k in sorted(m):
        print(f"{k:28s} {m[k]:18.6g}   per record {m[k] / recs:9.4f}")
    res = {"counters_mean_per_full_launch": m, "records_per_launch": recs, "bytes_per_launch": nbytes}
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        b = {k: m[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                     "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA",
                                     "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS") if k in m}
        res["fraction_of_wave_cycles"] = b
        print("fractions of SQ_WAVE_CYCLES:", json.dumps({k: round(v, 4) for k, v in b.items()}))
        if all(k in b for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")):
            s = b["SQ_WAIT_ANY"] + b["SQ_WAIT_INST_ANY"] + b["SQ_ACTIVE_INST_ANY"]
            print(f"WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = {s:.4f} of WAVE_CYCLES")
            res["bucket_sum"] = s
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
