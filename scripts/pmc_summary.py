"""Sum the pmc_sq.sh counter groups for fr::chunk_kernel and print per-record figures."""
import csv, glob, os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
tot = {}
for f in sorted(glob.glob(os.path.join(R, "gpurun_out/pmc/g*/**/*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if "fr::chunk_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k:32s} {tot[k]:16.4g}  per record {tot[k] / n:10.3f}")
