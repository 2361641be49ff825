#!/bin/bash
# Where the tally kernel's wave-cycles go (SQ wait/active counters, one --pmc pass), per record.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out/pmcw; export TMPDIR=/tmp
N=${N:-20000000}
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS \
   --output-format csv -d "$R/gpurun_out/pmcw/w" -o run -- python3 "$R/scripts/diag_scale.py" $N 1024 > "$R/gpurun_out/pmcw/w.log" 2>&1 || { echo "pmc failed"; tail -3 "$R/gpurun_out/pmcw/w.log"; exit 1; }
cd "$R"
python3 - <<'PY'
import csv, glob, os
n = int(os.environ.get("N", "20000000"))
tot = {}
for f in glob.glob("gpurun_out/pmcw/w/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("fr::chunk_kernel"):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print("per record:", " ".join(f"{k}={v / n:.2f}" for k, v in sorted(tot.items())))
PY
