#!/bin/bash
# Tally-kernel SQ counters per record, one --pmc pass per counter group (PASSES="c1 c2 ...;c3 ...").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out/pmcw; export TMPDIR=/tmp
N=${N:-20000000}
PASSES=${PASSES:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS"}
i=0
IFS=';' read -ra GROUPS_ <<< "$PASSES"
for g in "${GROUPS_[@]}"; do
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$R/gpurun_out/pmcw/p$i" -o run \
     -- python3 "$R/scripts/diag_scale.py" $N ${CH:-4095} > "$R/gpurun_out/pmcw/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -3 "$R/gpurun_out/pmcw/p$i.log"; exit 1; }
  cd "$R"; i=$((i+1))
done
python3 - <<'PY'
import csv, glob, os
n = int(os.environ.get("N", "20000000"))
tot = {}
for f in glob.glob("gpurun_out/pmcw/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("fr::chunk_kernel"):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print("per record:", " ".join(f"{k}={v / n:.3f}" for k, v in sorted(tot.items())))
PY
