#!/bin/bash
# Round-2 tally-kernel probe: timing under FR_ABLATE settings (1 no parse, 2 no encode, 4 no insert,
# 8 no HBM flush) on the diag workload, then SQ instruction counters (one --pmc pass per group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out/probe; export TMPDIR=/tmp
N=${N:-100000000}; CH=${CH:-4095}
for ab in ${ABL:-0 1 2 4 8 12}; do
  FR_ABLATE=$ab timeout -k 10 120 python scripts/diag_scale.py $N $CH > gpurun_out/probe/ab$ab.log 2>&1 || { echo "ablate $ab failed"; tail -3 gpurun_out/probe/ab$ab.log; exit 1; }
  echo "ablate=$ab $(grep -o 'launches=[0-9]* scan_ms=[0-9.]*' gpurun_out/probe/ab$ab.log)"
done
if [[ ${SQ:-1} == 1 ]]; then
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/probe/sq$i" -o run \
      -- python3 "$R/scripts/diag_scale.py" $N $CH > "$R/gpurun_out/probe/sq$i.log" 2>&1 || { echo "sq group $i failed"; tail -3 "$R/gpurun_out/probe/sq$i.log"; exit 1; }
done
cd "$R"
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/probe/sq*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "chunk_kernel" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:24s} per launch {sum(v)/len(v):.4g} ({len(v)} launches)")
PY
fi
