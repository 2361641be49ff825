#!/bin/bash
# SQ instruction/cycle/i-cache counters for the tally kernel (diag workload), one --pmc pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
N=${N:-20000000}
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VSKIPPED"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmc/g$i" -o run \
      -- python3 "$R/scripts/diag_scale.py" $N 1024 > "$R/gpurun_out/pmc/g$i.log" 2>&1 || { echo "group $i failed"; tail -3 "$R/gpurun_out/pmc/g$i.log"; exit 1; }
done
echo done
