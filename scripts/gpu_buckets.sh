#!/bin/bash
# SQ wave-cycle buckets of the tally kernel (MI355X_MICROARCH.md "rocprofv3 PMC slots": SQ_WAIT_ANY,
# SQ_WAIT_INST_ANY and SQ_ACTIVE_INST_ANY are disjoint and sum to ~SQ_WAVE_CYCLES), plus the issue
# counters per instruction class.  One rocprofv3 --pmc pass per counter group (<= 8 SQ counters each),
# each under its own hard time limit; counters the box does not list are dropped from a pass.
#   LIB: library suffix (frender_amd/libfrender_hip_exp_<LIB>.so), default the product library
#   ARGS: bench.py arguments (default the config-2 headline, 3 steps)
#   OUT: output directory under gpurun_out (default gpurun_out/buckets)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/buckets}
mkdir -p "$OUT"
ARGS=${ARGS:---steps 3 --warmup 1 --no-cpu --no-pin}
if [[ -n "${LIB:-}" ]]; then export FRENDER_HIP_LIB="$R/frender_amd/libfrender_hip_exp_${LIB}.so"; fi
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$R/$OUT/counters.txt" 2>&1 || true
cd "$R"
PASSES=(  # (not GROUPS: bash's own array of the user's group ids)
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES"
  "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS"
  "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
  "SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL"
)
i=0
for g in "${PASSES[@]}"; do
  i=$((i + 1))
  keep=""
  for c in $g; do
    if grep -qw "$c" "$OUT/counters.txt"; then keep="$keep $c"; fi
  done
  if [[ -z "$keep" ]]; then echo "group $i: no listed counter"; continue; fi
  echo "group $i:$keep"
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc $keep --output-format csv -d "$R/$OUT/g$i" -o run \
      -- python3 "$R/bench.py" $ARGS > "$R/$OUT/g$i.log" 2>&1
  rc=$?
  cd "$R"
  if [[ $rc -ne 0 ]]; then echo "pass $i failed ($rc)"; tail -5 "$OUT/g$i.log"; exit $rc; fi
done
python3 scripts/bucket_summary.py "$OUT" > "$OUT/summary.txt" 2>&1 || true
cat "$OUT/summary.txt"
