#!/bin/bash
# Per-stage dynamic instruction counts of the tally kernel by compile-time ablation:
# for the product library and each scripts/build_exp.sh variant named in VARIANTS (default: ab1 ab2 ab4 ab8 =
# FR_ABLATE 1 no header parse, 2 no code encode, 4 no LDS insert, 8 no commit flush), one rocprofv3 --pmc pass
# (SQ counters) and one timed bench run.  Each GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=${OUT:-gpurun_out/ablate}; mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${ARGS:---steps 3 --warmup 1 --no-cpu --no-pin}
CTRS=${CTRS:-SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY}
for v in product ${VARIANTS:-ab1 ab2 ab4 ab8}; do
  if [[ $v == product ]]; then unset FRENDER_HIP_LIB; else export FRENDER_HIP_LIB="$R/frender_amd/libfrender_hip_exp_$v.so"; fi
  timeout -k 10 240 python3 bench.py $ARGS > "$OUT/$v.bench.log" 2>&1 || { echo "bench $v failed"; tail -5 "$OUT/$v.bench.log"; exit 1; }
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d "$R/$OUT/$v" -o run -- python3 "$R/bench.py" $ARGS \
      > "$R/$OUT/$v.pmc.log" 2>&1
  rc=$?; cd "$R"
  if [[ $rc -ne 0 ]]; then echo "pmc $v failed ($rc)"; tail -5 "$OUT/$v.pmc.log"; exit $rc; fi
  python3 scripts/bucket_summary.py "$OUT/$v" > "$OUT/$v.summary.txt" 2>&1
  echo "== $v: $(grep -o '"avg_launch_ms": [0-9.]*' "$OUT/$v.bench.log" | head -1)"
  grep -E "SQ_INSTS_VALU|SQ_INSTS_SALU|SQ_INSTS_LDS|SQ_WAVE_CYCLES|fractions" "$OUT/$v.summary.txt"
done
