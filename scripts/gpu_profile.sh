#!/bin/bash
# rocprofv3 kernel-trace summary of the bench (profiles/), then PMC passes (FETCH_SIZE / WRITE_SIZE)
# in their own runs, per MI355X_MICROARCH.md (separate --pmc passes, no trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${PROF_ARGS:---steps 5 --warmup 1 --no-cpu}
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace" -o run --output-format csv \
    -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof_trace.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/prof_trace.log"; exit 1; }
if [[ ${PMC:-1} == 1 ]]; then
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof_fetch" -o run \
      -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof_fetch.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof_write" -o run \
      -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof_write.log" 2>&1 || { echo "pmc write failed"; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d "$R/gpurun_out/prof_valu" -o run \
      -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof_valu.log" 2>&1 || { echo "pmc valu failed"; exit 1; }
fi
if [[ ${STREAM:-0} == 1 ]]; then  # calibration: FETCH_SIZE of the stream-only ablation (no parse, no table):
  # the experiment build scripts/build_exp.sh stream "-DFR_ABLATE=1" (ablations are compile-time only)
  FRENDER_HIP_LIB="$R/frender_amd/libfrender_hip_exp_stream.so" timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof_fetch_stream" -o run \
      -- python3 "$R/bench.py" $ARGS --pin-json "$R/no-pin-for-the-ablation.json" > "$R/gpurun_out/prof_fetch_stream.log" 2>&1 || { echo "pmc stream fetch failed"; exit 1; }
fi
cd "$R"
find gpurun_out/prof_trace -name "*kernel_stats.csv" | head -1 | xargs cat | head -20
