#!/bin/bash
# Kernel trace of the bench with every commit logged (FR_LOG_MIN=0): the launch-log aggregation's own
# kernels (split, reduce) per launch, beside the tally.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
FR_LOG_MIN=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/logtrace" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/logtrace.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/logtrace.log"; exit 1; }
cd "$R"
grep -E "chunk_kernel|log_split|log_reduce" gpurun_out/logtrace/run_kernel_stats.csv | cut -c1-160
