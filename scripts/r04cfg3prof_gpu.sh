#!/bin/bash
# rocprof kernel trace of the config-3 shape bench (384 samples, 10+10, -rc).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/cfg3prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --samples 384 --index-len 10 --rc --no-cpu --steps 5 --warmup 1 > "$R/gpurun_out/cfg3prof.log" 2>&1 || { tail -5 "$R/gpurun_out/cfg3prof.log"; exit 1; }
echo done
