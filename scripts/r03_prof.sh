#!/bin/bash
# r03 profiles of this tree: config 2 (kernel trace --stats, FETCH_SIZE, WRITE_SIZE, stream-only
# FETCH_SIZE calibration), then the config-3 shape (trace + FETCH + WRITE), each set under gpurun_out/<name>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
rm -rf gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/prof_fetch_stream gpurun_out/c2 gpurun_out/c3
STREAM=1 bash scripts/gpu_profile.sh || exit 1
mkdir -p gpurun_out/c2 && mv gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/prof_fetch_stream gpurun_out/c2/
PROF_ARGS="--steps 5 --warmup 1 --no-cpu --samples 384 --index-len 10 --rc" bash scripts/gpu_profile.sh || exit 1
mkdir -p gpurun_out/c3 && mv gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/c3/
