#!/bin/bash
# Round 4: the other BASELINE config shapes on one GPU (per-GPU shapes of the 8-GPU configs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --samples 384 --index-len 10 --rc --no-cpu > gpurun_out/r04_cfg3_shape.log 2>&1 || { tail -5 gpurun_out/r04_cfg3_shape.log; exit 1; }
tail -1 gpurun_out/r04_cfg3_shape.log | cut -c1-200
timeout -k 10 400 python -u bench.py --combinatorial --nsubs 2 --no-cpu > gpurun_out/r04_cfg4_shape.log 2>&1 || { tail -5 gpurun_out/r04_cfg4_shape.log; exit 1; }
tail -1 gpurun_out/r04_cfg4_shape.log | cut -c1-200
timeout -k 10 400 python -u bench.py --read-len 150 --reads 20000000 --no-cpu > gpurun_out/r04_r150.log 2>&1 || { tail -5 gpurun_out/r04_r150.log; exit 1; }
tail -1 gpurun_out/r04_r150.log | cut -c1-200
