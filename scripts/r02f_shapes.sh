#!/bin/bash
# r02f: the other BASELINE config shapes on one GPU + the 2-rank rehearsal (gloo, one GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --samples 384 --index-len 10 --rc > gpurun_out/cfg3.log 2>&1 || { echo cfg3 failed; tail -5 gpurun_out/cfg3.log; exit 1; }
grep '^{' gpurun_out/cfg3.log | cut -c1-600
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --combinatorial --nsubs 2 > gpurun_out/cfg4.log 2>&1 || { echo cfg4 failed; tail -5 gpurun_out/cfg4.log; exit 1; }
grep '^{' gpurun_out/cfg4.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --reads 20000000 --read-len 150 > gpurun_out/r150.log 2>&1 || { echo r150 failed; tail -5 gpurun_out/r150.log; exit 1; }
grep '^{' gpurun_out/r150.log | cut -c1-300
bash scripts/gpu_check.sh dist
