#!/bin/bash
# Round-end pass on one box: the GPU suite, the default bench line, the PMC passes and shape lines
# (scripts/final_shapes.sh), then the config-5 line.  Every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh test || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r05_bench_final.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r05_bench_final.log; exit 1; }
grep "^{" gpurun_out/r05_bench_final.log | tail -1 | cut -c1-300
bash scripts/final_shapes.sh || exit $?
timeout -k 10 900 python -u bench.py --cfg5 --cfg5-pairs 20000000 --cfg5-files 16 > gpurun_out/r05_cfg5_final.log 2>&1 || { echo cfg5 failed; tail -5 gpurun_out/r05_cfg5_final.log; exit 1; }
grep "^{" gpurun_out/r05_cfg5_final.log | tail -1 | cut -c1-300
