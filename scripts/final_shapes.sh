#!/bin/bash
# Round-end measurements on one box: PMC passes at config 2 and at the config-3 shape (their own
# gpurun_out dirs), then the other config shapes and the multi-file step as bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/shapes
if [[ ${MAIN:-1} == 1 ]]; then bash scripts/gpu_profile.sh || exit $?; fi   # MAIN=0: config 2's passes already collected
CFG3="--samples 384 --index-len 10 --rc"
mkdir -p gpurun_out/cfg3
PROF_ARGS="--steps 5 --warmup 1 --no-cpu $CFG3" bash scripts/gpu_profile.sh > gpurun_out/cfg3/profile.log 2>&1 || { echo cfg3 profile failed; exit 1; }
for d in prof_trace prof_fetch prof_write prof_valu; do rm -rf gpurun_out/cfg3/$d; mv gpurun_out/$d gpurun_out/cfg3/$d; done
if [[ ${MAIN:-1} == 1 ]]; then bash scripts/gpu_profile.sh > /dev/null 2>&1 || exit 1; fi   # config 2's passes back in place
run() {  # name, args
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu $2 > gpurun_out/shapes/$1.log 2>&1 || { echo "$1 failed"; tail -3 gpurun_out/shapes/$1.log; exit 1; }
  grep "^{" gpurun_out/shapes/$1.log | tail -1 | cut -c1-200
}
run cfg3 "$CFG3"
run cfg4 "--combinatorial --nsubs 2"
run r150 "--read-len 150 --reads 20000000"
run files8 "--files 8"
run files1 ""
