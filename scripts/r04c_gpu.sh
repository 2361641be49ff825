#!/bin/bash
# Round 4, call c: the VALU microbenchmark with real-time clock stamps, the -m gpu suite, the default
# bench, and an interleaved A/B of the tally-kernel variants built by scripts/build_exp.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04c}
if [[ ${UBENCH:-1} == 1 ]]; then
  timeout -k 10 240 ./scripts/ubench_valu 20000 > gpurun_out/${TAG}_ubench_valu.txt 2>&1 || { tail -5 gpurun_out/${TAG}_ubench_valu.txt; exit 1; }
  echo ubench done
fi
if [[ ${TESTS:-1} == 1 ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest.log
fi
if [[ ${BENCH:-1} == 1 ]]; then
  timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
fi
if [[ -n ${VARIANTS:-} ]]; then
  ROUNDS=${ROUNDS:-2} timeout -k 10 600 python -u scripts/exp_variants.py $VARIANTS > gpurun_out/${TAG}_variants.log 2>&1 || { tail -5 gpurun_out/${TAG}_variants.log; exit 1; }
  tail -1 gpurun_out/${TAG}_variants.log | cut -c1-1500
fi
if [[ ${E2E:-0} == 1 ]]; then
  timeout -k 10 400 python -u scripts/e2e_profile.py > gpurun_out/${TAG}_e2e_profile.txt 2>&1 || { tail -5 gpurun_out/${TAG}_e2e_profile.txt; exit 1; }
  grep "scan s" gpurun_out/${TAG}_e2e_profile.txt
fi
if [[ ${TRACE:-0} == 1 ]]; then
  PMC=${PMC:-0} bash scripts/gpu_profile.sh > gpurun_out/${TAG}_prof.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
  tail -12 gpurun_out/${TAG}_prof.log | cut -c1-250
fi
if [[ ${CFG5:-0} == 1 ]]; then
  timeout -k 10 600 python -u bench.py --cfg5 > gpurun_out/${TAG}_cfg5.log 2>&1 || { tail -5 gpurun_out/${TAG}_cfg5.log; exit 1; }
  tail -1 gpurun_out/${TAG}_cfg5.log | cut -c1-400
fi
