#!/bin/bash
# GPU: the tally-kernel GPU tests (scan parity) with the product library, then an A/B of the product
# library against frender_amd/libfrender_hip_exp*.so on the diag workload (scripts/exp.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [[ ${TESTS:-1} == 1 ]]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider ${PYTEST_K:-} > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [[ $rc -ne 0 ]] && { grep -E "FAIL|Error|assert" gpurun_out/ab_tests.log | head -20; exit $rc; }
fi
REPS=${REPS:-2} bash scripts/exp.sh
