#!/bin/bash
# Round-4 GPU check: the -m gpu suite, the default bench (config 2 + cpu_baseline + e2e + the
# reference pin), and a rocprofv3 kernel-trace summary of the bench.  TAG names the outputs.
set -o pipefail
TAG=${TAG:-r04}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ ${TESTS:-1} == 1 ]]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/${TAG}_pytest.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
fi
if [[ ${BENCH:-1} == 1 ]]; then
  timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
fi
if [[ ${TRACE:-1} == 1 ]]; then
  rm -rf gpurun_out/prof_trace
  PMC=0 bash scripts/gpu_profile.sh > gpurun_out/${TAG}_prof.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
  head -4 gpurun_out/${TAG}_prof.log | cut -c1-200
fi
