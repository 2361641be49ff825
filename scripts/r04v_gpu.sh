#!/bin/bash
# Round 4, call v: GPU suite on the static-first-chunk / parameterized-ramp tree, the A/B of ticket
# and ramp variants, and the timeline of the new default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04v_pytest.log 2>&1 || { tail -20 gpurun_out/r04v_pytest.log; exit 1; }
tail -1 gpurun_out/r04v_pytest.log
ROUNDS=2 timeout -k 10 900 python -u scripts/exp_variants.py $VARIANTS > gpurun_out/r04v_variants.log 2>&1 || { tail -5 gpurun_out/r04v_variants.log; exit 1; }
echo variants done
FRENDER_HIP_LIB=frender_amd/libfrender_hip_exp_tl.so timeout -k 10 180 python -u scripts/chunk_timeline.py > gpurun_out/r04v_timeline.json 2> gpurun_out/r04v_timeline.err || { tail -5 gpurun_out/r04v_timeline.err; exit 1; }
echo timeline done
