#!/bin/bash
# Round 4, call aa: the heavy geometry's shorter ramp-down as the default -- GPU suite, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04aa_pytest.log 2>&1 || { tail -20 gpurun_out/r04aa_pytest.log; exit 1; }
tail -1 gpurun_out/r04aa_pytest.log
ROUNDS=3 timeout -k 10 900 python -u scripts/exp_variants.py $VARIANTS > gpurun_out/r04aa_variants.log 2>&1 || { tail -5 gpurun_out/r04aa_variants.log; exit 1; }
echo variants done
