#!/bin/bash
# Round 4, call ab: ramp-up start sizes, interleaved A/B (4 rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUNDS=${ROUNDS:-4} timeout -k 10 1000 python -u scripts/exp_variants.py $VARIANTS > gpurun_out/r04ab_variants.log 2>&1 || { tail -5 gpurun_out/r04ab_variants.log; exit 1; }
echo variants done
