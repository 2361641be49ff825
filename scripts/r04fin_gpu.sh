#!/bin/bash
# Round 4, final call: GPU suite, default bench, rocprof trace + PMC passes + stream calibration, and the
# collective census of a 2-rank scan (gloo on one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04fin} bash scripts/r04y_gpu.sh || exit 1
GPUS="1 2" FILES=4 READS=1000000 timeout -k 10 400 python -u scripts/census.py > gpurun_out/${TAG:-r04fin}_census.json 2> gpurun_out/${TAG:-r04fin}_census.err || { tail -5 gpurun_out/${TAG:-r04fin}_census.err; exit 1; }
echo census done
