#!/bin/bash
# Round 4, call u: the commit's phases (FR_STAMPS=2 build), then A/B of the joint resolve.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
FRENDER_HIP_LIB=frender_amd/libfrender_hip_exp_cs.so timeout -k 10 180 python -u scripts/commit_stamps.py > gpurun_out/r04u_commit_stamps.json 2> gpurun_out/r04u_commit_stamps.err || { tail -5 gpurun_out/r04u_commit_stamps.err; exit 1; }
echo stamps done
ROUNDS=3 timeout -k 10 600 python -u scripts/exp_variants.py main joint > gpurun_out/r04u_variants.log 2>&1 || { tail -5 gpurun_out/r04u_variants.log; exit 1; }
tail -1 gpurun_out/r04u_variants.log | cut -c1-1500
