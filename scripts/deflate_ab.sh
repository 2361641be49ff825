#!/bin/bash
# A/B of deflate variants built by scripts/build_exp.sh: scripts/deflate_ab.sh OUT NAME... (each
# runs scripts/deflate_bench.py 512 97 3 against libfrender_hip_exp_NAME.so; FRD_PROF builds also
# print their phase ticks)
set -eu
cd "$(dirname "$0")/.."
out=$1
shift
mkdir -p "$(dirname "$out")"
for v in "$@"; do
  echo "== $v" >> "$out"
  FRENDER_HIP_LIB=frender_amd/libfrender_hip_exp_$v.so timeout -k 10 180 python -u scripts/deflate_bench.py 512 97 3 >> "$out" 2>&1
done
