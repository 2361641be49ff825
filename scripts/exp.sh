#!/bin/bash
# A/B: the product library and experimental builds frender_amd/libfrender_hip_exp*.so on the diag
# workload (CH = launch MiB, EXP_ENV applied to every arm).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
N=${N:-100000000}; CH=${CH:-4095}
for rep in $(seq ${REPS:-1}); do
for lib in frender_amd/libfrender_hip.so frender_amd/libfrender_hip_exp*.so; do
  b=$(basename $lib .so)
  env ${EXP_ENV:-} FRENDER_HIP_LIB=$(pwd)/$lib timeout -k 10 120 python scripts/diag_scale.py $N $CH > gpurun_out/$b.log 2>&1 || { echo $b failed; tail -3 gpurun_out/$b.log; exit 1; }
  echo "$b $(grep -o 'launches=[0-9]* scan_ms=[0-9.]*' gpurun_out/$b.log)"
done
done
