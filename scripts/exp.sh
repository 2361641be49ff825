#!/bin/bash
# A/B: the product library and experimental builds frender_amd/libfrender_hip_exp*.so on the diag workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
N=${N:-100000000}
timeout -k 10 120 python scripts/diag_scale.py $N 1024 > gpurun_out/exp_base.log 2>&1 || { echo base failed; tail -3 gpurun_out/exp_base.log; exit 1; }
echo "base $(grep -o 'records=[0-9]* .*scan_ms=[0-9.]*' gpurun_out/exp_base.log)"
for lib in frender_amd/libfrender_hip_exp*.so; do
  b=$(basename $lib .so)
  env ${EXP_ENV:-} FRENDER_HIP_LIB=$(pwd)/$lib timeout -k 10 120 python scripts/diag_scale.py $N 1024 > gpurun_out/$b.log 2>&1 || { echo $b failed; tail -3 gpurun_out/$b.log; exit 1; }
  echo "$b $(grep -o 'records=[0-9]* .*scan_ms=[0-9.]*' gpurun_out/$b.log)"
done
