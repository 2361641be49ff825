#!/bin/bash
# A/B over (library, env) arms on the diag workload: ARMS="lib1|ENV=1 ENV2=2;lib2|" (lib relative to
# frender_amd/, env may be empty).  DIAG_S / DIAG_L select the sheet shape, N the reads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
N=${N:-100000000}; CH=${CH:-4095}
IFS=';' read -ra A <<< "$ARMS"
for rep in $(seq ${REPS:-2}); do
  for arm in "${A[@]}"; do
    lib=${arm%%|*}; envs=${arm#*|}
    env $envs FRENDER_HIP_LIB=$(pwd)/frender_amd/$lib timeout -k 10 120 python scripts/diag_scale.py $N $CH > gpurun_out/ab_env.log 2>&1 || { echo "$arm failed"; tail -3 gpurun_out/ab_env.log; exit 1; }
    echo "$lib [$envs] $(grep -o 'launches=[0-9]* scan_ms=[0-9.]* log_ms=[0-9.]*' gpurun_out/ab_env.log)"
  done
done
