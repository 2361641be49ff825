#!/bin/bash
# Tally-kernel time under env settings: VAR="v1 v2 ..." NAME=FR_FLUSH_AT bash scripts/env_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
N=${N:-100000000}
for v in $VALS; do
  env $NAME=$v timeout -k 10 120 python scripts/diag_scale.py $N ${CH:-4095} > gpurun_out/env_${NAME}_$v.log 2>&1 || { echo "$NAME=$v failed"; tail -3 gpurun_out/env_${NAME}_$v.log; exit 1; }
  echo "$NAME=$v $(grep -o 'scan_ms=[0-9.]*' gpurun_out/env_${NAME}_$v.log) $(grep -o "'spin_total': [0-9]*" gpurun_out/env_${NAME}_$v.log)"
done
