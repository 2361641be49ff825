#!/bin/bash
# A/B of commit modes on the config-2 and config-3 diag shapes (scan_ms = tally launches, log_ms =
# launch-log aggregation), env arms in ARMS (e.g. "FR_LOG=0 FR_LOG_MIN=432").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for shape in "96 8" "384 10"; do
  set -- $shape
  for lib in frender_amd/libfrender_hip.so ${LIBS:-}; do
  for arm in ${ARMS:-FR_LOG=0 FR_LOG_MIN=2600}; do
    env $arm FRENDER_HIP_LIB=$(pwd)/$lib DIAG_S=$1 DIAG_L=$2 timeout -k 10 120 python scripts/diag_scale.py 100000000 4095 > gpurun_out/cfg_ab.log 2>&1 || { echo "$arm S=$1 failed"; tail -3 gpurun_out/cfg_ab.log; exit 1; }
    echo "S=$1 L=$2 $(basename $lib .so) $arm $(grep -o 'U=[0-9]* launches=[0-9]* scan_ms=[0-9.]* log_ms=[0-9.]*' gpurun_out/cfg_ab.log)"
  done
  done
done
