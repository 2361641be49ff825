#!/bin/bash
# Timing-stamp build under several FR_ABLATE settings (per-phase wave cycles incl. commit / guess)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
N=${N:-100000000}
for ab in ${ABL:-0}; do
  FR_ABLATE=$ab FRENDER_HIP_LIB=$(pwd)/frender_amd/libfrender_hip_stamps.so timeout -k 10 120 python scripts/diag_scale.py $N ${CH:-4095} > gpurun_out/stamps_$ab.log 2>&1 || { echo "stamps $ab failed"; exit 1; }
  echo "ablate=$ab $(grep -o "scan_ms=[0-9.]*" gpurun_out/stamps_$ab.log) $(grep -o "'stamps'.*" gpurun_out/stamps_$ab.log)"
done
