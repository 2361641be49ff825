#!/bin/bash
# Tally-kernel phase breakdown: ablations (FR_ABLATE bits: 1 no header parse, 2 no encode,
# 4 no insert) with the product library, then per-phase s_memtime stamps (stamps build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
N=${N:-100000000}
for ab in ${ABL:-0 1 8 2 4}; do
  FR_ABLATE=$ab timeout -k 10 120 python scripts/diag_scale.py $N ${CH:-4095} > gpurun_out/ablate_$ab.log 2>&1 || { echo "ablate $ab failed"; tail -3 gpurun_out/ablate_$ab.log; exit 1; }
  echo "ablate=$ab $(grep -o 'scan_ms=[0-9.]*' gpurun_out/ablate_$ab.log)"
done
[ -n "${NOSTAMP:-}" ] && exit 0
FRENDER_HIP_LIB=$(pwd)/frender_amd/libfrender_hip_stamps.so timeout -k 10 120 python scripts/diag_scale.py $N ${CH:-4095} > gpurun_out/stamps.log 2>&1 || { echo "stamps failed"; exit 1; }
tail -2 gpurun_out/stamps.log
