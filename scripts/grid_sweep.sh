#!/bin/bash
# Tally-kernel time vs grid size (chunks per launch) on the diag workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
N=${N:-100000000}
for g in ${GRIDS:-1024 2048 4096 8192}; do
  FR_GRID=$g timeout -k 10 120 python scripts/diag_scale.py $N ${CH:-4095} > gpurun_out/grid_$g.log 2>&1 || { echo "grid $g failed"; tail -3 gpurun_out/grid_$g.log; exit 1; }
  echo "grid=$g $(grep -o 'scan_ms=[0-9.]*' gpurun_out/grid_$g.log)"
done
