#!/bin/bash
# config-3 shape: chunk size x launch-log threshold (bench.py, 10 steps); prints ms/step and tally ms/launch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C3="--samples 384 --index-len 10 --rc"
for arm in ${ARMS:-"80 2600" "112 2600" "128 2600" "128 3200" "160 3200" "160 4000" "80 2600" "112 2600"}; do
  set -- ${arm/_/ }
  FR_CHUNK_TILES=$1 FR_LOG_MIN=$2 timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu $C3 > gpurun_out/c3s_$1_$2.log 2>&1 || { echo "$arm failed"; exit 1; }
  echo "c3 C=$1 log_min=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c3s_$1_$2.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/c3s_$1_$2.log) $(grep -o '"log_aggregation_ms_per_launch": [0-9.]*' gpurun_out/c3s_$1_$2.log) $(grep -o '"table_checksum": "[0-9a-f]*"' gpurun_out/c3s_$1_$2.log)"
done
