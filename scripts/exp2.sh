#!/bin/bash
# diag_scale timings of the product library at several launch sizes (MiB) and env settings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
N=${N:-100000000}
i=0
for spec in "$@"; do   # each arg: "CHUNK_MIB ENV=VAL ..."
  set -- $spec; ch=$1; shift
  env "$@" timeout -k 10 120 python scripts/diag_scale.py $N $ch > gpurun_out/exp2_$i.log 2>&1 || { echo "[$spec] failed"; tail -3 gpurun_out/exp2_$i.log; exit 1; }
  echo "[$spec] $(grep -o 'launches=[0-9]* scan_ms=[0-9.]*' gpurun_out/exp2_$i.log) $(grep -o "'spin_total': [0-9]*" gpurun_out/exp2_$i.log) $(grep -o "'spec_replays': [0-9]*" gpurun_out/exp2_$i.log)"
  i=$((i+1))
done
