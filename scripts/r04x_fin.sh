#!/bin/bash
# Round 4, call x: kernel traces of the bench with each finalize pipeline (FR_FIN_OLD=1: a global atomic
# per code; 0: coarse buckets counted in LDS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
for f in 1 0; do
  FR_FIN_OLD=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/fin$f" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$R/gpurun_out/fin$f.log" 2>&1 || { echo "trace $f failed"; tail -5 "$R/gpurun_out/fin$f.log"; exit 1; }
  echo "fin_old=$f: $(tail -1 $R/gpurun_out/fin$f.log | cut -c1-160)"
done
