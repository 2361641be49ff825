#!/bin/bash
# Calibrate FETCH_SIZE / WRITE_SIZE on the tally's table access patterns (scripts/ubench_table.hip):
# one counter per run (MI355X_MICROARCH.md: separate --pmc passes), each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/tab_fetch" -o run -- "$R/scripts/ubench_table" > "$R/gpurun_out/tab_fetch.log" 2>&1 || { echo fetch failed; tail -5 "$R/gpurun_out/tab_fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/tab_write" -o run -- "$R/scripts/ubench_table" > "$R/gpurun_out/tab_write.log" 2>&1 || { echo write failed; tail -5 "$R/gpurun_out/tab_write.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/tab_trace" -o run -- "$R/scripts/ubench_table" > "$R/gpurun_out/tab_trace.log" 2>&1 || { echo trace failed; exit 1; }
cd "$R"
for f in $(find gpurun_out/tab_fetch gpurun_out/tab_write -name "*counter_collection.csv"); do echo "== $f"; cut -d, -f1-30 "$f" | head -20; done
