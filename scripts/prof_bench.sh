#!/bin/bash
# rocprofv3 kernel-trace stats of one bench.py run (BENCH_ARGS): per-kernel calls and average us
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_bench}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$R/$OUT.log" 2>&1 || { echo "prof failed"; tail -3 "$R/$OUT.log"; exit 1; }
cd "$R"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:48]:48s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:9.1f} us {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
