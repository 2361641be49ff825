#!/bin/bash
# One launch per device feed (chunk offsets, ranges over 4 GiB): GPU suite, then the bench with
# 16-GiB launches against 4-GiB ones, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04one_pytest.log 2>&1 || { tail -30 gpurun_out/r04one_pytest.log; exit 1; }
tail -1 gpurun_out/r04one_pytest.log
for r in 1 2; do
  for g in 16 4; do
    timeout -k 10 300 python -u bench.py --no-cpu --launch-gib $g > gpurun_out/r04one_bench_$g.$r.log 2>&1 || { tail -5 gpurun_out/r04one_bench_$g.$r.log; exit 1; }
    echo "gib=$g round $r $(tail -1 gpurun_out/r04one_bench_$g.$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"], r["launches_per_step"], r["frac"])')"
  done
done
