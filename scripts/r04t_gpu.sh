#!/bin/bash
# Round 4, call t: the tally launches' timeline (FR_STAMPS=3 build), then the bench step with each
# finalize pipeline, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
FRENDER_HIP_LIB=frender_amd/libfrender_hip_exp_tl.so timeout -k 10 180 python -u scripts/chunk_timeline.py > gpurun_out/r04t_timeline.json 2> gpurun_out/r04t_timeline.err || { tail -5 gpurun_out/r04t_timeline.err; exit 1; }
echo timeline done
for r in 1 2; do
  for f in 1 0; do
    FR_FIN_OLD=$f timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r04t_bench_fin$f.$r.log 2>&1 || { tail -5 gpurun_out/r04t_bench_fin$f.$r.log; exit 1; }
    echo "fin_old=$f round $r $(tail -1 gpurun_out/r04t_bench_fin$f.$r.log | cut -c1-200)"
  done
done
