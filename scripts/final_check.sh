set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_check.sh test || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r05_bench_pre.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r05_bench_pre.log; exit 1; }
tail -1 gpurun_out/r05_bench_pre.log | cut -c1-400
bash scripts/gpu_profile.sh || exit $?
