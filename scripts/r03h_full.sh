# full GPU suite, bench (config 2, with CPU baseline and e2e), the config-3 shape, and a rocprofv3
# kernel-trace summary of the bench (profiles/); logs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03h_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r03h_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03h_pytest.log | head -20; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r03h_bench.log 2>&1 || { tail -5 gpurun_out/r03h_bench.log; exit 1; }
tail -1 gpurun_out/r03h_bench.log
timeout -k 10 300 python -u bench.py --no-cpu --samples 384 --index-len 10 --rc > gpurun_out/r03h_bench_cfg3.log 2>&1 || { tail -5 gpurun_out/r03h_bench_cfg3.log; exit 1; }
tail -1 gpurun_out/r03h_bench_cfg3.log | cut -c1-200
R=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03h_prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/r03h_prof.log 2>&1 || { tail -5 $R/gpurun_out/r03h_prof.log; exit 1; }
cd $R && head -4 gpurun_out/r03h_prof/run_kernel_stats.csv | cut -c1-160
