# full GPU suite, bench (with CPU baseline) and a rocprofv3 kernel-trace of the bench (profiles/)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03_pytest_full.log 2>&1; rc=$?
tail -3 gpurun_out/r03_pytest_full.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03_pytest_full.log | head -20; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r03_bench_full.log 2>&1 || { tail -5 gpurun_out/r03_bench_full.log; exit 1; }
tail -1 gpurun_out/r03_bench_full.log
R=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03_prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/r03_prof.log 2>&1 || { tail -5 $R/gpurun_out/r03_prof.log; exit 1; }
cd $R && find gpurun_out/r03_prof -name "*kernel_stats.csv" | head -1 | xargs head -8
