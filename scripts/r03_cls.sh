# classify neighbourhood maps: parity tests, then the config-3 shape bench under a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 200 --timeout-method thread -k "classify or golden" > gpurun_out/r03_cls_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r03_cls_pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r03_cls_pytest.log | head -20; exit $rc; }
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03_cls_prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --samples 384 --index-len 10 --rc > $R/gpurun_out/r03_cls_bench.log 2>&1 || { tail -5 $R/gpurun_out/r03_cls_bench.log; exit 1; }
cd $R && tail -1 gpurun_out/r03_cls_bench.log | cut -c1-400 && find gpurun_out/r03_cls_prof -name "*kernel_stats.csv" | xargs grep -E "classify|nbr|chunk_kernel|log_" | cut -c1-200
