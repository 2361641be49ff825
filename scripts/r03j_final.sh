# final tree: GPU suite, bench (config 2 with CPU baseline + e2e), config-3/config-4/R=150 shapes,
# rocprofv3 trace + PMC passes (FETCH_SIZE, WRITE_SIZE, SQ VALU; stream-only FETCH calibration)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03j_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r03j_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r03j_pytest.log | head -20; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r03j_bench.log 2>&1 || { tail -5 gpurun_out/r03j_bench.log; exit 1; }
tail -1 gpurun_out/r03j_bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --no-cpu --samples 384 --index-len 10 --rc > gpurun_out/r03j_bench_cfg3.log 2>&1 || { tail -5 gpurun_out/r03j_bench_cfg3.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --combinatorial --nsubs 2 > gpurun_out/r03j_bench_cfg4.log 2>&1 || { tail -5 gpurun_out/r03j_bench_cfg4.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --read-len 150 --reads 20000000 > gpurun_out/r03j_bench_r150.log 2>&1 || { tail -5 gpurun_out/r03j_bench_r150.log; exit 1; }
for f in cfg3 cfg4 r150; do tail -1 gpurun_out/r03j_bench_$f.log | cut -c1-160; done
rm -rf gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/prof_valu gpurun_out/prof_fetch_stream
STREAM=1 bash scripts/gpu_profile.sh > gpurun_out/r03j_prof.log 2>&1 || { tail -5 gpurun_out/r03j_prof.log; exit 1; }
head -3 gpurun_out/r03j_prof.log | cut -c1-160
