# bucketed launch log: GPU suite, then tally timing at several log thresholds (config 3 shape, config 2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_log2_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r03_log2_pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r03_log2_pytest.log | head -20; exit $rc; }
out=gpurun_out/r03_log2.log; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3900 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
run DIAG_S=384 DIAG_L=10
run DIAG_S=384 DIAG_L=10 FR_LOG_MIN=1500
run DIAG_S=96 DIAG_L=8
run DIAG_S=96 DIAG_L=8 FR_LOG_MIN=1500
run DIAG_S=96 DIAG_L=8 FR_LOG_MIN=0
run DIAG_S=384 DIAG_L=10 FR_LOG_MIN=0
grep -v amdgpu.ids $out | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*'grid'/grid/"
