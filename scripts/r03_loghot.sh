# hot-code split of logged commits: GPU launch-log tests, then config-3 shape / config 2 at several FR_LOG_HOT
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 200 --timeout-method thread -k "launch_log or golden or random or heavy or speculative or many_tiles or device_scale" > gpurun_out/r03_loghot_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r03_loghot_pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r03_loghot_pytest.log | head -20; exit $rc; }
out=gpurun_out/r03_loghot.log; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3900 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
run DIAG_S=384 DIAG_L=10
run DIAG_S=384 DIAG_L=10 FR_LOG_HOT=2
run DIAG_S=384 DIAG_L=10 FR_LOG_HOT=16
run DIAG_S=384 DIAG_L=10 FR_LOG_HOT=1000000
run DIAG_S=384 DIAG_L=10 FR_LOG_MIN=1500
run DIAG_S=96 DIAG_L=8 FR_LOG_MIN=1500
run DIAG_S=96 DIAG_L=8 FR_LOG_MIN=0
run DIAG_S=96 DIAG_L=8 FR_LOG_MIN=0 FR_LOG_HOT=2
grep -v amdgpu.ids $out | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*//"
