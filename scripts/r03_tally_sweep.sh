# tally kernel sweep on the GPU box: config-2 diag (stamps when the library is built with
# FR_STAMPS), optional experimental libraries (scripts/build_exp.sh), config-3 shape, spot tests.
mkdir -p gpurun_out
out=gpurun_out/r03_sweep.log; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3700 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
run FR_ABLATE=0
for lib in frender_amd/libfrender_hip_exp*.so; do [ -e "$lib" ] && run FRENDER_HIP_LIB=$PWD/$lib FR_ABLATE=0; done
run DIAG_S=384 DIAG_L=10 FR_ABLATE=0
grep -v amdgpu.ids $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 200 --timeout-method thread -k "golden or random or heavy or speculative or launch_log or many_tiles or device_scale or growth" > gpurun_out/r03_pytest_spot.log 2>&1; tail -3 gpurun_out/r03_pytest_spot.log
