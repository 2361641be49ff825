# commit sub-phase stamps (FR_STAMPS=2 build) for the config-3 shape and config 2 with every commit logged
mkdir -p gpurun_out
out=gpurun_out/r03_st2.log; : > $out
L=$PWD/frender_amd/libfrender_hip_exp_st2.so
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3900 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
run FRENDER_HIP_LIB=$L DIAG_S=384 DIAG_L=10
run FRENDER_HIP_LIB=$L DIAG_S=96 DIAG_L=8 FR_LOG_MIN=0
run FRENDER_HIP_LIB=$L DIAG_S=384 DIAG_L=10 FR_LOG=0
grep -v amdgpu.ids $out | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*'stamps'/stamps/"
out2=gpurun_out/r03_st2b.log; : > $out2
run2() { echo "== $*" >> $out2; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3900 >> $out2 2>&1 || { echo "FAILED $*" >> $out2; exit 1; }; }
run2 DIAG_S=384 DIAG_L=10
run2 DIAG_S=96 DIAG_L=8
run2 DIAG_S=96 DIAG_L=8 FR_LOG_MIN=0
run2 DIAG_S=96 DIAG_L=8 FR_LOG_MIN=1500
grep -v amdgpu.ids $out2 | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*//"
