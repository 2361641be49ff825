# config-3 shape: split workgroups per region 32 (default build) vs 64 / 128 (exp builds), with ablation 768
mkdir -p gpurun_out
out=gpurun_out/r03_logab2.log; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3900 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
run DIAG_S=384 DIAG_L=10
for w in 64 128; do
run DIAG_S=384 DIAG_L=10 FRENDER_HIP_LIB=$PWD/frender_amd/libfrender_hip_exp_w$w.so
run DIAG_S=384 DIAG_L=10 FRENDER_HIP_LIB=$PWD/frender_amd/libfrender_hip_exp_w$w.so FR_ABLATE=768
done
grep -v amdgpu.ids $out | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*//"
