# launch-log threshold on the config-3 shape (384 samples, 10+10) and config 2 with the current commit
mkdir -p gpurun_out
out=gpurun_out/r03_logmin.log; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3900 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
run DIAG_S=384 DIAG_L=10
run DIAG_S=384 DIAG_L=10 FR_LOG_MIN=3200
run DIAG_S=384 DIAG_L=10 FR_LOG_MIN=4000
run DIAG_S=384 DIAG_L=10 FR_LOG=0
run DIAG_S=96 DIAG_L=8 FR_LOG=0
grep -v amdgpu.ids $out | sed -e 's/diag.*//' 
