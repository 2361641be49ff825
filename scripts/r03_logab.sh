# launch-log reduce ablations on the config-3 shape: 1024 = loads + filter only, 512 = no loads/fold,
# 256 = no flush to the table
mkdir -p gpurun_out
out=gpurun_out/r03_logab.log; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3900 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
run DIAG_S=384 DIAG_L=10
run DIAG_S=384 DIAG_L=10 FR_ABLATE=1024
run DIAG_S=384 DIAG_L=10 FR_ABLATE=512
run DIAG_S=384 DIAG_L=10 FR_ABLATE=256
run DIAG_S=384 DIAG_L=10 FR_ABLATE=768
grep -v amdgpu.ids $out | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*//"
