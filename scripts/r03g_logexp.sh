# commit cost bounds at config 2 / config-3 shape: default, everything logged (no direct hot inserts),
# and the no-flush ablation (FR_ABLATE=8: nothing reaches the HBM table; wrong counts, timing only)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r03g_logexp.log; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3900 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
for S in "DIAG_S=96 DIAG_L=8" "DIAG_S=384 DIAG_L=10"; do
  run $S
  run $S FR_LOG_MIN=0 FR_LOG_HOT=1000000
  run $S FR_ABLATE=8
done
grep -v amdgpu.ids $out | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*//"
