# per-phase wave cycles of the tally kernel (FR_STAMPS=1: walk / commit / guess; FR_STAMPS=2: the
# commit's own phases), config 2 and the config-3 shape, 100M reads, one launch per 4 GiB
set -o pipefail
mkdir -p gpurun_out
for v in st1 st2; do
  for cfg in "96 8" "384 10"; do
    set -- $cfg
    DIAG_S=$1 DIAG_L=$2 FRENDER_HIP_LIB=$(pwd)/frender_amd/libfrender_hip_exp_$v.so timeout -k 10 120 \
      python scripts/diag_scale.py 100000000 4095 > gpurun_out/stamps_${v}_$1.log 2>&1 || { echo "stamps $v $1 failed"; tail -5 gpurun_out/stamps_${v}_$1.log; exit 1; }
    echo "$v S=$1: $(grep -o "scan_ms=[0-9.]*" gpurun_out/stamps_${v}_$1.log) $(grep -o "'stamps'.*" gpurun_out/stamps_${v}_$1.log)"
  done
done
