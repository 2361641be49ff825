# launch-log aggregation kernels with every commit logged (config 2 and the config-3 shape): kernel
# trace per FR_ABLATE setting (0 full, 256 no table inserts, 1024 loads only, 512 no fold)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
for S in "96 8" "384 10"; do
  set -- $S
  for ab in 0 256 1024 512; do
    cd /tmp
    DIAG_S=$1 DIAG_L=$2 FR_LOG_MIN=0 FR_LOG_HOT=1000000 FR_ABLATE=$ab timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/r03g_agg_${1}_$ab" -o run -- python3 "$R/scripts/diag_scale.py" 100000000 3900 > "$R/gpurun_out/r03g_agg_${1}_$ab.log" 2>&1 || { tail -5 "$R/gpurun_out/r03g_agg_${1}_$ab.log"; exit 1; }
    cd "$R"
    echo "S=$1 ablate=$ab: $(grep -o "scan_ms=[0-9.]* log_ms=[0-9.]*" gpurun_out/r03g_agg_${1}_$ab.log)"
    grep -h "log_\|chunk_kernel" gpurun_out/r03g_agg_${1}_$ab/run_kernel_stats.csv | cut -d, -f1-4
  done
done
