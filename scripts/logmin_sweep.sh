set -o pipefail
for m in 2600 2000 1600 1200; do
  FR_LOG_MIN=$m timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/sw_c2_$m.log 2>&1 || exit 1
  echo "c2 $m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw_c2_$m.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/sw_c2_$m.log)"
done
for m in 2600 2000 1600; do
  FR_LOG_MIN=$m timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu --samples 384 --index-len 10 --rc > gpurun_out/sw_c3_$m.log 2>&1 || exit 1
  echo "c3 $m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw_c3_$m.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/sw_c3_$m.log)"
done
