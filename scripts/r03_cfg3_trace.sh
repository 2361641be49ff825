# kernel trace of the config-3 shape bench: per-kernel time and idle gaps of one step
R=$PWD; export TMPDIR=/tmp; mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03c3_prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --samples 384 --index-len 10 --rc > $R/gpurun_out/r03c3_prof.log 2>&1 || exit 1
