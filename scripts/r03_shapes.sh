# bench lines of every BASELINE shape on this tree + a kernel trace of the config-3 shape (profiles/)
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
b() { timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" | grep '"metric"'; }
b > gpurun_out/r03s_cfg2.json && \
b --samples 384 --index-len 10 --rc > gpurun_out/r03s_cfg3.json && \
b --combinatorial --nsubs 2 > gpurun_out/r03s_cfg4.json && \
b --reads 20000000 --read-len 150 > gpurun_out/r03s_r150.json || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03s_cfg3_prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --samples 384 --index-len 10 --rc > $R/gpurun_out/r03s_cfg3_prof.log 2>&1 || exit 1
cd $R
for f in cfg2 cfg3 cfg4 r150; do python3 -c "import json,sys; d=json.load(open('gpurun_out/r03s_$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline']['log_aggregation_ms_per_launch'])"; done
find gpurun_out/r03s_cfg3_prof -name "*kernel_stats.csv" | xargs head -14 | cut -c1-150
