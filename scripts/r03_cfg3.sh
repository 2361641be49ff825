# config-3 shape: launch-log tests, diag split, bench line and a kernel trace
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 200 --timeout-method thread -k "launch_log or heavy or golden_case or classify" > gpurun_out/r03c3_pytest.log 2>&1 || { tail -5 gpurun_out/r03c3_pytest.log; exit 1; }
tail -1 gpurun_out/r03c3_pytest.log
timeout -k 5 120 env DIAG_S=384 DIAG_L=10 python -u scripts/diag_scale.py 100000000 3900 2>&1 | grep -v amdgpu.ids | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*//"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --samples 384 --index-len 10 --rc | grep '"metric"' > gpurun_out/r03c3.json || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r03c3.json')); print('cfg3', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['log_aggregation_ms_per_launch'])"
