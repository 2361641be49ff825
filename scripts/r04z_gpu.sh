#!/bin/bash
# Round 4, call z: a shorter ramp-down (FR_RAMP_DOWN_PCT) -- parity on the bench geometry, A/B, timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
FR_RAMP_DOWN_PCT=70 timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bench_geometry or speculative or heavy_chunk or launch_log or many_tiles" > gpurun_out/r04z_pytest.log 2>&1 || { tail -20 gpurun_out/r04z_pytest.log; exit 1; }
tail -1 gpurun_out/r04z_pytest.log
ROUNDS=3 timeout -k 10 900 python -u scripts/exp_variants.py main main@FR_RAMP_DOWN_PCT=85 main@FR_RAMP_DOWN_PCT=70 main@FR_RAMP_DOWN_PCT=50 > gpurun_out/r04z_variants.log 2>&1 || { tail -5 gpurun_out/r04z_variants.log; exit 1; }
echo variants done
FR_RAMP_DOWN_PCT=${TL_PCT:-70} FRENDER_HIP_LIB=frender_amd/libfrender_hip_exp_tl.so timeout -k 10 180 python -u scripts/chunk_timeline.py > gpurun_out/r04z_timeline.json 2> gpurun_out/r04z_timeline.err || { tail -5 gpurun_out/r04z_timeline.err; exit 1; }
echo timeline done
