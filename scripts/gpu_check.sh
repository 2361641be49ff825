#!/bin/bash
# On-box check: GPU parity tests, a short bench, and a rocprofv3 kernel-trace of the bench.
# Every GPU step has its own time limit; a crash/timeout ends the script.
#   stage: all | test | bench | prof | dist
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}

if [[ $STAGE == all || $STAGE == test ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout=300 --timeout-method thread -rf \
      -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -30 gpurun_out/pytest_gpu.log
  echo "pytest exit $rc"
  if [[ $rc -ne 0 ]]; then exit $rc; fi
fi

if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  b=$?; tail -5 gpurun_out/bench.log; echo "bench exit $b"
  if [[ $b -ne 0 ]]; then exit $b; fi
fi

if [[ $STAGE == all || $STAGE == prof ]]; then
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS:-} \
      > "$ROOT/gpurun_out/prof.log" 2>&1
  p=$?; tail -3 "$ROOT/gpurun_out/prof.log"; echo "prof exit $p"
  cd "$ROOT"
  if [[ $p -ne 0 ]]; then exit $p; fi
  find gpurun_out/prof -name "*kernel_stats.csv" -exec head -20 {} \;
fi

if [[ $STAGE == dist ]]; then  # multi-rank rehearsal on this box's GPU (gloo): merged table == one-GPU table
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --reads 10000000 --no-cpu --dist-backend gloo \
      ${DIST_ARGS:-} > gpurun_out/dist2.log 2>&1 || { echo "dist run failed"; tail -5 gpurun_out/dist2.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --reads 20000000 --no-cpu ${DIST_ARGS:-} \
      > gpurun_out/dist1.log 2>&1 || { echo "single run failed"; exit 1; }
  python - <<'PY'
import json
a = [json.loads(l) for l in open("gpurun_out/dist2.log") if l.startswith("{")][0]
b = [json.loads(l) for l in open("gpurun_out/dist1.log") if l.startswith("{")][0]
print("merged uniques", a["config"]["unique_codes"], "single", b["config"]["unique_codes"])
print("merged checksum", a["config"]["table_checksum"], "single", b["config"]["table_checksum"])
print("N=2 roofline", a["roofline"])
assert a["config"]["unique_codes"] == b["config"]["unique_codes"]
assert a["config"]["table_checksum"] == b["config"]["table_checksum"]  # every (key, count, first) row
assert a["roofline"]["achieved"] > 0 and a["roofline"]["launches_per_step"] > 0
PY
  exit $?
fi
exit 0
