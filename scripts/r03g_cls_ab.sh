# classify kernel A/B at the config-3 shape: kernel trace of bench.py per library build (main = the
# in-tree library, NAME = libfrender_hip_exp_NAME.so); prints per-dispatch classify durations
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-main cls}; do
  lib=$R/frender_amd/libfrender_hip.so; [ $v != main ] && lib=$R/frender_amd/libfrender_hip_exp_$v.so
  cd /tmp
  FRENDER_HIP_LIB=$lib timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/cls_$v" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --samples 384 --index-len 10 --rc > "$R/gpurun_out/cls_$v.log" 2>&1 || { tail -5 "$R/gpurun_out/cls_$v.log"; exit 1; }
  cd "$R"
  python3 - "$v" <<'PY'
import csv, glob, json, sys
v = sys.argv[1]
d = []
for f in glob.glob(f"gpurun_out/cls_{v}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "classify_kernel" in r["Kernel_Name"]:
            d.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
d.sort()
line = [l for l in open(f"gpurun_out/cls_{v}.log") if l.startswith("{")]
ms = json.loads(line[-1])["ms_per_step"] if line else None
print(v, "ms_per_step", ms, "classify us (last 6):", [round(x[1], 1) for x in d[-6:]])
PY
done
