# SQ wave-state split of fr::chunk_kernel at config 2 (one PMC pass of 8 SQ counters, no trace domains)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU \
  --output-format csv -d "$R/gpurun_out/r03_sq" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu > "$R/gpurun_out/r03_sq.log" 2>&1 || { tail -5 "$R/gpurun_out/r03_sq.log"; exit 1; }
cd "$R"
python3 - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/r03_sq/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = collections.defaultdict(float); disp = set()
for r in rows:
    if r["Kernel_Name"].startswith("fr::chunk_kernel"):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
n = len(disp)
for k, v in sorted(acc.items()):
    print(f"{k:24s} {v / n:.4g} per dispatch")
w = acc["SQ_WAVE_CYCLES"]
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
    print(f"{k:24s} {acc[k] / w:.3f} of wave cycles")
PY
