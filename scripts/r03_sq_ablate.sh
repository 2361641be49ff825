# VALU / SALU / LDS instruction counts of fr::chunk_kernel per FR_ABLATE setting (config 2 bench, one
# PMC pass each): 0 full, 8 no HBM flush, 4 no LDS insert/commit, 2 locate only, 1 no parse
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
for ab in 0 8 4 2 1; do
  cd /tmp
  FR_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$R/gpurun_out/r03_sqa_$ab" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu > "$R/gpurun_out/r03_sqa_$ab.log" 2>&1 || { tail -5 "$R/gpurun_out/r03_sqa_$ab.log"; exit 1; }
  cd "$R"
done
python3 - <<'PY'
import csv, glob, collections
for ab in (0, 8, 4, 2, 1):
    rows = []
    for f in glob.glob(f"gpurun_out/r03_sqa_{ab}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    acc = collections.defaultdict(float); disp = set()
    for r in rows:
        if r["Kernel_Name"].startswith("fr::chunk_kernel"):
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    n = max(len(disp), 1)
    rec = 50e6
    print(f"ablate={ab:2d} " + " ".join(f"{k[3:]}={acc[k] / n / rec:.2f}" for k in sorted(acc)) + " (per record)")
PY
