# instruction mix of fr::chunk_kernel per FR_ABLATE setting (0 full, 8 no commit flush, 4 no LDS insert,
# 2 no encode, 1 no header parse): one PMC pass of SQ counters each, no trace domains
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
export TMPDIR=/tmp
for ab in ${ABL:-0 8 4 2 1}; do
  cd /tmp
  FR_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
    --kernel-trace --output-format csv -d "$R/gpurun_out/r03g_sqab_$ab" -o run -- python3 "$R/scripts/diag_scale.py" 100000000 3900 > "$R/gpurun_out/r03g_sqab_$ab.log" 2>&1 || { tail -5 "$R/gpurun_out/r03g_sqab_$ab.log"; exit 1; }
  cd "$R"
  python3 - "$ab" <<'PY'
import csv, glob, collections, sys
ab = sys.argv[1]
rows = []
for f in glob.glob(f"gpurun_out/r03g_sqab_{ab}/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = collections.defaultdict(float); disp = set()
for r in rows:
    if r["Kernel_Name"].startswith("fr::chunk_kernel"):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
dur = []
for f in glob.glob(f"gpurun_out/r03g_sqab_{ab}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("fr::chunk_kernel"):
            dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
n = len(disp)
recs = 50e6 * n  # the diag run's launches are 50M records each (100M reads, 2 launches) x2 runs
print(f"ablate={ab} dispatches={n} " + " ".join(f"{k[3:]}={v / recs * 1e0:.3f}/rec" for k, v in sorted(acc.items())),
      f"kernel_ms_last2={[round(d/1e6,3) for d in dur[-2:]]}")
PY
done
