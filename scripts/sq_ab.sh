#!/bin/bash
# SQ instruction counters of the tally kernel for the product library and every
# frender_amd/libfrender_hip_exp*.so (one --pmc pass per library, diag workload), per record.
set -u; shopt -s nullglob
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out/sq; export TMPDIR=/tmp
N=${N:-100000000}; CH=${CH:-4095}
CTRS=${CTRS:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"}
cd /tmp
for lib in "$R"/frender_amd/libfrender_hip.so "$R"/frender_amd/libfrender_hip_exp*.so; do
for ab in ${ABL:-0}; do
  b=$(basename $lib .so)_ab$ab
  FR_ABLATE=$ab FRENDER_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$R/gpurun_out/sq/$b" -o run \
      -- python3 "$R/scripts/diag_scale.py" $N $CH > "$R/gpurun_out/sq/$b.log" 2>&1 || { echo "$b failed"; tail -3 "$R/gpurun_out/sq/$b.log"; exit 1; }
done
done
cd "$R"
N=$N python3 - <<'PY'
import csv, glob, collections, os
n = int(os.environ["N"]) / 2  # records per launch (two launches)
for d in sorted(glob.glob("gpurun_out/sq/*/")):
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "chunk_kernel" in r.get("Kernel_Name", ""):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d.rstrip("/")), " ".join(f"{k.replace('SQ_','')}={sum(v)/len(v)/n:.3f}" for k, v in sorted(acc.items())))
PY
