#!/bin/bash
# VALU / SALU / LDS instruction counts of the tally kernel under each FR_ABLATE setting (one --pmc pass each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out/pmcph; export TMPDIR=/tmp
N=${N:-20000000}
cd /tmp
for ab in ${ABL:-0 1 2 4}; do
  FR_ABLATE=$ab timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d "$R/gpurun_out/pmcph/a$ab" -o run \
      -- python3 "$R/scripts/diag_scale.py" $N 1024 > "$R/gpurun_out/pmcph/a$ab.log" 2>&1 || { echo "ablate $ab failed"; tail -3 "$R/gpurun_out/pmcph/a$ab.log"; exit 1; }
done
cd "$R"
python3 - <<'PY'
import csv, glob, os
n = int(os.environ.get("N", "20000000"))
for d in sorted(glob.glob("gpurun_out/pmcph/a*/")):
    tot = {}
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("fr::chunk_kernel"):
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(d, " ".join(f"{k}={v / n:.2f}" for k, v in sorted(tot.items())))
PY
