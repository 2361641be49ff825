#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the tally kernel under FR_ABLATE settings (diag workload, one --pmc pass
# per counter and setting): how much of the HBM traffic each parse stage adds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out/pmcab; export TMPDIR=/tmp
N=${N:-100000000}
cd /tmp
for ab in ${ABL:-0 2}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    FR_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmcab/${c}_$ab" -o run \
        -- python3 "$R/scripts/diag_scale.py" $N 4095 > "$R/gpurun_out/pmcab/${c}_$ab.log" 2>&1 || { echo "$c $ab failed"; exit 1; }
  done
done
cd "$R"
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/pmcab/*/run_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if "chunk_kernel" in r.get("Kernel_Name", "")]
    vals = [float(r["Counter_Value"]) for r in rows]
    print(f.split("/")[2], len(vals), "avg KiB per launch", sum(vals) / max(len(vals), 1))
PY
