#!/bin/bash
# On-box A/B of bench.py variants, interleaved rounds (box-to-box and run-to-run drift hits every variant alike).
#   VARIANTS: newline-separated "label|bench.py arguments[|library suffix[|environment assignments]]" (e.g. "logall|--tuning log_min=0",
#             "noins|--tuning log_min=0|noins" runs frender_amd/libfrender_hip_exp_noins.so: scripts/build_exp.sh)
#   ROUNDS (default 2), STEPS (10), OUT (gpurun_out/variants.jsonl), TIMEOUT per run (240 s)
# Every run: --no-cpu; a run that fails or times out ends the script (nothing more runs on the GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/variants.jsonl}
: > "$OUT"
for r in $(seq 1 "${ROUNDS:-2}"); do
  while IFS='|' read -r label args libs envs; do
    [[ -z "$label" ]] && continue
    lib=frender_amd/libfrender_hip.so
    [[ -n "${libs:-}" ]] && lib=frender_amd/libfrender_hip_exp_${libs}.so
    env ${envs:-} FRENDER_HIP_LIB=$(pwd)/$lib timeout -k 10 "${TIMEOUT:-240}" python bench.py --steps "${STEPS:-10}" --warmup 2 \
        --no-cpu $args > gpurun_out/variant_run.log 2>&1
    rc=$?
    if [[ $rc -ne 0 ]]; then echo "variant $label failed ($rc)"; tail -20 gpurun_out/variant_run.log; exit $rc; fi
    python - "$label" "$r" "$OUT" <<'PY'
import json, sys
label, rnd, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
line = [l for l in open("gpurun_out/variant_run.log") if l.startswith("{")][-1]
d = json.loads(line)
rf = d["roofline"]
rec = {"label": label, "round": rnd, "value": d["value"], "ms_per_step": d["ms_per_step"],
       "tally_ms": rf["avg_launch_ms"], "launches": rf["launches_per_step"], "frac": rf["frac"],
       "log_ms_per_launch": rf["log_aggregation_ms_per_launch"], "unique": d["config"]["unique_codes"],
       "checksum": d["config"]["table_checksum"], "pin": (d["config"].get("reference_pin") or {}).get("equal")}
open(out, "a").write(json.dumps(rec) + "\n")
print(json.dumps(rec), flush=True)
PY
  done <<< "$VARIANTS"
done
