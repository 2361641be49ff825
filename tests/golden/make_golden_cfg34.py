#!/usr/bin/env python3
"""Pin the benchmarked config-3 and config-4 SHAPES to the REFERENCE itself.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden_cfg34.py --config 3 [--reads 100000000] [--workers 8]
    python tests/golden/make_golden_cfg34.py --config 4 [--reads 100000000] [--workers 8]

bench.py's config-3 shape (`--samples 384 --index-len 10 --rc`) and config-4 shape
(`--combinatorial --nsubs 2`) scan 100M SYN-v1 records (R=8, seed 1) per GPU as one logical
file resident in HBM.  This script writes the same records (host SYN-v1 generator,
frender_amd/synth.py, byte-identical to the device one) as `--workers` consecutive level-1
.fastq.gz files, imports /root/reference/frender.py (spec_from_file_location; the CLI sits
behind `__main__`, frender.py:817) and runs the reference's own frender_scan sequence
(frender.py:606-630).  In the config-3 shape the reads of synth.CFG3_RC_NAMES carry rc(idx2), so the
reference's call flips those 8 names and pass B classifies against the rewritten idx2 list:

    counter = tally_barcodes(W, files)                                       (:183-207)
    results = process(W, counter["total"], indexes, n, rc)                   (:391-426)
    # config 3 only (-rc):
    rc_calls = call_rc_mode_per_id(flatten_results(results), indexes["id"]) (:354-388, :482-492)
    indexes["idx2"] = [rc(idx2) if rc_calls[id]["call"] else idx2 ...]      (:618-623)
    results = process(W, counter["total"], indexes, n, rc_mode=False)       (:628-630)

Consecutive files keep the merged table's order and counts those of the single stream (R5).
It commits tests/golden/cfg{3,4}_pin.json with the unique-code count, the total reads, a
sha256 over every final row in the reference's order

    f"{code}\\t{reads}\\t{matched_idx1}\\t{matched_idx2}\\t{read_type}\\t{sample_name}\\n"

(the row format of cfg2_pin.json), the first and last 1000 rows verbatim, and for config 3
the pass-A digest over rows that also carry the rc columns

    f"...\\t{sample_name}\\t{matched_rc_idx2}\\t{rc_read_type}\\t{rc_sample_name}\\n"

plus every per-name rc call (name, reads_f, reads_rc, call).  Only data is committed.
"""
from __future__ import annotations

import argparse
import hashlib
import importlib.util
import json
import os
import sys
import tempfile
import time
import zlib
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from frender_amd import synth  # noqa: E402

REF_PATH = "/root/reference/frender.py"
BLOCK = 1 << 20

SHAPES = {
    3: {"samples": 384, "L": 10, "combinatorial": None, "n": 1, "rc": True, "rc_names": synth.CFG3_RC_NAMES,
        "workload": "BASELINE config 3 shape: SYN-v1 records [0, reads), 384 samples (synth.make_sheet(384, 10, 10), "
                    "seed 42), 10+10 bp, R=8, seed 1, n=1, -rc (pass A, per-name call, pass B); the reads of the "
                    "8 samples synth.CFG3_RC_NAMES carry rc(idx2), so the per-name call flips them"},
    4: {"samples": 96, "L": 8, "combinatorial": (12, 8), "n": 2, "rc": False, "rc_names": None,
        "workload": "BASELINE config 4 shape: SYN-v1 records [0, reads), 96 combinatorial dual indexes "
                    "(synth.make_sheet(96, 8, 8, combinatorial=(12, 8)), seed 42), 8+8 bp, R=8, seed 1, n=2, no -rc"},
}


def sheet_of(cfg: int):
    s = SHAPES[cfg]
    return synth.make_sheet(s["samples"], s["L"], s["L"], combinatorial=s["combinatorial"])


def _write_part(job):
    path, cfg, r0, n = job
    sheet = sheet_of(cfg)
    co = zlib.compressobj(1, zlib.DEFLATED, 31)  # gzip container, level 1
    with open(path, "wb") as f:
        for a in range(r0, r0 + n, BLOCK):
            b = min(BLOCK, r0 + n - a)
            f.write(co.compress(synth.generate_records(sheet, a, b, R=8, seed=1,
                                                       rc_names=SHAPES[cfg]["rc_names"]).tobytes()))
        f.write(co.flush())
    return path


def row_line(code, r) -> str:
    return f"{code}\t{r['reads']}\t{r['matched_idx1']}\t{r['matched_idx2']}\t{r['read_type']}\t{r['sample_name']}\n"


def row_line_rc(code, r) -> str:
    return row_line(code, r)[:-1] + f"\t{r['matched_rc_idx2']}\t{r['rc_read_type']}\t{r['rc_sample_name']}\n"


def digest(results, fmt, keep):
    h = hashlib.sha256()
    rows = []
    for code, r in results.items():
        line = fmt(code, r)
        h.update(line.encode())
        rows.append(line)
    return h.hexdigest(), rows[:keep], rows[-keep:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, choices=(3, 4), required=True)
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--keep", default=None, help="scratch dir to keep the .fastq.gz files in")
    ap.add_argument("--out", default=None, help="fixture path (default tests/golden/cfg{3,4}_pin.json)")
    ap.add_argument("--rows", type=int, default=1000, help="rows kept verbatim at each end")
    a = ap.parse_args()
    shape = SHAPES[a.config]
    out_path = a.out or os.path.join(HERE, f"cfg{a.config}_pin.json")
    spec = importlib.util.spec_from_file_location("frender_reference", REF_PATH)
    ref = importlib.util.module_from_spec(spec)
    sys.modules["frender_reference"] = ref  # its Pool workers (fork) pickle the module's functions by name
    spec.loader.exec_module(ref)
    sheet = sheet_of(a.config)
    d = a.keep or tempfile.mkdtemp(prefix=f"cfg{a.config}pin_")
    os.makedirs(d, exist_ok=True)
    W = a.workers
    cuts = [a.reads * i // W for i in range(W + 1)]
    files = [os.path.join(d, f"syn_L{i + 1:03d}_R1_001.fastq.gz") for i in range(W)]
    t0 = time.time()
    if not all(os.path.exists(p) for p in files):
        with Pool(W) as pool:
            pool.map(_write_part, [(files[i], a.config, cuts[i], cuts[i + 1] - cuts[i]) for i in range(W)])
    print(f"inputs written in {time.time() - t0:.1f} s", flush=True)
    sheet_csv = os.path.join(d, "sheet.csv")
    sheet.write_csv(sheet_csv)
    indexes = ref.get_indexes(sheet_csv)
    n = shape["n"]
    secs = {"workers": W}
    t0 = time.time()
    counter = ref.tally_barcodes(W, files)
    secs["tally"] = round(time.time() - t0, 1)
    print(f"tally {secs['tally']} s, {len(counter['total'])} codes", flush=True)
    t0 = time.time()
    results = ref.process(W, counter["total"], indexes, n, shape["rc"])
    secs["process"] = round(time.time() - t0, 1)
    print(f"process {secs['process']} s", flush=True)
    out = {"workload": shape["workload"], "config": a.config, "reads": a.reads,
           "total_reads": int(sum(counter["total"].values())), "unique_codes": len(results),
           "row_format": "code\\treads\\tmatched_idx1\\tmatched_idx2\\tread_type\\tsample_name\\n, reference order"}
    if shape["rc"]:
        ha, fa, la = digest(results, row_line_rc, a.rows)
        out["pass_a"] = {"row_format": "as row_format, then \\tmatched_rc_idx2\\trc_read_type\\trc_sample_name "
                                       "before the \\n (analyze_barcodes_with_rc, frender.py:294-351)",
                         "rows_sha256": ha, "first_rows": fa, "last_rows": la}
        rc_calls = ref.call_rc_mode_per_id(ref.flatten_results(results), indexes["id"])
        out["rc_calls"] = [[name, c["reads_f"], c["reads_rc"], bool(c["call"])] for name, c in rc_calls.items()]
        indexes["idx2"] = [ref.reverse_complement(indexes["idx2"][i]) if rc_calls[i_d]["call"] else indexes["idx2"][i]
                           for i, i_d in enumerate(indexes["id"])]
        t0 = time.time()
        results = ref.process(W, counter["total"], indexes, n, rc_mode=False)
        secs["process_b"] = round(time.time() - t0, 1)
        print(f"pass B {secs['process_b']} s", flush=True)
    h, first, last = digest(results, row_line, a.rows)
    out.update({"rows_sha256": h, "first_rows": first, "last_rows": last,
                "generated_by": "tests/golden/make_golden_cfg34.py: reference frender.py tally_barcodes + process "
                                "(+ call_rc_mode_per_id and pass B with -rc), imported",
                "reference_seconds": secs})
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("first_rows", "last_rows", "pass_a", "rc_calls")}))


if __name__ == "__main__":
    main()
