"""Pin the CPU oracle against the reference's own outputs (golden vectors).

Every case under tests/golden/cases was produced by running reference frender
(tests/golden/make_golden.py).  The oracle must reproduce each output file
byte for byte, and raise the same exception class (and message) where the
reference crashed.
"""
import gzip
import hashlib
import os
import tempfile

import pytest

from harness import build_inputs, case_names, load_spec, run_case
from oracle import frender_oracle


@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_reference(name):
    diffs = run_case(name, frender_oracle.scan)
    assert not diffs, "\n".join(diffs)


@pytest.mark.parametrize("name", [n for n in case_names() if load_spec(n)["synthetic"]])
def test_synthetic_inputs_are_stable(name):
    """The synthetic inputs are rebuilt on every machine: pin their decoded bytes."""
    with tempfile.TemporaryDirectory() as d:
        spec = build_inputs(name, d)
        for f, md5 in spec["synthetic"]["decoded_md5"].items():
            with gzip.open(os.path.join(d, f), "rb") as g:
                assert hashlib.md5(g.read()).hexdigest() == md5, f


def test_oracle_multicore_identical():
    """frender.py:189-193 / :395-411: the Pool fan-out must not change the output."""
    assert not run_case("s96_n1_4files", frender_oracle.scan, extra={"c": 4.0}, check_stdout=False)


def test_oracle_cfg2_prefix_pinned():
    """The oracle on the first 1M records of the benchmarked workload (BASELINE config 2) reproduces
    the reference's own tally_barcodes + process rows (tests/golden/cfg2_pin_1m.json, made by
    tests/golden/make_golden_cfg2.py with the reference imported)."""
    import json
    from multiprocessing import Pool

    from frender_amd import synth
    from oracle import frender_oracle as O

    with open(os.path.join(os.path.dirname(__file__), "golden", "cfg2_pin_1m.json")) as f:
        pin = json.load(f)
    sheet = synth.make_sheet(96, 8, 8)
    counts, records = O.tally_text(synth.generate_bytes(sheet, 0, pin["reads"], R=8, seed=1).decode())
    assert records == pin["total_reads"] and len(counts) == pin["unique_codes"]
    codes = list(counts)
    with Pool(4) as pool:
        res = pool.starmap(O.classify_code, [(c, counts[c], sheet.idx1, sheet.idx2, sheet.ids, 1, False) for c in codes])
    out = {"m1": [sheet.idx1.index(r["matched_idx1"]) if r["matched_idx1"] else -1 for r in res],
           "m2": [sheet.idx2.index(r["matched_idx2"]) if r["matched_idx2"] else -1 for r in res],
           "cls": [synth.CLASS_NAMES.index(r["read_type"]) for r in res],
           "row": [sheet.ids.index(r["sample_name"]) if r["sample_name"] else -1 for r in res]}
    digest, first, last = synth.rows_digest(codes, [counts[c] for c in codes], out, sheet.idx1, sheet.idx2,
                                            sheet.ids, keep=len(pin["first_rows"]))
    assert first == pin["first_rows"] and last == pin["last_rows"]
    assert digest == pin["rows_sha256"]


def _rows(codes, counts, res, rc):
    lines = []
    for c, r in zip(codes, res):
        line = f"{c}\t{counts[c]}\t{r['matched_idx1']}\t{r['matched_idx2']}\t{r['read_type']}\t{r['sample_name']}"
        if rc:
            line += f"\t{r['matched_rc_idx2']}\t{r['rc_read_type']}\t{r['rc_sample_name']}"
        lines.append(line + "\n")
    return hashlib.sha256("".join(lines).encode()).hexdigest(), lines


@pytest.mark.parametrize("cfg", [3, 4])
def test_oracle_cfg34_prefix_pinned(cfg):
    """The oracle on the first records of the config-3 shape (384 samples, 10+10, -rc: pass A, the
    per-name call, pass B) and the config-4 shape (12x8 combinatorial, n=2) reproduces the reference's
    own frender_scan sequence (tests/golden/cfg{3,4}_pin_1m.json, made by tests/golden/make_golden_cfg34.py
    with the reference imported)."""
    import json
    from multiprocessing import Pool

    from frender_amd import synth
    from frender_amd.host import reverse_complement
    from oracle import frender_oracle as O

    path = os.path.join(os.path.dirname(__file__), "golden", f"cfg{cfg}_pin_1m.json")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated")
    with open(path) as f:
        pin = json.load(f)
    rc = cfg == 3
    nsubs = 1 if cfg == 3 else 2
    L, S = (10, 384) if cfg == 3 else (8, 96)
    sheet = synth.make_sheet(S, L, L, combinatorial=(12, 8) if cfg == 4 else None)
    rc_names = synth.CFG3_RC_NAMES if cfg == 3 else None  # their reads carry rc(idx2): the call flips them
    counts, records = O.tally_text(synth.generate_bytes(sheet, 0, pin["reads"], R=8, seed=1,
                                                        rc_names=rc_names).decode())
    assert records == pin["total_reads"] and len(counts) == pin["unique_codes"]
    codes = list(counts)
    keep = len(pin["first_rows"])
    idx2 = list(sheet.idx2)
    with Pool(8) as pool:
        res = pool.starmap(O.classify_code, [(c, counts[c], sheet.idx1, idx2, sheet.ids, nsubs, rc) for c in codes])
        if rc:
            digest, lines = _rows(codes, counts, res, True)
            assert lines[:keep] == pin["pass_a"]["first_rows"] and lines[-keep:] == pin["pass_a"]["last_rows"]
            assert digest == pin["pass_a"]["rows_sha256"]
            sums = {n: [0, 0] for n in dict.fromkeys(sheet.ids)}
            for r in res:
                if r["sample_name"]:
                    sums[r["sample_name"]][0] += r["reads"]
                if r["rc_sample_name"]:
                    sums[r["rc_sample_name"]][1] += r["reads"]
            calls = [[n, f, b, f < b] for n, (f, b) in sums.items()]
            assert calls == pin["rc_calls"]
            assert sorted(n for n, _, _, c in calls if c) == sorted(synth.CFG3_RC_NAMES)
            use = {n: c for n, _, _, c in calls}
            idx2 = [reverse_complement(x) if use[i] else x for i, x in zip(sheet.ids, idx2)]
            res = pool.starmap(O.classify_code, [(c, counts[c], sheet.idx1, idx2, sheet.ids, nsubs, False)
                                                 for c in codes])
    digest, lines = _rows(codes, counts, res, False)
    assert lines[:keep] == pin["first_rows"] and lines[-keep:] == pin["last_rows"]
    assert digest == pin["rows_sha256"]
