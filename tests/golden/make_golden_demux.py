#!/usr/bin/env python3
"""Generate the `demux` golden fixtures by running REFERENCE frender
here (build container only; the reference never travels to the GPU box):

    python tests/golden/make_golden_demux.py [case ...]

Each case writes tests/golden/demux/<name>/:
    inputs/      the paired .fastq.gz inputs and the results CSV (README column order)
    spec.json    the demux arguments
    expected/    every output file the reference created, DECODED (gzip -> content, then
                 re-gzipped with mtime 0 so the fixture is byte-stable), stdout.txt, and
                 error.json when the reference raised

The reference's open_files() reads the module-global `args` (frender.py:671), which only
exists when it runs as a script; the generator sets that global before calling
frender_demux(args).  Only data is committed, none of the reference's source.
"""
from __future__ import annotations

import argparse
import contextlib
import gzip
import io
import json
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from frender_amd import synth  # noqa: E402
from oracle import frender_oracle as O  # noqa: E402
sys.path.insert(0, HERE)
from make_golden import load_reference  # noqa: E402

CASES_DIR = os.path.join(HERE, "demux")
README_COLS = ["idx1", "idx2", "reads", "matched_idx1", "matched_idx2", "read_type", "sample_name", "demux_ok"]


def r2_of(r1_text: str) -> str:
    """A mate file: headers with ' 2:' instead of ' 1:', reversed sequence/quality lines."""
    out = []
    for i, line in enumerate(r1_text.split("\n")):
        if i % 4 == 0:
            out.append(line.replace(" 1:N:", " 2:N:", 1))
        elif i % 4 in (1, 3):
            out.append(line[::-1])
        else:
            out.append(line)
    return "\n".join(out)


def results_rows(r1_texts, sheet_idx1, sheet_idx2, ids, n):
    total = {}
    for t in r1_texts:
        c, _ = O.tally_text(t)
        for k, v in c.items():
            total[k] = total.get(k, 0) + v
    rows = []
    for code, reads in total.items():
        i1, i2 = code.split("+")[0:2]
        r = O.classify_code(code, reads, sheet_idx1, sheet_idx2, ids, n, False)
        rows.append([i1, i2, str(reads), r["matched_idx1"], r["matched_idx2"], r["read_type"], r["sample_name"],
                     "True"])
    return rows


SCAN_COLS = ["idx1", "idx2", "matched_idx1", "matched_idx2", "read_type", "sample_name", "reads", "demux_ok"]


def write_results(path, rows, header=README_COLS):
    """rows are README-ordered; a header naming the same columns in another order (scan's own CSV)
    gets each row's fields in that order."""
    perm = [README_COLS.index(h) for h in header] if sorted(header) == sorted(README_COLS) else None
    with open(path, "w", newline="") as f:
        f.write(",".join(header) + "\r\n")
        for r in rows:
            f.write(",".join([r[i] for i in perm] if perm else r) + "\r\n")


def readme_order_copy(src, dst):
    """The build accepts scan's column order; the reference does not
    (frender.py:649-657), so its expected outputs for such a case come from the same rows in
    README order."""
    import csv
    with open(src, newline="") as f:
        rows = list(csv.reader(f))
    idx = [rows[0].index(c) for c in README_COLS]
    with open(dst, "w", newline="") as f:
        for r in rows:
            f.write(",".join(r[i] for i in idx) + "\r\n")


def syn_pair_case(name, S, n_reads, n_pairs, n=1, flags=None, nl="\n", r2_trim_lines=0, drop_codes=0,
                  results_header=README_COLS, tamper=None):
    def build(d):
        sheet = synth.make_sheet(S, 8, 8)
        r1s = []
        per = n_reads // n_pairs
        for p in range(n_pairs):
            t1 = synth.generate_bytes(sheet, p * per, per, R=8, seed=3).decode()
            t2 = r2_of(t1)
            if r2_trim_lines:
                t2 = "\n".join(t2.split("\n")[:-1 - r2_trim_lines]) + "\n"
            if nl != "\n":
                t1, t2 = t1.replace("\n", nl), t2.replace("\n", nl)
            synth.write_fastq_gz(os.path.join(d, f"syn_L{p + 1:03d}_R1_001.fastq.gz"), t1.encode(), level=1)
            synth.write_fastq_gz(os.path.join(d, f"syn_L{p + 1:03d}_R2_001.fastq.gz"), t2.encode(), level=1)
            r1s.append(t1.replace("\r\n", "\n"))
        rows = results_rows(r1s, sheet.idx1, sheet.idx2, sheet.ids, n)
        if drop_codes:
            rows = rows[:-drop_codes]
        if tamper:
            rows = tamper(rows)
        write_results(os.path.join(d, "results.csv"), rows, results_header)
    return name, build, dict(flags or {})


def hand_case(name, r1: str, r2: str, rows, flags=None):
    def build(d):
        synth.write_fastq_gz(os.path.join(d, "h_R1_001.fq.gz"), r1.encode(), level=6)
        synth.write_fastq_gz(os.path.join(d, "h_R2_001.fq.gz"), r2.encode(), level=6)
        write_results(os.path.join(d, "results.csv"), rows)
    return name, build, dict(flags or {})


def all_cases():
    def hop_to_weird(rows):
        return [r[:5] + (["weird", ""] if r[5] == "index_hop" else r[5:7]) + r[7:] for r in rows]

    hdr = "@M1:1:FC:1:1101:{}:{} 2:N:0:{}"
    rec = lambda h, s="ACGT": f"{h}\n{s}\n+\n{'F' * len(s)}\n"  # noqa: E731
    rows4 = [["AAAA", "CCCC", "5", "AAAA", "CCCC", "demuxable", "S1", "True"],
             ["GGGG", "TTTT", "5", "GGGG", "TTTT", "demuxable", "S2", "True"],
             ["AAAA", "TTTT", "2", "AAAA", "TTTT", "index_hop", "", "True"],
             ["ACGT", "ACGT", "1", "", "", "undetermined", "", "True"],
             ["acgt", "TTTT", "1", "", "", "ambiguous", "", "True"]]
    r1 = "".join(rec(hdr.format(i, i, c).replace(" 2:", " 1:")) for i, c in
                 enumerate(["AAAA+CCCC", "GGGG+TTTT", "AAAA+TTTT", "ACGT+ACGT", "acgt+TTTT", "AAAA+CCCC"]))
    r2 = "".join(rec(hdr.format(i, i, c), "TTGCA") for i, c in
                 enumerate(["AAAA+CCCC", "GGGG+TTTT", "AAAA+TTTT", "ACGT+ACGT", "acgt+TTTT", "AAAA+CCCC"]))
    return [
        syn_pair_case("syn_basic", 24, 3000, 2),
        syn_pair_case("syn_no_hop", 24, 2000, 1, flags={"no_index_hop": True}),
        syn_pair_case("syn_no_hop_amb", 24, 2000, 1, flags={"no_index_hop": True, "no_ambiguous": True}),
        syn_pair_case("syn_infix", 24, 1500, 1, flags={"o": "run7"}),
        syn_pair_case("syn_crlf", 12, 1000, 1, nl="\r\n"),
        syn_pair_case("syn_r2_short", 12, 1000, 1, r2_trim_lines=5),
        syn_pair_case("syn_missing_code", 12, 1000, 1, drop_codes=1),
        syn_pair_case("syn_no_undet", 12, 1000, 1, flags={"no_undeter": True}),
        syn_pair_case("syn_no_samples", 12, 1000, 1, flags={"no_samples": True}),
        syn_pair_case("syn_scan_order_csv", 12, 1000, 1, results_header=SCAN_COLS,
                      flags={"reference_reads_readme_order": True}),
        # the reference itself on scan's own column order: its AssertionError (strict parity)
        syn_pair_case("syn_scan_order_strict", 12, 1000, 1, results_header=SCAN_COLS,
                      flags={"strict_header": True}),
        # BASELINE config 5 shape: 96 samples, scan's own CSV fed to demux (paired, 2 lanes)
        syn_pair_case("syn96_scan_csv", 96, 20000, 2, results_header=SCAN_COLS,
                      flags={"reference_reads_readme_order": True}),
        syn_pair_case("syn_bad_header", 12, 500, 1,
                      results_header=["idx1", "idx2", "reads", "matched_idx1", "read_type", "matched_idx2",
                                      "sample_name", "demux_ok"]),
        syn_pair_case("syn_bad_type", 12, 1000, 1, tamper=hop_to_weird),
        hand_case("hand_mixed", r1, r2, rows4),
        hand_case("hand_extra_colons", r1, r2.replace(" 2:N:0:", " 2:N:0:x:y:"), rows4),
        hand_case("hand_partial_last", r1 + "@M1:1:FC:1:1101:9:9 1:N:0:AAAA+CCCC\nAC\n",
                  r2 + "@M1:1:FC:1:1101:9:9 2:N:0:AAAA+CCCC\nAC", rows4),
        hand_case("hand_lone_cr", r1.replace("\n", "\r"), r2.replace("\n", "\r"), rows4),
    ]


def run_reference(ref, d, flags):
    results = os.path.join(d, "inputs", "results.csv")
    if flags.get("reference_reads_readme_order"):
        results = os.path.join(d, "results_readme_order.csv")
        readme_order_copy(os.path.join(d, "inputs", "results.csv"), results)
    args = argparse.Namespace(r=results, d=os.path.join(d, "out"),
                              o=flags.get("o"), no_index_hop=flags.get("no_index_hop", False),
                              no_ambiguous=flags.get("no_ambiguous", False),
                              no_undeter=flags.get("no_undeter", False), no_samples=flags.get("no_samples", False),
                              strict_header=flags.get("strict_header", False),
                              files=[os.path.join(d, "inputs", f) for f in sorted(os.listdir(os.path.join(d, "inputs")))
                                     if f.endswith(".gz")])
    ref.args = args  # open_files() reads the module-global args (frender.py:671)
    buf = io.StringIO()
    err = None
    with contextlib.redirect_stdout(buf):
        try:
            ref.frender_demux(args)
        except BaseException as e:  # noqa: BLE001 - recorded as the expected failure
            err = {"type": type(e).__name__, "message": str(e)}
    return buf.getvalue(), err


def main(names):
    ref = load_reference()
    os.makedirs(CASES_DIR, exist_ok=True)
    for name, build, flags in all_cases():
        if names and name not in names:
            continue
        with tempfile.TemporaryDirectory() as tmp:
            inp = os.path.join(tmp, "inputs")
            os.makedirs(inp)
            build(inp)
            stdout, err = run_reference(ref, tmp, flags)
            case = os.path.join(CASES_DIR, name)
            shutil.rmtree(case, ignore_errors=True)
            shutil.copytree(inp, os.path.join(case, "inputs"))
            exp = os.path.join(case, "expected")
            os.makedirs(exp)
            # normalise the temp paths in messages / stdout
            stdout = stdout.replace(tmp, "<case>")
            with open(os.path.join(exp, "stdout.txt"), "w") as f:
                f.write(stdout)
            if err:
                err["message"] = err["message"].replace(tmp, "<case>")
                with open(os.path.join(exp, "error.json"), "w") as f:
                    json.dump(err, f, indent=1)
            outd = os.path.join(tmp, "out")
            if not err and os.path.isdir(outd):
                for fn in sorted(os.listdir(outd)):
                    with gzip.open(os.path.join(outd, fn), "rb") as g:
                        content = g.read()
                    with open(os.path.join(exp, fn + ".content.gz"), "wb") as f:
                        f.write(gzip.compress(content, compresslevel=6, mtime=0))
            with open(os.path.join(case, "spec.json"), "w") as f:
                json.dump({"flags": flags}, f, indent=1, sort_keys=True)
            print(f"{name}: {'error ' + err['type'] if err else 'ok'}")


if __name__ == "__main__":
    main(sys.argv[1:])
