#!/usr/bin/env python3
"""Generate the golden parity fixtures by running REFERENCE frender here.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden.py            # all cases
    python tests/golden/make_golden.py cfg1 crlf  # some cases

For every case it builds the inputs in a scratch dir (synthetic SYN-v1 inputs
from frender_amd.synth, or small hand-written FASTQ files for the edge cases of
SURVEY.md §4.2), imports /root/reference/frender.py with
importlib.util.spec_from_file_location (the CLI sits behind `__main__`,
frender.py:817, so importing runs nothing), calls `frender_scan(args)`
(frender.py:567) with an argparse Namespace, and commits under
tests/golden/cases/<name>/:

    spec.json       how to rebuild the inputs + the scan arguments
    inputs/         hand-written input files (synthetic inputs are rebuilt)
    expected/       the reference's output files (scan CSV, index-2-calls CSV),
                    stdout.txt, and error.json when the reference raised

Only DATA is committed: inputs and expected outputs.  Nothing of the
reference's source is copied.
"""
from __future__ import annotations

import argparse
import contextlib
import gzip
import hashlib
import importlib.util
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

REF_PATH = "/root/reference/frender.py"
CASES_DIR = os.path.join(HERE, "cases")


def load_reference():
    spec = importlib.util.spec_from_file_location("frender_reference", REF_PATH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# --------------------------------------------------------------------------------------
# helpers to write hand-made inputs
# --------------------------------------------------------------------------------------

def rec(header: str, seq: str = "ACGTACGT", qual: str = "FFFFFFFF", nl: str = "\n") -> str:
    return f"{header}{nl}{seq}{nl}+{nl}{qual}{nl}"


def hdr(code: str, i: int = 0, comment_prefix: str = "1:N:0:") -> str:
    return f"@M1:1:FC:1:1101:{1000 + i}:{2000 + i} {comment_prefix}{code}"


class RawGz(bytes):
    """A .gz input given as its exact file bytes (corrupt / truncated / padded streams)."""


def write_gz(path: str, text_or_bytes, members: int = 1) -> None:
    if isinstance(text_or_bytes, RawGz):
        with open(path, "wb") as f:
            f.write(bytes(text_or_bytes))
        return
    data = text_or_bytes.encode() if isinstance(text_or_bytes, str) else text_or_bytes
    synth.write_fastq_gz(path, data, level=6, members=members)


def write_sheet(path: str, rows, header=("Sample_ID", "index", "index2"), pre: str = "") -> None:
    with open(path, "w", newline="") as f:
        f.write(pre)
        f.write(",".join(header) + "\n")
        for r in rows:
            f.write(",".join(r) + "\n")


SHEET4 = [("S1", "AAAACCCC", "GGGGTTTT"), ("S2", "CCCCGGGG", "TTTTAAAA"),
          ("S3", "GGGGTTTT", "AAAACCCC"), ("S4", "TTTTAAAA", "CCCCGGGG")]


def codes_mix(n: int, seed: int = 7):
    """A small, deterministic mixture of demuxable / hop / 1-mismatch / junk codes."""
    import random
    rng = random.Random(seed)
    out = []
    for i in range(n):
        s = rng.randrange(4)
        a, b = SHEET4[s][1], SHEET4[s][2]
        u = rng.random()
        if u < 0.1:
            b = SHEET4[rng.randrange(4)][2]
        elif u < 0.2:
            j = rng.randrange(8)
            a = a[:j] + rng.choice("ACGTN") + a[j + 1:]
        elif u < 0.25:
            a = "".join(rng.choice("ACGT") for _ in range(8))
            b = "".join(rng.choice("ACGT") for _ in range(8))
        out.append(f"{a}+{b}")
    return out


# --------------------------------------------------------------------------------------
# case builders: each returns the spec dict after writing inputs into `d`
# --------------------------------------------------------------------------------------

def syn_case(name, S, L, n_reads, n_files, n, rc=False, R=8, seed=1, comb=None, rc_names=None,
             dup_row=False, s=None, p=None, o=None, name_fmt="syn_L{f:03d}_R1_001.fastq.gz"):
    def build(d):
        sheet = synth.make_sheet(S, L, L, seed=42, combinatorial=comb)
        if dup_row:
            sheet.ids.append(sheet.ids[3]); sheet.idx1.append(sheet.idx1[3]); sheet.idx2.append(sheet.idx2[3])
        sheet.write_csv(os.path.join(d, "sheet.csv"))
        return {
            "synthetic": {"S": S, "L": L, "n_reads": n_reads, "n_files": n_files, "R": R, "seed": seed,
                          "comb": comb, "rc_names": sorted(rc_names) if rc_names else None,
                          "name_fmt": name_fmt, "dup_row": dup_row},
            "args": {"n": n, "rc": rc, "c": 1.0, "s": s, "o": o, "p": p, "b": "sheet.csv",
                     "files": [name_fmt.format(f=f + 1) for f in range(n_files)]},
        }
    return name, build


def build_synthetic_inputs(d: str, syn: dict) -> None:
    """Rebuild the synthetic FASTQ inputs of a case into directory d."""
    sheet = synth.make_sheet(syn["S"], syn["L"], syn["L"], seed=42,
                             combinatorial=tuple(syn["comb"]) if syn["comb"] else None)
    rc_names = set(syn["rc_names"]) if syn.get("rc_names") else None
    synth.make_dataset(d, sheet, syn["n_reads"], syn["n_files"], R=syn["R"], seed=syn["seed"],
                       rc_names=rc_names, name_fmt=syn["name_fmt"])


def hand_case(name, files: dict, args: dict, sheet_rows=SHEET4, sheet_header=("Sample_ID", "index", "index2"),
              sheet_pre="", members=None, raw=False):
    def build(d):
        write_sheet(os.path.join(d, "sheet.csv"), sheet_rows, sheet_header, sheet_pre)
        for fn, content in files.items():
            path = os.path.join(d, fn)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            if fn.endswith(".gz"):
                write_gz(path, content, members=(members or {}).get(fn, 1))
            else:
                with open(path, "wb" if isinstance(content, bytes) else "w") as f:
                    f.write(content)
        a = {"n": 1, "rc": False, "c": 1.0, "s": None, "o": None, "p": None, "b": "sheet.csv",
             "files": sorted(k for k in files if k.endswith(".gz"))}
        a.update(args)
        return {"synthetic": None, "args": a, "inputs": sorted(files.keys()) + ["sheet.csv"]}
    return name, build


def all_cases():
    mix = codes_mix(400)
    lines = "".join(rec(hdr(c, i)) for i, c in enumerate(mix))
    cases = [
        # BASELINE config 1 (the CPU plumbing case)
        syn_case("cfg1_10k_s4_n0", 4, 8, 10_000, 1, 0),
        syn_case("s96_n1_4files", 96, 8, 60_000, 4, 1),
        syn_case("s96_n1_rc", 96, 8, 40_000, 2, 1, rc=True, rc_names={"Sample_005", "Sample_017"}),
        syn_case("s96_n2", 96, 8, 20_000, 1, 2),
        syn_case("s384_l10_n1_rc_dup", 384, 10, 30_000, 2, 1, rc=True,
                 rc_names={"Sample_002", "Sample_100", "Sample_300"}, dup_row=True),
        syn_case("comb96_n2", 96, 8, 20_000, 1, 2, comb=(12, 8)),
        syn_case("comb96_n1_rc", 96, 8, 20_000, 1, 1, rc=True, comb=(12, 8), rc_names={"Sample_010", "Sample_011"}),
        syn_case("s96_r150_n1", 96, 8, 5_000, 1, 1, R=150),
        syn_case("s96_sample2k", 96, 8, 20_000, 2, 1, s=2000),
        # demux_ok: files named after samples / undetermined, -p prefix removal
        syn_case("demuxok_names", 4, 8, 8_000, 4, 1, p="Sample_",
                 name_fmt="{f:03d}_Undetermined_R1_001.fastq.gz"),
        hand_case("mix_plain", {"a_R1.fastq.gz": lines}, {"n": 1}),
        hand_case("mix_n0", {"a_R1.fastq.gz": lines}, {"n": 0}),
        hand_case("mix_n3", {"a_R1.fastq.gz": lines}, {"n": 3}),
        hand_case("mix_neg", {"a_R1.fastq.gz": lines}, {"n": -1}),
        hand_case("crlf", {"a_R1.fq.gz": "".join(rec(hdr(c, i), nl="\r\n") for i, c in enumerate(mix[:50]))}, {}),
        hand_case("cr_only", {"a_R1.fq.gz": "".join(rec(hdr(c, i), nl="\r") for i, c in enumerate(mix[:50]))}, {}),
        hand_case("mixed_newlines", {"a_R1.fq.gz": "".join(
            rec(hdr(c, i), nl=["\n", "\r\n", "\r"][i % 3]) for i, c in enumerate(mix[:60]))}, {}),
        hand_case("lone_cr_in_seq", {"a_R1.fq.gz": rec(hdr(mix[0])) + rec(hdr(mix[1]), seq="ACGT\rACGT") +
                                     rec(hdr(mix[2])) + rec(hdr(mix[3]))}, {}),
        hand_case("no_trailing_newline", {"a_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[:20]))[:-1]}, {}),
        hand_case("truncated_record", {"a_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[:20])) +
                                       hdr(mix[21], 21) + "\nACGT\n"}, {}),
        hand_case("lowercase", {"a_R1.fq.gz": "".join(rec(hdr(c.lower() if i % 3 == 0 else c, i))
                                                      for i, c in enumerate(mix[:90]))}, {}),
        hand_case("n_in_index", {"a_R1.fq.gz": "".join(rec(hdr("NAAACCCC+GGGGTTTN", i)) for i in range(5)) +
                                 "".join(rec(hdr("AAAACCCC+GGGGTTTT", i)) for i in range(5))},
                  {"n": 1}, sheet_rows=SHEET4 + [("SN", "NNNNNNNN", "NNNNNNNN")]),
        hand_case("three_part_code", {"a_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(
            ["AAAACCCC+GGGGTTTT+ACGT", "AAAACCCC+GGGGTTTT", "AAAACCCC+GGGGTTTT+ACGT", "CCCCGGGG+TTTTAAAA+"]))}, {}),
        hand_case("third_field_ignored", {"a_R1.fq.gz": "".join(
            rec(f"@M1:1:FC:1:1101:{i}:1 1:N:0:{c} extra:ZZZ") for i, c in enumerate(mix[:30]))}, {}),
        hand_case("tab_tags", {"a_R1.fq.gz": "".join(
            rec(f"@M1:1:FC:1:1101:{i}:1 1:N:0:{c}\tBX:Z:AAA") for i, c in enumerate(mix[:10]))}, {}),
        hand_case("no_colon_token", {"a_R1.fq.gz": "".join(rec(f"@read{i} {c}") for i, c in enumerate(mix[:30]))}, {}),
        hand_case("no_space_header", {"a_R1.fq.gz": rec(hdr(mix[0])) + rec("@M1:1:FC:1:1101:1:2:AAAACCCC+GGGGTTTT")}, {}),
        hand_case("empty_header_line", {"a_R1.fq.gz": rec(hdr(mix[0])) + "\nACGT\n+\nFFFF\n"}, {}),
        hand_case("single_index", {"a_R1.fq.gz": "".join(rec(hdr("AAAACCCC", i)) for i in range(3))}, {}),
        hand_case("len_mismatch", {"a_R1.fq.gz": rec(hdr("AAAACCCCA+GGGGTTTT"))}, {}),
        hand_case("dup_sheet_row", {"a_R1.fq.gz": lines}, {"n": 1}, sheet_rows=SHEET4 + [SHEET4[1]]),
        hand_case("rc_basic", {"a_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(
            ["AAAACCCC+AAAACCCC"] * 30 + ["CCCCGGGG+TTTTAAAA"] * 10 + ["GGGGTTTT+GGTTTTTT"] * 5 +
            ["AAAACCCC+GGGGTTTT"] * 7 + ["TTTTAAAA+CCGGGGCC"] * 3))}, {"rc": True}),
        hand_case("rc_palindrome_ambig", {"a_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(
            ["AAAACCCC+ACGTACGT"] * 4 + ["CCCCGGGG+AACCGGTT"] * 3 + ["AAAACCCC+ACGTTTTT"] * 2))},
            {"rc": True, "n": 1},
            sheet_rows=[("P1", "AAAACCCC", "ACGTACGT"), ("P2", "CCCCGGGG", "AACCGGTT"),
                        ("P3", "AAAACCCC", "AAAAACGT")]),
        hand_case("sample_limit", {"a_R1.fq.gz": lines, "b_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[100:300]))},
                  {"s": 37, "files": ["a_R1.fq.gz", "b_R1.fq.gz"]}),
        hand_case("two_files_order", {"x_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[200:300])),
                                      "y_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[:200]))},
                  {"files": ["y_R1.fq.gz", "x_R1.fq.gz"]}),
        hand_case("same_file_twice", {"a_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[:50]))},
                  {"files": ["a_R1.fq.gz", "a_R1.fq.gz"]}),
        hand_case("same_basename_two_dirs", {"d1/S1_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[:40])),
                                             "d2/S1_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[40:60]))},
                  {"files": ["d1/S1_R1.fq.gz", "d2/S1_R1.fq.gz"]}),
        hand_case("multi_member_gz", {"a_R1.fq.gz": lines}, {}, members={"a_R1.fq.gz": 7}),
        hand_case("non_fastq_ignored", {"a_R1.fq.gz": lines, "notes.txt": "hello\n"},
                  {"files": ["a_R1.fq.gz", "notes.txt"]}),
        hand_case("missing_file_dropped", {"a_R1.fq.gz": lines}, {"files": ["a_R1.fq.gz", "nope_R1.fq.gz"]}),
        hand_case("demux_ok_samples", {
            "S1_R1_001.fastq.gz": "".join(rec(hdr("AAAACCCC+GGGGTTTT", i)) for i in range(20)),
            "S2_R1_001.fastq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(["CCCCGGGG+TTTTAAAA"] * 9 + ["AAAACCCC+GGGGTTTT"])),
            "Undetermined_S0_R1_001.fastq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[:60])),
            "Index-hop_R1.fastq.gz": "".join(rec(hdr("AAAACCCC+TTTTAAAA", i)) for i in range(4)),
        }, {"files": ["S1_R1_001.fastq.gz", "S2_R1_001.fastq.gz", "Undetermined_S0_R1_001.fastq.gz",
                      "Index-hop_R1.fastq.gz"]}),
        hand_case("demux_ok_prefix", {
            "1_R1.fq.gz": "".join(rec(hdr("AAAACCCC+GGGGTTTT", i)) for i in range(5)),
            "2_R1.fq.gz": "".join(rec(hdr("CCCCGGGG+TTTTAAAA", i)) for i in range(5)),
        }, {"files": ["1_R1.fq.gz", "2_R1.fq.gz"], "p": "Lib-"},
            sheet_rows=[("Lib-1", "AAAACCCC", "GGGGTTTT"), ("Lib-2", "CCCCGGGG", "TTTTAAAA")]),
        hand_case("illumina_sheet", {"a_R1.fq.gz": lines}, {},
                  sheet_header=("Sample_ID", "Sample_Name", "I7_Index_ID", "index", "I5_Index_ID", "index2"),
                  sheet_rows=[(s, s + "_name", "i7", a, "i5", b) for s, a, b in SHEET4],
                  sheet_pre="[Header]\nIEMFileVersion,4\nDate,1/1/2020\n[Reads]\n151\n151\n[Data]\n"),
        hand_case("sheet_lowercase_idx", {"a_R1.fq.gz": lines}, {},
                  sheet_rows=[(s, a.lower(), b) for s, a, b in SHEET4]),
        hand_case("empty_fastq", {"a_R1.fq.gz": ""}, {}),
        hand_case("output_infix", {"a_R1.fq.gz": lines}, {"o": "run7"}),
        hand_case("dir_mode", {"run/a_R1_001.fq.gz": lines,
                               "run/a_R2_001.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[:7]))},
                  {"files": ["run"], "b": "sheet.csv"}),
        hand_case("at_in_quality", {"a_R1.fq.gz": "".join(rec(hdr(c, i), qual="@@@@FFFF") for i, c in enumerate(mix[:40]))}, {}),
        hand_case("long_code", {"a_R1.fq.gz": "".join(rec(hdr("A" * 20 + "+" + "C" * 20, i)) for i in range(3))}, {},
                  sheet_rows=[("L1", "A" * 20, "C" * 20), ("L2", "C" * 20, "A" * 20)]),
        hand_case("unicode_header", {"a_R1.fq.gz": rec(hdr("AAAACCCC+GGGGTTTT")) + rec("@M1:ü:1 1:N:0:AAAACCCC+GGGGTTTT")}, {}),
        hand_case("bad_utf8", {"a_R1.fq.gz": (rec(hdr("AAAACCCC+GGGGTTTT")).encode() + b"@M1:\xff 1:N:0:AAAACCCC+GGGGTTTT\nAC\n+\nFF\n")}, {}),
        # UTF-8 errors far into a file: the message's position is relative to the reader's decode chunk;
        # with -s the reference fails only if the bad bytes are decoded before the sample ends
        hand_case("bad_utf8_deep", {"a_R1.fq.gz": lines.encode() + b"@M1:x 1:N:0:AAAA\xc3\x28CCCC+GGGGTTTT\nAC\n+\nFF\n" +
                                    lines.encode()}, {}),
        hand_case("bad_utf8_past_sample", {"a_R1.fq.gz": lines.encode() + b"@M1:x 1:N:0:AAAACCCC+GGGGTTTT\xff\nAC\n+\nFF\n",
                                           "b_R1.fq.gz": lines.encode()},
                  {"s": 5, "files": ["a_R1.fq.gz", "b_R1.fq.gz"]}),
        hand_case("bad_utf8_in_sample_chunk", {"a_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(mix[:40])).encode() +
                                               b"@M1:x 1:N:0:AAAACCCC+GGGGTTTT\xe2\x82\nAC\n+\nFF\n" + lines.encode()},
                  {"s": 30}),
        # gzip stream edge cases (native inflate): the reference's gzip reader decides
        hand_case("gz_truncated", {"a_R1.fq.gz": RawGz(gzip.compress(lines.encode(), 6)[:-900])}, {}),
        hand_case("gz_corrupt", {"a_R1.fq.gz": RawGz(gzip.compress(lines.encode(), 6)[:300] + b"\xff" * 64 +
                                                     gzip.compress(lines.encode(), 6)[364:])}, {}),
        hand_case("gz_nul_padding", {"a_R1.fq.gz": RawGz(gzip.compress(lines.encode()[:9000], 6) + b"\0" * 4096 +
                                                         gzip.compress(lines.encode()[9000:], 1) + b"\0" * 7)}, {}),
        hand_case("gz_trailing_garbage", {"a_R1.fq.gz": RawGz(gzip.compress(lines.encode(), 6) + b"garbage")}, {}),
        hand_case("gz_not_gzip", {"a_R1.fq.gz": RawGz(lines.encode()[:5000])}, {}),
        hand_case("gz_empty_file", {"a_R1.fq.gz": RawGz(b""), "b_R1.fq.gz": lines},
                  {"files": ["a_R1.fq.gz", "b_R1.fq.gz"]}),
        hand_case("gz_bad_crc", {"a_R1.fq.gz": RawGz(gzip.compress(lines.encode(), 6)[:-8] + b"\0\0\0\0" +
                                                     gzip.compress(lines.encode(), 6)[-4:])}, {}),
        hand_case("wide_codes_12", {"a_R1.fq.gz": "".join(rec(hdr(c, i)) for i, c in enumerate(
            ["AAAACCCCGGGG+TTTTAAAACCCC", "AAAACCCCGGGG+TTTTAAAACCCN", "aaaaccccgggg+ttttaaaacccc", "AAAACCCCGGGG+TTTTAAAACCCC",
             "CCCCGGGGTTTT+AAAACCCCGGGG", "ACGTACGTACGT+ACGTACGTACGT", "AAAACCCCGGGa+TTTTAAAACCCC", "NNNNNNNNNNNN+NNNNNNNNNNNN",
             "CCCCGGGGTTTT+AAAACCCCGGGG+ACGT", "AAAACCCCGGGG+TTTTAAAACCCG"] * 3))}, {"n": 1},
            sheet_rows=[("W1", "AAAACCCCGGGG", "TTTTAAAACCCC"), ("W2", "CCCCGGGGTTTT", "AAAACCCCGGGG")]),
    ]
    return cases


def run_reference(ref, d: str, args: dict):
    """Run reference frender_scan in directory d; return (stdout, error|None)."""
    ns = argparse.Namespace(**args)
    buf = io.StringIO()
    cwd = os.getcwd()
    os.chdir(d)
    err = None
    try:
        with contextlib.redirect_stdout(buf):
            try:
                ref.frender_scan(ns)
            except SystemExit as e:
                err = {"type": "SystemExit", "msg": str(e.code)}
            except Exception as e:  # noqa: BLE001 - we record the reference's failure mode
                err = {"type": type(e).__name__, "msg": str(e)}
    finally:
        os.chdir(cwd)
    return buf.getvalue(), err


def main(argv):
    ref = load_reference()
    names = set(argv[1:])
    os.makedirs(CASES_DIR, exist_ok=True)
    for name, build in all_cases():
        if names and name not in names:
            continue
        out = os.path.join(CASES_DIR, name)
        shutil.rmtree(out, ignore_errors=True)
        os.makedirs(os.path.join(out, "expected"))
        with tempfile.TemporaryDirectory() as d:
            spec = build(d)
            if spec["synthetic"]:
                build_synthetic_inputs(d, spec["synthetic"])
            before = set(os.listdir(d))
            stdout, err = run_reference(ref, d, spec["args"])
            produced = sorted(set(os.listdir(d)) - before)
            # commit hand-written inputs and the sheet
            os.makedirs(os.path.join(out, "inputs"))
            for fn in spec.get("inputs", ["sheet.csv"]):
                dst = os.path.join(out, "inputs", fn)
                os.makedirs(os.path.dirname(dst), exist_ok=True)
                shutil.copyfile(os.path.join(d, fn), dst)
            if spec["synthetic"]:
                md5 = {}
                for f in spec["args"]["files"]:
                    with gzip.open(os.path.join(d, f), "rb") as g:
                        md5[f] = hashlib.md5(g.read()).hexdigest()
                spec["synthetic"]["decoded_md5"] = md5
            outputs = []
            for fn in produced:
                src = os.path.join(d, fn)
                if os.path.isfile(src):
                    with open(src, "rb") as f:
                        data = f.read()
                    kind = "rc_csv" if fn.startswith("frender-index-2-calls_") else "scan_csv"
                    store = kind + ".csv.gz"
                    with gzip.open(os.path.join(out, "expected", store), "wb", compresslevel=9) as g:
                        g.write(data)
                    outputs.append({"kind": kind, "name": fn, "file": store})
            spec["expected"] = {"outputs": outputs, "error": err}
            with open(os.path.join(out, "expected", "stdout.txt"), "w") as f:
                f.write(stdout)
            with open(os.path.join(out, "spec.json"), "w") as f:
                json.dump(spec, f, indent=1, sort_keys=True)
        print(f"{name:28s} outputs={[o['kind'] for o in outputs]} error={err}")


if __name__ == "__main__":
    main(sys.argv)
