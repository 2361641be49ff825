"""Shared golden-case runner: rebuild a case's inputs, run an implementation's
`scan(args)` in a scratch CWD, and compare its outputs with the reference's.

The expected outputs under tests/golden/cases/*/expected were produced by the
reference itself (tests/golden/make_golden.py).  This file reads them as data;
it never touches /root/reference (which is absent on the GPU box).
"""
from __future__ import annotations

import argparse
import contextlib
import glob
import gzip
import io
import json
import os
import re
import shutil
import tempfile

from frender_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = os.path.join(HERE, "golden", "cases")
TS = re.compile(r"\d{4}-\d{2}-\d{2}_\d{4}_UTC")


def case_names():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(CASES, "*")) if os.path.isdir(p))


def load_spec(name: str) -> dict:
    with open(os.path.join(CASES, name, "spec.json")) as f:
        return json.load(f)


def build_inputs(name: str, d: str) -> dict:
    spec = load_spec(name)
    src = os.path.join(CASES, name, "inputs")
    for root, _, files in os.walk(src):
        for fn in files:
            rel = os.path.relpath(os.path.join(root, fn), src)
            os.makedirs(os.path.dirname(os.path.join(d, rel)) or d, exist_ok=True)
            shutil.copyfile(os.path.join(root, fn), os.path.join(d, rel))
    syn = spec["synthetic"]
    if syn:
        sheet = synth.make_sheet(syn["S"], syn["L"], syn["L"], seed=42,
                                 combinatorial=tuple(syn["comb"]) if syn["comb"] else None)
        rc_names = set(syn["rc_names"]) if syn.get("rc_names") else None
        synth.make_dataset(d, sheet, syn["n_reads"], syn["n_files"], R=syn["R"], seed=syn["seed"],
                           rc_names=rc_names, name_fmt=syn["name_fmt"])
    return spec


def run_impl(scan_fn, d: str, args: dict, extra: dict | None = None):
    a = dict(args)
    if extra:
        a.update(extra)
    ns = argparse.Namespace(**a)
    buf = io.StringIO()
    cwd = os.getcwd()
    before = set(os.listdir(d))
    os.chdir(d)
    err = None
    try:
        with contextlib.redirect_stdout(buf):
            try:
                scan_fn(ns)
            except SystemExit as e:
                err = {"type": "SystemExit", "msg": str(e.code)}
            except Exception as e:  # noqa: BLE001
                err = {"type": type(e).__name__, "msg": str(e)}
    finally:
        os.chdir(cwd)
    outs = {}
    for fn in sorted(set(os.listdir(d)) - before):
        p = os.path.join(d, fn)
        if os.path.isfile(p):
            with open(p, "rb") as f:
                outs[fn] = f.read()
    return outs, err, buf.getvalue()


def expected(name: str):
    spec = load_spec(name)
    outs = {}
    for o in spec["expected"]["outputs"]:
        with gzip.open(os.path.join(CASES, name, "expected", o["file"]), "rb") as g:
            outs[o["name"]] = g.read()
    with open(os.path.join(CASES, name, "expected", "stdout.txt")) as f:
        stdout = f.read()
    return outs, spec["expected"]["error"], stdout


def _norm_name(n: str) -> str:
    return TS.sub("<TS>", n)


def found_lines(stdout: str):
    return re.findall(r"found \d+ new barcodes? in \d+ reads\.", stdout)


def compare(name: str, outs: dict, err, stdout: str, check_stdout: bool = True) -> list:
    """Return a list of human-readable differences (empty = identical)."""
    exp_outs, exp_err, exp_stdout = expected(name)
    diffs = []
    if (err or {}).get("type") != (exp_err or {}).get("type"):
        diffs.append(f"error: got {err} expected {exp_err}")
    elif err and err["msg"] != exp_err["msg"]:
        diffs.append(f"error message: got {err['msg']!r} expected {exp_err['msg']!r}")
    got = {_norm_name(k): v for k, v in outs.items()}
    exp = {_norm_name(k): v for k, v in exp_outs.items()}
    if sorted(got) != sorted(exp):
        diffs.append(f"output files: got {sorted(got)} expected {sorted(exp)}")
    for k in sorted(set(got) & set(exp)):
        if got[k] != exp[k]:
            gl, el = got[k].split(b"\r\n"), exp[k].split(b"\r\n")
            first = next((i for i, (a, b) in enumerate(zip(gl, el)) if a != b), min(len(gl), len(el)))
            diffs.append(f"{k}: differs at line {first}: got {gl[first:first + 2]} expected {el[first:first + 2]} "
                         f"(rows got {len(gl)} expected {len(el)})")
    if check_stdout and found_lines(stdout) != found_lines(exp_stdout):
        diffs.append(f"per-file tally lines: got {found_lines(stdout)} expected {found_lines(exp_stdout)}")
    return diffs


def run_case(name: str, scan_fn, extra: dict | None = None, check_stdout: bool = True) -> list:
    with tempfile.TemporaryDirectory() as d:
        spec = build_inputs(name, d)
        outs, err, stdout = run_impl(scan_fn, d, spec["args"], extra)
    return compare(name, outs, err, stdout, check_stdout)
