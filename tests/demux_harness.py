"""Shared runner for the demux golden cases (tests/golden/demux/*, made by the reference).

Cases whose spec has "reference_reads_readme_order" feed `scan`'s own CSV column order, which the
reference rejects (frender.py:649-657): the reference was run on a README-order copy, so those cases
pin the build's documented deviation (accepting scan's order), not parity.  Parity for that input is
pinned by syn_scan_order_strict: strict_header=True, the reference fed the scan-order CSV itself,
expected = its AssertionError."""
import argparse
import contextlib
import gzip
import io
import json
import os
import shutil
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = os.path.join(HERE, "golden", "demux")


def case_names():
    return sorted(os.listdir(CASES)) if os.path.isdir(CASES) else []


def run_case(name, demux_fn):
    """Run demux_fn(args) on the case's inputs; return a list of differences (empty = parity)."""
    case = os.path.join(CASES, name)
    flags = json.load(open(os.path.join(case, "spec.json")))["flags"]
    exp_dir = os.path.join(case, "expected")
    diffs = []
    with tempfile.TemporaryDirectory() as tmp:
        shutil.copytree(os.path.join(case, "inputs"), os.path.join(tmp, "inputs"))
        inp = os.path.join(tmp, "inputs")
        args = argparse.Namespace(r=os.path.join(inp, "results.csv"), d=os.path.join(tmp, "out"), o=flags.get("o"),
                                  no_index_hop=flags.get("no_index_hop", False),
                                  no_ambiguous=flags.get("no_ambiguous", False),
                                  no_undeter=flags.get("no_undeter", False),
                                  no_samples=flags.get("no_samples", False),
                                  strict_header=flags.get("strict_header", False),
                                  files=[os.path.join(inp, f) for f in sorted(os.listdir(inp)) if f.endswith(".gz")])
        buf = io.StringIO()
        err = None
        with contextlib.redirect_stdout(buf):
            try:
                demux_fn(args)
            except BaseException as e:  # noqa: BLE001
                err = {"type": type(e).__name__, "message": str(e).replace(tmp, "<case>")}
        want_err = None
        if os.path.exists(os.path.join(exp_dir, "error.json")):
            want_err = json.load(open(os.path.join(exp_dir, "error.json")))
        if err != want_err:
            diffs.append(f"error: got {err} want {want_err}")
        want_out = open(os.path.join(exp_dir, "stdout.txt")).read()
        if buf.getvalue().replace(tmp, "<case>") != want_out:
            diffs.append(f"stdout: got {buf.getvalue()!r} want {want_out!r}")
        if want_err is None:
            outd = os.path.join(tmp, "out")
            got = sorted(os.listdir(outd)) if os.path.isdir(outd) else []
            want = sorted(f[:-len(".content.gz")] for f in os.listdir(exp_dir) if f.endswith(".content.gz"))
            if got != want:
                diffs.append(f"output files: got {got} want {want}")
            for fn in set(got) & set(want):
                with gzip.open(os.path.join(outd, fn), "rb") as g:
                    a = g.read()
                with gzip.open(os.path.join(exp_dir, fn + ".content.gz"), "rb") as g:
                    b = g.read()
                if a != b:
                    diffs.append(f"{fn}: content differs ({len(a)} vs {len(b)} bytes)")
    return diffs


def run_case_cli(name, gpus=2):
    """The case through `python -m frender_amd demux --gpus N` (N ranks rehearsed on this box's GPU over
    gloo): the same comparisons as run_case; an expected error must end the command with its message."""
    import subprocess
    import sys
    case = os.path.join(CASES, name)
    flags = json.load(open(os.path.join(case, "spec.json")))["flags"]
    exp_dir = os.path.join(case, "expected")
    diffs = []
    with tempfile.TemporaryDirectory() as tmp:
        shutil.copytree(os.path.join(case, "inputs"), os.path.join(tmp, "inputs"))
        inp = os.path.join(tmp, "inputs")
        cmd = [sys.executable, "-m", "frender_amd", "demux", "--gpus", str(gpus), "-r", os.path.join(inp, "results.csv"),
               "-d", os.path.join(tmp, "out")]
        if flags.get("o"):
            cmd += ["-o", flags["o"]]
        for f, opt in (("no_index_hop", "-i"), ("no_ambiguous", "-a"), ("no_undeter", "-u"), ("no_samples", "-s"),
                       ("strict_header", "--strict-header")):
            if flags.get(f):
                cmd.append(opt)
        cmd += [os.path.join(inp, f) for f in sorted(os.listdir(inp)) if f.endswith(".gz")]
        env = dict(os.environ, FRENDER_DIST_BACKEND="gloo", PYTHONPATH=os.path.dirname(HERE))
        r = subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True, timeout=240)
        want_err = None
        if os.path.exists(os.path.join(exp_dir, "error.json")):
            want_err = json.load(open(os.path.join(exp_dir, "error.json")))
        if want_err is None and r.returncode:
            diffs.append(f"exit {r.returncode}: {r.stderr[-1500:]}")
        if want_err is not None and (not r.returncode or want_err["message"].replace("<case>", tmp) not in r.stderr):
            diffs.append(f"error: want {want_err}, exit {r.returncode}, stderr {r.stderr[-1500:]}")
        want_out = open(os.path.join(exp_dir, "stdout.txt")).read()
        out = "".join(ln for ln in r.stdout.splitlines(True) if not ln.startswith("[Gloo]"))  # gloo's banner
        if out.replace(tmp, "<case>") != want_out:
            diffs.append(f"stdout: got {out!r} want {want_out!r}")
        if want_err is None:
            outd = os.path.join(tmp, "out")
            got = sorted(os.listdir(outd)) if os.path.isdir(outd) else []
            want = sorted(f[:-len(".content.gz")] for f in os.listdir(exp_dir) if f.endswith(".content.gz"))
            if got != want:
                diffs.append(f"output files: got {got} want {want}")
            for fn in set(got) & set(want):
                with gzip.open(os.path.join(outd, fn), "rb") as g:
                    a = g.read()
                with gzip.open(os.path.join(exp_dir, fn + ".content.gz"), "rb") as g:
                    b = g.read()
                if a != b:
                    diffs.append(f"{fn}: content differs ({len(a)} vs {len(b)} bytes)")
    return diffs
