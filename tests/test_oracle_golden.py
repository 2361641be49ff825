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
