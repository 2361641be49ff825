"""fr_write_scan_csv (frender_amd/csrc/fr_csv.cpp, host only) against the row loop it replaces in
report_analysis (Python's csv module over the code strings, frender.py:482-501): byte-identical files
for fast keys (one, two and three '+' parts), wide keys (12+12, lowercase, '+' at either end), exotic
codes that need CSV quoting, sheet strings that need quoting, empty matches, with and without the
demux_ok column; and the refusal (nothing written) for a code without '+'."""
import csv
import os

import numpy as np
import pytest

from frender_amd import _lib, scan

SYM = {"A": 1, "C": 2, "G": 3, "T": 4, "N": 5, "+": 6}


def fast_key(code):
    return sum(SYM[c] << (3 * i) for i, c in enumerate(code))


def python_rows(path, header, codes, counts, m1, m2, cls, row, dok, idx1, idx2, ids):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        for j, code in enumerate(codes):
            parts = code.split("+")
            r = [parts[0], parts[1], idx1[m1[j]] if m1[j] >= 0 else "", idx2[m2[j]] if m2[j] >= 0 else "",
                 scan.CLASS_NAMES[cls[j]], ids[row[j]] if row[j] >= 0 else "", int(counts[j])]
            if dok is not None:
                r.append(bool(dok[j]))
            w.writerow(r)


def case(rng, n):
    idx1 = ["ACGTACGT", "TTGCA,CG", 'AC"GT', "", "acgtnacg"]
    idx2 = ["GGGGCCCC", "AT\rAT", "CCCC"]
    ids = ["S1", "sample 2", "a,b", 'q"uote', "S1"]
    codes, keys, exo = [], [], []
    for j in range(n):
        k = rng.integers(0, 10)
        if k < 6:  # fast: 1-3 '+' separated groups
            parts = ["".join(rng.choice(list("ACGTN"), rng.integers(0, 9))) for _ in range(rng.integers(2, 4))]
            c = "+".join(parts)
            if len(c) > 21 or not c.replace("+", ""):
                c = "ACGT+ACGT"
            codes.append(c)
            keys.append(fast_key(c))
        elif k < 8:  # wide
            a = "".join(rng.choice(list("ACGTN"), 12))
            b = "".join(rng.choice(list("ACGTN"), rng.integers(0, 13)))
            c = a + "+" + b
            if rng.integers(0, 2):
                c = c.lower()
            if rng.integers(0, 4) == 0 and len(c) <= 22:  # '+' first: <= 21 letters after it
                c = "+" + c.replace("+", "")
            w = _lib.encode_wide(c)
            assert w is not None and _lib.decode_keys(np.array([w], np.uint64))[0] == c
            codes.append(c)
            keys.append(w)
        else:  # exotic: needs quoting, or several '+'
            c = rng.choice(['AC,GT+TT"A', "xyz+é,q", "AB+CD+EF", 'a"b+', "Ac+gT"])
            codes.append(str(c))
            keys.append(0)
            exo.append(j)
    m1 = rng.integers(-1, len(idx1), n).astype(np.int16)
    m2 = rng.integers(-1, len(idx2), n).astype(np.int16)
    cls = rng.integers(0, 4, n).astype(np.uint8)
    row = rng.integers(-1, len(ids), n).astype(np.int16)
    counts = rng.integers(1, 1 << 40, n).astype(np.uint64)
    dok = rng.integers(0, 2, n).astype(bool)
    return codes, np.array(keys, np.uint64), np.array(exo, np.int64), counts, m1, m2, cls, row, dok, idx1, idx2, ids


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("with_dok", [True, False])
def test_native_csv_equals_python_csv(tmp_path, seed, with_dok):
    rng = np.random.default_rng(seed)
    codes, keys, exo, counts, m1, m2, cls, row, dok, idx1, idx2, ids = case(rng, 3000)
    dok = dok if with_dok else None
    header = ["idx1", "idx2", "matched_idx1", "matched_idx2", "read_type", "sample_name", "reads"]
    if dok is not None:
        header.append("demux_ok")
    a, b = str(tmp_path / "py.csv"), str(tmp_path / "native.csv")
    python_rows(a, header, codes, counts, m1, m2, cls, row, dok, idx1, idx2, ids)
    # exotic positions given out of order: the writer takes them sorted
    perm = rng.permutation(exo.size)
    ok = scan._write_csv_native(b, scan._csv_fields(*header) + "\r\n", keys, exo[perm], [codes[j] for j in exo[perm]],
                                counts, m1, m2, cls, row, dok, idx1, idx2, ids)
    assert ok
    assert open(a, "rb").read() == open(b, "rb").read()


def test_native_csv_refuses_code_without_plus(tmp_path):
    p = str(tmp_path / "x.csv")
    keys = np.array([fast_key("ACGT+AC"), fast_key("ACGTAC")], np.uint64)
    z16, z8 = np.zeros(2, np.int16), np.zeros(2, np.uint8)
    args = (keys, np.zeros(0, np.int64), [], np.ones(2, np.uint64), z16, z16, z8, z16, None, ["A"], ["C"], ["S"])
    assert not scan._write_csv_native(p, "h\r\n", *args)
    assert not os.path.exists(p)
    # an exotic code without '+' is refused the same way
    args = (np.array([fast_key("ACGT+AC"), 0], np.uint64), np.array([1]), ["x,y"], *args[3:])
    assert not scan._write_csv_native(p, "h\r\n", *args)
    assert not os.path.exists(p)
