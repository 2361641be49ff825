"""Host plumbing of `scan`: core policy, sample-sheet and input discovery.

Same names, argument meaning and failure behaviour as the reference's helpers
(frender.py:9-151); these are configuration rules, not hot-path work.
"""
from __future__ import annotations

import csv
import os
import re
from math import floor
from pathlib import Path


def get_cores(cores: float) -> int:
    """frender.py:9-22 — 0: all available, (0,1): fraction (>= 1), >= 1: int(cores)."""
    assert cores >= 0, "Number of cores is negative... what does that mean?"
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    if cores == 0:
        return avail
    if 0 < cores < 1:
        return max(floor(cores * avail), 1)
    return int(cores)


def find_barcode_file(directory) -> Path:
    """frender.py:25-49 — note the code keeps the lexicographically LARGEST match (:42)."""
    d = Path(directory)
    assert Path.is_dir(d), "The specified directory does not exist"
    hits = [p for p in d.rglob("**/*")
            if bool(re.search("barcode.*association", str(p), re.IGNORECASE))
            | bool(re.search("sample.*sheet", str(p), re.IGNORECASE))]
    hits = [p for p in hits if re.search(r"\.csv$|\.txt$", str(p), re.IGNORECASE)]
    hits.sort(reverse=True)
    if not hits:
        raise SystemExit("I couldn't find a barcode table in that directory. Please either specify one with the argment "
                         "-b or specify a directory including a barcode table. File names matching "
                         "'.*barcode.*association.*' or '.*sample.*sheet.*' (case insensitive) are accepted.")
    print(f"Found barcode association file {os.path.basename(hits[0])}")
    return hits[0]


def handle_illumina_csv(barcode_file) -> int:
    """frender.py:52-62 — rows to skip: through the "[Data]" row when row 0 is "[Header]"."""
    with open(barcode_file, "r") as f:
        reader = csv.reader(f)
        header = next(reader)
        if re.search(r"\[Header\]", header[0]):
            i = 1
            while not re.search(r"\[Data\]", next(reader)[0]):
                i += 1
            return i + 1
        return 0


def get_col(match_pattern: str, cols, discard_pattern: str | None = None) -> int:
    """frender.py:65-87 — index of the first column matching (and not discard_pattern)."""
    for i, s in enumerate(cols):
        if re.search(match_pattern, s, flags=re.IGNORECASE) and not (
                discard_pattern and re.search(discard_pattern, s, flags=re.IGNORECASE)):
            return i
    raise ValueError(
        f"""Couldn't find column matching "{match_pattern}"{' but not "' + discard_pattern + '"' if discard_pattern is not None else ''} in csv header {cols}""")


def get_indexes(barcode_file) -> dict:
    """frender.py:90-116 — {"id": [...], "idx1": [...], "idx2": [...]} in sheet row order."""
    skip = handle_illumina_csv(barcode_file)
    with open(barcode_file, "r") as f:
        reader = csv.reader(f)
        for _ in range(skip):
            next(reader)
        header = next(reader)
        try:
            id_col = get_col("id|name", header)
            idx1_col = get_col("index", header, "id|2")
            idx2_col = get_col("index.*2", header)
        except ValueError as e:
            print("Error finding columns in provided barcode file:")
            raise SystemExit(e)
        out = {"id": [], "idx1": [], "idx2": []}
        for row in reader:
            out["id"].append(row[id_col])
            out["idx1"].append(row[idx1_col])
            out["idx2"].append(row[idx2_col])
        return out


def parse_files(file_dict: dict, just_r1: bool) -> list:
    """frender.py:119-151 — the input order defines the output row order (R5)."""
    kind = list(file_dict.keys())[0]
    paths = []
    if kind == "dir":
        print(f"Scanning {file_dict['dir']} for fastq files. {'Using read 1 files only for speed...' if just_r1 else ''}")
        paths = [p for p in Path(file_dict["dir"]).rglob("**/*") if Path.is_file(p)]
    elif kind == "file":
        v = file_dict["file"]
        paths = [Path(a) for a in v if Path.is_file(Path(a))] if isinstance(v, list) else [v]
    kept = []
    for p in paths:
        if re.search(r"\.f[ast]*q\.gz$", str(p), re.IGNORECASE):
            kept.append(p)
        else:
            print(f"Ignoring non-fastq file {os.path.basename(p)}")
    if kind == "dir" and just_r1:
        kept = [p for p in kept if re.search("R1", os.path.basename(p), re.IGNORECASE)]
    return kept


def reverse_complement(s: str) -> str:
    """frender.py:210-211."""
    return s.translate(str.maketrans("ATGCNatgcn", "TACGNtacgn"))[::-1]
