"""ORACLE — CPU restatement of reference frender `scan` (TEST INFRASTRUCTURE ONLY).

This module is the parity checker.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it; the product path (frender_amd/) never
does, and must fail loudly when its HIP library is missing.

It restates the behaviour of /root/reference/frender.py (njspix/frender @ v1) in
independent code, rule by rule.  Parity is PINNED: it is
checked against golden vectors produced by running the reference itself in the
build container (tests/golden/make_golden.py -> tests/golden/cases/*), see
tests/test_oracle_golden.py.

Reference anchors (file:line in frender.py):
  sheet discovery/parsing ........ find_barcode_file :25-49, handle_illumina_csv :52-62,
                                   get_col :65-87, get_indexes :90-116
  input file rules ............... parse_files :119-151
  per-read tally (R1-R4) ......... scan_file :154-181
  fan-out + merge (R4/R5) ........ tally_barcodes :183-207
  reverse complement ............. reverse_complement :210-211
  Hamming matcher (R7) ........... get_indexes_of_approx_matches :214-234
  classifier (R8) ................ analyze_barcode :237-291
  rc wrapper (R6, R9 pass A) ..... analyze_barcodes_with_rc :294-351
  per-sample rc call (R9) ........ call_rc_mode_per_id :354-388, rewrite :618-623
  classify fan-out ............... process :391-426
  outputs (R11, R12) ............. report_rc_call_info :429-479, flatten_results :482-492,
                                   report_analysis :495-501
  demux_ok (R10) ................. call_barcodes_correctly_distributed :504-564
  driver ......................... frender_scan :567-642
"""
from __future__ import annotations

import csv
import gzip
import os
import re
from datetime import datetime, timezone
from itertools import islice
from math import floor
from multiprocessing import Pool
from pathlib import Path

LINE_END = re.compile(r"\r\n|\r|\n")
_RC = str.maketrans("ATGCNatgcn", "TACGNtacgn")


class OracleError(Exception):
    pass


# ---------------------------------------------------------------------------------------
# host configuration rules (frender.py:9-151)
# ---------------------------------------------------------------------------------------

def resolve_cores(c: float) -> int:
    """frender.py:9-22: 0 = all, (0,1) = fraction (>=1), >=1 = int(c)."""
    if c < 0:
        raise AssertionError("Number of cores is negative... what does that mean?")
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    if c == 0:
        return avail
    if 0 < c < 1:
        return max(floor(c * avail), 1)
    return int(c)


def discover_sheet(directory) -> Path:
    """frender.py:25-49: lexicographically LARGEST matching .csv/.txt path wins."""
    d = Path(directory)
    if not d.is_dir():
        raise AssertionError("The specified directory does not exist")
    hits = [p for p in d.rglob("**/*")
            if re.search("barcode.*association", str(p), re.I) or re.search("sample.*sheet", str(p), re.I)]
    hits = sorted((p for p in hits if re.search(r"\.csv$|\.txt$", str(p), re.I)), reverse=True)
    if not hits:
        raise SystemExit("I couldn't find a barcode table in that directory. Please either specify one with the "
                         "argment -b or specify a directory including a barcode table. File names matching "
                         "'.*barcode.*association.*' or '.*sample.*sheet.*' (case insensitive) are accepted.")
    print(f"Found barcode association file {os.path.basename(hits[0])}")
    return hits[0]


def _first_col(pattern: str, cols, discard: str | None = None) -> int:
    for i, name in enumerate(cols):
        if re.search(pattern, name, re.I) and not (discard and re.search(discard, name, re.I)):
            return i
    extra = f' but not "{discard}"' if discard is not None else ""
    raise ValueError(f'Couldn\'t find column matching "{pattern}"{extra} in csv header {cols}')


def read_sheet(path) -> dict:
    """frender.py:52-116.  Returns {"id": [...], "idx1": [...], "idx2": [...]} in row order."""
    with open(path, "r") as f:
        rows = csv.reader(f)
        first = next(rows)
        skip = 0
        if re.search(r"\[Header\]", first[0]):
            skip = 1
            while not re.search(r"\[Data\]", next(rows)[0]):
                skip += 1
            skip += 1
    with open(path, "r") as f:
        rows = csv.reader(f)
        for _ in range(skip):
            next(rows)
        header = next(rows)
        try:
            c_id = _first_col("id|name", header)
            c_1 = _first_col("index", header, "id|2")
            c_2 = _first_col("index.*2", header)
        except ValueError as e:
            print("Error finding columns in provided barcode file:")
            raise SystemExit(e)
        out = {"id": [], "idx1": [], "idx2": []}
        for row in rows:
            out["id"].append(row[c_id])
            out["idx1"].append(row[c_1])
            out["idx2"].append(row[c_2])
    return out


def list_inputs(spec: dict, just_r1: bool = True) -> list:
    """frender.py:119-151.  spec = {"dir": path} or {"file": path | [paths]}."""
    kind = next(iter(spec))
    if kind == "dir":
        print(f"Scanning {spec['dir']} for fastq files. {'Using read 1 files only for speed...' if just_r1 else ''}")
        paths = [p for p in Path(spec["dir"]).rglob("**/*") if p.is_file()]
    else:
        v = spec["file"]
        paths = [Path(a) for a in v if Path(a).is_file()] if isinstance(v, list) else [v]
    kept = []
    for p in paths:
        if re.search(r"\.f[ast]*q\.gz$", str(p), re.I):
            kept.append(p)
        else:
            print(f"Ignoring non-fastq file {os.path.basename(p)}")
    if kind == "dir" and just_r1:
        kept = [p for p in kept if re.search("R1", os.path.basename(p), re.I)]
    return kept


# ---------------------------------------------------------------------------------------
# R1-R4: per-read tally (frender.py:154-207)
# ---------------------------------------------------------------------------------------

def header_lines(text: str):
    """R1: universal newlines (\\r\\n, \\r, \\n end a line); yield lines 0, 4, 8, ..."""
    pos = 0
    k = 0
    n = len(text)
    while pos < n:
        m = LINE_END.search(text, pos)
        end = m.start() if m else n
        if k % 4 == 0:
            yield text[pos:end]
        k += 1
        pos = m.end() if m else n


def code_of(line: str) -> str:
    """R2: token between the 1st and 2nd ' ' (IndexError if no ' '), suffix after its last ':'."""
    return line.split(" ")[1].split(":")[-1]


def tally_text(text: str, sample=None):
    """R1-R4 on decoded text -> ({code: count} in first-occurrence order, records)."""
    return tally_headers(header_lines(text), sample)


def tally_headers(headers, sample=None):
    """R3/R4 over an iterable of header lines (line terminator stripped or "\n"-terminated)."""
    counts: dict = {}
    records = 0
    for line in headers:
        if sample and records >= sample:
            break
        records += 1
        code = code_of(line.rstrip("\n"))
        counts[code] = counts.get(code, 0) + 1
    return counts, records


def tally_file(path, sample=None):
    """R1-R4 for one file -> (basename, {code: count} in first-occurrence order, records)."""
    name = os.path.basename(str(path))
    print(f"Tallying barcodes from {name}...", end="")
    # R1 through the same text-mode reader (frender.py:159): decode errors surface chunk by chunk
    # as the reader advances, so their message and whether -s stops before them match exactly
    with gzip.open(path, "rt") as f:
        counts, records = tally_headers(islice(f, 0, None, 4), sample)
    new = len(counts)
    print(f"found {new} new barcode{'' if new == 1 else 's'} in {records} reads.")
    return name, counts, records


def tally(cores: int, paths, sample=None) -> dict:
    """R4/R5: {"total": merged in (file, first-occurrence) order, basename: per-file table}."""
    print(f"Scanning {len(paths)} files with {cores} core{'' if cores == 1 else 's'}...")
    if sample:
        if not sample >= 1:
            raise AssertionError("Number of reads to sample must be ≥ 1!")
        print(f"Sampling {sample} reads from the head of each file...")
    if cores > 1:
        with Pool(processes=cores) as pool:
            per_file = pool.starmap(tally_file, [(p, sample) for p in paths])
    else:
        per_file = [tally_file(p, sample) for p in paths]
    print(type(per_file), len(per_file))
    out = {"total": {}}
    for _, counts, _ in per_file:
        tot = out["total"]
        for k, v in counts.items():
            tot[k] = tot.get(k, 0) + v
    for name, counts, _ in per_file:
        out[name] = counts
    return out


# ---------------------------------------------------------------------------------------
# R6-R9: classification (frender.py:210-426)
# ---------------------------------------------------------------------------------------

def revcomp(s: str) -> str:
    return s.translate(_RC)[::-1]


def within(query: str, entries, n: int) -> list:
    """R7: rows whose case-folded Hamming distance to query is <= n (length must match)."""
    if not entries:
        return []
    q = query.lower()
    rows = []
    for i, e in enumerate(entries):
        t = e.lower()
        if len(q) != len(t):
            raise AssertionError(f"Barcode {q} doesn't match length of supplied barcode {t}")
        if sum(1 for a, b in zip(q, t) if a != b) <= n:
            rows.append(i)
    return rows


def classify_pair(i1: str, i2: str, idx1, idx2, ids, n: int) -> dict:
    """R8: first-row matched strings and the class from |M1 ∩ M2|."""
    m1 = within(i1, idx1, n)
    m2 = within(i2, idx2, n)
    if m1 and m2:
        both = set(m1) & set(m2)
        if not both:
            t, name = "index_hop", ""
        elif len(both) == 1:
            t, name = "demuxable", ids[next(iter(both))]
        else:
            t, name = "ambiguous", ""
        return {"matched_idx1": idx1[m1[0]], "matched_idx2": idx2[m2[0]], "read_type": t, "sample_name": name}
    return {"matched_idx1": "", "matched_idx2": "", "read_type": "undetermined", "sample_name": ""}


def classify_code(code: str, reads: int, idx1, idx2, ids, n: int, rc: bool) -> dict:
    """R6 + R9 pass A (frender.py:294-351)."""
    i1, i2 = code.split("+")[0:2]
    res = classify_pair(i1, i2, idx1, idx2, ids, n)
    res["reads"] = reads
    if rc:
        alt = classify_pair(i1, i2, idx1, [revcomp(x) for x in idx2], ids, n)
        res["matched_idx1"] = res["matched_idx1"] or alt["matched_idx1"]
        res["matched_rc_idx2"] = alt["matched_idx2"]
        res["rc_read_type"] = alt["read_type"]
        res["rc_sample_name"] = alt["sample_name"]
        if res["read_type"] == "demuxable" and alt["read_type"] == "demuxable" \
                and res["sample_name"] != alt["sample_name"]:
            res.update(read_type="ambiguous", sample_name="", rc_read_type="ambiguous", rc_sample_name="")
    return res


def classify_all(cores: int, total: dict, sheet: dict, n: int, rc: bool) -> dict:
    args = [(code, reads, sheet["idx1"], sheet["idx2"], sheet["id"], n, rc) for code, reads in total.items()]
    if cores > 1:
        with Pool(processes=cores) as pool:
            print(f"Multiprocessing with {cores} cores")
            res = pool.starmap(classify_code, args)
    else:
        res = [classify_code(*a) for a in args]
    return dict(zip(total.keys(), res))


def rc_calls(rows: list, ids: list) -> dict:
    """R9: per unique name (first-appearance order): use_rc = f < rc."""
    if "rc_read_type" not in rows[0]:
        raise AssertionError("It looks like this frender result csv was not generated with the -rc flag. "
                             "Either specify a different result csv, or run this command without setting the -rc flag.")
    acc = {i: [0, 0] for i in ids}
    for r in rows:
        if r["sample_name"] != "":
            acc[r["sample_name"]][0] += int(r["reads"])
        if r["rc_sample_name"] != "":
            acc[r["rc_sample_name"]][1] += int(r["reads"])
    return {k: {"call": f < b, "reads_f": f, "reads_rc": b} for k, (f, b) in acc.items()}


# ---------------------------------------------------------------------------------------
# R10-R12: outputs (frender.py:429-564)
# ---------------------------------------------------------------------------------------

def flatten(results: dict) -> list:
    rows = []
    for code, r in results.items():
        parts = code.split("+")
        d = {"idx1": parts[0], "idx2": parts[1]}
        d.update(r)
        rows.append(d)
    return rows


def write_rc_report(calls: dict, sheet: dict, out_csv: str) -> None:
    name = out_csv.replace("frender-scan-results_", "frender-index-2-calls_")
    print("Based on the barcodes in the supplied fastq file, the following index 2 sequences will be used\n"
          f"(also recorded in {name}):\n")
    print("Sample Name", "Supplied Index 2", "Reads supporting (forward)", "Reverse complement Index 2",
          "Reads supporting (rev comp)", "Final call", sep="\t")
    for a, c in calls.items():
        i2 = sheet["idx2"][sheet["id"].index(a)]
        print(a, i2, c["reads_f"], revcomp(i2), c["reads_rc"], "reverse complement" if c["call"] else "forward", sep="\t")
    with open(name, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["sample_name", "supplied_index_2", "reads_supplied_index_2", "rc_index_2", "reads_rc_index_2", "use_rc"])
        for a, c in calls.items():
            i2 = sheet["idx2"][sheet["id"].index(a)]
            w.writerow([a, i2, c["reads_f"], revcomp(i2), c["reads_rc"], "TRUE" if c["call"] else "FALSE"])


def mark_demux_ok(counter: dict, results: dict, prefix: str):
    """R10 (frender.py:504-564)."""
    files = [k for k in counter if k != "total"]
    bad = set()
    for code, r in results.items():
        t = r["read_type"]
        oks = []
        for fn in files:
            present = bool(counter[fn].get(code, 0))
            if t == "undetermined":
                m = bool(re.search(re.compile("undetermined", re.I), fn))
            elif t == "index_hop":
                m = bool(re.search(re.compile("undetermined|index-hop", re.I), fn))
            elif t == "ambiguous":
                m = bool(re.search(re.compile("undetermined|ambiguous", re.I), fn))
            else:
                if t != "demuxable":
                    raise AssertionError(f"Strange read type ('{t}') found")
                m = bool(re.search(re.compile(r["sample_name"].removeprefix(prefix), re.I), fn))
            oks.append((not present) | m)
            r["demux_ok"] = len(oks) == sum(oks)
        bad.update(files[i] for i, ok in enumerate(oks) if not ok)
    return results, bad


def write_scan_csv(rows: list, out_csv: str) -> None:
    print(f"Analysis complete! Writing results to {out_csv}")
    keys = rows[0].keys()
    with open(out_csv, "w", newline="") as f:
        w = csv.DictWriter(f, keys)
        w.writeheader()
        w.writerows(rows)


def output_name(n: int, infix: str, files: list) -> tuple:
    """R11 naming (frender.py:587-601); returns (name, input spec)."""
    if len(files) == 1:
        p = Path(files[0])
        if p.is_dir():
            spec, tail = {"dir": p}, p.parts[-1]
        elif p.is_file():
            spec, tail = {"file": p}, p.name
        else:
            raise SystemExit("Specified directory or file path doesn't seem to exist!")
    else:
        spec = {"file": [Path(f) for f in files]}
        tail = datetime.strftime(datetime.now(timezone.utc), "%Y-%M-%d_%H%M_%Z")
    return f"frender-scan-results_{n}-mismatches_{infix}_{tail}.csv".replace("__", "_"), spec


def scan(args) -> dict:
    """R1-R12 end to end (frender.py:567-642); writes the CSVs into the CWD."""
    n = args.n
    cores = resolve_cores(args.c)
    infix = args.o if args.o else ""
    prefix = args.p if args.p else ""
    if args.b is None:
        if len(args.files) != 1:
            raise SystemExit("You have not specified a barcode table. Please either specify one with the argment -b "
                             "or specify a directory including a barcode table")
        sheet_path = discover_sheet(Path(args.files[0]))
    else:
        sheet_path = Path(args.b)
    sheet = read_sheet(sheet_path)
    out_csv, spec = output_name(n, infix, args.files)
    paths = list_inputs(spec, just_r1=True)
    counter = tally(cores, paths, args.s)
    print("Scanning complete! Analyzing barcodes...")
    results = classify_all(cores, counter["total"], sheet, n, args.rc)
    if args.rc:
        calls = rc_calls(flatten(results), sheet["id"])
        print("First round of analysis complete.")
        write_rc_report(calls, sheet, out_csv)
        sheet["idx2"] = [revcomp(x) if calls[i]["call"] else x for x, i in zip(sheet["idx2"], sheet["id"])]
        print("\nRe-analyzing barcodes with corrected index 2 sequences...")
        results = classify_all(cores, counter["total"], sheet, n, False)
    results, bad = mark_demux_ok(counter, results, prefix)
    if bad:
        print("Incorrectly demultiplexed barcodes found! Affected files:")
        for b in bad:
            print(b)
    else:
        print("It appears that all files are already correctly demultiplexed.")
    write_scan_csv(flatten(results), out_csv)
    return {"counter": counter, "results": results, "out_csv": out_csv}
