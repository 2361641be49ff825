"""ORACLE — CPU restatement of reference frender `demux` (TEST INFRASTRUCTURE ONLY).

Parity checker for SURVEY.md §8.1 row (f-1).  Only tests/ may import it; the product path
(frender_amd/demux.py) never does.  Restates /root/reference/frender.py (njspix/frender @ v1)
in independent code; pinned to golden vectors produced by running the reference here
(tests/golden/make_golden_demux.py -> tests/golden/demux/*, checked by
tests/test_demux_oracle.py).

Reference anchors (file:line in frender.py):
  results file ............. parse_results_file :645-664 (README column order asserted)
  output writers ........... open_files :667-676 (gzip "wb"), close_files :679-682
  R1/R2 pairing ............ is_read_mate :685-693, get_paired_files :696-716
  record grouping .......... grouper :719-723 (zip_longest, fill "")
  record writes ............ write_reads :726-730
  driver + hot loop ........ frender_demux :733-814 (code = R2 header .split(":")[-1].rstrip("\\n"))

Semantics restated (D1-D7):
  D1  text mode: gzip.open(...,"rt") decodes UTF-8 with universal newlines, so "\\r\\n" and a
      lone "\\r" end lines and every written line ends in "\\n" (except a last line without one).
  D2  records are groups of 4 lines; the last group of a file may be short; R1/R2 groups are
      paired by position and pairing stops at the shorter file (zip).
  D3  the code is the text after the last ':' of the R2 group's first line, "\\n" stripped.
  D4  routing by the results row's read_type: demuxable -> the sample's writers (if sample
      output is on and any sample id exists), index_hop / ambiguous -> their writers, or the
      Undetermined writers when -i / -a, undetermined -> Undetermined writers (unless -u);
      anything else -> SystemExit "Unrecognized read type ...".
  D5  a code missing from the results (or a demuxable row whose sample has no writers) ->
      SystemExit "Couldn't find barcode {code} in supplied frender result file!".
  D6  every writer is opened (created) up front; names
      {dir}/{name}_frender-demux_{o_}{R1|R2}.fq.gz with name in sample ids,
      Undetermined[-ambiguous][-index-hop], Index-hop, Ambiguous.
  D7  the results file must start with the README header order (idx1, idx2, reads,
      matched_idx1, matched_idx2, read_type, sample_name) -> else AssertionError.  Deviation
      shared with the build: scan's own column order (idx1, idx2,
      matched_idx1, matched_idx2, read_type, sample_name, reads) is accepted by name; its
      expected outputs are the reference's on the same rows in README order.
"""
from __future__ import annotations

import csv
import os
import re
from itertools import zip_longest
from pathlib import Path

from . import frender_oracle as scan_oracle

RESULTS_HEADER = ["idx1", "idx2", "reads", "matched_idx1", "matched_idx2", "read_type", "sample_name"]
SCAN_HEADER = ["idx1", "idx2", "matched_idx1", "matched_idx2", "read_type", "sample_name", "reads"]


def read_results(path, strict: bool = False) -> dict:
    """D7, frender.py:645-664: code -> (read_type, sample_id).  strict: the reference exactly."""
    with open(path, newline="") as f:
        rd = csv.reader(f)
        header = next(rd)
        if header[0:7] == SCAN_HEADER and not strict:  # the build's documented deviation: scan's own order
            return {row[0] + "+" + row[1]: (row[4], row[5]) for row in rd}
        if header[0:7] != RESULTS_HEADER:
            raise AssertionError(f"${path} does not appear to be a valid frender result file!")
        return {row[0] + "+" + row[1]: (row[5], row[6]) for row in rd}


def mate_of(a: str, b: str) -> bool:
    """frender.py:685-693: paths differing in exactly one character whose _R[12]_ are 1 and 2."""
    if sum(1 for x, y in zip(a, b) if x != y) != 1:
        return False
    ra = int(re.search("_R[12]_", a)[0].strip("_").lstrip("R"))
    rb = int(re.search("_R[12]_", b)[0].strip("_").lstrip("R"))
    return {ra, rb} == {1, 2}


def pair_files(paths: list) -> list:
    """frender.py:696-716."""
    out = []
    for p in paths:
        if not re.search("_R1_", str(p), re.IGNORECASE):
            continue
        mates = [q for q in paths if mate_of(str(p), str(q))]
        if len(mates) > 1:
            raise SystemExit(f"Found more than one potential read 2 file for {p}")
        if not mates:
            raise SystemExit(f"Couldn't find a read 2 file for {p}")
        out.append((p, mates[0]))
    return out


def text_lines(path) -> list:
    """D1: the decoded lines of a .gz file as Python's text mode yields them."""
    import gzip

    with gzip.open(path, "rt") as f:
        return list(f)


def groups(lines: list):
    """D2, frender.py:719-723."""
    it = [iter(lines)] * 4
    return zip_longest(*it, fillvalue="")


def out_name(d: str, name: str, infix, read: str) -> str:
    if not d.endswith("/"):
        d += "/"
    return f"{d}{name}_frender-demux_{infix + '_' if infix else ''}{read}.fq.gz"


def demux(args, write_files: bool = False) -> dict:
    """frender.py:733-814.  Returns {output file path: decoded bytes written} (all writers,
    including empty ones); raises like the reference does.  write_files: also write every output
    the way the reference does (gzip.open(..., "wb") writers at gzip's default level 9, one write per
    line, open_files / write_reads :667-676, :726-730) -- the CPU baseline timing of bench.py --cfg5."""
    want_hop = not args.no_index_hop
    want_amb = not args.no_ambiguous
    want_und = not args.no_undeter
    want_samples = not args.no_samples
    und_name = f"Undetermined{'-ambiguous' if want_amb else ''}{'-index-hop' if want_hop else ''}"
    if not Path(args.r).is_file():
        raise SystemExit(f"File {Path(args.r)} not found")
    results = read_results(Path(args.r), strict=getattr(args, "strict_header", False))
    ids = sorted({sid for _, sid in results.values()} - {""})
    if not ids and want_samples:
        print("Warning: no demuxable sample ids found in the supplied frender result file!")
    os.mkdir(args.d)
    out: dict = {}

    import gzip

    gz: dict = {}

    def writers(name):
        pair = (out_name(args.d, name, args.o, "R1"), out_name(args.d, name, args.o, "R2"))
        for p in pair:
            out[p] = bytearray()
            if write_files:
                gz[p] = gzip.open(p, "wb")
        return pair

    sample_w = {sid: writers(sid) for sid in ids} if want_samples else None
    und_w = writers(und_name) if want_und else None
    hop_w = writers("Index-hop") if want_hop else und_w
    amb_w = writers("Ambiguous") if want_amb else und_w

    if len(args.files) == 1:
        f = Path(args.files[0])
        if f.is_dir():
            spec = {"dir": f}
        elif f.is_file():
            spec = {"file": f}
        else:
            raise SystemExit("Specified directory or file path doesn't seem to exist!")
    else:
        spec = {"file": [Path(x) for x in args.files]}
    for r1, r2 in pair_files(scan_oracle.list_inputs(spec, just_r1=False)):
        print(f"Demultiplexing {r1.name}...")
        for g1, g2 in zip(groups(text_lines(r1)), groups(text_lines(r2))):
            code = g2[0].split(":")[-1].rstrip("\n")
            row = results.get(code)
            if row is None:
                raise SystemExit(f"Couldn't find barcode {code} in supplied frender result file!")
            rtype, sid = row
            if rtype == "demuxable" and sample_w:
                if sid not in sample_w:
                    raise SystemExit(f"Couldn't find barcode {code} in supplied frender result file!")
                w = sample_w[sid]
            elif rtype == "index_hop" and hop_w:
                w = hop_w
            elif rtype == "ambiguous" and amb_w:
                w = amb_w
            elif rtype == "undetermined" and und_w:
                w = und_w
            else:
                raise SystemExit("Unrecognized read type found in supplied frender result file!")
            for lines, p in zip((g1, g2), w):
                for line in lines:
                    if write_files:
                        gz[p].write(str(line).encode("utf-8"))
                    else:
                        out[p] += line.encode("utf-8")
    for f in gz.values():
        f.close()
    return {p: bytes(b) for p, b in out.items()}
