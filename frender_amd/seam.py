"""The reference's seam with the reference's data shapes.

frender's `frender_scan` (frender.py:567-642) calls three functions that hold the hot path:

    barcode_counter = tally_barcodes(cores, files, sample)                      frender.py:606
    results = process(cores, barcode_counter["total"], indexes, num_subs, rc)   frender.py:610, :628
    rc_calls = call_rc_mode_per_id(flatten_results(results), indexes["id"])     frender.py:614

and hands what they return to its own host code: flatten_results (:482-492),
report_rc_call_info (:429-479), call_barcodes_correctly_distributed (:504-564) and
report_analysis (:495-501).  The functions below have the same names, arguments and return
shapes, with the work done on the GPU through the C ABI (frender_amd/scan.py ->
frender_amd/_lib.py -> libfrender_hip.so), so replacing those three names is the whole
integration:

* tally_barcodes returns a BarcodeCounter: a read-only Mapping with the reference's keys,
  "total" first, then every scanned file's basename (a later file of the same basename replaces
  the earlier one's table, frender.py:204-205).  ["total"] maps code -> reads in first-occurrence
  order (:199-203); [basename] maps code -> reads in that file (scan_file's file_barcodes,
  :171-177; the counts come from fr_get_presence_counts).
* process returns a ResultsMapping: code -> the reference's per-code dict (analyze_barcodes_with_rc,
  :286-291, :311, :325-332, :336-349), keys in the reference's order.  Each dict is built on first
  access and then kept, so the reference's call_barcodes_correctly_distributed can add
  "demux_ok" to it (:556) and report_analysis finds it there.
* call_rc_mode_per_id takes the reference's flattened list of dicts (summed on the host, as the
  reference sums it, :369-373) or a ResultsMapping (the GPU's per-name sums, fr_rc_counts).

Both mappings keep the GPU arrays (`.table`: frender_amd.scan.UniqueTable; `.results`:
frender_amd.scan.Results), which frender_amd.scan.frender_scan uses directly: the product CLI never
builds a Python dict per code.

Iteration order: "total" and the results iterate in the reference's order.  A per-file table
holds exactly the reference's codes and counts, but iterates in the scan's first-occurrence order;
the reference iterates it in that file's own first-occurrence order, which differs only for codes
first seen in an earlier file.  The reference's own consumers only look codes up in it.
"""
from __future__ import annotations

from collections.abc import Mapping

import numpy as np

from . import _lib
from . import scan as _scan
from .host import reverse_complement


class _CodeIndex:
    """code -> merged position, built once on first lookup."""

    def __init__(self, codes):
        self._codes = codes
        self._pos = None

    def get(self, code):
        if self._pos is None:
            self._pos = {c: j for j, c in enumerate(self._codes)}
        return self._pos.get(code)


class TotalCounts(Mapping):
    """barcode_counter["total"] (frender.py:199-203): code -> reads over all files."""

    def __init__(self, table: "_scan.UniqueTable", index: _CodeIndex):
        self.table = table
        self._index = index

    def __getitem__(self, code):
        j = self._index.get(code)
        if j is None:
            raise KeyError(code)
        return int(self.table.counts[j])

    def __iter__(self):
        return iter(self.table.codes)

    def __len__(self):
        return len(self.table.codes)

    def __contains__(self, code):
        return self._index.get(code) is not None


class FileCounts(Mapping):
    """barcode_counter[basename] (scan_file's file_barcodes, frender.py:171-177): code -> reads of
    the code in that file."""

    def __init__(self, table: "_scan.UniqueTable", file_index: int):
        self.table = table
        self.file_index = file_index
        self._d = None

    def _dict(self) -> dict:
        if self._d is None:
            t = self.table
            sel = np.nonzero(np.asarray(t.pres_f) == self.file_index)[0]
            u = np.asarray(t.pres_u, dtype=np.int64)[sel]
            n = np.asarray(t.pres_n, dtype=np.uint64)[sel]
            o = np.argsort(u, kind="stable")
            self._d = {t.codes[j]: int(c) for j, c in zip(u[o].tolist(), n[o].tolist())}
        return self._d

    def __getitem__(self, code):
        return self._dict()[code]

    def __iter__(self):
        return iter(self._dict())

    def __len__(self):
        return len(self._dict())

    def __contains__(self, code):
        return code in self._dict()


class BarcodeCounter(Mapping):
    """tally_barcodes' return value (frender.py:200-207): {"total": ..., basename: ..., ...}."""

    def __init__(self, table: "_scan.UniqueTable"):
        if table.group is not None:
            raise NotImplementedError("the reference-shaped views cover one process's scan; a multi-GPU "
                                      "scan's table is one key partition (use frender_amd.scan.frender_scan)")
        self.table = table
        self._index = _CodeIndex(table.codes)
        self._total = TotalCounts(table, self._index)
        last = {}
        for i, name in enumerate(table.files):
            last[name] = i  # a later file of the same basename replaces the earlier table (:204-205)
        self._last = last  # insertion order = first appearance of each basename
        self._files = {}

    def __getitem__(self, key):
        if key == "total":
            return self._total
        i = self._last.get(key)
        if i is None:
            raise KeyError(key)
        v = self._files.get(key)
        if v is None:
            v = self._files[key] = FileCounts(self.table, i)
        return v

    def __iter__(self):
        yield "total"
        yield from self._last

    def __len__(self):
        return 1 + len(self._last)

    def __contains__(self, key):
        return key == "total" or key in self._last


class ResultsMapping(Mapping):
    """process' return value (frender.py:411, :414-425): code -> the reference's result dict."""

    def __init__(self, table: "_scan.UniqueTable", results: "_scan.Results", index: _CodeIndex):
        self.table = table
        self.results = results
        self._index = index
        self._cache: dict = {}
        self._rc_idx2 = [reverse_complement(x) for x in results.idx2] if results.rc else None

    def _build(self, j: int) -> dict:
        r, names = self.results, _scan.CLASS_NAMES
        idx1, idx2, ids = r.idx1, r.idx2, r.ids
        m1, m2, row = int(r.m1[j]), int(r.m2[j]), int(r.row[j])
        d = {"matched_idx1": idx1[m1] if m1 >= 0 else "",
             "matched_idx2": idx2[m2] if m2 >= 0 else "",
             "read_type": names[int(r.cls[j])],
             "sample_name": ids[row] if row >= 0 else "",
             "reads": int(self.table.counts[j])}
        if r.rc:
            rm2, rrow = int(r.rc_m2[j]), int(r.rc_row[j])
            d["matched_rc_idx2"] = self._rc_idx2[rm2] if rm2 >= 0 else ""
            d["rc_read_type"] = names[int(r.rc_cls[j])]
            d["rc_sample_name"] = ids[rrow] if rrow >= 0 else ""
        return d

    def __getitem__(self, code):
        d = self._cache.get(code)
        if d is None:
            j = self._index.get(code)
            if j is None:
                raise KeyError(code)
            d = self._cache[code] = self._build(j)
        return d

    def __iter__(self):
        return iter(self.table.codes)

    def __len__(self):
        return len(self.table.codes)

    def __contains__(self, code):
        return self._index.get(code) is not None


def _table_of(counter) -> tuple:
    """The UniqueTable behind barcode_counter["total"] (and its code index), or one built from any
    other {code: reads} mapping (classified by the code-point classifier, fr_classify_cp)."""
    if isinstance(counter, TotalCounts):
        return counter.table, counter._index
    codes = list(counter)
    counts = np.array([int(counter[c]) for c in codes], dtype=np.uint64)
    n = len(codes)
    first = np.arange(n, dtype=np.uint64)
    table = _scan.UniqueTable(codes, counts, first, np.full(n, -1, np.int64), np.arange(n, dtype=np.int64),
                              np.zeros(0, np.int64), np.zeros(0, np.int64), [], [], np.zeros(n, np.uint64),
                              np.zeros(0, np.uint64))
    return table, _CodeIndex(codes)


def tally_barcodes(cores, files, sample=None, ctx=None) -> BarcodeCounter:
    """frender.py:183-207 on the GPU (frender_amd.scan.tally_barcodes), the reference's shape.  A seam
    caller is a long-lived process that may scan once: the inflate's cached decode buffers (up to 4 GiB)
    go back to the OS afterwards (fr_gz_trim)."""
    try:
        return BarcodeCounter(_scan.tally_barcodes(cores, files, sample, ctx=ctx))
    finally:
        _lib.gz_trim()


def process(cores, barcode_counter, indexes, num_subs, rc_mode, ctx=None) -> ResultsMapping:
    """frender.py:391-426 on the GPU (frender_amd.scan.process), the reference's shape."""
    table, index = _table_of(barcode_counter)
    return ResultsMapping(table, _scan.process(cores, table, indexes, num_subs, rc_mode, ctx=ctx), index)


def call_rc_mode_per_id(results_list, ids) -> dict:
    """frender.py:354-388.  The reference passes flatten_results(results): a list of dicts, summed
    here per sample name as the reference sums it (:369-373).  A ResultsMapping (or Results) takes
    the GPU's per-name sums (fr_rc_counts) instead."""
    if isinstance(results_list, ResultsMapping):
        return _scan.call_rc_mode_per_id(results_list.results, ids)
    if isinstance(results_list, _scan.Results):
        return _scan.call_rc_mode_per_id(results_list, ids)
    assert "rc_read_type" in results_list[0].keys(), (
        "It looks like this frender result csv was not generated with the -rc flag. Either specify a different "
        "result csv, or run this command without setting the -rc flag.")
    sums = {name: [0, 0] for name in ids}
    for rec in results_list:
        if rec["sample_name"] != "":
            sums[rec["sample_name"]][0] += int(rec["reads"])
        if rec["rc_sample_name"] != "":
            sums[rec["rc_sample_name"]][1] += int(rec["reads"])
    return {name: {"call": f < r, "reads_f": f, "reads_rc": r} for name, (f, r) in sums.items()}
