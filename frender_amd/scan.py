"""frender `scan` on MI355X — host driver around the C ABI (include/frender_amd.h).

Mirrors the reference's scan interface (frender.py:154-642): the same function
names, argument meaning, stdout lines, CSV formats and failure modes.  The hot
path — per-read tally (scan_file/tally_barcodes), Hamming classification
(process -> analyze_barcodes_with_rc -> analyze_barcode ->
get_indexes_of_approx_matches) and the -rc per-name sums — runs in HIP kernels
on the GPU through frender_amd._lib; nothing here falls back to a CPU path.

Data model: the merged tally (`barcode_counter["total"]`, frender.py:199-203) is a
UniqueTable of codes in first-occurrence order with counts and per-file presence;
classification results are arrays aligned with it.  Codes over {A,C,G,T,N,+} up
to 21 chars ("fast" keys) and codes whose letters are all ACGTN or all acgtn with
at most one '+' and <= 24 letters ("wide" keys: 12+12 dual indexes, lowercase
files) are counted and classified entirely on the GPU.  Anything else ("exotic":
mixed case, other bytes, longer codes) is captured verbatim by the GPU, merged by
string inside the library (C++), and classified on the GPU by the code-point
classifier.
"""
from __future__ import annotations

import csv
import gzip
import io
import operator
import os
import re
from collections.abc import Sequence
from itertools import islice
from datetime import datetime, timezone
from pathlib import Path

import numpy as np

from . import _lib
from .host import find_barcode_file, get_cores, get_indexes, parse_files, reverse_complement

UNDET, HOP, DEMUX, AMBIG = 0, 1, 2, 3
CLASS_NAMES = _lib.CLASS_NAMES
ORD_SHIFT = 44

_CTX = None


def default_context() -> _lib.Context:
    """This process's GPU context: LOCAL_RANK's device (one process per GPU; ranks share a GPU
    only in single-GPU rehearsals of a multi-rank run)."""
    global _CTX
    if _CTX is None:
        dev = int(os.environ.get("LOCAL_RANK", "0"))
        n = _lib.torch.cuda.device_count() if _lib.torch is not None else 0
        _CTX = _lib.Context(device=dev % n if n else dev)
        _CTX.set_timing(False)  # the product reads no kernel timings: no event bubbles on its stream
    return _CTX


class UniqueTable:
    """The merged tally: codes in (file, first occurrence) order (R4/R5)."""

    def __init__(self, codes, counts, first, fast_idx, exo_idx, pres_u, pres_f, files, records, key_of=None,
                 pres_n=None):
        self.codes = codes            # list[str], merged order
        self.counts = counts          # uint64
        self.first = first            # uint64 ordinals (file_index+1) << 44 | byte offset
        self.fast_idx = fast_idx      # merged -> index in the GPU's finalized table, or -1
        self.exo_idx = exo_idx        # merged -> index in the exotic list, or -1
        self.pres_u = pres_u          # (unique, file) presence pairs
        self.pres_f = pres_f
        self.pres_n = pres_n          # reads of the pair's code in the pair's file (per-file tables)
        self.files = files            # basenames in input order
        self.records = records        # records per file
        self.key_of = key_of          # merged -> packed key (fast / wide codes), 0 for exotic codes
        self.group = None             # multi-GPU scans: torch.distributed; this table is one key partition
        self.wire = None              # and the device its exchange tensors live on

    def __len__(self):
        return len(self.codes)

    def as_dict(self) -> dict:
        """barcode_counter["total"] as a plain dict (small inputs / tests)."""
        return {c: int(n) for c, n in zip(self.codes, self.counts)}


def _replay_decode_error(path, sample):
    """Error path only, after the GPU flagged invalid UTF-8 in a file (or the native inflate
    rejected it: truncated or corrupt gzip, whose EOFError / BadGzipFile / zlib.error the same
    re-read raises).  The reference's exception
    text (byte, position, reason) is relative to the chunk its text-mode reader handed the decoder
    (frender.py:159: gzip.open(..., "rt"), whose chunk boundaries depend on the compressed
    stream), and with -s it raises only if the bad bytes lie in a chunk read before the sample
    ends (islice over the lines, :160-166).  So re-open the file the same way and read the same
    lines: this raises exactly what the reference raises (UnicodeDecodeError, or the IndexError
    of an earlier header without ' ', :169), or returns when the reference would not fail.
    Nothing it reads feeds the tally."""
    with gzip.open(path, "rt") as f:
        for i, line in enumerate(islice(f, 0, None, 4)):
            if sample and i >= sample:
                return
            if " " not in line:
                raise IndexError("list index out of range")


def _file_done(st, path=None, sample=None):
    """Per-file epilogue of scan_file (frender.py:160-181): the reference's exceptions for bad
    input.  Exotic codes are merged inside the library (fr_get_exotic_table) and counted in
    st.new_keys."""
    if st.utf8_bad:  # gzip.open(..., "rt") decode (frender.py:159)
        if path is None:
            raise UnicodeDecodeError("utf-8", b"", 0, 1, "invalid start byte")
        _replay_decode_error(path, sample)
    if st.error == _lib.FR_SCAN_NO_SPACE:  # frender.py:169 split(" ")[1]
        raise IndexError("list index out of range")


def scan_files(ctx, files, indices, sample, cores, on_file=None, after_file=None):
    """scan_file (frender.py:154-181) for files[i], i in `indices` (increasing), into ctx's table.
    The bytes come from the library's native inflate (fr_gz_*): up to `cores` files inflate ahead
    in host threads while the GPU tallies them in order (the reference's Pool over files,
    :189-193).  Every file is opened at its global index, so any subset of a scan's files, on any
    GPU, yields the single-GPU ordinals.  on_file(i, name) runs before a file is read (the
    reference's "Tallying barcodes from ..." line), after_file(i, records, new barcodes) once it is
    tallied.  Returns {i: (records, new barcodes)}."""
    out = {}
    paths = [files[i] for i in indices]
    pool = _lib.GzPool(paths, threads=max(1, int(cores)), ahead=_lib.inflate_ahead(paths, max(1, int(cores))))
    try:
        for k, fi in enumerate(indices):
            path = files[fi]
            if on_file:
                on_file(fi, str(os.path.basename(path)))
            ctx.begin_file(sample, file_index=fi)
            try:
                pool.feed(k, ctx)
            except _lib.GzError as e:  # not a valid gzip stream: the reference's reader fails on it
                _replay_decode_error(path, sample)
                raise RuntimeError(f"native inflate rejected {path} but Python's gzip reads it: {e}") from e
            st = ctx.end_file()
            _file_done(st, path, sample)
            out[fi] = (int(st.records), int(st.new_keys))
            if after_file:
                after_file(fi, *out[fi])
    finally:
        pool.close()
    return out


def found_line(new_here, records) -> str:
    return f"found {new_here} new barcode{'' if new_here == 1 else 's'} in {records} reads."


def local_table(ctx) -> dict:
    """This context's finalized tally as host arrays: fast/wide keys in first-occurrence order with
    counts and first ordinals, their (unique index, file index) presence pairs, and the exotic codes
    the library aggregated (bytes, counts, firsts, (code, file) presence)."""
    ctx.finalize()
    keys, counts, first = ctx.unique()
    pu, pf = ctx.presence()
    ecodes, ecounts, efirst, epc, epf = ctx.exotic_table()
    pn, epn = ctx.presence_counts(len(epc))
    return {"keys": keys, "counts": counts, "first": first, "pu": pu, "pf": pf, "pn": pn,
            "ecodes": ecodes, "ecounts": ecounts, "efirst": efirst, "epc": epc, "epf": epf, "epn": epn}


class Codes(Sequence):
    """UniqueTable.codes: the code strings in merged order, decoded from the packed keys only when
    someone reads them (the CSV writer works from the keys: a config-2 scan has ~10^6 codes, and
    decoding them all to Python strings cost more host time than the GPU's whole tally).  Exotic
    codes are held as text at their merged positions."""

    def __init__(self, key_of, exo_pos, exo_codes):
        self._keys = np.asarray(key_of, dtype=np.uint64)
        self._exo = dict(zip(np.asarray(exo_pos, dtype=np.int64).tolist(), exo_codes))
        self._list = None

    def __len__(self):
        return int(self._keys.size)

    def _all(self) -> list:
        if self._list is None:
            out = _lib.decode_keys(self._keys)
            for j, c in self._exo.items():
                out[j] = c
            self._list = out
        return self._list

    def __getitem__(self, j):
        if self._list is not None or isinstance(j, slice):
            return self._all()[j]
        j = operator.index(j)
        n = len(self)
        if j < 0:
            j += n
        if not 0 <= j < n:
            raise IndexError("list index out of range")
        c = self._exo.get(j)
        return c if c is not None else _lib.decode_keys(self._keys[j:j + 1])[0]

    def __iter__(self):
        return iter(self._all())


def build_table(t: dict, names, records) -> UniqueTable:
    """barcode_counter["total"] (frender.py:199-203) from a finalized tally: keyed and exotic codes
    interleaved in (file, first occurrence) order."""
    keys, counts, first = t["keys"], t["counts"], t["first"]
    exo_codes = [c.decode("utf-8") for c in t["ecodes"]]
    exo_counts = np.asarray(t["ecounts"], dtype=np.uint64)
    exo_first = np.asarray(t["efirst"], dtype=np.uint64)
    all_first = np.concatenate([first, exo_first])
    order = np.argsort(all_first, kind="stable")
    nf = len(keys)
    pos = np.empty(order.size, dtype=np.int64)
    pos[order] = np.arange(order.size)
    fast_idx = np.where(order < nf, order, -1)
    exo_idx = np.where(order >= nf, order - nf, -1)
    pu, pf = np.asarray(t["pu"], dtype=np.int64), np.asarray(t["pf"], dtype=np.int64)
    epc, epf = np.asarray(t["epc"], dtype=np.int64), np.asarray(t["epf"], dtype=np.int64)
    pres_u = np.concatenate([pos[pu], pos[nf + epc]])
    pres_f = np.concatenate([pf, epf])
    pres_n = np.concatenate([np.asarray(t["pn"], dtype=np.uint64), np.asarray(t["epn"], dtype=np.uint64)])
    key_of = np.concatenate([np.asarray(keys, dtype=np.uint64), np.zeros(len(exo_codes), np.uint64)])[order]
    codes = Codes(key_of, pos[nf:], exo_codes)
    return UniqueTable(codes, np.concatenate([counts, exo_counts])[order], all_first[order], fast_idx, exo_idx,
                       pres_u, pres_f, list(names), list(records), key_of, pres_n)


def tally_barcodes(cores, files, sample=None, ctx=None) -> UniqueTable:
    """frender.py:183-207 (+ scan_file :154-181) on the GPU: files in order, one context.  With a
    torch.distributed group of N > 1 ranks (one per GPU) the record stream is sharded over the GPUs
    and every rank returns its key partition of the merged table (frender_amd/dist.py:
    sharded_tally); the functions below take such a partition and run their collectives."""
    from .dist import sharded_tally, world_group
    group = world_group()
    lead = group is None or group.get_rank() == 0  # the lines rank 0 prints for the whole job
    if lead:
        print(f"Scanning {len(files)} files with {cores} core{'' if cores == 1 else 's'}...")
    if sample:
        assert sample >= 1, "Number of reads to sample must be ≥ 1!"
        if lead:
            print(f"Sampling {sample} reads from the head of each file...")
    ctx = ctx or default_context()
    if group is not None:
        return sharded_tally(group, ctx, files, sample, cores)
    ctx.reset()
    names = [str(os.path.basename(p)) for p in files]

    per = scan_files(ctx, files, list(range(len(files))), sample, cores,
                     on_file=lambda fi, name: print(f"Tallying barcodes from {name}...", end=""),
                     after_file=lambda fi, records, new: print(found_line(new, records)))
    print(type([]), len(files))
    return build_table(local_table(ctx), names, [per[i][0] for i in range(len(files))])


class Results:
    """process() output: arrays aligned with the UniqueTable (frender.py:286-291, :325-332)."""

    def __init__(self, n, rc):
        self.m1 = np.full(n, -1, np.int16)
        self.m2 = np.full(n, -1, np.int16)
        self.cls = np.zeros(n, np.uint8)
        self.row = np.full(n, -1, np.int16)
        self.rc = rc
        if rc:
            self.rc_m2 = np.full(n, -1, np.int16)
            self.rc_cls = np.zeros(n, np.uint8)
            self.rc_row = np.full(n, -1, np.int16)
        self.rc_f = None
        self.rc_r = None
        self.n_total = n              # codes of the whole scan (all key partitions of a multi-GPU scan)
        self.idx1 = self.idx2 = self.ids = None
        self.names = None


def _sheet_names(ids):
    names = list(dict.fromkeys(ids))
    where = {n: i for i, n in enumerate(names)}
    return names, [where[i] for i in ids]


def _length_error(q: str, entries) -> AssertionError:
    ql = q.lower()
    for e in entries:
        if len(ql) != len(e.lower()):
            return AssertionError(f"Barcode {ql} doesn't match length of supplied barcode {e.lower()}")
    return AssertionError("length mismatch")  # pragma: no cover


def _lead(table) -> bool:
    return table.group is None or table.group.get_rank() == 0


def process(cores, table: UniqueTable, indexes: dict, num_subs: int, rc_mode: bool, ctx=None) -> Results:
    """frender.py:391-426 on the GPU: classify every unique code (fast keys by packed
    Hamming, exotic codes by the code-point classifier); raise the reference's first error.
    On a key partition (multi-GPU): each rank classifies its partition; the -rc per-name sums are
    all-reduced and the first error in first-occurrence order over all partitions is raised."""
    ctx = ctx or default_context()
    idx1, idx2, ids = list(indexes["idx1"]), list(indexes["idx2"]), list(indexes["id"])
    names, name_id = _sheet_names(ids)
    ctx.set_sheet(idx1, idx2, [reverse_complement(x) for x in idx2], name_id, len(names))
    if cores > 1 and _lead(table):
        print(f"Multiprocessing with {cores} cores")
    n = len(table)
    res = Results(n, rc_mode)
    res.idx1, res.idx2, res.ids, res.names = idx1, idx2, ids, names
    errs = []  # (merged position, exception)
    fsel = np.nonzero(table.fast_idx >= 0)[0]
    if fsel.size:
        out = ctx.classify(num_subs, rc_mode)
        fi = table.fast_idx[fsel]
        res.m1[fsel], res.m2[fsel], res.cls[fsel], res.row[fsel] = out["m1"][fi], out["m2"][fi], out["cls"][fi], out["row"][fi]
        if rc_mode:
            res.rc_m2[fsel], res.rc_cls[fsel], res.rc_row[fsel] = out["rc_m2"][fi], out["rc_cls"][fi], out["rc_row"][fi]
        if out["err_unique"] >= 0:
            j = int(np.nonzero(table.fast_idx == out["err_unique"])[0][0])
            errs.append((j, out["err_which"]))
    esel = np.nonzero(table.exo_idx >= 0)[0]
    f_add = np.zeros(len(names), np.uint64)
    r_add = np.zeros(len(names), np.uint64)
    if esel.size:
        split_ok, q1, q2, js = [], [], [], []
        for j in esel.tolist():
            parts = table.codes[j].split("+")
            if len(parts) < 2:
                errs.append((j, 3))
                continue
            js.append(j)
            q1.append(parts[0].lower())
            q2.append(parts[1].lower())
        if js:
            out = ctx.classify_cp(q1, q2, num_subs, rc_mode)
            ja = np.array(js)
            res.m1[ja], res.m2[ja], res.cls[ja], res.row[ja] = out["m1"], out["m2"], out["cls"], out["row"]
            if rc_mode:
                res.rc_m2[ja], res.rc_cls[ja], res.rc_row[ja] = out["rc_m2"], out["rc_cls"], out["rc_row"]
                for k, j in enumerate(js):
                    if out["cls"][k] == DEMUX:
                        f_add[name_id[out["row"][k]]] += table.counts[j]
                    if out["rc_cls"][k] == DEMUX:
                        r_add[name_id[out["rc_row"][k]]] += table.counts[j]
            for k, j in enumerate(js):
                if out["err"][k]:
                    errs.append((j, int(out["err"][k])))
    if table.group is not None:
        errs = _first_error_everywhere(table, errs)
    if errs:
        j, which = min(errs)
        code = table.codes[j] if isinstance(j, int) else j[1]
        if which == 3:  # idx1, idx2 = barcode.split("+")[0:2]  (frender.py:306)
            raise ValueError("not enough values to unpack (expected 2, got 1)")
        parts = code.split("+")
        raise _length_error(parts[0], idx1) if which == 1 else _length_error(parts[1], idx2)
    if rc_mode:
        f, r = ctx.rc_counts() if fsel.size else (np.zeros(len(names), np.uint64), np.zeros(len(names), np.uint64))
        res.rc_f = f + f_add
        res.rc_r = r + r_add
        if table.group is not None:  # the per-name sums of every partition (frender.py:367-373), one reduce
            from .dist import reduce_sum
            k = len(names)
            v = reduce_sum(table.group, table.wire, np.concatenate([res.rc_f.astype(np.int64), res.rc_r.astype(np.int64),
                                                                  [n]]))
            res.rc_f, res.rc_r, res.n_total = v[:k].astype(np.uint64), v[k:2 * k].astype(np.uint64), int(v[2 * k])
    return res


def _first_error_everywhere(table, errs):
    """Multi-GPU: the classification error the reference meets first (its Pool over the uniques in
    first-occurrence order) among every partition's first error.  Rank 0 gets [((first, code), which)]
    for it; the other ranks raise PeerFailed; no error anywhere -> []."""
    from .dist import PeerFailed, gather_bytes, reduce_max

    g = table.group
    mine = b""
    if errs:
        j, which = min(errs, key=lambda e: int(table.first[e[0]]))
        mine = f"{int(table.first[j])}\t{which}\t".encode() + table.codes[j].encode("utf-8", "surrogateescape")
    any_err = int(reduce_max(g, table.wire, [1 if errs else 0])[0])
    if not any_err:
        return []
    got = gather_bytes(g, table.wire, mine)
    if g.get_rank() != 0:
        raise PeerFailed("classification failed (rank 0 reports it)")
    cands = []
    for b in got:
        if b:
            f, w, c = b.split(b"\t", 2)
            cands.append(((int(f), c.decode("utf-8", "surrogateescape")), int(w)))
    return [min(cands)]


def call_rc_mode_per_id(results: Results, ids) -> dict:
    """frender.py:354-388: per distinct name, use rc idx2 iff its reads beat the forward ones."""
    if results.n_total == 0:  # an empty partition of a non-empty multi-GPU scan is not an empty scan
        raise IndexError("list index out of range")  # results_list[0] on an empty scan (:364)
    assert results.rc, ("It looks like this frender result csv was not generated with the -rc flag. Either specify a "
                        "different result csv, or run this command without setting the -rc flag.")
    return {name: {"call": bool(int(f) < int(r)), "reads_f": int(f), "reads_rc": int(r)}
            for name, f, r in zip(results.names, results.rc_f, results.rc_r)}


def report_rc_call_info(rc_calls: dict, indexes: dict, out_csv_name: str) -> None:
    """frender.py:429-479 (stdout table + frender-index-2-calls_*.csv)."""
    rc_name = out_csv_name.replace("frender-scan-results_", "frender-index-2-calls_")
    print("Based on the barcodes in the supplied fastq file, the following index 2 sequences will be used\n"
          f"(also recorded in {rc_name}):\n")
    print("Sample Name", "Supplied Index 2", "Reads supporting (forward)", "Reverse complement Index 2",
          "Reads supporting (rev comp)", "Final call", sep="\t")
    first_row = {}
    for i, a in enumerate(indexes["id"]):
        first_row.setdefault(a, i)
    for a, c in rc_calls.items():
        i2 = indexes["idx2"][first_row[a]]
        print(a, i2, c["reads_f"], reverse_complement(i2), c["reads_rc"],
              "reverse complement" if c["call"] else "forward", sep="\t")
    with open(rc_name, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["sample_name", "supplied_index_2", "reads_supplied_index_2", "rc_index_2", "reads_rc_index_2",
                    "use_rc"])
        for a, c in rc_calls.items():
            i2 = indexes["idx2"][first_row[a]]
            w.writerow([a, i2, c["reads_f"], reverse_complement(i2), c["reads_rc"], "TRUE" if c["call"] else "FALSE"])


def call_barcodes_correctly_distributed(table: UniqueTable, results: Results, prefix: str):
    """frender.py:504-564 (R10): per unique, every scanned file (by basename; the last
    file of a basename wins, :204-205) holding it must match its class's pattern."""
    basenames = list(dict.fromkeys(table.files))
    if not basenames:
        return None, set()
    bidx = {b: i for i, b in enumerate(basenames)}
    last_file = {b: i for i, b in enumerate(table.files)}
    file_b = np.array([bidx[b] for b in table.files], dtype=np.int64)
    file_live = np.array([last_file[b] == i for i, b in enumerate(table.files)], dtype=bool)
    # the demuxable patterns are compiled per (barcode, file) by the reference: an invalid
    # one raises at the first demuxable barcode in order
    rows = results.row.astype(np.int64)
    demux = np.nonzero(results.cls == DEMUX)[0]
    names = results.names
    name_of = {n: k for k, n in enumerate(names)}
    order = [results.ids[rows[j]] for j in demux.tolist()]
    if table.group is not None:  # every partition's demuxable names, by their first demuxable code
        from .dist import reduce_min
        big = (1 << 63) - 1
        firsts = np.full(len(names), big, np.int64)
        for j in demux.tolist():
            k = name_of[results.ids[rows[j]]]
            firsts[k] = min(firsts[k], int(table.first[j]))
        firsts = reduce_min(table.group, table.wire, firsts)
        order = [names[k] for k in np.argsort(firsts, kind="stable").tolist() if firsts[k] != big]
    pat = {}
    for nm in order:
        if nm not in pat:
            try:
                pat[nm] = re.compile(nm.removeprefix(prefix), re.I)
            except re.error:
                if table.group is not None and table.group.get_rank() != 0:
                    from .dist import PeerFailed
                    raise PeerFailed("sample pattern failed to compile (rank 0 reports it)") from None
                raise
    groups = [re.compile("undetermined", re.I), re.compile("undetermined|index-hop", re.I),
              re.compile("undetermined|ambiguous", re.I)] + [pat.get(n) for n in names]
    ok = np.ones((len(groups), len(basenames)), dtype=bool)
    for g, rx in enumerate(groups):
        if rx is None:
            continue
        for b, fn in enumerate(basenames):
            ok[g, b] = bool(re.search(rx, fn))
    grp = np.array([0, 1, -1, 2], dtype=np.int64)[results.cls.astype(np.int64)]  # undet, hop, -, ambiguous
    if demux.size:
        grp[demux] = 3 + np.array([name_of[results.ids[r]] for r in rows[demux].tolist()], dtype=np.int64)
    pu, pf = table.pres_u, table.pres_f
    keep = file_live[pf] if pf.size else np.zeros(0, bool)
    pu, pf = pu[keep], pf[keep]
    pair_ok = ok[grp[pu], file_b[pf]] if pu.size else np.zeros(0, bool)
    demux_ok = np.ones(len(table), dtype=bool)
    demux_ok[pu[~pair_ok]] = False
    bad_b = np.zeros(len(basenames), np.int64)
    bad_b[np.unique(file_b[pf[~pair_ok]])] = 1
    if table.group is not None:  # the mismatching files of every partition
        from .dist import reduce_max
        bad_b = reduce_max(table.group, table.wire, bad_b)
    bad = {basenames[b] for b in np.nonzero(bad_b)[0].tolist()}
    return demux_ok, bad


def _gather_partitions(table: UniqueTable, results: Results, demux_ok):
    """Multi-GPU: every partition's classified rows on rank 0, in first-occurrence order (int64 rows
    over RCCL: first, key, count, m1, m2, class, row, demux_ok; exotic codes are rank 0's already).
    Returns (keys, exotic positions, exotic codes, counts, m1, m2, cls, row, demux_ok) arrays on
    rank 0 (key 0 at an exotic code's position), None elsewhere."""
    from .dist import gather_rows

    import torch

    fast = np.nonzero(table.fast_idx >= 0)[0]
    dok = np.ones(len(table), bool) if demux_ok is None else np.asarray(demux_ok, bool)
    cols = [table.first.view(np.int64)[fast], table.key_of.view(np.int64)[fast], table.counts.view(np.int64)[fast],
            results.m1[fast], results.m2[fast], results.cls[fast], results.row[fast], dok[fast]]
    rows = torch.from_numpy(np.stack([np.asarray(c, np.int64) for c in cols], 1) if fast.size
                            else np.zeros((0, 8), np.int64))
    got = gather_rows(table.group, table.wire, rows)
    if got is None:
        return None
    allr = np.concatenate(got, 0)
    exo = np.nonzero(table.exo_idx >= 0)[0]
    first = np.concatenate([allr[:, 0].view(np.uint64), table.first[exo]])
    keys = np.concatenate([allr[:, 1].view(np.uint64), np.zeros(exo.size, np.uint64)])
    counts = np.concatenate([allr[:, 2].view(np.uint64), table.counts[exo]])
    rest = [np.concatenate([allr[:, 3 + i], np.asarray(c, np.int64)[exo]])
            for i, c in enumerate((results.m1, results.m2, results.cls, results.row, dok))]
    o = np.argsort(first, kind="stable")
    pos = np.empty(o.size, np.int64)
    pos[o] = np.arange(o.size)
    exo_pos = pos[allr.shape[0]:]
    return (keys[o], exo_pos, [table.codes[j] for j in exo.tolist()], counts[o], rest[0][o].astype(np.int16),
            rest[1][o].astype(np.int16), rest[2][o].astype(np.uint8), rest[3][o].astype(np.int16),
            rest[4][o].astype(bool))


def _csv_fields(*fields) -> str:
    """The fields as Python's csv module (excel dialect) writes them inside a row, joined by ','."""
    buf = io.StringIO()
    csv.writer(buf).writerow([*fields, "x"])
    return buf.getvalue()[:-len(",x\r\n")]


def _write_csv_native(path, header, keys, exo_pos, exo_codes, counts, m1, m2, cls, row, dok, idx1, idx2, ids) -> bool:
    """fr_write_scan_csv (fr_csv.cpp): the rows formatted from the packed keys and the classification
    arrays.  False, with nothing written, when some code does not split on '+' (the caller's row
    loop then raises the reference's IndexError where the reference does)."""
    texts = []
    for c in exo_codes:
        parts = c.split("+")
        if len(parts) < 2:
            return False
        texts.append(_csv_fields(parts[0], parts[1]).encode("utf-8", "surrogateescape"))
    ents = [_csv_fields(x).encode("utf-8", "surrogateescape") for x in (*idx1, *idx2, *ids, *CLASS_NAMES)]
    dict_off = np.concatenate([[0], np.cumsum([len(e) for e in ents])]).astype(np.uint64)
    dict_n = np.array([len(idx1), len(idx2), len(ids), len(CLASS_NAMES)], np.uint32)
    eo = np.argsort(np.asarray(exo_pos, np.int64), kind="stable")
    exo_rows = np.ascontiguousarray(np.asarray(exo_pos, np.uint64)[eo])
    exo_text = b"".join(texts[i] for i in eo.tolist())
    exo_off = np.concatenate([[0], np.cumsum([len(texts[i]) for i in eo.tolist()])]).astype(np.uint64)
    arr = [np.ascontiguousarray(keys, np.uint64), np.ascontiguousarray(counts, np.uint64),
           np.ascontiguousarray(m1, np.int16), np.ascontiguousarray(m2, np.int16), np.ascontiguousarray(cls, np.uint8),
           np.ascontiguousarray(row, np.int16)]
    d = None if dok is None else np.ascontiguousarray(dok, np.uint8)
    rc = _lib.lib.fr_write_scan_csv(os.fsencode(path), header.encode(), len(arr[0]), *[_lib._ptr(a) for a in arr],
                                    _lib._ptr(d), b"".join(ents), _lib._ptr(dict_off), _lib._ptr(dict_n),
                                    len(exo_rows), _lib._ptr(exo_rows), exo_text, _lib._ptr(exo_off))
    if rc == _lib.FR_ERR_INVALID:
        return False
    if rc != 0:
        raise OSError(f"fr_write_scan_csv failed ({rc}) writing {path}")
    return True


def report_analysis(table: UniqueTable, results: Results, demux_ok, out_csv_name: str) -> None:
    """frender.py:482-501: the scan CSV (excel dialect, columns in the code's order).  On a key
    partition (multi-GPU) rank 0 gathers every partition's rows and writes the file.  The rows are
    formatted natively from the packed keys (fr_write_scan_csv); the row loop below is kept for the
    codes that do not split on '+', where it raises the reference's IndexError at the same row."""
    if table.group is not None:
        got = _gather_partitions(table, results, demux_ok)
        if got is None:
            return
        keys, exo_pos, exo_codes, counts, m1, m2, cls, row, dok = got
        dok = dok if demux_ok is not None else None
    else:
        keys, counts = table.key_of, table.counts
        exo_pos = np.nonzero(table.exo_idx >= 0)[0]
        exo_codes = [table.codes[j] for j in exo_pos.tolist()]
        m1, m2, cls, row, dok = results.m1, results.m2, results.cls, results.row, demux_ok
    print(f"Analysis complete! Writing results to {out_csv_name}")
    if len(keys) == 0:
        raise IndexError("list index out of range")  # results[0].keys() on an empty scan (:497)
    idx1, idx2, ids = results.idx1, results.idx2, results.ids
    header = ["idx1", "idx2", "matched_idx1", "matched_idx2", "read_type", "sample_name", "reads"]
    if dok is not None:
        header.append("demux_ok")
    if _write_csv_native(out_csv_name, _csv_fields(*header) + "\r\n", keys, exo_pos, exo_codes, counts, m1, m2, cls,
                         row, dok, idx1, idx2, ids):
        return
    codes = Codes(keys, exo_pos, exo_codes)
    m1, m2, cls, row, counts = m1.tolist(), m2.tolist(), cls.tolist(), row.tolist(), counts.tolist()
    dok = None if dok is None else dok.tolist()

    def rows():
        for j, code in enumerate(codes):
            parts = code.split("+")
            r = [parts[0], parts[1], idx1[m1[j]] if m1[j] >= 0 else "", idx2[m2[j]] if m2[j] >= 0 else "",
                 CLASS_NAMES[cls[j]], ids[row[j]] if row[j] >= 0 else "", counts[j]]
            if dok is not None:
                r.append(dok[j])
            yield r

    with open(out_csv_name, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows())


def output_name(num_subs, user_infix, files_arg):
    """frender.py:587-601."""
    if len(files_arg) == 1:
        p = Path(files_arg[0])
        if Path.is_dir(p):
            spec, tail = {"dir": p}, p.parts[-1]
        elif Path.is_file(p):
            spec, tail = {"file": p}, p.name
        else:
            raise SystemExit("Specified directory or file path doesn't seem to exist!")
    else:
        spec = {"file": [Path(f) for f in files_arg]}
        tail = datetime.strftime(datetime.now(timezone.utc), "%Y-%M-%d_%H%M_%Z")
    return f"frender-scan-results_{num_subs}-mismatches_{user_infix}_{tail}.csv".replace("__", "_"), spec


def frender_scan(args, ctx=None) -> dict:
    """frender.py:567-642 with the hot path on the GPU."""
    num_subs = args.n
    rc_mode = args.rc
    cores = get_cores(args.c)
    sample = args.s
    user_infix = args.o if args.o else ""
    prefix = args.p if args.p else ""
    if args.b is None:
        if len(args.files) != 1:
            raise SystemExit("You have not specified a barcode table. Please either specify one with the argment -b or "
                             "specify a directory including a barcode table")
        barcode_file = find_barcode_file(Path(args.files[0]))
    else:
        barcode_file = Path(args.b)
    indexes = get_indexes(barcode_file)
    out_csv_name, spec = output_name(num_subs, user_infix, args.files)
    files = parse_files(spec, just_r1=True)
    ctx = ctx or default_context()
    table = tally_barcodes(cores, files, sample, ctx=ctx)
    lead = _lead(table)  # multi-GPU: every rank holds a key partition; rank 0 prints and writes
    if lead:
        print("Scanning complete! Analyzing barcodes...")
    results = process(cores, table, indexes, num_subs, rc_mode, ctx=ctx)
    if rc_mode:
        rc_calls = call_rc_mode_per_id(results, indexes["id"])
        if lead:
            print("First round of analysis complete.")
            report_rc_call_info(rc_calls, indexes, out_csv_name)
        indexes["idx2"] = [reverse_complement(indexes["idx2"][i]) if rc_calls[i_d]["call"] else indexes["idx2"][i]
                           for i, i_d in enumerate(indexes["id"])]
        if lead:
            print("\nRe-analyzing barcodes with corrected index 2 sequences...")
        results = process(cores, table, indexes, num_subs, False, ctx=ctx)
    demux_ok, mismatching = call_barcodes_correctly_distributed(table, results, prefix)
    if lead:
        if mismatching:
            print("Incorrectly demultiplexed barcodes found! Affected files:")
            for a in mismatching:
                print(a)
        else:
            print("It appears that all files are already correctly demultiplexed.")
    report_analysis(table, results, demux_ok, out_csv_name)
    if getattr(table, "group", None) is not None and os.environ.get("FRENDER_DIST_CENSUS"):
        import json
        import sys

        from .dist import CENSUS
        print("census " + json.dumps({"rank": table.group.get_rank(), "collectives": CENSUS}), file=sys.stderr)
    return {"table": table, "results": results, "out_csv": out_csv_name} if lead else None


# the name the golden harness calls
scan = frender_scan
