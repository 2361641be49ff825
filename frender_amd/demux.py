"""frender `demux` with the record routing on the GPU.

Mirrors frender.py:645-814: the same results-file check, writer names, R1/R2 pairing, stdout
lines and failure modes.  Per file pair, the decoded R1 and R2 text goes to the GPU
(libfrender_hip.so, fr_dmx_* in include/frender_amd.h), which finds every record, resolves the
R2 code of each pair against the results and gathers both mates' records destination-major;
the host inflates, resolves the rare codes outside the fast alphabet, raises the reference's
errors and gzips each destination's bytes into its writer pair (threads: zlib releases the GIL).
"""
from __future__ import annotations

import csv
import gc
import gzip
import json
import os
import re
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

from . import _lib
from .host import parse_files

RESULTS_HEADER = ["idx1", "idx2", "reads", "matched_idx1", "matched_idx2", "read_type", "sample_name"]
# the column order `scan` itself writes (frender.py:482-501, report_analysis)
SCAN_HEADER = ["idx1", "idx2", "matched_idx1", "matched_idx2", "read_type", "sample_name", "reads"]


def parse_results_file(result_file, strict: bool = False) -> dict:
    """frender.py:645-664: code -> (read_type, sample_id).

    The reference asserts the README's column order, which its own `scan` does not write, so its
    demux rejects its own scan CSV.  Documented deviation, on by default so that
    scan -> demux chains (BASELINE config 5) work: a header in `scan`'s order is
    accepted too, its columns taken by name.  strict=True (`demux --strict-header`) is the
    reference's behaviour exactly: that header raises its AssertionError (golden case
    syn_scan_order_strict).  Any other header fails with the reference's AssertionError, and
    README-order files behave exactly as in the reference, in both modes."""
    with open(result_file, newline="") as f:
        rd = csv.reader(f)
        header = next(rd)
        top = header[0:7]
        if top == SCAN_HEADER and not strict:
            ti, si = top.index("read_type"), top.index("sample_name")
        else:
            assert top == RESULTS_HEADER, f"${result_file} does not appear to be a valid frender result file!"
            ti, si = 5, 6
        # (a scan's results file holds a row per distinct code: hundreds of thousands of tuples, which
        # the cyclic collector would walk again and again while the dict grows)
        enabled = gc.isenabled()
        gc.disable()
        try:
            return {line[0] + "+" + line[1]: (line[ti], line[si]) for line in rd}
        finally:
            if enabled:
                gc.enable()


def _load_libdeflate():
    """libdeflate (whole-buffer DEFLATE, 2-4x zlib's speed), when the image has it; None otherwise."""
    import ctypes

    try:
        ld = ctypes.CDLL("libdeflate.so.0")
    except OSError:
        return None
    ld.libdeflate_alloc_compressor.restype = ctypes.c_void_p
    ld.libdeflate_alloc_compressor.argtypes = [ctypes.c_int]
    ld.libdeflate_gzip_compress_bound.restype = ctypes.c_size_t
    ld.libdeflate_gzip_compress_bound.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    ld.libdeflate_gzip_compress.restype = ctypes.c_size_t
    ld.libdeflate_gzip_compress.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_size_t]
    return ld


_LD = _load_libdeflate()
_LD_TLS = threading.local()


class _GzMembers:
    """A .fq.gz writer that compresses every write into its own gzip member with libdeflate (ctypes
    releases the GIL, so the writers of one window compress in parallel threads).  A multi-member
    gzip file decompresses to the concatenation of its members, which is how gzip.open -- and the
    reference -- read it; the writes of one file arrive in order (the caller waits for a window's
    jobs before it submits the next window's).  A file nothing was written to gets one empty member,
    as gzip.open's writer leaves it."""

    def __init__(self, path: str, level: int):
        self.f = open(path, "wb")
        self.level = level
        self.wrote = False

    def _compressor(self):
        c = getattr(_LD_TLS, "c", None)
        if c is None:
            c = _LD_TLS.c = {}
        h = c.get(self.level)
        if h is None:
            h = c[self.level] = _LD.libdeflate_alloc_compressor(self.level)
            if not h:
                raise MemoryError("libdeflate_alloc_compressor")
        return h

    def write_from(self, arr: np.ndarray, start: int, end: int) -> None:
        import ctypes

        n = end - start
        if n <= 0:
            return
        comp = self._compressor()
        bound = _LD.libdeflate_gzip_compress_bound(comp, n)
        out = np.empty(bound, dtype=np.uint8)
        k = _LD.libdeflate_gzip_compress(comp, ctypes.c_void_p(arr.ctypes.data + start), n,
                                         ctypes.c_void_p(out.ctypes.data), bound)
        if k == 0:
            raise RuntimeError("libdeflate_gzip_compress: output bound too small")
        self.f.write(memoryview(out)[:k])
        self.wrote = True

    def close(self) -> None:
        if not self.wrote:
            self.f.write(gzip.compress(b"", compresslevel=self.level))
        self.f.close()


class _GzDevice:
    """A .fq.gz writer of gzip members whose deflate streams the GPU made (fr_dmx_deflate): one member
    per window, header + stream + (CRC-32, length) trailer.  A file nothing was written to gets one
    empty member, as gzip.open's writer leaves it."""

    def __init__(self, path: str, level: int):
        self.f = open(path, "wb")
        self.level = level
        self.wrote = False

    def write_member(self, arr: np.ndarray, start: int, end: int, crc: int, isize: int) -> None:
        if end <= start:
            return
        head, tail = _lib.gzip_frame(int(crc), int(isize))
        self.f.write(head)
        self.f.write(memoryview(arr)[start:end])
        self.f.write(tail)
        self.wrote = True

    def close(self) -> None:
        if not self.wrote:
            self.f.write(gzip.compress(b"", compresslevel=9))
        self.f.close()


class _GzFile:
    """gzip.open writer with the same write_from interface (the image has no libdeflate)."""

    def __init__(self, path: str, level: int):
        self.f = gzip.open(path, "wb", compresslevel=level)

    def write_from(self, arr: np.ndarray, start: int, end: int) -> None:
        if end > start:
            self.f.write(memoryview(arr)[start:end])

    def close(self) -> None:
        self.f.close()


def out_path(name, out_dir, infix, read) -> str:
    """frender.py:667-676's file name of one writer."""
    if not out_dir.endswith("/"):
        out_dir += "/"
    return f"{out_dir}{name}_frender-demux_{infix + '_' if infix else ''}{read}.fq.gz"


_WRITERS = {"gpu": _GzDevice, "libdeflate": _GzMembers, "zlib": _GzFile}


def writer_kind(name: str):
    """The writer class of --gz-writer (libdeflate falls back to zlib where the image has none)."""
    if name == "libdeflate" and _LD is None:
        name = "zlib"
    return _WRITERS[name]


def open_files(name, out_dir, infix, level, kind=_GzDevice):
    """frender.py:667-676."""
    return {read: kind(out_path(name, out_dir, infix, read), level) for read in ("R1", "R2")}


_MATE_TAG = re.compile("_R([12])_")


def is_read_mate(str1, str2) -> bool:
    """frender.py:685-693: the two paths differ at exactly one position (compared over the shorter
    one's length) and their first `_R1_`/`_R2_` tags are one of each.  A path without such a tag
    fails the way the reference does (TypeError on the missing match)."""
    diff = sum(map(str.__ne__, str1, str2))
    if diff != 1:
        return False
    mates = {_MATE_TAG.search(s)[1] for s in (str1, str2)}
    return mates == {"1", "2"}


def get_paired_files(files_list) -> list:
    """frender.py:696-716."""
    pairs = []
    for path in [p for p in files_list if re.search("_R1_", str(p), re.IGNORECASE)]:
        mates = [i for i, f in enumerate(files_list) if is_read_mate(str(path), str(f))]
        if len(mates) > 1:
            raise SystemExit(f"Found more than one potential read 2 file for {path}")
        if not mates:
            raise SystemExit(f"Couldn't find a read 2 file for {path}")
        pairs.append((path, files_list[mates[0]]))
    return pairs


def _replay_gz_error(path):
    """Error path only: the native inflate rejected the file.  The reference's text-mode reader
    (frender.py:776-777) raises on it as Python's gzip does: re-read it that way to raise the same."""
    with gzip.open(path, "rt") as f:
        for _ in f:
            pass


def text_chunks(path, pool=None, index=0):
    """Decoded bytes of a .gz file as the reference's text-mode reader sees them (frender.py:776),
    streamed from the native inflate pool (fr_gz_next; a one-file pool when none is given): strict
    UTF-8 (UnicodeDecodeError otherwise, sequences may straddle blocks) and universal newlines folded
    to '\n' (a '\r' ending a block waits for the next one)."""
    import codecs

    own = pool is None
    if own:
        pool = _lib.GzPool([path], threads=1)
        index = 0
    dec = None
    hold = b""
    try:
        try:
            for raw in pool.blocks(index):
                data = hold + raw
                hold = b""
                if data.endswith(b"\r"):
                    hold, data = b"\r", data[:-1]
                if dec is not None or not data.isascii():
                    dec = dec or codecs.getincrementaldecoder("utf-8")()
                    dec.decode(data)  # raises like gzip.open(..., "rt")
                if b"\r" in data:
                    data = data.replace(b"\r\n", b"\n").replace(b"\r", b"\n")
                if data:
                    yield data
        except _lib.GzError as e:
            _replay_gz_error(path)
            raise RuntimeError(f"native inflate rejected {path} but Python's gzip reads it: {e}") from e
        if dec is not None:
            dec.decode(b"", final=True)
        if hold:
            yield b"\n"
    finally:
        if own:
            pool.close()


def read_text(path) -> bytes:
    """The whole decoded file (text-mode view): see text_chunks."""
    return b"".join(text_chunks(path))


def _line_at(parts, start: int) -> bytes:
    """The line that starts at byte `start` of the concatenation of `parts` (without its '\n')."""
    for k, p in enumerate(parts):
        if start >= len(p):
            start -= len(p)
            continue
        e = p.find(b"\n", start)
        if e >= 0:
            return p[start:e]
        out = [p[start:]]
        break
    else:
        return b""
    for q in parts[k + 1:]:
        e = q.find(b"\n")
        if e >= 0:
            out.append(q[:e])
            break
        out.append(q)
    return b"".join(out)


def _tail(parts, start: int) -> list:
    """The bytes of the concatenation of `parts` from `start` on, as parts (no copy of whole parts)."""
    for k, p in enumerate(parts):
        if start < len(p):
            return ([p[start:]] if start else [p]) + parts[k + 1:]
        start -= len(p)
    return []


STAGE_TIMES = {}  # seconds per stage of _demux_pair's windows (demux --stage-times prints them)


def _demux_pair(dmx, pool, gz, i1, i2, read1_file, read2_file, results, route_of, writers, window):
    """One R1/R2 pair in record-aligned windows: the GPU indexes both windows, the complete
    record pairs are routed, and the bytes after the last routed record carry into the next
    window.  Pairing stops when either mate runs out of records (zip, frender.py:777).  The mates
    inflate on the native pool gz (files i1, i2)."""
    streams = [text_chunks(read1_file, gz, i1), text_chunks(read2_file, gz, i2)]
    bufs = [[], []]  # each mate's window as a list of decoded blocks (never joined on the host)
    eof = [False, False]
    pending = []  # the previous window's gzip jobs: overlap with this window's inflate and GPU work
    st = STAGE_TIMES
    clock = time.perf_counter
    try:
        while True:
            t0 = clock()
            for m in (0, 1):
                size = sum(len(p) for p in bufs[m])
                while size < window and not eof[m]:
                    try:
                        c = next(streams[m])
                    except StopIteration:
                        eof[m] = True
                        break
                    bufs[m].append(c)
                    size += len(c)
            t1 = clock()
            n = [dmx.load_parts(0, bufs[0]), dmx.load_parts(1, bufs[1])]
            t2 = clock()
            # the last record of a window may continue in the next one unless its file ended
            done = [n[m] if eof[m] else max(n[m] - 1, 0) for m in (0, 1)]
            n_pairs = min(done)
            if n_pairs == 0:
                if eof[0] or eof[1] or (not n[0] and not n[1]):
                    break
                window *= 2  # a record longer than the window: widen it
                continue
            ex = dmx.exotic(n_pairs)
            if ex.size:  # codes outside the fast alphabet: resolve by string
                starts, _ = dmx.records(1, ex)
                dest = []
                for s in starts.tolist():
                    code = _line_at(bufs[1], s).split(b":")[-1].decode("utf-8")
                    row = results.get(code)
                    dest.append(_lib.FR_DMX_MISSING if row is None else route_of(row))
                dmx.patch(ex, np.array(dest, dtype=np.int32))
            first, val, b1, b2 = dmx.route(len(writers), n_pairs)
            t3 = clock()
            if first >= 0:
                s, _ = dmx.records(1, [first])
                code = _line_at(bufs[1], int(s[0])).split(b":")[-1].decode("utf-8")
                if val == _lib.FR_DMX_MISSING:
                    raise SystemExit(f"Couldn't find barcode {code} in supplied frender result file!")
                raise SystemExit("Unrecognized read type found in supplied frender result file!")
            if isinstance(writers[0]["R1"], _GzDevice):  # the GPU deflates every destination's bytes
                z1, k1, o1 = dmx.deflate(0, len(writers))
                z2, k2, o2 = dmx.deflate(1, len(writers))
                t4 = clock()
                for j in pending:
                    j.result()
                c1 = np.concatenate([[0], np.cumsum(z1)]).astype(np.int64)
                c2 = np.concatenate([[0], np.cumsum(z2)]).astype(np.int64)
                pending = []
                for k, w in enumerate(writers):
                    if b1[k]:
                        pending.append(pool.submit(w["R1"].write_member, o1, int(c1[k]), int(c1[k + 1]), k1[k], b1[k]))
                    if b2[k]:
                        pending.append(pool.submit(w["R2"].write_member, o2, int(c2[k]), int(c2[k + 1]), k2[k], b2[k]))
            else:
                o1 = dmx.fetch(0, int(b1.sum()))
                o2 = dmx.fetch(1, int(b2.sum()))
                t4 = clock()
                for j in pending:
                    j.result()
                c1 = np.concatenate([[0], np.cumsum(b1)]).astype(np.int64)
                c2 = np.concatenate([[0], np.cumsum(b2)]).astype(np.int64)
                pending = []
                for k, w in enumerate(writers):
                    if b1[k]:
                        pending.append(pool.submit(w["R1"].write_from, o1, int(c1[k]), int(c1[k + 1])))
                    if b2[k]:
                        pending.append(pool.submit(w["R2"].write_from, o2, int(c2[k]), int(c2[k + 1])))
            t5 = clock()
            for k, v in (("inflate+join", t1 - t0), ("load+index", t2 - t1), ("route", t3 - t2), ("deflate/fetch", t4 - t3),
                         ("wait writers", t5 - t4)):
                st[k] = st.get(k, 0.0) + v
            st["windows"] = st.get("windows", 0) + 1
            # carry the bytes after the routed records
            for m in (0, 1):
                if n_pairs < n[m]:
                    s, _ = dmx.records(m, [n_pairs])
                    bufs[m] = _tail(bufs[m], int(s[0]))
                else:
                    bufs[m] = []
            if (eof[0] and n_pairs == n[0]) or (eof[1] and n_pairs == n[1]):
                break
    finally:
        for j in pending:
            j.result()
        for st in streams:
            st.close()


def frender_demux(args, dev=None) -> None:
    """frender.py:733-814 with the per-record loop on the GPU."""
    t_start = time.perf_counter()
    index_hop = not args.no_index_hop
    ambiguous = not args.no_ambiguous
    undeter = not args.no_undeter
    samples = not args.no_samples
    level = getattr(args, "gz_level", None) or 9  # gzip.open's default, as the reference writes
    kind = writer_kind(getattr(args, "gz_writer", None) or "gpu")
    if kind is _GzDevice and getattr(args, "gz_level", None) not in (None, 9):
        print(f"Warning: --gz-level {args.gz_level} has no effect with --gz-writer gpu (the GPU writer's streams "
              "are no larger than level 9's); use --gz-writer libdeflate or zlib for another level", file=sys.stderr)
    infix = args.o
    undeter_name = f"Undetermined{'-ambiguous' if ambiguous else ''}{'-index-hop' if index_hop else ''}"

    from .dist import world_group
    group = None if dev is not None else world_group()  # demux --gpus N: one rank of N
    lead = group is None or group.get_rank() == 0

    result_file = Path(args.r)
    if not Path.is_file(result_file):
        raise SystemExit(f"File {result_file} not found")
    results = parse_results_file(result_file, strict=getattr(args, "strict_header", False))
    ids = sorted({sid for _, sid in results.values()} - {""})
    if (not ids) & samples and lead:
        print("Warning: no demuxable sample ids found in the supplied frender result file!")

    if group is None:
        os.mkdir(args.d)
    else:
        _mkdir_everywhere(group, args.d)
    writers = []  # destination id -> writer pair (N ranks: its name; rank 0 writes the files at the end)

    def new_writers(name):
        writers.append(open_files(name, args.d, infix, level, kind) if group is None else name)
        return len(writers) - 1

    sample_dest = {sid: new_writers(sid) for sid in ids} if samples else None
    undeter_dest = new_writers(undeter_name) if undeter else None
    hop_dest = new_writers("Index-hop") if index_hop else undeter_dest
    amb_dest = new_writers("Ambiguous") if ambiguous else undeter_dest

    def route_of(row) -> int:  # frender.py:779-810
        rtype, sid = row
        if rtype == "demuxable" and sample_dest:
            return sample_dest.get(sid, _lib.FR_DMX_MISSING)  # KeyError -> "Couldn't find barcode"
        if rtype == "index_hop" and hop_dest is not None:
            return hop_dest
        if rtype == "ambiguous" and amb_dest is not None:
            return amb_dest
        if rtype == "undetermined" and undeter_dest is not None:
            return undeter_dest
        return _lib.FR_DMX_BADTYPE

    codes = list(results.keys())
    keys, fast = _lib.pack_fast(codes)
    vals = np.array([route_of(results[c]) for c in codes], dtype=np.int32)

    if len(args.files) == 1:
        file = Path(args.files[0])
        if Path.is_dir(file):
            spec = {"dir": file}
        elif Path.is_file(file):
            spec = {"file": file}
        else:
            raise SystemExit("Specified directory or file path doesn't seem to exist!")
    else:
        spec = {"file": [Path(f) for f in args.files]}
    pairs = get_paired_files(parse_files(spec, just_r1=False))

    window = int(getattr(args, "window", None) or (512 << 20))  # decoded bytes per mate per GPU pass
    if group is not None:
        return _demux_ranks(group, args, dev, pairs, results, route_of, keys[fast], vals[fast], writers, window, level,
                            infix, kind)
    # with the GPU compressing, the host's cores inflate (a big single-member file in parallel); the
    # pool's workers start at once, so the first blocks decode while the device context comes up
    paths = [str(f) for pr in pairs for f in pr]
    nt = _inflate_threads(kind)
    gz = _lib.GzPool(paths, threads=nt, ahead=_lib.inflate_ahead(paths, nt))
    STAGE_TIMES["setup: results, writers"] = time.perf_counter() - t_start
    try:
        dmx = dev or _lib.Demux(_device_index(None))
    except BaseException:
        gz.close()
        raise
    pool = ThreadPoolExecutor(max_workers=max(2, min(32, len(writers) * 2)))
    try:
        dmx.set_table(keys[fast], vals[fast])
        STAGE_TIMES["setup"] = time.perf_counter() - t_start  # results, writers, device table, pool
        for k, (read1_file, read2_file) in enumerate(pairs):
            print(f"Demultiplexing {read1_file.name}...")
            _demux_pair(dmx, pool, gz, 2 * k, 2 * k + 1, read1_file, read2_file, results, route_of, writers, window)
    finally:
        t_end = time.perf_counter()
        gz.close()
        t_gz = time.perf_counter()
        pool.shutdown(wait=True)
        STAGE_TIMES["finish: inflate pool"] = t_gz - t_end
        STAGE_TIMES["finish: writer pool"] = time.perf_counter() - t_gz
        for w in writers:
            for f in w.values():
                f.close()
        t_files = time.perf_counter()
        if dev is None:
            dmx.close()
        STAGE_TIMES["finish: files"] = t_files - t_end - STAGE_TIMES["finish: inflate pool"] - STAGE_TIMES["finish: writer pool"]
        STAGE_TIMES["finish"] = time.perf_counter() - t_end  # last writes, closes
        STAGE_TIMES["total"] = time.perf_counter() - t_start
        if getattr(args, "stage_times", False):
            print(json.dumps({k: round(v, 3) for k, v in STAGE_TIMES.items()}), file=sys.stderr)


# ---- demux --gpus N ------------------------------------------------------------------------------
# The reference demultiplexes its file pairs one after another into one writer pair per destination
# (frender.py:776-814).  Here rank r of N takes pairs r, r + N, ... (whole pairs: both mates of a pair
# must be read in lockstep), writes each pair's destinations into part files of its own, and rank 0
# concatenates the parts in pair order into the final files.  The writers emit gzip members, so a
# concatenation is a valid gzip stream whose text is the concatenation of the pairs' texts: the
# reference's file content.  The first failing pair (in pair order) decides the error, raised by the
# rank that met it, after rank 0 has written the pairs up to it.

def _inflate_threads(kind) -> int:
    """Inflate threads of the demux's GzPool: 4 beside host compressors; with the GPU writers, the
    process's CPUs up to 16.  The pool inflates as many files at once as fit its block budget (4 of
    the config-5 shape's 443-MB mates: this pair's and the next), each big single-member file split
    over its share of the threads."""
    if kind is not _GzDevice:
        return 4
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 4)
    return max(4, min(16, n))


def _device_index(group) -> int:
    """This rank's GPU: LOCAL_RANK, folded onto the visible GPUs for gloo rehearsals on one GPU."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if group is not None and group.get_backend() == "gloo":
        import torch
        local %= max(torch.cuda.device_count(), 1)
    return local


def _wire(group):
    return "cpu" if group.get_backend() == "gloo" else f"cuda:{_device_index(group)}"


def _mkdir_everywhere(group, path):
    """Rank 0 creates the output directory (FileExistsError as the reference raises it); every rank
    learns the outcome before anyone writes."""
    from .dist import PeerFailed, reduce_max
    err = None
    if group.get_rank() == 0:
        try:
            os.mkdir(path)
        except OSError as e:
            err = e
    if int(reduce_max(group, _wire(group), [1 if err is not None else 0])[0]):
        if err is not None:
            raise err
        raise PeerFailed()


def _demux_ranks(group, args, dev, pairs, results, route_of, keys, vals, names, window, level, infix, kind):
    import shutil

    from .dist import PeerFailed, reduce_min
    rank, world = group.get_rank(), group.get_world_size()
    parts = os.path.join(args.d, ".frender-parts")
    mine = list(range(rank, len(pairs), world))
    gz = dmx = None
    pool = ThreadPoolExecutor(max_workers=max(2, min(32, len(names) * 2)))
    failed, exc = len(pairs), None
    try:
        # opened inside the try: a rank whose pool or device fails still joins the collectives below
        paths = [str(f) for k in mine for f in pairs[k]]
        nt = _inflate_threads(kind)
        gz = _lib.GzPool(paths, threads=nt, ahead=_lib.inflate_ahead(paths, nt))
        dmx = _lib.Demux(_device_index(group))
        dmx.set_table(keys, vals)
        for j, k in enumerate(mine):
            d = os.path.join(parts, str(k))
            os.makedirs(d, exist_ok=True)
            writers = [open_files(n, d, infix, level, kind) for n in names]
            try:
                _demux_pair(dmx, pool, gz, 2 * j, 2 * j + 1, pairs[k][0], pairs[k][1], results, route_of, writers,
                            window)
            except (Exception, SystemExit) as e:  # re-raised below if it is the first in pair order
                failed, exc = k, e
            finally:
                for w in writers:
                    for f in w.values():
                        f.close()
            if exc is not None:
                break
    except (Exception, SystemExit) as e:  # before any pair (the device, the table): this rank's first pair
        if exc is None:
            failed, exc = (mine[0] if mine else len(pairs)), e
    finally:
        pool.shutdown(wait=True)
        if gz is not None:
            gz.close()
        if dmx is not None:
            dmx.close()
    first = int(reduce_min(group, _wire(group), [failed])[0])  # every rank's pairs are done here
    last = min(first, len(pairs) - 1)
    if rank == 0:
        for k in range(last + 1):
            print(f"Demultiplexing {pairs[k][0].name}...")
        for n in names:
            for read in ("R1", "R2"):
                final = out_path(n, args.d, infix, read)
                with open(final, "wb") as out:
                    for k in range(last + 1):
                        part = out_path(n, os.path.join(parts, str(k)), infix, read)
                        if os.path.exists(part):
                            with open(part, "rb") as f:
                                shutil.copyfileobj(f, out, 16 << 20)
                    if out.tell() == 0:  # no pair reached it: an empty gzip file, as the reference's writer
                        out.write(gzip.compress(b"", compresslevel=level))
    reduce_min(group, _wire(group), [0])  # the parts are read: remove them
    if rank == 0:
        shutil.rmtree(parts, ignore_errors=True)
    if first < len(pairs):
        if failed == first:
            raise exc
        raise PeerFailed()
