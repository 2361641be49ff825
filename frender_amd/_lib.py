"""ctypes binding of libfrender_hip.so (include/frender_amd.h).

There is no fallback: if the HIP library is missing or does not load, importing
this module raises.  Build it with `python -c "import __graft_entry__ as g; g.build()"`.

PyTorch (when importable) is imported first so that this process holds a single
HIP runtime: torch ships its own libamdhip64.so.7 and our library's NEEDED entry
then binds to that same copy, which lets torch.distributed (RCCL) move buffers
that this library wrote.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _runtime

torch = None
if _runtime.USE_TORCH:  # one HIP runtime per process (see module doc)
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is plumbing only
        torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FRENDER_HIP_LIB", os.path.join(HERE, "libfrender_hip.so"))


def source_tree_hash() -> str:
    """sha256 (16 hex digits) of the sources libfrender_hip.so is built from (csrc/ + the C header):
    measurements kept under profiles/ (the PMC traffic file) name the tree they were taken on, and
    bench.py refuses one taken on another tree."""
    import hashlib

    h = hashlib.sha256()
    csrc = os.path.join(HERE, "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".cpp", ".h")))
    files.append(os.path.join(os.path.dirname(HERE), "include", "frender_amd.h"))
    for p in files:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]

FR_OK = 0
FR_ERR_INVALID = 1
FR_SAMPLE_DONE = 5
FR_ERR_IO = 6
FR_SCAN_OK, FR_SCAN_NO_SPACE, FR_SCAN_UTF8 = 0, 1, 2
CLASS_NAMES = ("undetermined", "index_hop", "demuxable", "ambiguous")


class FrenderError(RuntimeError):
    pass


class FileStats(C.Structure):
    _fields_ = [("records", C.c_uint64), ("lines", C.c_uint64), ("new_keys", C.c_uint64),
                ("exotic", C.c_uint64), ("error", C.c_int32), ("utf8_bad", C.c_int32),
                ("error_offset", C.c_uint64)]


class Timing(C.Structure):
    _fields_ = [("scan_launches", C.c_uint64), ("scan_bytes", C.c_uint64), ("scan_ms", C.c_double),
                ("last_scan_ms", C.c_double), ("classify_ms", C.c_double), ("finalize_ms", C.c_double),
                ("log_ms", C.c_double)]


class Tuning(C.Structure):
    """fr_tuning (include/frender_amd.h): the tally's geometry and thresholds.  Results never depend on
    them; tests and A/B runs pass them on purpose (Context(tuning={...})), nothing reads the environment."""
    _fields_ = [("size", C.c_uint32), ("grid", C.c_int32), ("flush_at", C.c_uint32), ("cold_cap", C.c_uint32),
                ("log", C.c_int32), ("log_min", C.c_uint32), ("log_hot", C.c_uint32), ("chunk_tiles", C.c_uint32),
                ("chunk_tiles_heavy", C.c_uint32), ("ramp", C.c_int32), ("ramp_up_s", C.c_uint32),
                ("ramp_down_s", C.c_uint32), ("ramp_down_pct", C.c_uint32), ("ramp_down_pct_h", C.c_uint32),
                ("spec_commit", C.c_int32), ("nbr", C.c_int32), ("ovf_cap", C.c_uint64)]


if not os.path.exists(LIB_PATH):
    raise ImportError(f"frender_amd: HIP library {LIB_PATH} is not built (run __graft_entry__.build())")
lib = C.CDLL(LIB_PATH)

P = C.c_void_p
u64p = C.POINTER(C.c_uint64)
_SIGS = {
    "fr_create": (P, [C.c_int, C.c_uint64, C.c_uint64]),
    "fr_tuning_defaults": (None, [C.POINTER(Tuning)]),
    "fr_create_tuned": (P, [C.c_int, C.c_uint64, C.c_uint64, C.POINTER(Tuning)]),
    "fr_destroy": (None, [P]),
    "fr_last_error": (C.c_char_p, [P]),
    "fr_get_timing": (C.c_int, [P, C.POINTER(Timing)]),
    "fr_sync": (C.c_int, [P]),
    "fr_set_timing": (C.c_int, [P, C.c_int]),
    "fr_get_diag": (C.c_int, [P, P, C.c_int]),
    "fr_set_sheet": (C.c_int, [P, C.c_int, P, P, P, P, P, P, C.c_int, P, P, P, C.c_int]),
    "fr_reset": (C.c_int, [P]),
    "fr_begin_file": (C.c_int, [P, C.c_int64]),
    "fr_begin_file_at": (C.c_int, [P, C.c_int64, C.c_uint64, C.c_int64]),
    "fr_feed": (C.c_int, [P, P, C.c_uint64]),
    "fr_feed_device": (C.c_int, [P, P, C.c_uint64]),
    "fr_end_file": (C.c_int, [P, C.POINTER(FileStats)]),
    "fr_finalize": (C.c_int, [P, u64p, u64p, u64p]),
    "fr_get_unique": (C.c_int, [P, P, P, P]),
    "fr_get_presence": (C.c_int, [P, P, P]),
    "fr_get_presence_counts": (C.c_int, [P, P, P]),
    "fr_exotic_sizes": (C.c_int, [P, u64p, u64p, u64p]),
    "fr_get_exotic_table": (C.c_int, [P, P, P, P, P, P, P]),
    "fr_classify": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P, P, P, P, P]),
    "fr_rc_counts": (C.c_int, [P, P, P]),
    "fr_classify_cp": (C.c_int, [P, C.c_int, P, P, P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P, P, P]),
    "fr_export_unique_device": (C.c_int, [P, P, P, P, C.c_uint64]),
    "fr_merge_unique_device": (C.c_int, [P, P, P, P, C.c_uint64]),
    "fr_export_partitioned_device": (C.c_int, [P, C.c_int, P, P, C.c_uint64]),
    "fr_merge_rows_device": (C.c_int, [P, P, C.c_uint64]),
    "fr_device_alloc": (P, [P, C.c_uint64]),
    "fr_device_free": (C.c_int, [P, P]),
    "fr_copy_to_host": (C.c_int, [P, P, P, C.c_uint64]),
    "fr_copy_to_device": (C.c_int, [P, P, P, C.c_uint64]),
    "fr_synth_device": (C.c_int, [P, P, C.c_uint64, C.c_uint64, C.c_int, C.c_uint64, C.c_char_p, C.c_char_p,
                                  C.c_int, C.c_int, C.c_int]),
    # native inflate (row f-2)
    "fr_gz_open": (P, [C.POINTER(C.c_char_p), C.c_int, C.c_int]),
    "fr_gz_open_ahead": (P, [C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_int]),
    "fr_gz_feed": (C.c_int, [P, C.c_int, P]),
    "fr_gz_next": (C.c_int, [P, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    "fr_gz_feed_part": (C.c_int, [P, C.c_int, P, C.c_int64, C.c_int, C.c_int, C.c_uint64, C.POINTER(C.c_uint64)]),
    "fr_gz_size_hint": (C.c_uint64, [C.c_char_p]),
    "fr_write_scan_csv": (C.c_int, [C.c_char_p, C.c_char_p, C.c_uint64, P, P, P, P, P, P, P, C.c_char_p, P, P,
                                    C.c_uint64, P, C.c_char_p, P]),
    "fr_gz_part_bounds": (C.c_int, [C.c_char_p, C.c_int, C.c_uint64, C.POINTER(C.c_uint64)]),
    "fr_gz_error": (C.c_char_p, [P]),
    "fr_gz_part_open": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int),
                                  u64p, u64p]),
    "fr_gz_part_data": (C.c_int, [P, C.c_uint64, C.POINTER(C.c_void_p), u64p, u64p, u64p]),
    "fr_gz_part_feed": (C.c_int, [P, P, C.c_int64, C.c_uint64, u64p]),
    "fr_gz_part_error": (C.c_char_p, [P]),
    "fr_gz_part_close": (None, [P]),
    "fr_gz_close": (None, [P]),
    "fr_gz_trim": (None, []),
    "fr_gz_parallel_members": (C.c_uint64, []),
    # demux (row f-1)
    "fr_dmx_create": (P, [C.c_int]),
    "fr_dmx_destroy": (None, [P]),
    "fr_dmx_last_error": (C.c_char_p, [P]),
    "fr_dmx_set_table": (C.c_int, [P, P, P, C.c_uint64]),
    "fr_dmx_load": (C.c_int, [P, C.c_int, P, C.c_uint64, u64p]),
    "fr_dmx_load_device": (C.c_int, [P, C.c_int, P, C.c_uint64, u64p]),
    "fr_dmx_records": (C.c_int, [P, C.c_int, P, C.c_uint64, P, P]),
    "fr_dmx_exotic": (C.c_int, [P, C.c_uint64, P, C.c_uint64, u64p]),
    "fr_dmx_patch": (C.c_int, [P, P, P, C.c_uint64]),
    "fr_dmx_route": (C.c_int, [P, C.c_int, C.c_uint64, C.POINTER(C.c_int64), C.POINTER(C.c_int32), P, P]),
    "fr_dmx_fetch": (C.c_int, [P, C.c_int, P, C.c_uint64]),
    "fr_dmx_load_parts": (C.c_int, [P, C.c_int, P, P, C.c_int, C.POINTER(C.c_uint64)]),
    "fr_dmx_deflate": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "fr_dmx_fetch_deflated": (C.c_int, [P, C.c_int, P, C.c_uint64]),
    "fr_defl_create": (P, [C.c_int]),
    "fr_defl_destroy": (None, [P]),
    "fr_defl_last_error": (C.c_char_p, [P]),
    "fr_defl_run": (C.c_int, [P, P, P, C.c_int, P, P]),
    "fr_defl_run_host": (C.c_int, [P, P, C.c_uint64, P, C.c_int, P, P]),
    "fr_defl_out_bytes": (C.c_uint64, [P]),
    "fr_defl_stored_fallbacks": (C.c_uint64, [P]),
    "fr_defl_fetch": (C.c_int, [P, P, C.c_uint64]),
}
for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_SIGS)


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(P)


M21 = np.arange(21, dtype=np.uint64) * np.uint64(3)
SYM_LUT = np.frombuffer(b"\0ACGTN+\0", dtype=np.uint8)
WIDE_BIT = np.uint64(1 << 63)
WIDE_MAXN, WIDE_NOPLUS = 24, 31
WIDE_OFF = np.array([(5 ** n - 1) // 4 for n in range(WIDE_MAXN + 2)], dtype=np.uint64)  # length offsets


def _decode_wide(keys: np.ndarray) -> list:
    """Wide keys (include/frender_amd.h) -> code strings, vectorised over the keys."""
    V = keys & np.uint64((1 << 57) - 1)
    plus = ((keys >> np.uint64(57)) & np.uint64(31)).astype(np.int64)
    lower = ((keys >> np.uint64(62)) & np.uint64(1)).astype(bool)
    n = np.searchsorted(WIDE_OFF, V, side="right") - 1  # letters: the largest n with off[n] <= V
    D = V - WIDE_OFF[n]
    digits = np.empty((keys.size, WIDE_MAXN), dtype=np.uint8)
    for i in range(WIDE_MAXN):
        digits[:, i] = (D % np.uint64(5)).astype(np.uint8)
        D //= np.uint64(5)
    up = np.frombuffer(b"ACGTN", dtype=np.uint8)[digits]
    out = []
    for r, k, p, lo in zip(up.view(f"S{WIDE_MAXN}").ravel().tolist(), n.tolist(), plus.tolist(), lower.tolist()):
        s = r[:k].decode("ascii")
        if p != WIDE_NOPLUS:
            s = s[:p] + "+" + s[p:]
        out.append(s.lower() if lo else s)
    return out


def decode_keys(keys: np.ndarray) -> list:
    """Packed keys -> code strings: fast keys 3 bits per char (char i at bits [3i, 3i+3)), wide
    keys (bit 63) base 5 per letter (include/frender_amd.h)."""
    if keys.size == 0:
        return []
    wide = (keys & WIDE_BIT) != 0
    syms = ((keys[:, None] >> M21[None, :]) & np.uint64(7)).astype(np.uint8)
    raw = np.ascontiguousarray(SYM_LUT[syms]).view("S21").ravel()
    out = [b.decode("ascii") for b in raw.tolist()]
    if wide.any():
        w = np.nonzero(wide)[0]
        for i, c in zip(w.tolist(), _decode_wide(keys[w])):
            out[i] = c
    return out


def encode_wide(code: str):
    """The wide key of a code (None outside the wide form): the host statement of wide_encode in
    fr_kernels.hip, for tests and the demux results table."""
    if not 1 <= len(code) <= WIDE_MAXN + 1 or code.count("+") > 1:
        return None
    letters = code.replace("+", "")
    if not letters or not (set(letters) <= set("ACGTN") or set(letters) <= set("acgtn")):
        return None
    p = code.find("+")
    n1, n2 = (len(letters), 0) if p < 0 else (p, len(letters) - p)
    if len(letters) > WIDE_MAXN or n1 > 21 or n2 > 21:
        return None
    v = sum("acgtn".index(ch) * 5 ** i for i, ch in enumerate(letters.lower())) + (5 ** len(letters) - 1) // 4
    return (1 << 63) | (int(letters.islower()) << 62) | ((WIDE_NOPLUS if p < 0 else p) << 57) | v


def pack_lower(s: str) -> int:
    """Sheet entry -> 3-bit packed case-folded chars (a1 c2 g3 t4 n5 other 7); 0 if > 21 chars."""
    if len(s) > 21:
        return 0
    v = 0
    for i, ch in enumerate(s):
        v |= {"a": 1, "c": 2, "g": 3, "t": 4, "n": 5}.get(ch, 7) << (3 * i)
    return v


FR_DMX_MISSING, FR_DMX_BADTYPE, FR_DMX_EXOTIC = -1, -2, -3


_PACK_LUT = np.zeros(128, dtype=np.uint8)
for _i, _c in enumerate("ACGTN+"):
    _PACK_LUT[ord(_c)] = _i + 1


def pack_fast(codes) -> tuple:
    """Codes over {A,C,G,T,N,+} of 1..21 chars -> (3-bit packed keys, mask of the packable codes):
    character j of a code is bits 3j..3j+2 (A=1 C=2 G=3 T=4 N=5 +=6).  Vectorised over the codes (a
    per-character loop took 1.4 s for a 300k-row results file)."""
    n = len(codes)
    keys = np.zeros(n, dtype=np.uint64)
    ok = np.zeros(n, dtype=bool)
    if not n:
        return keys, ok
    lens = np.fromiter((len(c) for c in codes), dtype=np.int64, count=n)
    sel = np.nonzero((lens >= 1) & (lens <= 21))[0]
    if not sel.size:
        return keys, ok
    cp = np.array([codes[i] for i in sel.tolist()], dtype="<U21").view(np.uint32).reshape(-1, 21)
    # 0: not in the alphabet, or padding; one row per character position
    sym = np.ascontiguousarray(np.where(cp < 128, _PACK_LUT[np.minimum(cp, 127)], np.uint8(0)).T)
    nvalid = np.count_nonzero(sym, axis=0)
    good = nvalid == lens[sel]  # every character in the alphabet (padding is 0: it never counts)
    packed = np.zeros(sel.size, dtype=np.uint64)
    for j in range(21):
        packed |= sym[j].astype(np.uint64) << np.uint64(3 * j)
    keys[sel[good]] = packed[good]
    ok[sel[good]] = True
    return keys, ok


class GzError(FrenderError):
    """A .gz input the native inflate could not read (the caller replays it with Python's gzip)."""


def inflate_ahead(paths, threads: int, budget: int = 2 << 30) -> int:
    """Files a pool should inflate at once: as many as `threads` while their decoded sizes fit the pool's
    2-GiB block budget, fewer for big files (whose decode then splits over the idle threads: a consumer
    that reads the files in order otherwise waits on one thread per file).  A file's decoded size is its
    gzip trailer's ISIZE (the decoded length mod 2^32) lifted by whole 2^32 steps toward 4 x its size, as
    the native pool sizes it (fr_gz.cpp lift_isize): exact for a member of up to 4 GiB decoded, and a
    big member whose ISIZE wrapped, or a multi-member file's small last ISIZE, is not taken at its word."""
    big = 0
    for p in paths:
        try:
            with open(p, "rb") as f:
                f.seek(0, os.SEEK_END)
                n = f.tell()
                f.seek(max(n - 4, 0))
                isize = int.from_bytes(f.read(4), "little")
        except OSError:
            continue
        want = 4 * n
        big = max(big, isize + (((want - isize + (1 << 31)) >> 32) << 32 if want > isize else 0))
    if big <= 0:
        return max(1, threads)
    ahead = max(2, min(threads, budget // big)) if threads >= 2 else 1
    return max(1, min(ahead, len(paths)))  # one file: every thread splits it


class GzPool:
    """Native inflate of a scan's .gz files (fr_gz_*): `threads` host threads inflate the listed
    files in order ahead of the consumer; feed(i, ctx) hands file i's bytes to ctx.feed."""

    def __init__(self, paths, threads: int = 1, ahead: int = None):
        """`ahead`: files inflating at once (default `threads`); the other threads split big
        single-member files (fr_gz_open_ahead)."""
        self.paths = [str(p) for p in paths]
        enc = [os.fsencode(p) for p in self.paths]
        arr = (C.c_char_p * max(len(enc), 1))(*enc)
        threads = max(1, int(threads))
        self.h = lib.fr_gz_open_ahead(arr, len(enc), threads, max(1, int(ahead or threads)))
        if not self.h:
            raise FrenderError("fr_gz_open returned NULL")

    def feed(self, i: int, ctx) -> bool:
        """Feed file i into ctx's open file; True once the -s sample is complete."""
        return ctx.feed_gz(self, i)

    def _feed(self, i: int, ctx_handle) -> bool:
        rc = lib.fr_gz_feed(self.h, i, ctx_handle)
        if rc == FR_ERR_IO:
            raise GzError(lib.fr_gz_error(self.h).decode(errors="replace"))
        if rc not in (FR_OK, FR_SAMPLE_DONE):
            raise FrenderError(f"fr_gz_feed failed ({rc}): {lib.fr_gz_error(self.h).decode(errors='replace')}")
        return rc == FR_SAMPLE_DONE

    def blocks(self, i: int):
        """File i's decoded bytes, block by block (fr_gz_next; each block copied out before the next
        call).  GzError when the file is not a valid gzip stream."""
        ptr, n = C.c_void_p(), C.c_uint64()
        while True:
            rc = lib.fr_gz_next(self.h, i, C.byref(ptr), C.byref(n))
            if rc == FR_ERR_IO:
                raise GzError(lib.fr_gz_error(self.h).decode(errors="replace"))
            if rc != FR_OK:
                raise FrenderError(f"fr_gz_next failed ({rc}): {lib.fr_gz_error(self.h).decode(errors='replace')}")
            if not n.value:
                return
            yield C.string_at(ptr, n.value)

    def _feed_part(self, i: int, ctx_handle, file_index: int, part: int, nparts: int, hint: int) -> int:
        base = C.c_uint64(0)
        rc = lib.fr_gz_feed_part(self.h, i, ctx_handle, int(file_index), int(part), int(nparts), int(hint),
                                 C.byref(base))
        if rc == FR_ERR_IO:
            raise GzError(lib.fr_gz_error(self.h).decode(errors="replace"))
        if rc != FR_OK:
            raise FrenderError(f"fr_gz_feed_part failed ({rc}): {lib.fr_gz_error(self.h).decode(errors='replace')}")
        return int(base.value)

    @staticmethod
    def part_bounds(path, nparts: int, hint: int) -> list:
        """fr_gz_part_bounds: the record-aligned cuts [b_0 = 0, ..., b_nparts = size] of the file."""
        out = (C.c_uint64 * (nparts + 1))()
        rc = lib.fr_gz_part_bounds(os.fsencode(str(path)), int(nparts), int(hint), out)
        if rc == FR_ERR_IO:
            raise GzError(f"{path}: not a valid gzip stream")
        if rc != FR_OK:
            raise FrenderError(f"fr_gz_part_bounds failed ({rc})")
        return [int(x) for x in out]

    @staticmethod
    def size_hint(path) -> int:
        """fr_gz_size_hint: the decoded size the file's trailers promise (deterministic)."""
        return int(lib.fr_gz_size_hint(os.fsencode(str(path))))

    def close(self):
        if self.h:
            lib.fr_gz_close(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class GzPart:
    """One record part of a BGZF file decoded on its own, without inflating what precedes it
    (fr_gz_part_*, include/frender_amd.h).  open() returns None for a file that is not BGZF."""

    def __init__(self, h, lines: int, inflated: int):
        self.h, self.lines, self.inflated = h, lines, inflated
        self.base = None
        self.length = None

    @classmethod
    def open(cls, path, part: int, nparts: int, threads: int = 1):
        h, bg, lines, infl = C.c_void_p(), C.c_int(), C.c_uint64(), C.c_uint64()
        rc = lib.fr_gz_part_open(os.fsencode(str(path)), int(part), int(nparts), max(1, int(threads)), C.byref(h),
                                 C.byref(bg), C.byref(lines), C.byref(infl))
        if rc == FR_ERR_IO:
            raise GzError(f"{path}: a BGZF member does not decode")
        if rc != FR_OK:
            raise FrenderError(f"fr_gz_part_open failed ({rc})")
        return cls(h, int(lines.value), int(infl.value)) if bg.value else None

    def _ck(self, rc, what):
        if rc == FR_ERR_IO:
            raise GzError(lib.fr_gz_part_error(self.h).decode(errors="replace"))
        if rc not in (FR_OK, FR_SAMPLE_DONE):
            raise FrenderError(f"{what} failed ({rc}): {lib.fr_gz_part_error(self.h).decode(errors='replace')}")

    def _cut(self, lines_before: int):
        d, n, b, infl = C.c_void_p(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._ck(lib.fr_gz_part_data(self.h, int(lines_before), C.byref(d), C.byref(n), C.byref(b), C.byref(infl)),
                 "fr_gz_part_data")
        self.inflated, self.base, self.length = int(infl.value), int(b.value), int(n.value)
        return d, n.value

    def data(self, lines_before: int):
        """The part's records (bytes) and their file offset, given the terminators before its range."""
        d, n = self._cut(lines_before)
        return (C.string_at(d, n) if n else b""), self.base

    def feed(self, ctx_handle, file_index: int, lines_before: int) -> int:
        """fr_gz_part_feed into a context's scan; returns the part's byte base."""
        b = C.c_uint64()
        self._ck(lib.fr_gz_part_feed(self.h, ctx_handle, int(file_index), int(lines_before), C.byref(b)),
                 "fr_gz_part_feed")
        self._cut(lines_before)  # the cut is known now: records its size and the bytes inflated
        return int(b.value)

    def close(self):
        if self.h:
            lib.fr_gz_part_close(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Demux:
    """One GPU's demux state (fr_dmx): see include/frender_amd.h."""

    def __init__(self, device: int = 0):
        self.h = lib.fr_dmx_create(device)
        err = lib.fr_dmx_last_error(self.h) if self.h else b"fr_dmx_create returned NULL"
        if err:
            raise FrenderError(f"fr_dmx_create: {err.decode()}")

    def _ck(self, rc, what):
        if rc != FR_OK:
            raise FrenderError(f"{what}: {lib.fr_dmx_last_error(self.h).decode()} (rc={rc})")

    def close(self):
        if self.h:
            lib.fr_dmx_destroy(self.h)
            self.h = None

    def set_table(self, keys: np.ndarray, vals: np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        vals = np.ascontiguousarray(vals, dtype=np.int32)
        self._ck(lib.fr_dmx_set_table(self.h, _ptr(keys), _ptr(vals), keys.size), "fr_dmx_set_table")

    def load(self, mate: int, data) -> int:
        a = np.frombuffer(data, dtype=np.uint8)
        n = C.c_uint64()
        self._ck(lib.fr_dmx_load(self.h, mate, _ptr(a), a.size, C.byref(n)), "fr_dmx_load")
        return n.value

    def load_parts(self, mate: int, parts) -> int:
        """load() of the concatenation of a list of bytes objects, without joining them on the host."""
        ptrs = (C.c_void_p * max(len(parts), 1))(*[C.cast(C.c_char_p(p), C.c_void_p) for p in parts])
        lens = np.array([len(p) for p in parts] or [0], dtype=np.uint64)
        n = C.c_uint64()
        self._ck(lib.fr_dmx_load_parts(self.h, mate, ptrs, _ptr(lens), len(parts), C.byref(n)), "fr_dmx_load_parts")
        return n.value

    def load_device(self, mate: int, dev_ptr: int, nbytes: int) -> int:
        n = C.c_uint64()
        self._ck(lib.fr_dmx_load_device(self.h, mate, P(dev_ptr), nbytes, C.byref(n)), "fr_dmx_load_device")
        return n.value

    def records(self, mate: int, recs) -> tuple:
        r = np.ascontiguousarray(recs, dtype=np.uint64)
        s, e = np.empty(r.size, np.uint64), np.empty(r.size, np.uint64)
        self._ck(lib.fr_dmx_records(self.h, mate, _ptr(r), r.size, _ptr(s), _ptr(e)), "fr_dmx_records")
        return s, e

    def exotic(self, n_pairs: int) -> np.ndarray:
        n = C.c_uint64()
        self._ck(lib.fr_dmx_exotic(self.h, n_pairs, None, 0, C.byref(n)), "fr_dmx_exotic")
        out = np.empty(n.value, np.uint64)
        if n.value:
            self._ck(lib.fr_dmx_exotic(self.h, n_pairs, _ptr(out), n.value, C.byref(n)), "fr_dmx_exotic")
        return out

    def patch(self, recs, dest):
        r = np.ascontiguousarray(recs, dtype=np.uint64)
        d = np.ascontiguousarray(dest, dtype=np.int32)
        self._ck(lib.fr_dmx_patch(self.h, _ptr(r), _ptr(d), r.size), "fr_dmx_patch")

    def route(self, n_dest: int, n_pairs: int):
        fe, ev = C.c_int64(), C.c_int32()
        b1, b2 = np.zeros(n_dest, np.uint64), np.zeros(n_dest, np.uint64)
        self._ck(lib.fr_dmx_route(self.h, n_dest, n_pairs, C.byref(fe), C.byref(ev), _ptr(b1), _ptr(b2)),
                 "fr_dmx_route")
        return fe.value, ev.value, b1, b2

    def fetch(self, mate: int, nbytes: int) -> np.ndarray:
        out = np.empty(nbytes, np.uint8)
        self._ck(lib.fr_dmx_fetch(self.h, mate, _ptr(out), nbytes), "fr_dmx_fetch")
        return out

    def deflate(self, mate: int, n_dest: int) -> tuple:
        """The routed bytes of a mate as one raw deflate stream per destination (fr_dmx_deflate):
        (stream bytes per destination, CRC-32 per destination, the streams concatenated)."""
        comp, crc = np.zeros(n_dest, np.uint64), np.zeros(n_dest, np.uint32)
        self._ck(lib.fr_dmx_deflate(self.h, mate, n_dest, _ptr(comp), _ptr(crc)), "fr_dmx_deflate")
        out = np.empty(int(comp.sum()), np.uint8)
        self._ck(lib.fr_dmx_fetch_deflated(self.h, mate, _ptr(out), out.size), "fr_dmx_fetch_deflated")
        return comp, crc, out


class Deflater:
    """GPU deflate over byte ranges (fr_defl): see include/frender_amd.h."""

    def __init__(self, device: int = 0):
        self.h = lib.fr_defl_create(device)
        err = lib.fr_defl_last_error(self.h) if self.h else b"fr_defl_create returned NULL"
        if err:
            raise FrenderError(f"fr_defl_create: {err.decode()}")

    def close(self):
        if self.h:
            lib.fr_defl_destroy(self.h)
            self.h = None

    def compress(self, data, offsets=None) -> tuple:
        """Raw deflate streams of the ranges [offsets[s], offsets[s + 1]) of host bytes `data` (one
        range when offsets is None): (stream bytes per range, CRC-32 per range, the streams)."""
        a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        a = np.ascontiguousarray(a, dtype=np.uint8)
        offs = np.ascontiguousarray([0, a.size] if offsets is None else offsets, dtype=np.uint64)
        n = offs.size - 1
        comp, crc = np.zeros(n, np.uint64), np.zeros(n, np.uint32)
        rc = lib.fr_defl_run_host(self.h, _ptr(a), a.size, _ptr(offs), n, _ptr(comp), _ptr(crc))
        if rc != FR_OK:
            raise FrenderError(f"fr_defl_run_host: {lib.fr_defl_last_error(self.h).decode()} (rc={rc})")
        out = np.empty(int(lib.fr_defl_out_bytes(self.h)), np.uint8)
        rc = lib.fr_defl_fetch(self.h, _ptr(out), out.size)
        if rc != FR_OK:
            raise FrenderError(f"fr_defl_fetch: {lib.fr_defl_last_error(self.h).decode()} (rc={rc})")
        return comp, crc, out


def gzip_frame(crc: int, isize: int) -> tuple:
    """The header and trailer that make a raw deflate stream a gzip member (RFC 1952; XFL 2 and OS 255
    as Python's gzip writes them at level 9, mtime 0)."""
    import struct
    return b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x02\xff", struct.pack("<II", crc & 0xFFFFFFFF, isize & 0xFFFFFFFF)


def _torch_stream_done(device: int):
    """Wait for the work queued on torch's current stream of `device` (no-op without torch / CUDA)."""
    if torch is not None and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.current_stream(torch.device("cuda", device)).synchronize()


def tuning_defaults() -> Tuning:
    """The library's default fr_tuning (fr_tuning_defaults)."""
    t = Tuning()
    lib.fr_tuning_defaults(C.byref(t))
    return t


def gz_parallel_members() -> int:
    """Files this process decoded with the parallel single-member inflate (fr_gz_parallel_members)."""
    return int(lib.fr_gz_parallel_members())


def gz_trim():
    """Return the native inflate's cached decode buffers to the OS (fr_gz_trim)."""
    lib.fr_gz_trim()


class Context:
    """One GPU's scan state (fr_ctx)."""

    def __init__(self, device: int = 0, chunk_bytes: int = 256 << 20, table_slots: int = 1 << 20,
                 tuning: dict | None = None):
        """tuning: fr_tuning fields to change from the library's defaults (tests and A/B runs only; the
        product never passes any)."""
        self.device = int(device)
        if tuning:
            t = tuning_defaults()
            for k, v in tuning.items():
                if k == "size" or not hasattr(t, k):
                    raise ValueError(f"unknown fr_tuning field {k!r}")
                setattr(t, k, int(v))
            self.h = lib.fr_create_tuned(device, chunk_bytes, table_slots, C.byref(t))
        else:
            self.h = lib.fr_create(device, chunk_bytes, table_slots)
        if not self.h:
            raise FrenderError("fr_create returned NULL")
        err = lib.fr_last_error(self.h)
        if err:
            raise FrenderError(f"fr_create: {err.decode()}")
        self.n_names = 0
        self._sheet_cache: dict = {}

    def close(self):
        if self.h:
            lib.fr_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _ck(self, rc: int, what: str) -> int:
        if rc not in (FR_OK, FR_SAMPLE_DONE):
            raise FrenderError(f"{what} failed ({rc}): {lib.fr_last_error(self.h).decode()}")
        return rc

    # ---- sheet ----------------------------------------------------------------------
    def set_sheet(self, idx1: list, idx2: list, idx2rc: list, name_id: list, n_names: int):
        last = getattr(self, "_sheet_last", None)
        if last is not None and last[0] == [idx1, idx2, idx2rc, list(name_id), n_names]:
            packed = last[1]  # the same lists as the last call (compared by value, at C speed): no re-keying
        else:
            key = (tuple(idx1), tuple(idx2), tuple(idx2rc), tuple(name_id), n_names)
            packed = self._sheet_cache.get(key)
            if packed is None:
                packed = self._pack_sheet(idx1, idx2, idx2rc, name_id)
                if len(self._sheet_cache) >= 8:
                    self._sheet_cache.clear()
                self._sheet_cache[key] = packed
        self._sheet_last = ([list(idx1), list(idx2), list(idx2rc), list(name_id), n_names], packed)
        p1, p2, p2rc, len1, len2, nid, cp, stride = packed
        self.cp_stride = stride
        self._sheet_keep = packed
        self.n_names = n_names
        self._ck(lib.fr_set_sheet(self.h, len(idx1), _ptr(p1), _ptr(len1), _ptr(p2), _ptr(len2), _ptr(p2rc),
                                  _ptr(nid), n_names, _ptr(cp[0]), _ptr(cp[1]), _ptr(cp[2]), stride),
                 "fr_set_sheet")

    @staticmethod
    def _pack_sheet(idx1, idx2, idx2rc, name_id):
        """Host-side encoding of the sheet lists (case-folded, 3-bit packed + code points)."""
        S = len(idx1)
        l1 = [s.lower() for s in idx1]
        l2 = [s.lower() for s in idx2]
        l2rc = [s.lower() for s in idx2rc]
        p1 = np.array([pack_lower(s) for s in l1], dtype=np.uint64)
        p2 = np.array([pack_lower(s) for s in l2], dtype=np.uint64)
        p2rc = np.array([pack_lower(s) for s in l2rc], dtype=np.uint64)
        len1 = np.array([len(s) for s in l1], dtype=np.int32)
        len2 = np.array([len(s) for s in l2], dtype=np.int32)
        nid = np.array(name_id, dtype=np.int32)
        stride = max([1] + [len(s) for s in l1 + l2])
        cp = [np.zeros((S, stride), dtype=np.uint32) for _ in range(3)]
        for arr, strs in zip(cp, (l1, l2, l2rc)):
            for i, s in enumerate(strs):
                arr[i, :len(s)] = [ord(ch) for ch in s]
        return p1, p2, p2rc, len1, len2, nid, cp, stride

    # ---- tally ----------------------------------------------------------------------
    def reset(self):
        self._ck(lib.fr_reset(self.h), "fr_reset")

    def begin_file(self, max_records: int | None, file_index: int | None = None, byte_base: int = 0):
        """Open the next file (or, for sharded scans, file `file_index` of the whole scan from byte
        `byte_base` on: fr_begin_file_at)."""
        if file_index is None and not byte_base:
            self._ck(lib.fr_begin_file(self.h, int(max_records or 0)), "fr_begin_file")
        else:
            self._ck(lib.fr_begin_file_at(self.h, int(file_index or 0), int(byte_base), int(max_records or 0)),
                     "fr_begin_file_at")

    def feed(self, data) -> bool:
        """Feed decoded bytes; returns True once the -s sample limit is reached."""
        buf = C.c_char_p(data) if isinstance(data, bytes) else None
        if buf is not None:
            rc = lib.fr_feed(self.h, C.cast(buf, P), len(data))
        else:
            a = np.frombuffer(data, dtype=np.uint8)
            rc = lib.fr_feed(self.h, _ptr(a), a.size)
        return self._ck(rc, "fr_feed") == FR_SAMPLE_DONE

    def feed_gz(self, pool: "GzPool", i: int) -> bool:
        """Feed file i of a native inflate pool (GzPool); True once the -s sample is complete."""
        return pool._feed(i, self.h)

    def feed_gz_part(self, pool: "GzPool", i: int, file_index: int, part: int, nparts: int, hint: int) -> int:
        """Begin file_index at part `part` of `nparts` of pool file i's records and feed that part
        (fr_gz_feed_part; call fr_end_file after); returns the part's byte base."""
        return pool._feed_part(i, self.h, file_index, part, nparts, hint)

    def feed_gz_part_counted(self, part: "GzPart", file_index: int, lines_before: int) -> int:
        """Begin file_index at a BGZF part's first record and feed its records (fr_gz_part_feed; call
        fr_end_file after); returns the part's byte base."""
        base = part.feed(self.h, file_index, lines_before)
        part.base = base
        return base

    def feed_device(self, dev_ptr: int, nbytes: int):
        self._ck(lib.fr_feed_device(self.h, P(dev_ptr), nbytes), "fr_feed_device")

    def end_file(self) -> FileStats:
        st = FileStats()
        self._ck(lib.fr_end_file(self.h, C.byref(st)), "fr_end_file")
        return st

    # ---- unique table ---------------------------------------------------------------
    def finalize(self):
        u, p, e = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._ck(lib.fr_finalize(self.h, C.byref(u), C.byref(p), C.byref(e)), "fr_finalize")
        self.U, self.NP, self.NE = u.value, p.value, e.value
        return self.U, self.NP, self.NE

    def unique(self):
        keys = np.empty(self.U, dtype=np.uint64)
        counts = np.empty(self.U, dtype=np.uint64)
        first = np.empty(self.U, dtype=np.uint64)
        self._ck(lib.fr_get_unique(self.h, _ptr(keys), _ptr(counts), _ptr(first)), "fr_get_unique")
        return keys, counts, first

    def presence(self):
        u = np.empty(self.NP, dtype=np.uint32)
        f = np.empty(self.NP, dtype=np.uint32)
        self._ck(lib.fr_get_presence(self.h, _ptr(u), _ptr(f)), "fr_get_presence")
        return u, f

    def presence_counts(self, n_exotic_pairs: int):
        """Reads of each presence pair's code in the pair's file (fr_get_presence_counts): aligned with
        presence() and with exotic_table()'s pairs (n_exotic_pairs of them)."""
        c = np.empty(self.NP, dtype=np.uint64)
        e = np.empty(int(n_exotic_pairs), dtype=np.uint64)
        self._ck(lib.fr_get_presence_counts(self.h, _ptr(c), _ptr(e)), "fr_get_presence_counts")
        return c, e

    def exotic_table(self):
        """The scan's exotic codes aggregated by the library: (codes as bytes, counts, first
        ordinals, presence code indices, presence file indices)."""
        n, nb, npres = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._ck(lib.fr_exotic_sizes(self.h, C.byref(n), C.byref(nb), C.byref(npres)), "fr_exotic_sizes")
        counts = np.empty(n.value, np.uint64)
        first = np.empty(n.value, np.uint64)
        offs = np.empty(n.value + 1, np.uint64)
        data = np.empty(max(nb.value, 1), np.uint8)
        pc = np.empty(npres.value, np.uint32)
        pf = np.empty(npres.value, np.uint32)
        self._ck(lib.fr_get_exotic_table(self.h, _ptr(counts), _ptr(first), _ptr(offs), _ptr(data), _ptr(pc),
                                         _ptr(pf)), "fr_get_exotic_table")
        raw = data.tobytes()
        o = offs.tolist()
        codes = [raw[o[i]:o[i + 1]] for i in range(n.value)]
        return codes, counts, first, pc, pf

    # ---- classify -------------------------------------------------------------------
    def classify(self, num_subs: int, rc: bool, to_host: bool = True):
        """Classify the finalized table on the GPU; to_host=False leaves the results in HBM."""
        n = self.U if to_host else 0
        out = {k: (np.empty(n, dtype=np.int16) if to_host else None) for k in ("m1", "m2", "row", "rc_m2", "rc_row")}
        out["cls"] = np.empty(n, dtype=np.uint8) if to_host else None
        out["rc_cls"] = np.empty(n, dtype=np.uint8) if to_host else None
        eu, ew = C.c_int64(), C.c_int32()
        self._ck(lib.fr_classify(self.h, num_subs, 1 if rc else 0, _ptr(out["m1"]), _ptr(out["m2"]),
                                 _ptr(out["cls"]), _ptr(out["row"]), _ptr(out["rc_m2"]), _ptr(out["rc_cls"]),
                                 _ptr(out["rc_row"]), C.byref(eu), C.byref(ew)), "fr_classify")
        out["err_unique"], out["err_which"] = eu.value, ew.value
        return out

    def rc_counts(self):
        f = np.zeros(max(self.n_names, 1), dtype=np.uint64)
        r = np.zeros(max(self.n_names, 1), dtype=np.uint64)
        self._ck(lib.fr_rc_counts(self.h, _ptr(f), _ptr(r)), "fr_rc_counts")
        return f[:self.n_names], r[:self.n_names]

    def classify_cp(self, q1: list, q2: list, num_subs: int, rc: bool):
        n = len(q1)
        stride = self.cp_stride
        a1 = np.zeros((n, stride), dtype=np.uint32)
        a2 = np.zeros((n, stride), dtype=np.uint32)
        for i, (x, y) in enumerate(zip(q1, q2)):
            a1[i, :min(len(x), stride)] = [ord(c) for c in x[:stride]]
            a2[i, :min(len(y), stride)] = [ord(c) for c in y[:stride]]
        l1 = np.array([len(x) for x in q1], dtype=np.int32)
        l2 = np.array([len(y) for y in q2], dtype=np.int32)
        out = {k: np.empty(n, dtype=np.int16) for k in ("m1", "m2", "row", "rc_m2", "rc_row")}
        out["cls"] = np.empty(n, dtype=np.uint8)
        out["rc_cls"] = np.empty(n, dtype=np.uint8)
        out["err"] = np.zeros(n, dtype=np.int32)
        self._ck(lib.fr_classify_cp(self.h, n, _ptr(a1), _ptr(l1), _ptr(a2), _ptr(l2), stride, num_subs,
                                    1 if rc else 0, _ptr(out["m1"]), _ptr(out["m2"]), _ptr(out["cls"]),
                                    _ptr(out["row"]), _ptr(out["rc_m2"]), _ptr(out["rc_cls"]), _ptr(out["rc_row"]),
                                    _ptr(out["err"])), "fr_classify_cp")
        return out

    # ---- device memory / synthetic data / timing --------------------------------------
    def device_alloc(self, nbytes: int) -> int:
        p = lib.fr_device_alloc(self.h, nbytes)
        if not p:
            raise FrenderError(f"fr_device_alloc({nbytes}) failed")
        return p

    def device_free(self, p: int):
        self._ck(lib.fr_device_free(self.h, P(p)), "fr_device_free")

    def copy_to_host(self, dev_ptr: int, nbytes: int) -> bytes:
        out = np.empty(nbytes, dtype=np.uint8)
        self._ck(lib.fr_copy_to_host(self.h, _ptr(out), P(dev_ptr), nbytes), "fr_copy_to_host")
        return out.tobytes()

    def copy_to_device(self, dev_ptr: int, data: bytes):
        a = np.frombuffer(data, dtype=np.uint8)
        self._ck(lib.fr_copy_to_device(self.h, P(dev_ptr), _ptr(a), a.size), "fr_copy_to_device")

    def synth_device(self, dev_ptr: int, r0: int, n: int, R: int, seed: int, idx1: list, idx2: list):
        L1, L2 = len(idx1[0]), len(idx2[0])
        self._ck(lib.fr_synth_device(self.h, P(dev_ptr), r0, n, R, seed, "".join(idx1).encode(),
                                     "".join(idx2).encode(), len(idx1), L1, L2), "fr_synth_device")

    def timing(self) -> Timing:
        t = Timing()
        self._ck(lib.fr_get_timing(self.h, C.byref(t)), "fr_get_timing")
        return t

    def diag(self) -> dict:
        v = np.zeros(24, dtype=np.uint64)
        self._ck(lib.fr_get_diag(self.h, _ptr(v), 24), "fr_get_diag")
        d = dict(zip(("spin_max", "spin_total", "keys", "overflow", "presence", "exotic", "grid", "slots"),
                     v[:8].tolist()))
        d["spec_replays"] = int(v[16])
        d["exo_replays"] = int(v[17])
        d["chunk_tiles"] = int(v[18])  # full-chunk size of the next ramped launch (larger once commits log)
        d["heavy_launches"] = int(v[19])  # ramped launches since the reset that walked the heavy chunk size
        d["big_rollbacks"] = int(v[20])  # big feeds replayed in logged ranges (the table ran out of room)
        d["fold_max"] = int(v[21])  # the last device feed's fullest launch-log fold (of AGG_LNS = 4096 slots)
        d["fold_over"] = int(v[22])  # its entries that found their fold full
        d["feed_step"] = int(v[23])  # its range size (bytes per launch)
        if v[8:16].any():  # FR_TIMING build / FR_ABLATE=64: per-phase cycles or commit counts
            names = ("guess", "walk0", "wait0", "resolve", "walk1", "commit", "kernel", "chunks")
            d["stamps"] = dict(zip(names, v[8:].tolist()))
        return d

    def sync(self):
        self._ck(lib.fr_sync(self.h), "fr_sync")

    def set_timing(self, on: bool):
        """HIP timing events on (default) or off (fr_set_timing): off removes their stream bubbles."""
        self._ck(lib.fr_set_timing(self.h, 1 if on else 0), "fr_set_timing")

    def export_unique_device(self, keys_ptr: int, counts_ptr: int, first_ptr: int, cap: int):
        """Copy the finalized table into device buffers (fr_export_unique_device: queued on the library's
        stream, which it synchronises before returning).  Stream contract: buffers that
        torch allocated may still be in use by work queued on torch's stream (its caching allocator hands
        a block back as soon as its last use is QUEUED), so torch's stream is drained first; afterwards the
        rows are complete in HBM and any stream (torch's, RCCL's) may read them."""
        _torch_stream_done(self.device)
        self._ck(lib.fr_export_unique_device(self.h, P(keys_ptr), P(counts_ptr), P(first_ptr), cap),
                 "fr_export_unique_device")

    def merge_unique_device(self, keys_ptr: int, counts_ptr: int, first_ptr: int, n: int):
        self._ck(lib.fr_merge_unique_device(self.h, P(keys_ptr), P(counts_ptr), P(first_ptr), n),
                 "fr_merge_unique_device")

    def export_partitioned(self, world: int):
        """The finalized rows as an int64 tensor [U, 3] on this GPU, partitioned by owner rank (blocks of
        owners 0..world-1 in order; fr_export_partitioned_device), and the rows per owner (int64 [world], same
        device).  Same stream contract as export_unique_device."""
        U = int(self.U)
        dev = torch.device("cuda", self.device)
        rows = torch.empty((max(U, 1), 3), dtype=torch.int64, device=dev)
        cnt = torch.empty(2 * world, dtype=torch.int64, device=dev)
        _torch_stream_done(self.device)
        self._ck(lib.fr_export_partitioned_device(self.h, int(world), P(rows.data_ptr()), P(cnt.data_ptr()),
                                                  max(U, 1)), "fr_export_partitioned_device")
        return rows[:U], cnt[:world]

    def merge_rows_rowmajor(self, rows):
        """Merge (key, count, first) rows [n, 3] (int64, on this GPU, row-major) into the table
        (fr_merge_rows_device); torch's stream is drained first (the rows may come from an RCCL receive)."""
        n = int(rows.shape[0])
        if not n:
            return
        rows = rows.contiguous()
        torch.cuda.current_stream(rows.device).synchronize()
        self._ck(lib.fr_merge_rows_device(self.h, P(rows.data_ptr()), n), "fr_merge_rows_device")
        self.sync()  # rows goes back to torch's allocator after this

    # ---- tensor views for the multi-GPU merge (frender_amd/dist.py) ----------------------
    def export_rows(self, device):
        """The finalized table as an int64 tensor [U, 3] of (key, count, first) rows on `device`
        (this GPU's HBM: fr_export_unique_device; "cpu" stages through it for gloo rehearsals)."""
        U = int(self.U)
        cols = torch.empty((3, max(U, 1)), dtype=torch.int64, device=torch.device("cuda", self.device))
        if U:
            self.export_unique_device(cols[0].data_ptr(), cols[1].data_ptr(), cols[2].data_ptr(), U)
        return cols[:, :U].t().to(device)

    def merge_rows(self, rows):
        """Merge (key, count, first) rows [n, 3] into this context's table (count = sum, first = min:
        fr_merge_unique_device); the rows may live on any device."""
        n = int(rows.shape[0])
        if not n:
            return
        cols = rows.t().contiguous().to(torch.device("cuda", self.device))
        torch.cuda.current_stream(cols.device).synchronize()  # a transfer on torch's stream has landed
        self.merge_unique_device(cols[0].data_ptr(), cols[1].data_ptr(), cols[2].data_ptr(), n)
        self.sync()  # cols goes back to torch's allocator after this
