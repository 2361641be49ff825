"""A CPU stand-in for frender_amd._lib.Context (TEST INFRASTRUCTURE ONLY): the tally half of the
C ABI (reset / begin_file_at / feed / end_file / finalize / unique / presence / exotic_table /
device merge) restated in Python over the oracle's rules, so the multi-rank host logic
(frender_amd/dist.py: sharded_tally, merge_tables) runs under gloo on CPU.  Keys follow
include/frender_amd.h (fast 3-bit keys, wide base-5 keys, exotic codes by bytes); ordinals are
(file index + 1) << 44 | byte offset of the record's header."""
from __future__ import annotations

import re
import types

import numpy as np

from frender_amd import _lib

LINE = re.compile(rb"\r\n|\r|\n")
SYM = {"A": 1, "C": 2, "G": 3, "T": 4, "N": 5, "+": 6}


def fast_key(code: str):
    if not 1 <= len(code) <= 21 or any(ch not in SYM for ch in code):
        return None
    return sum(SYM[ch] << (3 * i) for i, ch in enumerate(code))


class FakeContext:
    def __init__(self):
        self.mem = {}
        self.reset()

    # ---- tally ------------------------------------------------------------------------
    def reset(self):
        self.tab = {}        # key -> [count, first, set(files)]
        self.exo = {}        # bytes -> [count, first, set(files)]
        self.merged = False

    def begin_file(self, sample, file_index=None, byte_base=0):
        self.fi = file_index
        self.base = byte_base
        self.sample = sample
        self.buf = bytearray()

    def feed(self, data) -> bool:
        self.buf += bytes(data)
        return False

    def feed_gz(self, pool, i) -> bool:
        import gzip
        with gzip.open(pool.paths[i], "rb") as g:
            return self.feed(g.read())

    def end_file(self):
        data = bytes(self.buf)
        st = types.SimpleNamespace(records=0, new_keys=0, exotic=0, error=0, utf8_bad=0, lines=0)
        try:
            data.decode("utf-8")
        except UnicodeDecodeError:
            st.utf8_bad = 1
        starts, pos, k = [], 0, 0
        for m in LINE.finditer(data):
            if k % 4 == 0:
                starts.append((pos, m.start()))
            pos, k = m.end(), k + 1
        if pos < len(data):
            if k % 4 == 0:
                starts.append((pos, len(data)))
        if self.sample:
            starts = starts[: self.sample]
        seen = set()
        tag = (self.fi + 1) << 44
        for s, e in starts:
            line = data[s:e].decode("utf-8", errors="replace")
            parts = line.split(" ")
            if len(parts) < 2:
                st.error = _lib.FR_SCAN_NO_SPACE
                break
            code = parts[1].split(":")[-1]
            key = fast_key(code)
            if key is None:
                key = _lib.encode_wide(code)
            ordv = tag | (self.base + s)
            if key is None:
                tab, key = self.exo, code.encode()
                st.exotic += 1
            else:
                tab = self.tab
            e = tab.setdefault(key, [0, 1 << 64, set()])
            e[0] += 1
            e[1] = min(e[1], ordv)
            e[2].add(self.fi)
            seen.add(key)
            st.records += 1
        st.new_keys = len(seen)
        return st

    def finalize(self):
        self.order = sorted(self.tab, key=lambda k: self.tab[k][1])
        return len(self.order), 0, len(self.exo)

    def unique(self):
        keys = np.array(self.order, dtype=np.uint64)
        counts = np.array([self.tab[k][0] for k in self.order], dtype=np.uint64)
        first = np.array([self.tab[k][1] for k in self.order], dtype=np.uint64)
        return keys, counts, first

    def presence(self):
        pu = [i for i, k in enumerate(self.order) for _ in self.tab[k][2]]
        pf = [f for k in self.order for f in sorted(self.tab[k][2])]
        return np.array(pu, dtype=np.uint32), np.array(pf, dtype=np.uint32)

    def exotic_table(self):
        codes = list(self.exo)
        pc = [i for i, c in enumerate(codes) for _ in self.exo[c][2]]
        pf = [f for c in codes for f in sorted(self.exo[c][2])]
        return (codes, np.array([self.exo[c][0] for c in codes], dtype=np.uint64),
                np.array([self.exo[c][1] for c in codes], dtype=np.uint64),
                np.array(pc, dtype=np.uint32), np.array(pf, dtype=np.uint32))

    # ---- "device" merge ----------------------------------------------------------------
    def device_alloc(self, n):
        h = len(self.mem) + 1
        self.mem[h] = b""
        return h

    def device_free(self, h):
        self.mem.pop(h, None)

    def copy_to_device(self, h, data):
        self.mem[h] = bytes(data)

    def sync(self):
        pass

    def merge_unique_device(self, kp, cp, fp, n):
        keys, counts, first = (np.frombuffer(self.mem[h], dtype=np.uint64)[:n] for h in (kp, cp, fp))
        for k, c, f in zip(keys.tolist(), counts.tolist(), first.tolist()):
            e = self.tab.setdefault(k, [0, 1 << 64, set()])
            e[0] += c
            e[1] = min(e[1], f)
