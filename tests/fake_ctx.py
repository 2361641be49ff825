"""A CPU stand-in for frender_amd._lib.Context (TEST INFRASTRUCTURE ONLY): the C ABI's tally
(reset / begin_file_at / feed / record parts / end_file / finalize / unique / presence /
exotic_table), merge (export_rows / merge_rows) and classify (set_sheet / classify / classify_cp /
rc_counts) restated in Python over the oracle's rules, so the multi-rank host logic
(frender_amd/dist.py, frender_amd/scan.py on key partitions) runs under gloo on CPU.  Keys follow
include/frender_amd.h (fast 3-bit keys, wide base-5 keys, exotic codes by bytes); ordinals are
(file index + 1) << 44 | byte offset of the record's header rounded down to a multiple of 4.  Record parts are cut by the library's
own host cutter (fr_gz_part_bounds), so that code is what these tests run."""
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
    device = "cpu"

    def __init__(self):
        self.mem = {}
        self.order = []
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

    def feed_gz_part(self, pool, i, file_index, part, nparts, hint) -> int:
        import gzip
        b = _lib.GzPool.part_bounds(pool.paths[i], nparts, hint)
        with gzip.open(pool.paths[i], "rb") as g:
            data = g.read()
        self.begin_file(None, file_index=file_index, byte_base=b[part])
        self.feed(data[b[part]:b[part + 1]])
        return b[part]

    def feed_gz_part_counted(self, part, file_index, lines_before) -> int:
        data, base = part.data(lines_before)
        self.begin_file(None, file_index=file_index, byte_base=base)
        self.feed(data)
        return base

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
            ordv = tag | ((self.base + s) & ~3)  # the library's ordinals: offsets rounded down to 4 B
            if key is None:
                tab, key = self.exo, code.encode()
                st.exotic += 1
            else:
                tab = self.tab
            e = tab.setdefault(key, [0, 1 << 64, {}])
            e[0] += 1
            e[1] = min(e[1], ordv)
            e[2][self.fi] = e[2].get(self.fi, 0) + 1
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

    def presence_counts(self, n_exotic_pairs):
        c = [self.tab[k][2][f] for k in self.order for f in sorted(self.tab[k][2])]
        e = [self.exo[k][2][f] for k in self.exo for f in sorted(self.exo[k][2])]
        assert len(e) == n_exotic_pairs
        return np.array(c, dtype=np.uint64), np.array(e, dtype=np.uint64)

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
            e = self.tab.setdefault(k, [0, 1 << 64, {}])
            e[0] += c
            e[1] = min(e[1], f)

    # ---- tensors for the key-partitioned merge (frender_amd/dist.py) ---------------------
    @property
    def U(self):
        return len(self.order)

    def export_rows(self, device):
        import torch
        keys, counts, first = self.unique()
        return torch.from_numpy(np.stack([keys.view(np.int64), counts.view(np.int64), first.view(np.int64)], 1)
                                if keys.size else np.zeros((0, 3), np.int64)).to(device)

    def merge_rows(self, rows):
        a = rows.cpu().numpy().view(np.uint64)
        for k, c, f in a.tolist():
            e = self.tab.setdefault(k, [0, 1 << 64, {}])
            e[0] += c
            e[1] = min(e[1], f)

    # ---- classification (R7-R9 over the oracle's rules) ---------------------------------
    def set_sheet(self, idx1, idx2, idx2rc, name_id, n_names):
        self.sheet = (list(idx1), list(idx2), list(idx2rc), list(name_id))
        self.n_names = n_names

    def _one(self, i1, i2, n, rc):
        from oracle.frender_oracle import within
        idx1, idx2, idx2rc, name_id = self.sheet

        def pair(l2):
            m1, m2 = within(i1, idx1, n), within(i2, l2, n)
            if not (m1 and m2):
                return -1, -1, 0, -1
            both = sorted(set(m1) & set(m2))
            cls = 1 if not both else 2 if len(both) == 1 else 3
            return m1[0], m2[0], cls, both[0] if len(both) == 1 else -1

        m1, m2, cls, row = pair(idx2)
        out = {"m1": m1, "m2": m2, "cls": cls, "row": row, "rc_m2": -1, "rc_cls": 0, "rc_row": -1}
        if rc:
            a1, a2, acls, arow = pair(idx2rc)
            out.update(m1=m1 if m1 >= 0 else a1, rc_m2=a2, rc_cls=acls, rc_row=arow)
            if cls == 2 and acls == 2 and name_id[row] != name_id[arow]:
                out.update(cls=3, row=-1, rc_cls=3, rc_row=-1)
        return out

    def _classify(self, pairs, n, rc):
        keys = ("m1", "m2", "row", "rc_m2", "rc_row")
        out = {k: np.full(len(pairs), -1, np.int16) for k in keys}
        out["cls"] = np.zeros(len(pairs), np.uint8)
        out["rc_cls"] = np.zeros(len(pairs), np.uint8)
        err = np.zeros(len(pairs), np.int32)
        for j, (i1, i2) in enumerate(pairs):
            if i2 is None:
                err[j] = 3
                continue
            try:
                r = self._one(i1, i2, n, rc)
            except AssertionError:
                from oracle.frender_oracle import within
                try:
                    within(i1, self.sheet[0], n)
                    err[j] = 2
                except AssertionError:
                    err[j] = 1
                continue
            for k, v in r.items():
                out[k][j] = v
        return out, err

    def classify(self, num_subs, rc, to_host=True):
        codes = _lib.decode_keys(np.array(self.order, dtype=np.uint64))
        pairs = [(c.split("+")[0], c.split("+")[1]) if "+" in c else (c, None) for c in codes]
        out, err = self._classify(pairs, num_subs, rc)
        bad = np.nonzero(err)[0]
        out["err_unique"] = int(bad[0]) if bad.size else -1
        out["err_which"] = int(err[bad[0]]) if bad.size else 0
        f = np.zeros(self.n_names, np.uint64)
        r = np.zeros(self.n_names, np.uint64)
        name_id = self.sheet[3]
        for j, k in enumerate(self.order):
            if err[j]:
                continue
            if out["cls"][j] == 2:
                f[name_id[out["row"][j]]] += self.tab[k][0]
            if rc and out["rc_cls"][j] == 2:
                r[name_id[out["rc_row"][j]]] += self.tab[k][0]
        self._rc = (f, r)
        return out

    def rc_counts(self):
        return self._rc

    def classify_cp(self, q1, q2, num_subs, rc):
        out, err = self._classify(list(zip(q1, q2)), num_subs, rc)
        out["err"] = err
        return out
