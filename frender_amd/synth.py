"""SYN-v1: the seeded synthetic Illumina-style FASTQ generator.

Every record is a pure function of (seed, global record index r), built from a
counter-based hash, so the host generator here and the device generator kernel
(`fr_synth_records` in csrc/fr_synth.hip) produce byte-identical streams, and a
file split is just a range of r.  Records have a fixed length:

    @SYN:1:FCX:1:{tile:04d}:{x:05d}:{y:05d} 1:N:0:{i1}+{i2}\\n   (36+L1+1+L2+1 B)
    {seq: R bases}\\n+\\n{qual: R chars '!'..'J'}\\n               (2R+4 B)

8+8 indexes, R=8 -> 74 B/record (the headline size); R=150 -> 358 B.

Per read (hash fields k):  k=0 sample; k=1,2 index hop (2 %, idx2 of a random
sample); k=3,4 fully random idx1+idx2 (1 %); k=8+j per index base j: 0.5 %
substitution, 0.2 % 'N'; k=80.. sequence bases; k=100.. quality bytes.

The sample sheets are generated with numpy's seeded PCG64 (seed 42 by default);
indexes are drawn with a pairwise Hamming distance >= 3 within each index list,
as real index kits are.
"""
from __future__ import annotations

import csv
import gzip
import io
import os
from dataclasses import dataclass

import numpy as np

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
RC_TABLE = bytes.maketrans(b"ATGCNatgcn", b"TACGNtacgn")

# per-10000 rates of SYN-v1
HOP_PER_10K = 200
JUNK_PER_10K = 100
SUB_PER_10K = 50
N_PER_10K = 20


def mix64_int(x: int) -> int:
    """splitmix64 finalizer on a python int (mod 2^64)."""
    x &= M64
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & M64
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & M64
    x ^= x >> 31
    return x


def _mix64(x: np.ndarray) -> np.ndarray:
    x = x.copy()
    x ^= x >> np.uint64(30)
    x *= np.uint64(0xBF58476D1CE4E5B9)
    x ^= x >> np.uint64(27)
    x *= np.uint64(0x94D049BB133111EB)
    x ^= x >> np.uint64(31)
    return x


def seed_base(seed: int) -> int:
    return mix64_int(seed + GOLDEN)


def _h(base: int, r: np.ndarray, k: int) -> np.ndarray:
    return _mix64(((r << np.uint64(8)) | np.uint64(k)) ^ np.uint64(base))


@dataclass
class Sheet:
    ids: list
    idx1: list
    idx2: list

    @property
    def S(self) -> int:
        return len(self.ids)

    def write_csv(self, path: str, illumina: bool = False) -> None:
        with open(path, "w", newline="") as f:
            if illumina:
                f.write("[Header]\nIEMFileVersion,4\nInvestigator Name,syn\n[Reads]\n151\n[Data]\n")
            w = csv.writer(f, lineterminator="\n")
            w.writerow(["Sample_ID", "Sample_Name", "index", "index2"])
            for i, a, b in zip(self.ids, self.idx1, self.idx2):
                w.writerow([i, i, a, b])


def _draw_indexes(rng: np.random.Generator, count: int, length: int, min_dist: int = 3) -> list:
    out: list = []
    arr = np.zeros((0, length), dtype=np.uint8)
    while len(out) < count:
        cand = rng.integers(0, 4, size=length, dtype=np.uint8)
        if arr.shape[0] and int(((arr != cand).sum(axis=1)).min()) < min_dist:
            continue
        arr = np.vstack([arr, cand[None, :]])
        out.append(BASES[cand].tobytes().decode())
    return out


def make_sheet(S: int = 96, L1: int = 8, L2: int = 8, seed: int = 42,
               combinatorial: tuple | None = None, prefix: str = "Sample_") -> Sheet:
    """Unique-dual (default) or combinatorial (n1 x n2 grid) sample sheet."""
    rng = np.random.default_rng(seed)
    if combinatorial:
        n1, n2 = combinatorial
        i1 = _draw_indexes(rng, n1, L1)
        i2 = _draw_indexes(rng, n2, L2)
        pairs = [(a, b) for a in i1 for b in i2][:S]
        idx1 = [p[0] for p in pairs]
        idx2 = [p[1] for p in pairs]
    else:
        idx1 = _draw_indexes(rng, S, L1)
        idx2 = _draw_indexes(rng, S, L2)
    ids = [f"{prefix}{i + 1:03d}" for i in range(len(idx1))]
    return Sheet(ids, idx1, idx2)


# The config-3 shape's (384 samples, 10+10, -rc) samples whose reads carry rc(idx2): the reference's
# per-name call flips exactly these (frender.py:375-379), so its idx2 rewrite (:618-623) and pass B
# (:628-630) run on a mixed list at the benchmarked geometry (tests/golden/cfg3_pin.json).
CFG3_RC_NAMES = ("Sample_004", "Sample_050", "Sample_099", "Sample_150",
                 "Sample_201", "Sample_256", "Sample_300", "Sample_377")


def read_idx2(sheet: Sheet, rc_names=None) -> list:
    """idx2 as the generated reads carry it: rc(idx2) for the samples in rc_names (the list the device
    generator fr_synth_device takes to produce the same records as generate_records(..., rc_names))."""
    return [(x.encode().translate(RC_TABLE)[::-1].decode() if rc_names and sheet.ids[i] in rc_names else x)
            for i, x in enumerate(sheet.idx2)]


def record_length(L1: int, L2: int, R: int) -> int:
    return 36 + L1 + 1 + L2 + 1 + 2 * R + 4


def _digits(v: np.ndarray, width: int) -> np.ndarray:
    out = np.empty((v.shape[0], width), dtype=np.uint8)
    v = v.copy()
    for i in range(width - 1, -1, -1):
        out[:, i] = (v % np.uint64(10)).astype(np.uint8) + ord("0")
        v //= np.uint64(10)
    return out


def generate_records(sheet: Sheet, r0: int, n: int, R: int = 8, seed: int = 1,
                     rc_names: set | None = None) -> np.ndarray:
    """Records r0 .. r0+n-1 as an (n, reclen) uint8 array.

    rc_names: samples whose reads carry the reverse complement of the sheet's
    idx2 (to exercise -rc; the sheet itself is unchanged)."""
    L1 = len(sheet.idx1[0])
    L2 = len(sheet.idx2[0])
    assert all(len(x) == L1 for x in sheet.idx1) and all(len(x) == L2 for x in sheet.idx2)
    assert L1 + L2 <= 32 and R <= 256
    S = sheet.S
    base = seed_base(seed)
    r = np.arange(r0, r0 + n, dtype=np.uint64)
    reclen = record_length(L1, L2, R)
    out = np.empty((n, reclen), dtype=np.uint8)

    lut1 = np.frombuffer("".join(sheet.idx1).encode(), dtype=np.uint8).reshape(S, L1)
    idx2_eff = read_idx2(sheet, rc_names)
    lut2 = np.frombuffer("".join(idx2_eff).encode(), dtype=np.uint8).reshape(S, L2)
    code_of = np.zeros(256, dtype=np.uint8)
    for c, v in zip(b"ACGT", range(4)):
        code_of[c] = v

    s = (_h(base, r, 0) % np.uint64(S)).astype(np.int64)
    idx = np.concatenate([lut1[s], lut2[s]], axis=1)  # (n, L1+L2) ascii
    hop = (_h(base, r, 1) % np.uint64(10000)) < np.uint64(HOP_PER_10K)
    s2 = (_h(base, r, 2) % np.uint64(S)).astype(np.int64)
    idx[hop, L1:] = lut2[s2[hop]]
    junk = (_h(base, r, 3) % np.uint64(10000)) < np.uint64(JUNK_PER_10K)
    if junk.any():
        hj = _h(base, r[junk], 4)
        jb = np.stack([((hj >> np.uint64(2 * j)) & np.uint64(3)).astype(np.uint8) for j in range(L1 + L2)], axis=1)
        idx[junk] = BASES[jb]
    for j in range(L1 + L2):
        v = _h(base, r, 8 + j)
        p = v % np.uint64(10000)
        sub = p < np.uint64(SUB_PER_10K)
        nn = (p >= np.uint64(SUB_PER_10K)) & (p < np.uint64(SUB_PER_10K + N_PER_10K))
        if sub.any():
            orig = code_of[idx[sub, j]]
            new = (orig.astype(np.uint64) + np.uint64(1) + (v[sub] >> np.uint64(32)) % np.uint64(3)) % np.uint64(4)
            idx[sub, j] = BASES[new.astype(np.int64)]
        idx[nn, j] = ord("N")

    pos = 0

    def put(b: bytes):
        nonlocal pos
        out[:, pos:pos + len(b)] = np.frombuffer(b, dtype=np.uint8)
        pos += len(b)

    put(b"@SYN:1:FCX:1:")
    out[:, pos:pos + 4] = _digits((r // np.uint64(10**10)) % np.uint64(10**4), 4); pos += 4
    put(b":")
    out[:, pos:pos + 5] = _digits((r // np.uint64(10**5)) % np.uint64(10**5), 5); pos += 5
    put(b":")
    out[:, pos:pos + 5] = _digits(r % np.uint64(10**5), 5); pos += 5
    put(b" 1:N:0:")
    out[:, pos:pos + L1] = idx[:, :L1]; pos += L1
    put(b"+")
    out[:, pos:pos + L2] = idx[:, L1:]; pos += L2
    put(b"\n")
    for w in range((R + 31) // 32):
        hv = _h(base, r, 80 + w)
        for j in range(32 * w, min(R, 32 * w + 32)):
            out[:, pos + j] = BASES[((hv >> np.uint64(2 * (j - 32 * w))) & np.uint64(3)).astype(np.int64)]
    pos += R
    put(b"\n+\n")
    for w in range((R + 7) // 8):
        hv = _h(base, r, 100 + w)
        for j in range(8 * w, min(R, 8 * w + 8)):
            out[:, pos + j] = (((hv >> np.uint64(8 * (j - 8 * w))) & np.uint64(0xFF)) % np.uint64(42)).astype(np.uint8) + 33
    pos += R
    put(b"\n")
    assert pos == reclen
    return out


def generate_bytes(sheet: Sheet, r0: int, n: int, R: int = 8, seed: int = 1, rc_names=None,
                   block: int = 1 << 20) -> bytes:
    parts = []
    for a in range(r0, r0 + n, block):
        b = min(block, r0 + n - a)
        parts.append(generate_records(sheet, a, b, R=R, seed=seed, rc_names=rc_names).tobytes())
    return b"".join(parts)


def write_fastq_gz(path: str, data: bytes, level: int = 1, members: int = 1) -> None:
    """Write decoded FASTQ bytes as gzip; members>1 writes a multi-member file
    (split at arbitrary byte points, which Python's gzip reader concatenates)."""
    with open(path, "wb") as f:
        if members <= 1:
            f.write(gzip.compress(data, compresslevel=level))
        else:
            cuts = np.linspace(0, len(data), members + 1).astype(np.int64)
            for a, b in zip(cuts[:-1], cuts[1:]):
                f.write(gzip.compress(data[a:b], compresslevel=level))


def bgzf_bytes(data: bytes, block: int = 65280, level: int = 1) -> bytes:
    """BGZF (the blocked gzip of htslib / bgzip): independent gzip members of <= 64 KiB of input, each
    carrying its compressed size in a 'BC' extra subfield, then the empty EOF member.  Python's gzip
    (and so the reference, frender.py:159) reads it as an ordinary multi-member gzip file."""
    import struct
    import zlib

    out = []
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        co = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = co.compress(chunk) + co.flush()
        bsize = 12 + 6 + len(body) + 8
        out.append(b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<HBBHH", 6, 66, 67, 2, bsize - 1)
                   + body + struct.pack("<II", zlib.crc32(chunk), len(chunk) & 0xFFFFFFFF))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))  # EOF member
    return b"".join(out)


def make_dataset(outdir: str, sheet: Sheet, n_reads: int, n_files: int = 1, R: int = 8, seed: int = 1,
                 rc_names=None, name_fmt: str = "syn_L{f:03d}_R1_001.fastq.gz", level: int = 1) -> list:
    """Split records [0, n_reads) into n_files gz files; return their paths."""
    os.makedirs(outdir, exist_ok=True)
    cuts = np.linspace(0, n_reads, n_files + 1).astype(np.int64)
    paths = []
    for f, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        p = os.path.join(outdir, name_fmt.format(f=f + 1))
        write_fastq_gz(p, generate_bytes(sheet, int(a), int(b - a), R=R, seed=seed, rc_names=rc_names), level=level)
        paths.append(p)
    return paths


CLASS_NAMES = ("undetermined", "index_hop", "demuxable", "ambiguous")


def rows_digest(codes, counts, out, idx1, idx2, ids, keep: int = 1000, idx2rc=None):
    """sha256 over a classified unique table in its order, one line per code
    f"{code}\\t{reads}\\t{matched_idx1}\\t{matched_idx2}\\t{read_type}\\t{sample_name}\\n" (the row format
    of tests/golden/cfg{2,3,4}_pin.json, which tests/golden/make_golden_cfg2.py / make_golden_cfg34.py
    computed from the reference's own tally_barcodes + process), plus the first and last `keep` lines.
    `out` holds fr_classify's m1 / m2 / cls / row arrays.  idx2rc given (an -rc pass A): each line also
    carries \\t{matched_rc_idx2}\\t{rc_read_type}\\t{rc_sample_name} before its \\n (the rc_* arrays), as
    the reference's analyze_barcodes_with_rc dicts do (frender.py:325-349)."""
    import hashlib

    m1, m2, cls, row = (np.asarray(out[k]).tolist() for k in ("m1", "m2", "cls", "row"))
    if idx2rc is not None:
        rm2, rcls, rrow = (np.asarray(out[k]).tolist() for k in ("rc_m2", "rc_cls", "rc_row"))
    h = hashlib.sha256()
    lines = []
    n = len(codes)
    for j, (c, k) in enumerate(zip(codes, np.asarray(counts).tolist())):
        line = (f"{c}\t{k}\t{idx1[m1[j]] if m1[j] >= 0 else ''}\t{idx2[m2[j]] if m2[j] >= 0 else ''}\t"
                f"{CLASS_NAMES[cls[j]]}\t{ids[row[j]] if row[j] >= 0 else ''}")
        if idx2rc is not None:
            line += (f"\t{idx2rc[rm2[j]] if rm2[j] >= 0 else ''}\t{CLASS_NAMES[rcls[j]]}\t"
                     f"{ids[rrow[j]] if rrow[j] >= 0 else ''}")
        line += "\n"
        h.update(line.encode())
        if j < keep or j >= n - keep:
            lines.append(line)
    return h.hexdigest(), lines[:keep], lines[-keep:] if n >= keep else lines


def pin_rows(ctx, sheet: Sheet, nsubs: int, rc: bool, keep: int = 1000) -> dict:
    """The reference's frender_scan sequence (frender.py:606-630) on ctx's finalized table, in the form
    of tests/golden/cfg{2,3,4}_pin.json (make_golden_cfg2.py / make_golden_cfg34.py): process (:610); with
    -rc its pass-A rows (with the rc columns), call_rc_mode_per_id's calls (:614, :367-388: use rc iff
    f < rc), the idx2 rewrite (:618-623) and pass B (:628-630).  Returns unique_codes, rows_sha256,
    first_rows, last_rows (the final pass) and, with -rc, pass_a and rc_calls [[name, f, rc, call]]."""
    from ._lib import decode_keys
    from .host import reverse_complement
    from .scan import _sheet_names

    names, nid = _sheet_names(sheet.ids)
    idx2rc = [reverse_complement(x) for x in sheet.idx2]
    keys, counts, _ = ctx.unique()
    codes = decode_keys(keys)
    ctx.set_sheet(sheet.idx1, sheet.idx2, idx2rc, nid, len(names))
    out = ctx.classify(nsubs, rc)
    res: dict = {"unique_codes": len(codes)}
    idx2_final = list(sheet.idx2)
    if rc:
        d, f, l = rows_digest(codes, counts, out, sheet.idx1, sheet.idx2, sheet.ids, keep, idx2rc=idx2rc)
        res["pass_a"] = {"rows_sha256": d, "first_rows": f, "last_rows": l}
        fr, rr = ctx.rc_counts()
        use = [int(a) < int(b) for a, b in zip(fr, rr)]
        res["rc_calls"] = [[n, int(a), int(b), u] for n, a, b, u in zip(names, fr, rr, use)]
        idx2_final = [reverse_complement(x) if use[nid[i]] else x for i, x in enumerate(sheet.idx2)]
        ctx.set_sheet(sheet.idx1, idx2_final, [reverse_complement(x) for x in idx2_final], nid, len(names))
        out = ctx.classify(nsubs, False)
    d, f, l = rows_digest(codes, counts, out, sheet.idx1, idx2_final, sheet.ids, keep)
    res.update({"rows_sha256": d, "first_rows": f, "last_rows": l})
    return res


def pin_differences(got: dict, pin: dict) -> list:
    """The fields of a pin_rows result that differ from a committed pin (empty list = equal)."""
    bad = [k for k in ("unique_codes", "rows_sha256", "first_rows", "last_rows") if got.get(k) != pin.get(k)]
    if "pass_a" in pin:
        bad += [f"pass_a.{k}" for k in ("rows_sha256", "first_rows", "last_rows")
                if (got.get("pass_a") or {}).get(k) != pin["pass_a"].get(k)]
        if got.get("rc_calls") != pin.get("rc_calls"):
            bad.append("rc_calls")
    return bad
