"""Native inflate (frender_amd/csrc/fr_gz.cpp, host only) against Python's gzip on the stream shapes
the scan meets: single-member files (libdeflate whole-file path), multi-member files with NUL
padding, BGZF files (member-parallel path), and a file past the whole-file budget's reach (zlib
stream).  Pools run back to back in one process, so decode buffers come from the process-wide
cache and are reused at other sizes: a stale byte from an earlier file would show up here."""
import gzip
import io
import os
import struct
import zlib

import numpy as np
import pytest

from frender_amd import _lib


def fastq(rng, n, R=8):
    out = io.BytesIO()
    for i in range(n):
        seq = bytes(rng.choice(list(b"ACGTN"), R))
        out.write(b"@r%d 1:N:0:%s+%s\n%s\n+\n%s\n" % (i, bytes(rng.choice(list(b"ACGT"), 8)),
                                                   bytes(rng.choice(list(b"ACGT"), 8)), seq, b"F" * R))
    return out.getvalue()


def bgzf(data, block=60000):
    out = io.BytesIO()
    for o in range(0, len(data), block):
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        body = c.compress(data[o:o + block]) + c.flush()
        bsize = 18 + len(body) + 8 - 1
        out.write(b"\x1f\x8b\x08\x04" + b"\0" * 4 + b"\0\xff" + struct.pack("<H", 6) + b"BC" +
                  struct.pack("<HH", 2, bsize) + body + struct.pack("<II", zlib.crc32(data[o:o + block]),
                                                                     len(data[o:o + block])))
    out.write(b"\x1f\x8b\x08\x04\0\0\0\0\0\xff\x06\0BC\x02\0\x1b\0\x03\0\0\0\0\0\0\0\0\0")  # EOF member
    return out.getvalue()


def decoded(paths, threads):
    pool = _lib.GzPool(paths, threads=threads)
    try:
        return [b"".join(pool.blocks(i)) for i in range(len(paths))]
    finally:
        pool.close()


@pytest.mark.parametrize("threads", [1, 3])
def test_native_inflate_equals_python_gzip(tmp_path, threads):
    rng = np.random.default_rng(threads)
    texts, paths = [], []
    for k, n in enumerate([8000, 3, 40000, 0, 20000]):
        t = fastq(rng, n)
        p = str(tmp_path / f"f{k}.fq.gz")
        if k == 1:  # multi-member with NUL padding between and after members
            blob = gzip.compress(t[:10]) + b"\0" * 5 + gzip.compress(t[10:]) + b"\0" * 3
        elif k == 2:
            blob = bgzf(t)
        else:
            blob = gzip.compress(t, compresslevel=1 + k)
        with open(p, "wb") as f:
            f.write(blob)
        texts.append(gzip.decompress(blob) if blob else b"")
        paths.append(p)
    for _ in range(3):  # later rounds reuse cached buffers, in another order of sizes
        assert decoded(paths, threads) == texts
        paths, texts = paths[::-1], texts[::-1]


def test_native_inflate_grows_past_the_trailer_hint(tmp_path):
    """A multi-member file whose last member is tiny: its ISIZE trailer under-promises the decoded
    size, so the whole-file decode outgrows its first buffer (a cached one, reused from the pools
    before) and must grow without losing bytes."""
    rng = np.random.default_rng(7)
    t = fastq(rng, 30000, R=40).replace(b"N", b"A") * 3  # compresses > 4x
    p = str(tmp_path / "grow.fq.gz")
    with open(p, "wb") as f:
        f.write(gzip.compress(t[:-10], compresslevel=9) + gzip.compress(t[-10:]))
    assert len(t) > 4 * os.path.getsize(p)
    for threads in (1, 2):
        assert decoded([p], threads) == [t]


@pytest.mark.parametrize("eol", [b"\n", b"\r", b"\r\n"])
def test_bgzf_parts_of_concatenated_files(tmp_path, eol):
    """BGZF files joined by `cat` leave an empty EOF member mid-file.  A part cut that lands on it (here
    the halfway point of two equal halves) must still decode the byte after it: with '\\r' line ends the
    terminator count looks at that byte (fr_gz_part_open).  Every part split gives back the whole text,
    each part starting at a record start, for LF, CR and CRLF records."""
    rng = np.random.default_rng(len(eol))
    half = fastq(rng, 3000).replace(b"\n", eol)
    other = fastq(rng, 3000).replace(b"\n", eol)
    other = other[:len(half)] if len(other) >= len(half) else other + b"@" * 0
    text = half + other
    p = str(tmp_path / "cat.fq.gz")
    with open(p, "wb") as f:
        f.write(bgzf(half, block=5000) + bgzf(other, block=5000))
    assert gzip.decompress(open(p, "rb").read()) == text
    starts = {0}
    lines = text.replace(b"\r\n", b"\n").replace(b"\r", b"\n").split(b"\n")
    off = 0
    for i, ln in enumerate(lines[:-1]):  # byte offsets of record starts (every 4th line) in `text`
        off += len(ln)
        off += 2 if text[off:off + 2] == b"\r\n" else 1
        if (i + 1) % 4 == 0:
            starts.add(off)
    for nparts in (2, 3, 4, 7):
        parts = [_lib.GzPart.open(p, j, nparts) for j in range(nparts)]
        try:
            assert all(x is not None for x in parts)
            before, got = 0, []
            for x in parts:
                data, base = x.data(before)
                assert base in starts or base == len(text), (nparts, base)
                got.append((base, data))
                before += x.lines
            assert b"".join(d for _, d in got) == text, nparts
            assert [b for b, _ in got] == sorted(b for b, _ in got)
        finally:
            for x in parts:
                x.close()


def test_gz_trim_releases_the_cache(tmp_path):
    """fr_gz_trim hands the cached decode buffers back; the next pool decodes into fresh ones."""
    rng = np.random.default_rng(3)
    t = fastq(rng, 20000)
    p = str(tmp_path / "t.fq.gz")
    with open(p, "wb") as f:
        f.write(gzip.compress(t, compresslevel=1))
    assert decoded([p], 1) == [t]
    _lib.gz_trim()
    assert decoded([p], 2) == [t]
