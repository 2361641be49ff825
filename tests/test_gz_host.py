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


@pytest.fixture(scope="module")
def big_text():
    """~90 MB of SYN-v1 FASTQ (1.2M records at R=8 plus R=40 ones): single members of > 16 MiB compressed."""
    from frender_amd import synth

    sheet = synth.make_sheet(96, 8, 8)
    return synth.generate_bytes(sheet, 0, 1_000_000, R=8, seed=31) + synth.generate_bytes(sheet, 0, 250_000, R=40,
                                                                                           seed=32)


def _gzip_member(text, level, name=None):
    co = zlib.compressobj(level, zlib.DEFLATED, -15)
    body = co.compress(text) + co.flush()
    flg = 8 if name else 0
    head = b"\x1f\x8b\x08" + bytes([flg]) + b"\0\0\0\0\0\xff" + ((name + b"\0") if name else b"")
    return head + body + struct.pack("<II", zlib.crc32(text), len(text) & 0xFFFFFFFF)


@pytest.mark.parametrize("level,name,pad", [(1, None, 0), (6, b"lane1.fastq", 7)])
def test_parallel_single_member(tmp_path, big_text, level, name, pad):
    """One big member (>= 16 MiB compressed: the parallel decoder, fr_pinflate.h) equals Python's gzip for
    levels 1 and 6, with an FNAME header field and NUL padding after the member; the pool's threads decode
    it together (fr_gz_parallel_members counts it)."""
    blob = _gzip_member(big_text, level, name) + b"\0" * pad
    assert len(blob) >= 16 << 20
    p = str(tmp_path / "big.fq.gz")
    with open(p, "wb") as f:
        f.write(blob)
    before = _lib.gz_parallel_members()
    assert decoded([p], 6) == [gzip.decompress(blob)]
    assert _lib.gz_parallel_members() == before + 1


@pytest.mark.parametrize("damage", ["flip", "crc", "isize", "truncate", "trailing", "second_member"])
def test_parallel_single_member_errors(tmp_path, big_text, damage):
    """A damaged big member never yields bytes Python's gzip would not: the parallel decoder refuses it and
    the one-thread decoders take the file (the same error, or the same bytes for a valid multi-member file)."""
    blob = bytearray(_gzip_member(big_text, 1))
    if damage == "flip":
        blob[len(blob) // 2] ^= 0x5A
    elif damage == "crc":
        blob[-8] ^= 1
    elif damage == "isize":
        blob[-1] ^= 1
    elif damage == "truncate":
        blob = blob[: len(blob) - 1000]
    elif damage == "trailing":
        blob += b"garbage!"
    else:
        blob += gzip.compress(b"@x 1:N:0:ACGT+TTTT\nA\n+\nF\n")
    p = str(tmp_path / "bad.fq.gz")
    with open(p, "wb") as f:
        f.write(bytes(blob))
    try:
        exp = gzip.decompress(bytes(blob))
    except Exception:  # noqa: BLE001 - Python's gzip rejects it
        exp = None
    before = _lib.gz_parallel_members()
    if exp is None:
        with pytest.raises(_lib.GzError):
            decoded([p], 6)
    else:
        assert decoded([p], 6) == [exp]
    assert _lib.gz_parallel_members() == before  # never the parallel decoder's output


def test_inflate_ahead(tmp_path):
    """Files inflating at once: all of them while their decoded sizes (gzip ISIZE) fit the 2-GiB block
    budget, fewer for big ones, never more than the files, one file gets every thread."""
    import gzip
    import struct

    from frender_amd import _lib

    def fake(name, isize, comp=64):  # a file whose trailer claims `isize` decoded bytes
        p = tmp_path / name
        p.write_bytes(b"\x1f\x8b" + b"\0" * (comp - 6) + struct.pack("<I", isize))
        return str(p)

    small = [fake(f"s{i}.gz", 200 << 20) for i in range(8)]
    assert _lib.inflate_ahead(small, 8) == 8
    big = [fake(f"b{i}.gz", 443 << 20) for i in range(32)]
    assert _lib.inflate_ahead(big, 16) == 4
    assert _lib.inflate_ahead(big, 8) == 4
    assert _lib.inflate_ahead([fake("huge.gz", 1800 << 20)], 16) == 1
    assert _lib.inflate_ahead(big[:2], 16) == 2
    assert _lib.inflate_ahead(big, 1) == 1
    real = tmp_path / "real.gz"
    real.write_bytes(gzip.compress(b"@r 1:N:0:AC+GT\nA\n+\nF\n" * 1000))
    assert _lib.inflate_ahead([str(real)] * 3, 4) == 3
