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
