"""The demux writers' compression on the GPU (fr_deflate.hip through fr_defl_* / fr_dmx_deflate).

Every stream must inflate (zlib) to its bytes with their CRC-32; on the demux's FASTQ shapes it must
be no larger than zlib level 9 makes it (the reference's writers are gzip.open(..., "wb"),
frender.py:667-676); and it must be the stream the host build of the same algorithm makes
(tests/native/frd_host.cpp), byte for byte.  The demux end-to-end tests (tests/test_gpu_scan.py) read
the GPU-written members through Python's gzip."""
import gzip
import zlib

import numpy as np
import pytest

from deflate_cases import DEFLATE_BLOCK, edge_cases, routed_fastq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dfl():
    from frender_amd import _lib
    z = _lib.Deflater(0)
    yield z
    z.close()


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    from test_deflate_host import build_host
    return build_host(tmp_path_factory.mktemp("frd"))


def _streams(comp, out):
    offs = np.concatenate([[0], np.cumsum(comp)]).astype(np.int64)
    return [out[offs[s]:offs[s + 1]].tobytes() for s in range(len(comp))]


@pytest.mark.parametrize("name", sorted(edge_cases()))
def test_roundtrip_and_host_equal(dfl, host, name):
    from test_deflate_host import host_deflate
    data = edge_cases()[name]
    comp, crc, out = dfl.compress(data)
    if not data:
        assert comp[0] == 0 and crc[0] == 0 and out.size == 0
        return
    body = out.tobytes()
    assert zlib.decompressobj(-15).decompress(body) == data
    assert int(crc[0]) == zlib.crc32(data)
    hb, hcrc = host_deflate(host, data)
    assert body == hb, f"GPU stream differs from the host build ({len(body)} vs {len(hb)} bytes)"


def test_many_streams(dfl):
    """Destination-major ranges of every size class, empty ones among them: each is its own stream."""
    rng = np.random.default_rng(3)
    sizes = [0, 1, 5, 0, 100, DEFLATE_BLOCK - 1, DEFLATE_BLOCK, DEFLATE_BLOCK + 7, 3 * DEFLATE_BLOCK + 11, 0, 2]
    sizes += rng.integers(0, 9000, 300).tolist()
    fq = routed_fastq(4000, 150)
    data = (fq * (sum(sizes) // len(fq) + 1))[: sum(sizes)]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    comp, crc, out = dfl.compress(data, offs)
    streams = _streams(comp, out)
    for s, n in enumerate(sizes):
        a, b = int(offs[s]), int(offs[s + 1])
        if n == 0:
            assert comp[s] == 0 and crc[s] == 0
            continue
        assert zlib.decompressobj(-15).decompress(streams[s]) == data[a:b], s
        assert int(crc[s]) == zlib.crc32(data[a:b]), s


@pytest.mark.parametrize("R,n", [(150, 30000), (100, 40000), (8, 200000)])
def test_fastq_no_larger_than_zlib9(dfl, R, n):
    data = routed_fastq(n, R)
    comp, crc, out = dfl.compress(data)
    assert zlib.decompressobj(-15).decompress(out.tobytes()) == data
    z9 = len(zlib.compress(data, 9)) - 6
    assert int(comp[0]) <= z9, (int(comp[0]), z9)


def test_gzip_member_frame(dfl):
    from frender_amd import _lib
    data = routed_fastq(3000, 150)
    comp, crc, out = dfl.compress(data)
    head, tail = _lib.gzip_frame(int(crc[0]), len(data))
    member = head + out.tobytes() + tail
    assert gzip.decompress(member + member) == data + data  # members concatenate (one file per window each)


def test_demux_writers_gpu_vs_host(tmp_path):
    """The demux with --gz-writer gpu and libdeflate: the same text in every file, the GPU's files no
    larger in total than the same text at zlib level 9."""
    import argparse
    import os

    from frender_amd import synth
    from frender_amd.demux import frender_demux

    sheet = synth.make_sheet(12, 8, 8)
    inp = tmp_path / "in"
    inp.mkdir()
    t1 = synth.generate_bytes(sheet, 0, 40_000, R=150, seed=9).decode()
    lines = t1.split("\n")
    t2 = "\n".join(ln.replace(" 1:N:", " 2:N:", 1) if i % 4 == 0 else (ln[::-1] if i % 4 in (1, 3) else ln)
                   for i, ln in enumerate(lines))
    for mate, text in (("R1", t1), ("R2", t2)):
        synth.write_fastq_gz(str(inp / f"syn_L001_{mate}_001.fastq.gz"), text.encode(), level=1)
    with open(tmp_path / "results.csv", "w") as f:
        f.write("idx1,idx2,reads,matched_idx1,matched_idx2,read_type,sample_name,demux_ok\n")
        codes = sorted({ln.rsplit(":", 1)[-1] for ln in lines[0::4] if ln})
        for i, c in enumerate(codes):  # every code the inputs hold; a few undetermined
            a, b = c.split("+")
            kind, sid = ("demuxable", sheet.ids[i % len(sheet.ids)]) if i % 7 else ("undetermined", "")
            f.write(f"{a},{b},1,{a},{b},{kind},{sid},True\n")
    files = sorted(str(p) for p in inp.iterdir())

    def run(writer):
        d = tmp_path / writer
        frender_demux(argparse.Namespace(r=str(tmp_path / "results.csv"), d=str(d), o=None, no_index_hop=False,
                                         no_ambiguous=False, no_undeter=False, no_samples=False, files=files,
                                         gz_writer=writer, gz_level=9, window=8 << 20))
        return d

    g, h = run("gpu"), run("libdeflate")
    assert sorted(os.listdir(g)) == sorted(os.listdir(h))
    gpu_total = z9_total = 0
    for fn in os.listdir(g):
        with gzip.open(g / fn, "rb") as a, gzip.open(h / fn, "rb") as b:
            text = a.read()
            assert text == b.read(), fn
        gpu_total += os.path.getsize(g / fn)
        z9_total += len(gzip.compress(text, 9))
    assert gpu_total <= z9_total, (gpu_total, z9_total)
