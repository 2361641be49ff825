"""The GPU deflate encoder's algorithm in its host build (tests/native/frd_host.cpp over
frender_amd/csrc/fr_deflate_core.h: the kernel's matchfinder batches, lane parses, passes and block
layout as loops).  Every stream must inflate (zlib) to its input with the input's CRC-32, and on the
demux writers' FASTQ shapes be no larger than zlib level 9 -- the reference's writer, gzip.open's
default (frender.py:667-676).  The GPU kernel itself is checked in tests/test_gpu_deflate.py."""
import ctypes
import os
import subprocess
import zlib

import pytest

from deflate_cases import edge_cases, routed_fastq

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "frd_host.cpp")


def build_host(tmp_dir) -> ctypes.CDLL:
    so = os.path.join(str(tmp_dir), "frd_host.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-o", so, SRC], check=True)
    lib = ctypes.CDLL(so)
    lib.frd_host_deflate.restype = ctypes.c_uint64
    lib.frd_host_deflate.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    return lib


def host_deflate(lib, data: bytes) -> tuple:
    """(raw deflate stream, crc32) with the kernel's settings: 3 passes, pass-1 length/distance 2 bits."""
    out = ctypes.create_string_buffer(len(data) + len(data) // 64 + 1024)
    crc = ctypes.c_uint32()
    k = lib.frd_host_deflate(data, len(data), out, len(out), 3, 2, 2, ctypes.byref(crc))
    assert k, "host build: output bound or bit accounting failed"
    return out.raw[:k], crc.value


@pytest.fixture(scope="module")
def frd(tmp_path_factory):
    return build_host(tmp_path_factory.mktemp("frd"))


@pytest.mark.parametrize("name", sorted(edge_cases()))
def test_roundtrip(frd, name):
    data = edge_cases()[name]
    body, crc = host_deflate(frd, data)
    assert zlib.decompressobj(-15).decompress(body) == data
    assert crc == zlib.crc32(data)
    if name.startswith("random"):
        assert len(body) <= len(data) + 5 * (len(data) // 65535 + 2) + 16  # stored, not expanded


@pytest.mark.parametrize("R,n", [(150, 12000), (100, 16000), (8, 60000)])
def test_fastq_no_larger_than_zlib9(frd, R, n):
    data = routed_fastq(n, R)
    body, _ = host_deflate(frd, data)
    assert zlib.decompressobj(-15).decompress(body) == data
    z9 = len(zlib.compress(data, 9)) - 6  # zlib header + adler trailer
    assert len(body) <= z9, (len(body), z9)
