"""The multi-GPU product path's host logic (frender_amd/dist.py: sharded_tally, merge_tables)
over gloo on CPU: N ranks, each with a CPU stand-in context (tests/fake_ctx.py), must give rank 0
exactly the single-rank table (codes, counts, firsts, presence, per-file records) and the same
per-file stdout lines, on multi-file inputs with fast, wide and exotic codes, -s, duplicate
files and a data error."""
import contextlib
import io
import os
import random
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from frender_amd import synth


def _inputs(d, seed):
    rng = random.Random(seed)
    sheet = synth.make_sheet(24, 8, 8)
    files = []
    for i in range(5):
        text = synth.generate_bytes(sheet, i * 3000, rng.randint(500, 3000), R=8, seed=seed).decode()
        extra = "".join(f"@x{j} 1:N:0:{c}\nAC\n+\nFF\n" for j, c in enumerate(
            rng.choice(["AAAACCCCGGGG+TTTTAAAACCCC", "acgtacgt+ttttcccc", "AcGt+TTTT", "ÄCGT+ACGT", "A+C+G"])
            for _ in range(rng.randint(0, 40))))
        p = os.path.join(d, f"f{i}_R1.fq.gz")
        synth.write_fastq_gz(p, (text + extra).encode(), level=1)
        files.append(p)
    files.append(files[1])  # the same file twice (two file indices)
    return files


def _run(world, rank, files, sample, port, q):
    from fake_ctx import FakeContext

    from frender_amd import scan
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = io.StringIO()
    err = None
    t = None
    with contextlib.redirect_stdout(buf):
        try:
            t = scan.tally_barcodes(2, files, sample, ctx=FakeContext())
        except Exception as e:  # noqa: BLE001
            err = (type(e).__name__, str(e))
    out = None
    if t is not None:
        pres = sorted(zip(t.pres_u.tolist(), t.pres_f.tolist()))
        out = (t.codes, t.counts.tolist(), t.first.tolist(), pres, t.records, t.files)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if q is not None:
        q.put((rank, out, err, buf.getvalue()))
    return out, err, buf.getvalue()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _multi(world, files, sample):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(world, r, files, sample, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (o, e, s)) for r, o, e, s in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(1, world):
        assert got[r][0] is None and got[r][2] == ""  # only rank 0 returns a table / prints
    return got[0]


@pytest.mark.parametrize("world,sample", [(2, None), (3, 700)])
def test_sharded_tally_equals_single(tmp_path, world, sample):
    files = _inputs(str(tmp_path), seed=world)
    one = _run(1, 0, files, sample, None, None)
    assert one[1] is None and one[0] is not None
    many = _multi(world, files, sample)
    assert many[1] is None
    assert many[0] == one[0]
    assert many[2] == one[2]  # the same stdout lines, in file order


def test_sharded_tally_error_in_file_order(tmp_path):
    files = _inputs(str(tmp_path), seed=7)
    with open(files[3], "wb") as f:  # a header without ' ' in file 3: IndexError there
        import gzip
        f.write(gzip.compress(b"@x 1:N:0:AAAA+CCCC\nA\n+\nF\n@nospace\nA\n+\nF\n"))
    one = _run(1, 0, files, None, None, None)
    many = _multi(2, files, None)
    assert one[1] == ("IndexError", "list index out of range")
    assert many[1] == one[1] and many[2] == one[2]
