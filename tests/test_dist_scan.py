"""The multi-GPU scan's host logic (frender_amd/dist.py + the key-partition paths of
frender_amd/scan.py) over gloo on CPU: N ranks, each with a CPU stand-in context
(tests/fake_ctx.py), must write exactly the single-rank outputs (scan CSV, -rc CSV, stdout) on
multi-file inputs with fast, wide and exotic codes, -s, duplicate files and data errors, and on a
SINGLE file, whose records every rank tallies a part of (record-aligned cuts by the library's own
host cutter, fr_gz_part_bounds)."""
import argparse
import contextlib
import gzip
import io
import os
import random
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from frender_amd import synth


def _inputs(d, seed, n_files=5, dup=True):
    rng = random.Random(seed)
    sheet = synth.make_sheet(24, 8, 8)
    sheet.write_csv(os.path.join(d, "sheet.csv"))
    files = []
    for i in range(n_files):
        text = synth.generate_bytes(sheet, i * 3000, rng.randint(500, 3000), R=8, seed=seed).decode()
        extra = "".join(f"@x{j} 1:N:0:{c}\nAC\n+\nFF\n" for j, c in enumerate(
            rng.choice(["acgtacgt+ttttcccc", "AcGtAcGt+TTTTCCCC", "ÄCGTACGT+ACGTACGT", "ACGTACGT+ACGTACGT+GG",
                        "ACGTNCGT+ACGTACGN"])
            for _ in range(rng.randint(0, 40))))
        p = os.path.join(d, f"f{i}_R1.fq.gz")
        synth.write_fastq_gz(p, (text + extra).encode(), level=1)
        files.append(p)
    if dup:
        files.append(files[1])  # the same file twice (two file indices)
    return files


def _run(world, rank, files, sheet, flags, out_dir, port, q):
    from fake_ctx import FakeContext

    from frender_amd import scan
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    os.makedirs(out_dir, exist_ok=True)
    cwd = os.getcwd()
    os.chdir(out_dir)
    buf = io.StringIO()
    err = None
    args = argparse.Namespace(n=flags.get("n", 1), rc=flags.get("rc", False), c=2.0, s=flags.get("s"), o="t",
                              p=None, b=sheet, files=list(files))
    ctx = FakeContext()
    if flags.get("boom_rank") == rank:  # a library failure on this rank (not a data error)
        def boom(*a, **k):
            raise RuntimeError("boom")
        ctx.end_file = boom
    with contextlib.redirect_stdout(buf):
        try:
            scan.frender_scan(args, ctx=ctx)
        except Exception as e:  # noqa: BLE001
            err = (type(e).__name__, str(e))
    os.chdir(cwd)
    outs = {f.split("_t_")[0]: open(os.path.join(out_dir, f), "rb").read() for f in sorted(os.listdir(out_dir))}
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    res = (outs, err, buf.getvalue())
    if q is not None:
        q.put((rank, res))
    return res


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _multi(world, files, sheet, flags, tmp):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(world, r, files, sheet, flags, os.path.join(tmp, f"rank{r}"), port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(1, world):
        outs, err, out = got[r]
        assert outs == {} and out == ""  # only rank 0 prints and writes
        assert err is None or err[0] == "PeerFailed"
    return got[0]


def _norm(out: str) -> str:
    """The affected-files lines come from a set (frender.py:636-638): their order follows string
    hashing, which differs per process (PYTHONHASHSEED), in the reference too.  Sort that block.  The
    output names carry the minute of the run (frender.py's strftime): runs may straddle a minute."""
    import re
    out = re.sub(r"\d{4}-\d{2}-\d{2}_\d{4}_UTC", "<time>", out)
    lines = out.split("\n")
    if "Incorrectly demultiplexed barcodes found! Affected files:" in lines:
        i = lines.index("Incorrectly demultiplexed barcodes found! Affected files:") + 1
        j = next(k for k in range(i, len(lines)) if lines[k].startswith("Analysis complete!"))
        lines[i:j] = sorted(lines[i:j])
    return "\n".join(lines)


def _check(tmp_path, world, files, flags):
    sheet = os.path.join(str(tmp_path), "sheet.csv")
    one = _run(1, 0, files, sheet, flags, os.path.join(str(tmp_path), "one"), None, None)
    many = _multi(world, files, sheet, flags, str(tmp_path))
    assert many[1] == one[1]
    assert _norm(many[2]) == _norm(one[2])  # the same stdout lines, in order
    assert many[0] == one[0]  # byte-identical CSVs
    return one


@pytest.mark.parametrize("world,flags", [(2, {}), (3, {"s": 700}), (2, {"rc": True, "n": 1}), (4, {"n": 2})])
def test_sharded_scan_equals_single(tmp_path, world, flags):
    files = _inputs(str(tmp_path), seed=world)
    one = _check(tmp_path, world, files, flags)
    assert one[1] is None and one[0]


@pytest.mark.parametrize("world", [2, 3])
def test_single_file_record_shards(tmp_path, world):
    """Fewer files than ranks: every rank tallies a record-aligned part of the one file (CRLF lines
    too), and the merged outputs are the single-rank ones."""
    files = _inputs(str(tmp_path), seed=11, n_files=1, dup=False)
    with gzip.open(files[0], "rb") as g:
        text = g.read()
    crlf = os.path.join(str(tmp_path), "crlf_R1.fq.gz")
    with gzip.open(crlf, "wb") as g:
        g.write(text.replace(b"\n", b"\r\n"))
    for fs in ([files[0]], [crlf]):
        one = _check(tmp_path, world, fs, {"rc": True})
        assert one[1] is None


def test_sharded_scan_error_in_file_order(tmp_path):
    files = _inputs(str(tmp_path), seed=7)
    with open(files[3], "wb") as f:  # a header without ' ' in file 3: IndexError there
        f.write(gzip.compress(b"@x 1:N:0:AAAA+CCCC\nA\n+\nF\n@nospace\nA\n+\nF\n"))
    one = _check(tmp_path, 2, files, {})
    assert one[1] == ("IndexError", "list index out of range")


def test_part_bounds_are_record_starts(tmp_path):
    """fr_gz_part_bounds (host only): cuts at record starts at or after j * hint / k, the same for
    any hint source; LF, CRLF and lone-CR files."""
    import re

    from frender_amd import _lib
    rng = random.Random(3)
    recs = [f"@r{i} 1:N:0:ACGT+TTTT\n{'A' * rng.randint(1, 90)}\n+\n" for i in range(4000)]
    recs = [r + "F" * (len(r.split("\n")[1])) + "\n" for r in recs]
    for nl in ("\n", "\r\n", "\r"):
        data = "".join(recs).replace("\n", nl).encode()
        p = os.path.join(str(tmp_path), f"t{len(nl)}{nl == chr(13)}.fq.gz")
        with gzip.open(p, "wb") as g:
            g.write(data)
        hint = _lib.GzPool.size_hint(p)
        assert hint == len(data)  # single member, < 4 GiB: exact
        ends = [m.end() for m in re.finditer(rb"\r\n|\r|\n", data)]
        starts = [0] + ends[3::4]  # line starts with index 0 mod 4
        for k in (1, 2, 3, 7):
            b = _lib.GzPool.part_bounds(p, k, hint)
            assert b[0] == 0 and b[-1] == len(data) and b == sorted(b)
            for j in range(1, k):
                t = hint * j // k
                assert b[j] == min([s for s in starts if s >= t] + [len(data)])


@pytest.mark.parametrize("world", [2, 4])
def test_rc_low_cardinality_empty_partitions(tmp_path, world):
    """-rc over N ranks when the scan has one or two distinct codes: most key partitions are empty, and
    an empty partition is not an empty scan (the rc call needs the global count)."""
    sheet = synth.make_sheet(4, 8, 8)
    sheet.write_csv(os.path.join(str(tmp_path), "sheet.csv"))
    files = []
    for i, codes in enumerate([[f"{sheet.idx1[0]}+{sheet.idx2[0]}"] * 5,
                               [f"{sheet.idx1[0]}+{sheet.idx2[0]}", f"{sheet.idx1[1]}+{sheet.idx2[1]}"] * 3]):
        p = os.path.join(str(tmp_path), f"f{i}_R1.fq.gz")
        synth.write_fastq_gz(p, "".join(f"@r{j} 1:N:0:{c}\nA\n+\nF\n" for j, c in enumerate(codes)).encode())
        files.append(p)
    for fs in ([files[0]], files):
        one = _check(tmp_path, world, fs, {"rc": True, "n": 1})
        assert one[1] is None and one[0]


def test_rank_failure_is_raised_not_hung(tmp_path):
    """A non-data failure on rank 1 (its context raises) is recorded, rank 1 still joins every
    collective and raises its own exception afterwards; rank 0 raises PeerFailed; nothing hangs."""
    files = _inputs(str(tmp_path), seed=5, n_files=3, dup=False)
    sheet = os.path.join(str(tmp_path), "sheet.csv")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(2, r, files, sheet, {"boom_rank": 1}, os.path.join(str(tmp_path), f"r{r}"),
                                            port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert got[1][1] == ("RuntimeError", "boom")
    assert got[0][1][0] == "PeerFailed"


def _bgzf_file(d, name, text: bytes, block=4000):
    p = os.path.join(d, name)
    with open(p, "wb") as f:
        f.write(synth.bgzf_bytes(text, block=block))
    return p


@pytest.mark.parametrize("nl", ["\n", "\r\n", "\r"])
def test_bgzf_part_cuts(tmp_path, nl):
    """fr_gz_part_open / fr_gz_part_data (host only): the parts of a BGZF file, each decoded on its
    own with the line counts of the parts before it, are record-aligned and concatenate to the whole
    decoded file; each part inflates little more than its own bytes (plus the members at its ends)."""
    import re

    from frender_amd import _lib
    rng = random.Random(len(nl))
    recs = [f"@r{i} 1:N:0:ACGT+TTTT\n{'A' * rng.randint(1, 90)}\n+\n" for i in range(6000)]
    recs = [r + "F" * (len(r.split("\n")[1])) + "\n" for r in recs]
    data = "".join(recs).replace("\n", nl).encode()
    p = _bgzf_file(str(tmp_path), "x.fq.gz", data, block=3000)
    ends = [m.end() for m in re.finditer(rb"\r\n|\r|\n", data)]
    starts = set([0] + ends[3::4])
    for k in (1, 2, 3, 7, 40):
        gps = [_lib.GzPart.open(p, j, k, threads=2) for j in range(k)]
        assert all(g is not None for g in gps)
        before, got = 0, b""
        for j, g in enumerate(gps):
            chunk, base = g.data(before)
            assert base == len(got) and (base in starts or base == len(data))
            got += chunk
            assert g.inflated <= len(chunk) + 3 * 3000 + 200, (k, j, g.inflated, len(chunk))
            before += g.lines
            g.close()
        assert got == data
    with open(os.path.join(str(tmp_path), "plain.fq.gz"), "wb") as f:
        f.write(gzip.compress(data))
    assert _lib.GzPart.open(os.path.join(str(tmp_path), "plain.fq.gz"), 0, 2) is None  # not BGZF


@pytest.mark.parametrize("world", [2, 3])
def test_single_bgzf_file_record_shards(tmp_path, world):
    """Fewer files than ranks, BGZF inputs: every rank decodes only its own part (fr_gz_part_open) and
    the merged outputs are the single-rank ones (LF and CRLF)."""
    files = _inputs(str(tmp_path), seed=13, n_files=1, dup=False)
    with gzip.open(files[0], "rb") as g:
        text = g.read()
    for name, t in (("bg_R1.fq.gz", text), ("bgcr_R1.fq.gz", text.replace(b"\n", b"\r\n"))):
        p = _bgzf_file(str(tmp_path), name, t)
        one = _check(tmp_path, world, [p], {"rc": True})
        assert one[1] is None


def _inflated_rank(world, rank, path, port, q):
    from fake_ctx import FakeContext

    from frender_amd import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with contextlib.redirect_stdout(io.StringIO()):
        t = D.sharded_tally(dist, FakeContext(), [path], None, 2)
    q.put((rank, t.inflated))
    dist.barrier()
    dist.destroy_process_group()


def test_bgzf_parts_inflate_only_their_part(tmp_path):
    """Each rank's inflated bytes <= 1.1 x its part plus the members at its ends (no prefix inflate)."""
    files = _inputs(str(tmp_path), seed=17, n_files=1, dup=False)
    with gzip.open(files[0], "rb") as g:
        text = g.read() * 4
    p = _bgzf_file(str(tmp_path), "big_R1.fq.gz", text, block=8000)
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_inflated_rank, args=(world, r, p, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for pr in procs:
        pr.join(60)
        assert pr.exitcode == 0
    total = 0
    for r in range(world):
        (inflated, part_len), = got[r].values()
        assert inflated <= 1.1 * part_len + 3 * 8000, (r, inflated, part_len)
        total += part_len
    assert total == len(text)
