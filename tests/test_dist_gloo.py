"""The multi-GPU merge protocol (frender_amd/dist.py) over gloo on CPU, world sizes 2-5.

Each rank holds a random table {key: (count, first)}; the tree merge must leave
rank 0 with the exact union (count = sum, first = min), as the reference's
parent-process dict merge does (frender.py:199-205).  The device merge kernel is
covered by tests/test_gpu_scan.py::test_merge_unique_device.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from frender_amd.dist import tree_merge


def _table(rank, seed):
    rng = np.random.default_rng(seed * 100 + rank)
    n = int(rng.integers(0, 50)) if rank % 3 != 2 else 0  # some ranks are empty
    keys = rng.choice(np.arange(1, 80), size=n, replace=False)
    return {int(k): (int(rng.integers(1, 1000)), int(rng.integers(0, 1 << 50))) for k in keys}


def _worker(rank, world, port, seed, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    table = dict(_table(rank, seed))

    def export(buf, n):
        ks = sorted(table)
        assert len(ks) == n
        buf[0] = torch.tensor(ks, dtype=torch.int64)
        buf[1] = torch.tensor([table[k][0] for k in ks], dtype=torch.int64)
        buf[2] = torch.tensor([table[k][1] for k in ks], dtype=torch.int64)

    def merge(buf, n):
        for k, c, f in zip(buf[0].tolist(), buf[1].tolist(), buf[2].tolist()):
            c0, f0 = table.get(k, (0, 1 << 62))
            table[k] = (c0 + c, min(f0, f))

    n = tree_merge(dist, "cpu", len(table), export, merge, lambda: len(table))
    if rank == 0:
        out.put((n, sorted(table.items())))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2), (4, 3), (5, 4)])
def test_tree_merge_gloo(world, seed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    n, got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    want = {}
    for r in range(world):
        for k, (c, f) in _table(r, seed).items():
            c0, f0 = want.get(k, (0, 1 << 62))
            want[k] = (c0 + c, min(f0, f))
    assert got == sorted(want.items())
    assert n == len(want)


def _worker_a2a(rank, world, port, seed, out):
    from frender_amd.dist import exchange, owner_of, reduce_sum
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    table = _table(rank, seed)
    rows = torch.tensor([[k, c, f] for k, (c, f) in sorted(table.items())], dtype=torch.int64).reshape(-1, 3)
    mine = exchange(dist, "cpu", rows, owner_of(rows[:, 0], world))
    part = {}
    for k, c, f in mine.tolist():
        assert int(owner_of(torch.tensor([k]), world)[0]) == rank  # only codes this rank owns
        c0, f0 = part.get(k, (0, 1 << 62))
        part[k] = (c0 + c, min(f0, f))
    total = int(reduce_sum(dist, "cpu", [len(part)])[0])
    out.put((rank, sorted(part.items()), total))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,seed", [(2, 5), (3, 6), (4, 7)])
def test_partition_exchange_gloo(world, seed):  # dist.exchange, as partition_merge_device uses it
    """The hash-partitioned all-to-all merge: every code lands on exactly one owner and the
    union of the merged partitions equals the merged table (count = sum, first = min)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_a2a, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    union = {}
    for _, items, _ in got:
        for k, v in items:
            assert k not in union
            union[k] = v
    want = {}
    for r in range(world):
        for k, (c, f) in _table(r, seed).items():
            c0, f0 = want.get(k, (0, 1 << 62))
            want[k] = (c0 + c, min(f0, f))
    assert union == want
    assert all(t == len(want) for _, _, t in got)


def _worker_a2a_partitioned(rank, world, port, seed, out):
    """exchange_partitioned's side of the RCCL merge: rows already in owner blocks (what
    fr_export_partitioned_device writes; here sorted by owner_of on the host) with per-owner counts."""
    from frender_amd.dist import exchange_partitioned, owner_of, reduce_sum
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    table = _table(rank, seed)
    rows = torch.tensor([[k, c, f] for k, (c, f) in sorted(table.items())], dtype=torch.int64).reshape(-1, 3)
    own = owner_of(rows[:, 0], world)
    order = torch.argsort(own, stable=True)
    mine = exchange_partitioned(dist, "cpu", rows[order], torch.bincount(own, minlength=world))
    part = {}
    for k, c, f in mine.tolist():
        assert int(owner_of(torch.tensor([k]), world)[0]) == rank
        c0, f0 = part.get(k, (0, 1 << 62))
        part[k] = (c0 + c, min(f0, f))
    total = int(reduce_sum(dist, "cpu", [len(part)])[0])
    out.put((rank, sorted(part.items()), total))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,seed", [(2, 8), (4, 9)])
def test_partitioned_exchange_gloo(world, seed):
    """dist.exchange_partitioned (the RCCL merge's all-to-all of rows in owner blocks): every code lands on
    its owner and the union of the partitions equals the merged table."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_a2a_partitioned, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    union = {}
    for _, items, _ in got:
        for k, v in items:
            assert k not in union
            union[k] = v
    want = {}
    for r in range(world):
        for k, (c, f) in _table(r, seed).items():
            c0, f0 = want.get(k, (0, 1 << 62))
            want[k] = (c0 + c, min(f0, f))
    assert union == want
    assert all(t == len(want) for _, _, t in got)


def _worker_census(rank, world, port, out):
    from frender_amd import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = torch.arange(12, dtype=torch.int64).reshape(4, 3) + 100 * rank
    D.exchange(dist, "cpu", rows, D.owner_of(rows[:, 0], world))
    D.reduce_sum(dist, "cpu", [1, 2])
    D.reduce_max(dist, "cpu", [rank])
    D.gather_rows(dist, "cpu", rows)
    out.put((rank, {k: (v["calls"], v["bytes"]) for k, v in D.CENSUS.items()}))
    dist.barrier()
    dist.destroy_process_group()


def test_collective_census_gloo():
    """dist.CENSUS counts every collective of the module per kind with the bytes it moves (what
    FRENDER_DIST_CENSUS prints after a multi-rank scan)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_census, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, c in got.items():
        assert c["exchange"] == (1, 4 * 3 * 8)  # every row sent once
        assert c["all_reduce"] == (2, 3 * 8)
        assert c["gather_rows"][0] == 1
    assert got[0]["gather_rows"][1] == 2 * 4 * 3 * 8 and got[1]["gather_rows"][1] == 4 * 3 * 8
