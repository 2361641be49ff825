"""Multi-GPU table merge: one process per GPU, torch.distributed over RCCL.

The record stream shards with no data-path collective: each rank tallies its own
records into its own device table.  The only exchange is the merge of the
compacted tables at the end, replacing the reference's parent-process dict merge
(frender.py:199-205):

    binary tree over ranks, log2(N) rounds: in round k, rank r with
    r % 2^(k+1) == 2^k sends its compacted (key, count, first) arrays to rank
    r - 2^k, which merges them into its own device table (count = sum,
    first = min) and re-compacts.  Rank 0 ends with the whole table.

The tree keeps every xGMI link busy at once in the early rounds (point-to-point
links, not a switch) and runs the merges of one round in parallel; rank 0
receives the same total bytes a gather would deliver.  Integer sums and mins
make the result identical for any N.

The device work is injected as callables so the same protocol runs over RCCL
with the HIP library (bench.py) and over gloo with CPU tables (tests).
"""
from __future__ import annotations

from typing import Callable


def tree_merge(dist, device, n_local: int,
               export: Callable[[object, int], None],
               merge: Callable[[object, int], None],
               refinalize: Callable[[], int]) -> int:
    """Merge every rank's table into rank 0's.  Returns this rank's table size after
    its last merge (on rank 0: the merged table's size).

    export(buf, n)  write this rank's compacted table into buf[3, n] (int64 tensor)
    merge(buf, n)   merge buf[3, n] received from a child into this rank's table
    refinalize()    re-compact after merges; returns the new size
    """
    import torch

    rank, world = dist.get_rank(), dist.get_world_size()
    # gloo moves host tensors only: stage device tables through host memory (rehearsal
    # runs of the multi-rank path on one GPU); RCCL sends device memory over xGMI
    wire = "cpu" if dist.get_backend() == "gloo" else device
    n = int(n_local)
    step = 1
    while step < world:
        if rank % (2 * step) == step:  # sender this round, then done
            parent = rank - step
            dist.send(torch.tensor([n], dtype=torch.int64, device=wire), dst=parent)
            if n:
                buf = torch.empty((3, n), dtype=torch.int64, device=device)
                export(buf, n)
                dist.send(buf.to(wire), dst=parent)
            return n
        if rank % (2 * step) == 0 and rank + step < world:  # receiver this round
            child = rank + step
            sz = torch.zeros(1, dtype=torch.int64, device=wire)
            dist.recv(sz, src=child)
            m = int(sz.item())
            if m:
                buf = torch.empty((3, m), dtype=torch.int64, device=wire)
                dist.recv(buf, src=child)
                merge(buf.to(device), m)
                n = refinalize()
        step *= 2
    return n


def device_callbacks(ctx):
    """tree_merge callables backed by the HIP library's export/merge entry points."""

    def export(buf, n):
        ctx.export_unique_device(buf[0].data_ptr(), buf[1].data_ptr(), buf[2].data_ptr(), n)

    def merge(buf, n):
        import torch

        torch.cuda.current_stream().synchronize()  # the recv landed on torch's stream
        ctx.merge_unique_device(buf[0].data_ptr(), buf[1].data_ptr(), buf[2].data_ptr(), n)
        ctx.sync()  # buf goes back to torch's allocator after this

    def refinalize():
        U, _, _ = ctx.finalize()
        return int(U)

    return export, merge, refinalize


# ---- hash-partitioned merge (all-to-all): the scalable form ---------------------------------
# Weak scaling wants every rank's work constant in N.  The tree leaves rank 0 merging and
# classifying the whole N-times-larger table; instead partition the key space: rank r owns the
# codes with part(key) == r.  One all-to-all over xGMI moves each compacted (key, count, first)
# row to its owner (every link busy at once, U x 24 B per rank in total), each rank merges and
# classifies its own partition, and only the -rc per-name (f, rc) sums (2 x names integers) need
# an all-reduce.  Counts are integer sums and firsts integer mins, so the union of the
# partitions is identical to a single-GPU scan of all records.

_MULT = -7046029254386353131  # 0x9E3779B97F4A7C15 as int64 (wrapping multiply)


def owner_of(keys, world: int):
    """Owning rank of each int64 code key: the top bits of a multiplicative hash, mod world."""
    import torch

    return ((keys * _MULT) >> 40).bitwise_and(0xFFFFFF).remainder(world)


def partition_exchange(dist, device, rows):
    """rows: [U, 3] int64 (key, count, first) on `device`.  Returns the rows this rank owns,
    gathered from every rank ([R, 3], same device; order: by source rank, then local order)."""
    import torch

    world = dist.get_world_size()
    wire = "cpu" if dist.get_backend() == "gloo" else device
    dest = owner_of(rows[:, 0], world) if rows.shape[0] else torch.zeros(0, dtype=torch.int64, device=rows.device)
    order = torch.argsort(dest, stable=True)
    send = rows[order].contiguous().to(wire)
    scount = torch.bincount(dest, minlength=world).to(torch.int64).to(wire)
    rcount = torch.empty_like(scount)
    dist.all_to_all_single(rcount, scount)
    sc, rc = scount.tolist(), rcount.tolist()
    recv = torch.empty((sum(rc), 3), dtype=torch.int64, device=wire)
    dist.all_to_all_single(recv.view(-1), send.view(-1), [3 * c for c in rc], [3 * c for c in sc])
    return recv.to(device)


def reduce_sum(dist, device, values):
    """All-reduce (sum) of a small int64 vector, e.g. the -rc per-name counts."""
    import torch

    wire = "cpu" if dist.get_backend() == "gloo" else device
    t = torch.as_tensor(values, dtype=torch.int64).to(wire)
    dist.all_reduce(t)
    return t.cpu().tolist()


def partition_merge_device(dist, device, ctx):
    """The hash-partitioned merge on the HIP library: export this rank's finalized table,
    exchange, rebuild the table from the rows this rank owns, and finalize it.  Returns the
    size of this rank's partition of the merged table."""
    import torch

    U = int(ctx.U)
    rows = torch.empty((3, max(U, 1)), dtype=torch.int64, device=device)
    if U:
        ctx.export_unique_device(rows[0].data_ptr(), rows[1].data_ptr(), rows[2].data_ptr(), U)
    mine = partition_exchange(dist, device, rows[:, :U].t())
    cols = mine.t().contiguous()
    torch.cuda.current_stream().synchronize()  # the exchange landed on torch's stream
    ctx.reset()
    if cols.shape[1]:
        ctx.merge_unique_device(cols[0].data_ptr(), cols[1].data_ptr(), cols[2].data_ptr(), int(cols.shape[1]))
    n, _, _ = ctx.finalize()
    ctx.sync()
    return int(n)
