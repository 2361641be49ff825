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
