"""Multi-GPU scan: one process per GPU, torch.distributed over RCCL.

Product path (`python -m frender_amd scan --gpus K`, or any torchrun launch): sharded_tally
deals the input files to the GPUs (the reference's unit of parallelism, its Pool over files,
frender.py:189-193), every GPU tallies its files at their global file indices
(fr_begin_file_at), and rank 0 gathers the per-GPU tables, merges them on its GPU (count = sum,
first = min) and continues with classification and the CSVs: byte-identical to one GPU.

Bench path (below): device-resident record shards merged by a tree or a hash-partitioned
all-to-all.

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


# ---- product path: files sharded over GPUs, merged on rank 0 ---------------------------------

def world_group():
    """torch.distributed when this process is one rank of N > 1, else None."""
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover
        return None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


def assign_files(files, world: int) -> list:
    """Deal file indices to ranks: longest (compressed size) first onto the least loaded rank,
    ties to the lower rank and index; each rank's list in increasing index order."""
    import os

    size = [os.path.getsize(f) if os.path.exists(f) else 0 for f in files]
    load = [0] * world
    out = [[] for _ in range(world)]
    for i in sorted(range(len(files)), key=lambda i: (-size[i], i)):
        r = min(range(world), key=lambda r: (load[r], r))
        out[r].append(i)
        load[r] += size[i] + 1
    return [sorted(x) for x in out]


def merge_tables(ctx, parts):
    """Rank 0: merge the gathered per-rank tallies on this GPU (fr_merge_unique_device: count =
    sum, first = min; the file indices in the ordinals are global) and order the result
    (fr_finalize).  Presence pairs travel as (key, file) and map onto the merged order; exotic
    codes merge by string.  Returns the table dict scan.build_table takes."""
    import numpy as np

    ctx.reset()
    for t in parts:
        n = int(t["keys"].size)
        if not n:
            continue
        bufs = [ctx.device_alloc(8 * n) for _ in range(3)]
        try:
            for b, a in zip(bufs, (t["keys"], t["counts"], t["first"])):
                ctx.copy_to_device(b, np.ascontiguousarray(a, dtype=np.uint64).tobytes())
            ctx.merge_unique_device(bufs[0], bufs[1], bufs[2], n)
            ctx.sync()
        finally:
            for b in bufs:
                ctx.device_free(b)
    ctx.finalize()
    keys, counts, first = ctx.unique()
    order = np.argsort(keys, kind="stable")
    sk = keys[order]
    pk = np.concatenate([t["keys"][t["pu"].astype(np.int64)] for t in parts] + [np.zeros(0, np.uint64)])
    pf = np.concatenate([t["pf"].astype(np.int64) for t in parts] + [np.zeros(0, np.int64)])
    pu = order[np.searchsorted(sk, pk)] if pk.size else np.zeros(0, np.int64)
    srt = np.lexsort((pf, pu))  # (unique, file) order, as one context would emit them
    pu, pf = pu[srt], pf[srt]
    exo: dict = {}
    for t in parts:
        for k, c in enumerate(t["ecodes"]):
            e = exo.setdefault(c, [0, (1 << 64) - 1, set()])
            e[0] += int(t["ecounts"][k])
            e[1] = min(e[1], int(t["efirst"][k]))
        for k, f in zip(t["epc"].tolist(), t["epf"].tolist()):
            exo[t["ecodes"][k]][2].add(int(f))
    ecodes = list(exo)
    epc = [i for i, c in enumerate(ecodes) for _ in exo[c][2]]
    epf = [f for c in ecodes for f in sorted(exo[c][2])]
    return {"keys": keys, "counts": counts, "first": first, "pu": pu, "pf": pf, "ecodes": ecodes,
            "ecounts": np.array([exo[c][0] for c in ecodes], dtype=np.uint64),
            "efirst": np.array([exo[c][1] for c in ecodes], dtype=np.uint64),
            "epc": np.array(epc, dtype=np.int64), "epf": np.array(epf, dtype=np.int64)}


def sharded_tally(dist, ctx, files, sample, cores):
    """tally_barcodes (frender.py:183-207) over N GPUs.  Every rank tallies its share of the files
    (assign_files) into its own context; the tables, per-file lines and any data error go to rank
    0, which prints the per-file lines in file order, raises the first file's error as one GPU
    would, and returns the merged UniqueTable.  Other ranks return None."""
    import os

    from . import scan

    rank, world = dist.get_rank(), dist.get_world_size()
    mine = assign_files(files, world)[rank]
    ctx.reset()
    err = None
    per = {}
    try:
        scan.scan_files(ctx, files, mine, sample, cores,
                        after_file=lambda fi, records, new: per.__setitem__(fi, (records, new)))
    except BaseException as e:  # noqa: BLE001 - rank 0 re-raises it in file order
        err = (next(i for i in mine if i not in per), e)
    try:
        table = scan.local_table(ctx) if err is None else None
    except BaseException as e:  # noqa: BLE001
        err, table = (min(mine) if mine else 0, e), None
    payload = {"rank": rank, "per": per, "err": err, "table": table}
    got = [None] * world if rank == 0 else None
    dist.gather_object(payload, got, dst=0)
    if rank != 0:
        return None
    per_all, errs = {}, []
    for p in got:
        per_all.update(p["per"])
        if p["err"] is not None:
            errs.append(p["err"])
    first_bad = min((e[0] for e in errs), default=None)
    for fi, path in enumerate(files):
        name = str(os.path.basename(path))
        print(f"Tallying barcodes from {name}...", end="")
        if first_bad is not None and fi >= first_bad:
            raise next(e for i, e in errs if i == first_bad)
        records, new = per_all[fi]
        print(scan.found_line(new, records))
    print(type([]), len(files))
    merged = merge_tables(ctx, [p["table"] for p in got])
    names = [str(os.path.basename(p)) for p in files]
    return scan.build_table(merged, names, [per_all[i][0] for i in range(len(files))])
