"""Multi-GPU scan: one process per GPU, torch.distributed over RCCL.

One design for the product (`python -m frender_amd scan --gpus N`, any torchrun launch) and the bench
(bench.py --gpus N):

1. Record shards.  The reference's unit of parallelism is the file (its Pool, frender.py:189-193);
   here every rank tallies a share of the RECORD stream into its own device table at global
   ordinals (fr_begin_file_at: (file index + 1) << 44 | byte offset).  The product deals whole files
   when there are at least as many files as GPUs, and otherwise cuts each file into record-aligned
   parts (fr_gz_feed_part: cuts at record starts, universal newlines), so even one file spreads over
   every GPU.  The bench's shards are records generated in each rank's HBM.
2. Key partition.  The only exchange: every rank exports its finalized (key, count, first) rows and
   its (key, file) presence pairs, and one all-to-all over xGMI moves each to the rank that owns the
   key (a multiplicative hash of the key, mod N).  Each rank merges its rows on its GPU
   (fr_merge_unique_device: count = sum, first = min) and orders its partition (fr_finalize).
3. Classification per partition, on each GPU; with -rc the per-name (f, rc) read sums are the only
   other collective (an all-reduce of 2 x names integers).
4. Rank 0 gathers the classified rows (fixed-width int64 rows: first, key, count, matches, class,
   demux_ok) over RCCL, orders them by first occurrence and writes the CSVs.  Exotic codes (outside
   the fast and wide key forms: rare) travel to rank 0 as a byte blob of their own.

Integer sums, mins and unions make every output identical for any N.  No Python objects are pickled:
every exchange is an int64 or uint8 tensor (device tensors over RCCL; host tensors over gloo, which
rehearses N ranks on one GPU or on CPU).

The tree merge (tree_merge) is kept as the alternative protocol for the bench (--merge tree).
"""
from __future__ import annotations

import time
from typing import Callable

# Collective census: every exchange / reduce / gather of this module, counted and timed per kind (wall
# clock around the blocking call).  `python -m frender_amd scan` prints it per rank to stderr when
# FRENDER_DIST_CENSUS is set.
CENSUS: dict = {}


def _census(kind: str, t0: float, nbytes: int = 0):
    c = CENSUS.setdefault(kind, {"calls": 0, "ms": 0.0, "bytes": 0})
    c["calls"] += 1
    c["ms"] += (time.perf_counter() - t0) * 1e3
    c["bytes"] += int(nbytes)


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


# ---- collectives on int64 / uint8 tensors (RCCL device buffers, or host tensors over gloo) -----

def wire_of(dist, ctx):
    """Where this rank's exchange tensors live: its GPU (RCCL), or the host (gloo rehearsals)."""
    import torch

    if dist.get_backend() == "gloo":
        return torch.device("cpu")
    return torch.device("cuda", getattr(ctx, "device", torch.cuda.current_device()))


def exchange(dist, wire, rows, dest):
    """All-to-all of int64 rows [n, k]: row i goes to rank dest[i].  Returns the rows this rank
    received, [m, k] on `wire`, ordered by source rank, then by their order at the source."""
    import torch

    t0 = time.perf_counter()
    world = dist.get_world_size()
    rows = rows.to(wire)
    k = int(rows.shape[1])
    dest = dest.to(wire)
    order = torch.argsort(dest, stable=True)
    send = rows[order].contiguous()
    scount = torch.bincount(dest, minlength=world).to(torch.int64)
    rcount = torch.empty_like(scount)
    dist.all_to_all_single(rcount, scount)
    sc, rc = scount.tolist(), rcount.tolist()
    recv = torch.empty((sum(rc), k), dtype=torch.int64, device=wire)
    dist.all_to_all_single(recv.view(-1), send.view(-1), [k * c for c in rc], [k * c for c in sc])
    _census("exchange", t0, 8 * k * sum(sc))
    return recv


def exchange_partitioned(dist, wire, send, scount):
    """All-to-all of int64 rows [n, k] already in owner blocks (ranks 0..world-1 in order, scount[r] rows for
    rank r: the library's partitioned export).  Returns the received rows [m, k], by source rank."""
    import torch

    t0 = time.perf_counter()
    k = int(send.shape[1]) if send.dim() == 2 else 3
    scount = scount.to(wire).to(torch.int64)
    rcount = torch.empty_like(scount)
    dist.all_to_all_single(rcount, scount)
    sc, rc = scount.tolist(), rcount.tolist()
    recv = torch.empty((sum(rc), k), dtype=torch.int64, device=wire)
    dist.all_to_all_single(recv.view(-1), send.contiguous().view(-1), [k * c for c in rc], [k * c for c in sc])
    _census("exchange", t0, 8 * k * sum(sc))
    return recv


def _reduce(dist, wire, values, op):
    import torch

    t0 = time.perf_counter()
    t = torch.as_tensor(list(values), dtype=torch.int64).to(wire)
    if t.numel():
        dist.all_reduce(t, op=op)
    out = t.cpu().numpy()
    _census("all_reduce", t0, 8 * t.numel())
    return out


def reduce_sum(dist, wire, values):
    """All-reduce (sum) of a small int64 vector (per-name -rc counts, per-file records, ...)."""
    return _reduce(dist, wire, values, dist.ReduceOp.SUM)


def reduce_max(dist, wire, values):
    return _reduce(dist, wire, values, dist.ReduceOp.MAX)


def reduce_min(dist, wire, values):
    return _reduce(dist, wire, values, dist.ReduceOp.MIN)


def gather_rows(dist, wire, rows):
    """Gather int64 rows [n_r, k] of every rank on rank 0 (point-to-point sends of each rank's rows).
    Returns the list of numpy arrays (rank order) on rank 0, None elsewhere."""
    import torch

    t0 = time.perf_counter()
    rank, world = dist.get_rank(), dist.get_world_size()
    rows = rows.to(wire).contiguous()
    k = int(rows.shape[1])
    sizes = [torch.zeros(1, dtype=torch.int64, device=wire) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([rows.shape[0]], dtype=torch.int64, device=wire))
    n = [int(x.item()) for x in sizes]
    if rank != 0:
        if n[rank]:
            dist.send(rows, dst=0)
        _census("gather_rows", t0, 8 * k * n[rank])
        return None
    out = [rows.cpu().numpy()]
    for r in range(1, world):
        buf = torch.empty((n[r], k), dtype=torch.int64, device=wire)
        if n[r]:
            dist.recv(buf, src=r)
        out.append(buf.cpu().numpy())
    _census("gather_rows", t0, 8 * k * sum(n))
    return out


def gather_bytes(dist, wire, blob: bytes):
    """Gather one byte string per rank on rank 0 (as int64 rows); a list on rank 0, None elsewhere."""
    import numpy as np
    import torch

    padded = blob + b"\0" * ((-len(blob)) % 8)
    rows = torch.from_numpy(np.frombuffer(padded, dtype=np.int64).copy().reshape(-1, 1))
    got = gather_rows(dist, wire, rows)
    lens = gather_rows(dist, wire, torch.tensor([[len(blob)]], dtype=torch.int64))
    if got is None:
        return None
    return [g.reshape(-1).view(np.uint8)[: int(n[0, 0])].tobytes() for g, n in zip(got, lens)]


# ---- bench path: the partition merge of device-resident shards ---------------------------------

def partition_merge_device(dist, device, ctx):
    """Steps 2 of the module doc on the HIP library: export this rank's finalized table, move every
    row to its owner, rebuild the table from the rows this rank owns and finalize it.  Returns the
    size of this rank's partition of the merged table."""
    import torch

    wire = "cpu" if dist.get_backend() == "gloo" else device
    if wire != "cpu":  # RCCL: rows partitioned by owner on the device (one library call), merged row-major
        rows, scount = ctx.export_partitioned(dist.get_world_size())
        mine = exchange_partitioned(dist, rows.device, rows, scount)
        ctx.reset()
        ctx.merge_rows_rowmajor(mine)
        n, _, _ = ctx.finalize()
        ctx.sync()
        return int(n)
    rows = ctx.export_rows(wire)
    mine = exchange(dist, wire, rows, owner_of(rows[:, 0], dist.get_world_size()) if rows.shape[0]
                    else torch.zeros(0, dtype=torch.int64, device=rows.device))
    ctx.reset()
    ctx.merge_rows(mine)
    n, _, _ = ctx.finalize()
    ctx.sync()
    return int(n)


# ---- product path ------------------------------------------------------------------------------

def launch_ranks(n: int, argv: list, cmd: list | None = None) -> int:
    """`scan|demux --gpus N` (and `bench.py --gpus N`): one child process per GPU (this process never
    touches a GPU), joined by torch.distributed over 127.0.0.1; rank 0's stdout is the command's.  A
    rank that fails ends the others; the exit status is rank 0's, or the first failure's.  cmd: the
    child's program (default `python -m frender_amd`)."""
    import os
    import socket
    import subprocess
    import sys
    import time

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([*(cmd or [sys.executable, "-m", "frender_amd"]), *argv], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    codes = [None] * n
    while any(c is None for c in codes):
        for r, p in enumerate(procs):
            if codes[r] is None:
                codes[r] = p.poll()
        if any(c not in (None, 0) for c in codes):  # a failed rank: the others cannot finish
            time.sleep(2)
            for r, p in enumerate(procs):
                if p.poll() is None:
                    p.terminate()
            for r, p in enumerate(procs):
                codes[r] = p.wait()
            break
        time.sleep(0.05)
    return codes[0] if codes[0] else next((c for c in codes if c), 0)



class PeerFailed(Exception):
    """Raised on ranks > 0 when a scan fails: rank 0 raises the reference's exception, in the
    reference's order, and the launcher exits with rank 0's status."""


class _Skip(Exception):
    """Internal: skip this rank's local table after a recorded failure."""


def world_group():
    """torch.distributed when this process is one rank of N > 1, else None.  A process that has not
    imported torch has no process group: the single-GPU commands do not pay the import here."""
    import sys

    if "torch" not in sys.modules:
        return None
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


def plan_shards(files, world: int, sample=None) -> list:
    """Record shards per rank: lists of (file index, part, parts), increasing file index.  Whole
    files (part 0 of 1) when there are at least as many files as ranks, or with -s (a sample is the
    head of each whole file); otherwise every file is cut into record-aligned parts so that every
    rank holds exactly one part: floor(N / F) parts per file, one more for the F' = N mod F largest."""
    import os

    F = len(files)
    if sample or F == 0 or F >= world:
        return [[(i, 0, 1) for i in lst] for lst in assign_files(files, world)]
    size = [os.path.getsize(f) if os.path.exists(f) else 0 for f in files]
    big = sorted(range(F), key=lambda i: (-size[i], i))[: world % F]
    nparts = [world // F + (1 if i in big else 0) for i in range(F)]
    units = [(i, j, nparts[i]) for i in range(F) for j in range(nparts[i])]
    return [[u] for u in units]


def _exo_blob(ecodes, ecounts, efirst, epc, epf, epn) -> bytes:
    """This rank's exotic-code table as bytes: counts, then per code (length, count, first), the
    (code, file, reads in the file) presence triples and the code bytes (no pickling)."""
    import numpy as np

    n, m = len(ecodes), len(epc)
    head = np.array([n, m], dtype=np.int64)
    meta = np.array([[len(c), int(k), int(f)] for c, k, f in zip(ecodes, ecounts, efirst)],
                    dtype=np.uint64).reshape(-1, 3)
    pairs = (np.stack([np.asarray(epc, np.int64), np.asarray(epf, np.int64), np.asarray(epn, np.int64)], 1) if m
             else np.zeros((0, 3), np.int64))
    return head.tobytes() + meta.tobytes() + pairs.tobytes() + b"".join(bytes(c) for c in ecodes)


def _exo_unblob(blob: bytes):
    import numpy as np

    n, m = np.frombuffer(blob[:16], dtype=np.int64).tolist()
    o = 16
    meta = np.frombuffer(blob[o:o + 24 * n], dtype=np.uint64).reshape(n, 3)
    o += 24 * n
    pairs = np.frombuffer(blob[o:o + 24 * m], dtype=np.int64).reshape(m, 3)
    o += 24 * m
    codes = []
    for ln in meta[:, 0].tolist():
        codes.append(blob[o:o + ln])
        o += ln
    return codes, meta[:, 1], meta[:, 2], pairs[:, 0], pairs[:, 1], pairs[:, 2]


def _merge_exotic(blobs):
    """Rank 0: the exotic codes of every rank merged by byte string (count = sum, first = min,
    presence = union, per-file reads = sum), in first-seen order (build_table orders them by first
    ordinal)."""
    import numpy as np

    exo: dict = {}
    for b in blobs:
        codes, counts, first, pc, pf, pn = _exo_unblob(b)
        for c, k, f in zip(codes, counts.tolist(), first.tolist()):
            e = exo.setdefault(c, [0, (1 << 64) - 1, {}])
            e[0] += int(k)
            e[1] = min(e[1], int(f))
        for c, f, k in zip(pc.tolist(), pf.tolist(), pn.tolist()):
            per = exo[codes[c]][2]
            per[int(f)] = per.get(int(f), 0) + int(k)
    ecodes = list(exo)
    return (ecodes, np.array([exo[c][0] for c in ecodes], dtype=np.uint64),
            np.array([exo[c][1] for c in ecodes], dtype=np.uint64),
            np.array([i for i, c in enumerate(ecodes) for _ in exo[c][2]], dtype=np.int64),
            np.array([f for c in ecodes for f in sorted(exo[c][2])], dtype=np.int64),
            np.array([exo[c][2][f] for c in ecodes for f in sorted(exo[c][2])], dtype=np.uint64))


ERR_NOSPACE, ERR_UTF8, ERR_GZ, ERR_OTHER = 0, 1, 2, 3  # columns of the per-file error flags


def sharded_tally(dist, ctx, files, sample, cores):
    """tally_barcodes (frender.py:183-207) over N GPUs: steps 1-2 of the module doc.  Every rank
    returns its PARTITION of the merged table as a UniqueTable (rank 0's also holds the exotic
    codes), with the global per-file records; rank 0 prints the reference's per-file lines.  A data
    error raises the reference's exception on rank 0 (files in order) and PeerFailed elsewhere."""
    import os

    import numpy as np
    import torch

    from . import _lib, scan

    rank, world = dist.get_rank(), dist.get_world_size()
    wire = wire_of(dist, ctx)
    F = len(files)
    plan = plan_shards(files, world, sample)
    mine = plan[rank]
    # Any failure on this rank is recorded, never raised before the collectives below (a rank that
    # left them would hang its peers): data errors by their file's flags, anything else (a device or
    # library error) as ERR_OTHER of its file, or of row F when it is tied to no file; the rank that
    # met it raises it once every rank knows, the others raise PeerFailed.
    records = np.zeros(F, np.int64)
    flags = np.zeros((F + 1, 4), np.int64)
    other: dict = {}  # file index (F: none) -> this rank's exception
    pool = None
    # Record parts of BGZF files decode on their own (fr_gz_part_open: no inflate of what precedes the
    # part); their cuts need the line count before each part, so the ranks first count their parts'
    # lines and exchange the counts (one all-reduce of an F x N matrix, run whenever the plan cuts a
    # file, so every rank joins it).  Parts of other gzip streams inflate from the file's start
    # (fr_gz_feed_part): a single deflate stream cannot be entered mid-way.
    bgzf: dict = {}  # unit index -> GzPart
    part_lines = np.zeros((F, world), np.int64)
    for k, (fi, part, nparts) in enumerate(mine):
        if nparts > 1:
            try:
                gp = _lib.GzPart.open(files[fi], part, nparts, threads=max(1, int(cores)))
                if gp is not None:
                    bgzf[k] = gp
                    part_lines[fi, part] = gp.lines
            except _lib.GzError:
                flags[fi, ERR_GZ] = 1
            except Exception as e:  # noqa: BLE001 - raised after the collectives
                flags[fi, ERR_OTHER] = 1
                other.setdefault(fi, e)
    if F and any(u[2] > 1 for units in plan for u in units):
        part_lines = reduce_sum(dist, wire, part_lines.reshape(-1)).reshape(F, world)
    inflated = {}  # BGZF parts: decoded bytes produced, and the part's record bytes (diagnostics)
    try:
        ctx.reset()
        streamed = [k for k in range(len(mine)) if k not in bgzf and not (flags[mine[k][0]].any())]
        paths = [files[mine[k][0]] for k in streamed]
        pool = _lib.GzPool(paths, threads=max(1, int(cores)), ahead=_lib.inflate_ahead(paths, max(1, int(cores))))
        slot = {k: j for j, k in enumerate(streamed)}
        for k, (fi, part, nparts) in enumerate(mine):
            if k not in bgzf and k not in slot:
                continue  # failed before the collectives (flagged)
            try:
                if k in bgzf:
                    ctx.feed_gz_part_counted(bgzf[k], fi, int(part_lines[fi, :part].sum()))
                    inflated[fi] = (bgzf[k].inflated, bgzf[k].length)
                elif nparts == 1:
                    ctx.begin_file(sample, file_index=fi)
                    pool.feed(slot[k], ctx)
                else:
                    ctx.feed_gz_part(pool, slot[k], fi, part, nparts, _lib.GzPool.size_hint(files[fi]))
                st = ctx.end_file()
                records[fi] += int(st.records)
                flags[fi, ERR_UTF8] |= 1 if st.utf8_bad else 0
                flags[fi, ERR_NOSPACE] |= 1 if st.error == _lib.FR_SCAN_NO_SPACE else 0
            except _lib.GzError:
                flags[fi, ERR_GZ] = 1
                try:
                    ctx.end_file()
                except Exception:  # noqa: BLE001 - the file is reported through its flag
                    pass
            except Exception as e:  # noqa: BLE001 - raised after the collectives
                flags[fi, ERR_OTHER] = 1
                other.setdefault(fi, e)
                break  # the context may be unusable: this rank stops tallying
    except Exception as e:  # noqa: BLE001 - the pool or the reset: no file to blame
        flags[F, ERR_OTHER] = 1
        other.setdefault(F, e)
    finally:
        if pool is not None:
            pool.close()
        for gp in bgzf.values():
            gp.close()
    # ---- the local table: rows, presence pairs, exotic codes ---------------------------------
    empty3 = np.zeros((0, 3), np.int64)
    try:
        if other:
            raise _Skip()
        ctx.finalize()
        keys, _, _ = ctx.unique()
        pu, pf = ctx.presence()
        exo_local = ctx.exotic_table()
        pn, epn = ctx.presence_counts(len(exo_local[3]))
        exo_local = (*exo_local, epn)
        rows = ctx.export_rows(wire)
        # (key, file, reads of the key in this rank's share of the file) presence triples
        pairs = torch.as_tensor(np.stack([keys[np.asarray(pu, np.int64)].view(np.int64), np.asarray(pf, np.int64),
                                          np.asarray(pn, np.uint64).view(np.int64)], 1)
                                if len(pu) else empty3)
    except Exception as e:  # noqa: BLE001 - this rank joins the exchange with nothing
        if not isinstance(e, _Skip):
            flags[F, ERR_OTHER] = 1
            other.setdefault(F, e)
        rows, pairs = torch.as_tensor(empty3), torch.as_tensor(empty3)
        exo_local = ([], np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.int64), np.zeros(0, np.int64),
                     np.zeros(0, np.uint64))
    # ---- step 2: every row and pair to the key's owner; the partition's table -----------------
    k64 = torch.zeros(0, dtype=torch.int64)
    my_rows = exchange(dist, wire, rows, owner_of(rows[:, 0], world) if rows.shape[0] else k64)
    my_pairs = exchange(dist, wire, pairs, owner_of(pairs[:, 0], world) if pairs.shape[0] else k64).cpu().numpy()
    pkeys = pcounts = pfirst = np.zeros(0, np.uint64)
    if other:  # a failed rank joins the exchange but keeps nothing
        my_pairs = my_pairs[:0]
    else:
        try:
            ctx.reset()
            ctx.merge_rows(my_rows)
            ctx.finalize()
            pkeys, pcounts, pfirst = ctx.unique()
        except Exception as e:  # noqa: BLE001 - raised after the collectives
            flags[F, ERR_OTHER] = 1
            other.setdefault(F, e)
            my_pairs = my_pairs[:0]
    if my_pairs.shape[0]:
        pk, inv = np.unique(my_pairs[:, :2], axis=0, return_inverse=True)  # (key, file), each once
        reads = np.zeros(pk.shape[0], np.int64)
        np.add.at(reads, inv.reshape(-1), my_pairs[:, 2])  # a file cut into parts: the parts' reads summed
        srt = np.argsort(pkeys.view(np.int64), kind="stable")
        idx = srt[np.searchsorted(pkeys.view(np.int64)[srt], pk[:, 0])]
        o = np.lexsort((pk[:, 1], idx))
        p_u, p_f, p_n = idx[o].astype(np.int64), pk[o, 1], reads[o].astype(np.uint64)
    else:
        p_u = p_f = np.zeros(0, np.int64)
        p_n = np.zeros(0, np.uint64)
    blobs = gather_bytes(dist, wire, _exo_blob(*exo_local))
    if rank == 0:
        ecodes, ecounts, efirst, epc, epf, epn = _merge_exotic(blobs)
    else:
        ecodes, ecounts, efirst, epc, epf, epn = [], np.zeros(0, np.uint64), np.zeros(0, np.uint64), \
            np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint64)
    # ---- global per-file numbers: records, distinct codes ("new barcodes"), errors -------------
    distinct = np.bincount(p_f, minlength=F)[:F] + np.bincount(epf, minlength=F)[:F] if F else np.zeros(0)
    # one reduce for records and distinct codes, one for the flags
    sums = reduce_sum(dist, wire, np.concatenate([records, np.asarray(distinct, np.int64)]))
    records, distinct = sums[:F], sums[F:]
    flags = reduce_max(dist, wire, flags.reshape(-1)).reshape(F + 1, 4)
    names = [str(os.path.basename(p)) for p in files]
    # rank 0 decides which file fails first, as one GPU would (a flagged file's replay through
    # Python's gzip may find that the reference reads it fine, e.g. bad bytes past a -s sample)
    failed, err = -1, None
    if rank == 0:
        for fi in range(F + 1):
            if flags[fi, ERR_OTHER]:  # a library / device failure on some rank: that rank raises it
                failed = fi
                break
            if fi == F:
                break
            print(f"Tallying barcodes from {names[fi]}...", end="")
            if flags[fi].any():
                try:
                    if flags[fi, ERR_UTF8] or flags[fi, ERR_GZ]:
                        scan._replay_decode_error(files[fi], sample)  # the reference's exception, if any
                        if flags[fi, ERR_GZ]:
                            raise RuntimeError(f"native inflate rejected {files[fi]} but Python's gzip reads it")
                    if flags[fi, ERR_NOSPACE]:
                        raise IndexError("list index out of range")  # frender.py:169 split(" ")[1]
                except BaseException as e:  # noqa: BLE001 - re-raised once the peers know
                    failed, err = fi, e
                    break
            print(scan.found_line(int(distinct[fi]), int(records[fi])))
    failed = int(reduce_max(dist, wire, [failed])[0])
    if failed >= 0:
        if failed in other:
            raise other[failed]
        if rank == 0 and err is not None:
            raise err
        raise PeerFailed("scan failed (the rank that met it reports it)")
    if rank == 0:
        print(type([]), F)
    t = {"keys": pkeys, "counts": pcounts, "first": pfirst, "pu": p_u, "pf": p_f, "pn": p_n, "ecodes": ecodes,
         "ecounts": ecounts, "efirst": efirst, "epc": epc, "epf": epf, "epn": epn}
    table = scan.build_table(t, names, [int(x) for x in records])
    table.group, table.wire = dist, wire
    table.inflated = inflated
    return table
