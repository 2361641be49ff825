#!/usr/bin/env python3
"""bench.py — frender `scan` hot path on MI355X (BASELINE.json metric).

metric: "M reads/sec scanned+classified (96 samples, 8+8bp, n=1)"; workload =
BASELINE config 2: 100M SYN-v1 reads (96 samples, 8+8 bp dual index, n=1,
R=8 -> 74 B/record) per GPU, decoded FASTQ bytes resident in HBM when the timed
region starts (generated on the device by the SYN-v1 kernel).

One step = the whole scan hot path over that batch: reset the device tables ->
tally kernel over every byte (header scan, code pack, LDS-privatised hash count)
-> compaction + first-occurrence ordering -> Hamming classification of every
unique code (+ with --rc the rc pass, per-name call and pass B).  With N>1 GPUs
(torchrun, one process per GPU) each rank scans its own 100M reads (weak
scaling) and the per-GPU tables are merged over RCCL (binary-tree send/recv of
the compacted tables, merged on the GPU, frender_amd/dist.py) into rank 0, which
classifies the merged table.

Prints ONE JSON line (rank 0): value = total reads of all ranks / max-over-ranks
step time, plus roofline (tally kernel, HIP events on the library's stream) and
cpu_baseline (the oracle's CPU port timed on a bounded sample on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=100_000_000, help="reads per GPU")
    ap.add_argument("--samples", type=int, default=96)
    ap.add_argument("--index-len", type=int, default=8)
    ap.add_argument("--read-len", type=int, default=8, help="R: bases per read (8 -> 74 B/record)")
    ap.add_argument("--nsubs", type=int, default=1)
    ap.add_argument("--rc", action="store_true")
    ap.add_argument("--combinatorial", action="store_true", help="12x8 combinatorial sheet (config 4 shape)")
    ap.add_argument("--cpu-reads", type=int, default=2_000_000, help="bounded sample for the CPU baseline")
    ap.add_argument("--cpu-cores", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"),
                    help="per-launch HBM bytes of the tally kernel from rocprofv3 PMC (null if absent)")
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle CPU port (tally + classify, same algorithm as the reference) on a bounded
    sample of the same workload, from decoded text in memory, `cores` worker processes
    over `cores` shards as the reference parallelises over files (frender.py:189-193)."""
    from multiprocessing import Pool

    from frender_amd import synth
    from oracle import frender_oracle as O

    sheet = synth.make_sheet(args.samples, args.index_len, args.index_len,
                             combinatorial=(12, 8) if args.combinatorial else None)
    n = args.cpu_reads
    cores = args.cpu_cores
    cuts = [n * i // cores for i in range(cores + 1)]
    shards = [synth.generate_bytes(sheet, cuts[i], cuts[i + 1] - cuts[i], R=args.read_len, seed=1).decode()
              for i in range(cores)]
    t0 = time.perf_counter()
    with Pool(cores) as pool:
        per = pool.starmap(O.tally_text, [(s, None) for s in shards])
        total = {}
        for counts, _ in per:
            for k, v in counts.items():
                total[k] = total.get(k, 0) + v
        items = [(c, r, sheet.idx1, sheet.idx2, sheet.ids, args.nsubs, args.rc) for c, r in total.items()]
        pool.starmap(O.classify_code, items, chunksize=max(1, len(items) // (4 * cores)))
    dt = time.perf_counter() - t0
    return {"value": round(n / dt / 1e6, 4), "unit": "M reads/s", "cores": cores, "kind": "port",
            "sample": f"{n} SYN-v1 reads ({args.samples} samples, {args.index_len}+{args.index_len}bp, "
                      f"n={args.nsubs}, R={args.read_len}) decoded in memory, {cores} shards; oracle tally + "
                      f"classify of {len(total)} uniques took {dt:.2f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if args.dist_backend == "gloo":  # rehearsal: every rank on this box's GPU(s)
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from frender_amd import _lib, synth
    from frender_amd.dist import device_callbacks, tree_merge
    from frender_amd.host import reverse_complement
    from frender_amd.scan import _sheet_names

    sheet = synth.make_sheet(args.samples, args.index_len, args.index_len,
                             combinatorial=(12, 8) if args.combinatorial else None)
    reclen = synth.record_length(args.index_len, args.index_len, args.read_len)
    n = args.reads
    nbytes = n * reclen
    ctx = _lib.Context(device=local, chunk_bytes=1 << 30, table_slots=1 << 22)
    buf = ctx.device_alloc(nbytes + 64)
    ctx.synth_device(buf, rank * n, n, args.read_len, 1, sheet.idx1, sheet.idx2)
    names, nid = _sheet_names(sheet.ids)
    merge_cbs = device_callbacks(ctx)
    idx2rc = [reverse_complement(x) for x in sheet.idx2]

    def step():
        ctx.reset()
        ctx.begin_file(None)
        ctx.feed_device(buf, nbytes)
        st = ctx.end_file()
        assert st.records == n and st.error == 0, (st.records, st.error)
        U, _, _ = ctx.finalize()
        if world > 1:  # weak-scaled shards, one exchange: tree merge of the tables (dist.py)
            U = tree_merge(dist, "cuda", U, *merge_cbs)
        if rank == 0 or world == 1:
            ctx.set_sheet(sheet.idx1, sheet.idx2, idx2rc, nid, len(names))
            ctx.classify(args.nsubs, args.rc, to_host=False)
            if args.rc:
                f, r = ctx.rc_counts()
                use = [int(a) < int(b) for a, b in zip(f, r)]
                idx2b = [reverse_complement(x) if use[nid[i]] else x for i, x in enumerate(sheet.idx2)]
                ctx.set_sheet(sheet.idx1, idx2b, [reverse_complement(x) for x in idx2b], nid, len(names))
                ctx.classify(args.nsubs, False, to_host=False)
        ctx.sync()
        return U

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        U = step()
    ctx.sync()
    barrier()
    dt = time.perf_counter() - t0
    t_after = ctx.timing()
    ms = dt / args.steps * 1e3
    if world > 1:
        import torch
        x = torch.tensor([ms], dtype=torch.float64, device="cpu" if args.dist_backend == "gloo" else "cuda")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        ms = float(x.item())

    # tally-kernel roofline from HIP events on the library's stream (timed steps only:
    # ctx.reset() clears the per-reset counters, so read the last step's launches)
    launches = t_after.scan_launches
    scan_ms = t_after.scan_ms
    per_launch_bytes = t_after.scan_bytes / max(launches, 1)
    per_launch_ms = scan_ms / max(launches, 1)
    achieved = per_launch_bytes / (per_launch_ms / 1e3) / 1e9 if per_launch_ms > 0 else 0.0
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if tj.get("reads") == n and tj.get("read_len") == args.read_len:
            traffic = tj.get("hbm_bytes_per_launch")
    except Exception:
        traffic = None

    if rank == 0:
        cpu = None if args.no_cpu else cpu_baseline(args)
        value = world * n / (ms / 1e3) / 1e6
        out = {
            "metric": "M reads/sec scanned+classified (96 samples, 8+8bp, n=1) at 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "M reads/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (SYN-v1, generated in HBM)",
            "config": {"workload": f"BASELINE config 2: {n} SYN-v1 reads/GPU, {args.samples} samples, "
                                   f"{args.index_len}+{args.index_len}bp, n={args.nsubs}"
                                   f"{', -rc' if args.rc else ''}, R={args.read_len} ({reclen} B/record), "
                                   f"decoded FASTQ resident in HBM",
                       "reads_per_gpu": n, "bytes_per_record": reclen, "samples": args.samples,
                       "nsubs": args.nsubs, "rc": bool(args.rc), "unique_codes": int(U),
                       "parallelism": f"dp{world} (record shards) + {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} tree merge of the tables" if world > 1 else "1 GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "fr::chunk_kernel", "bytes_per_launch": int(per_launch_bytes),
                         "avg_launch_ms": round(per_launch_ms, 4), "launches_per_step": int(launches)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ctx.device_free(buf)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
