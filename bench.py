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
scaling) and the per-GPU tables are merged over RCCL with one all-to-all: every
code goes to the rank that owns its hash partition, each rank merges (on the GPU)
and classifies its partition, and -rc adds an all-reduce of the per-name sums
(frender_amd/dist.py; --merge tree sends everything to rank 0 instead).

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
    ap.add_argument("--launch-gib", type=int, default=16, help="largest tally launch of a device feed (GiB)")
    ap.add_argument("--rc", action="store_true")
    ap.add_argument("--files", type=int, default=1,
                    help="feed each GPU's records as this many consecutive files (per-file presence scans and the "
                         "presence map in the timed step; the headline is one file, BASELINE config 2's one stream)")
    ap.add_argument("--combinatorial", action="store_true", help="12x8 combinatorial sheet (config 4 shape)")
    ap.add_argument("--cpu-reads", type=int, default=24_000_000, help="bounded sample for the CPU baseline (~10-20 s on 8 cores)")
    ap.add_argument("--cpu-cores", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pin", action="store_true", help="skip the reference-pin check (ablation builds only)")
    ap.add_argument("--no-single", action="store_true",
                    help="skip e2e.single_member (the cpu_baseline's records as one single-member .fastq.gz)")
    ap.add_argument("--merge", choices=["a2a", "tree"], default="a2a",
                    help="N>1 table merge: hash-partitioned all-to-all (every rank merges and classifies its "
                         "partition) or a binary tree into rank 0")
    ap.add_argument("--merge-leg", action="store_true",
                    help="N=1 only, not the headline: a one-rank nccl (RCCL) process group, and every step also runs "
                         "the N>1 merge leg on the full table (partition_merge_device's all-to-all and rebuild, then "
                         "classify, then gather_rows of the rows to rank 0, as the product's writer does); reports "
                         "merge_leg with the phases' ms per step")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--rank-check", action="store_true",
                    help="launcher check: every rank joins the process group over gloo, rank 0 prints the world "
                         "size it sees, nothing touches a GPU")
    ap.add_argument("--pin-json", default=None,
                    help="the reference's own rows for this shape (default tests/golden/cfg{2,3,4}_pin.json, made by "
                         "tests/golden/make_golden_cfg2.py / make_golden_cfg34.py): at N=1 on that exact shape and read "
                         "count the classified table must reproduce them (checked after timing)")
    ap.add_argument("--cfg5", action="store_true",
                    help="instead of the headline metric: BASELINE config 5's shape end to end (paired .fastq.gz, "
                         "R=150 -> scan + demux CLIs) beside the reference's CPU path (oracle port) on a bounded sample")
    ap.add_argument("--cfg5-pairs", type=int, default=2_000_000)
    ap.add_argument("--cfg5-files", type=int, default=4, help="file pairs")
    ap.add_argument("--cfg5-cpu-pairs", type=int, default=100_000)
    ap.add_argument("--tuning", default="",
                    help="A/B runs only: fr_tuning fields for the bench's context, e.g. 'log_min=0,chunk_tiles=400' "
                         "(results never change; a tuned run reports them in config.tuning)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r06.json"),
                    help="per-launch HBM bytes of the tally kernel from rocprofv3 PMC (scripts/make_traffic.py); "
                         "used only when taken on this source tree and this launch shape, else traffic is null")
    return ap.parse_args()


def config_name(args) -> str:
    """Which BASELINE.json config this run's shape is (configs 3/4 are quoted on 8 GPUs).  Only the
    exact shape gets the config's name: another read count or read length is a custom run."""
    std = args.read_len == 8
    if args.combinatorial and std and args.samples == 96 and args.index_len == 8 and args.nsubs == 2 and not args.rc:
        return "BASELINE config 4 shape (96 combinatorial, n=2)"
    if std and args.samples == 384 and args.index_len == 10 and args.rc and args.nsubs == 1 and not args.combinatorial:
        return "BASELINE config 3 shape (384 samples, 10+10, -rc)"
    if (std and args.reads == 100_000_000 and args.samples == 96 and args.index_len == 8 and args.nsubs == 1
            and not args.rc and not args.combinatorial):
        return "BASELINE config 2" + (f" as {args.files} files" if args.files > 1 else "")
    return "custom shape"


def table_checksum(ctx, U):
    """Order-independent checksum of a finalized (key, count, first) table: summed over the
    partitions of an N-rank merge it equals the single-GPU table's (count = sum, first = min are
    exact), so N>1 runs are checked against N=1 on every row, not just the unique count."""
    import torch

    if not U:
        return 0
    rows = torch.empty((3, U), dtype=torch.int64, device="cuda")
    ctx.export_unique_device(rows[0].data_ptr(), rows[1].data_ptr(), rows[2].data_ptr(), U)
    h = rows[0] * -7046029254386353131 + rows[1] * 0x2545F4914F6CDD1D + rows[2] * -4658895280553007687
    h = h ^ (h >> 29)
    return int(h.sum().item())


def reads_idx2(args, sheet):
    """idx2 as the synthetic reads carry it: with --rc the samples of synth.CFG3_RC_NAMES read rc(idx2)."""
    from frender_amd import synth
    return synth.read_idx2(sheet, synth.CFG3_RC_NAMES if args.rc else None)


def load_traffic(path, tree, per_launch_bytes, samples, index_len, combinatorial):
    """(HBM bytes per launch, note, VALU dict) from a PMC traffic file (scripts/make_traffic.py), or
    (None, why, None): a file measured on another source tree (frender_amd._lib.source_tree_hash) or
    launch shape is refused, never reported."""
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC traffic file", None
    name = os.path.basename(path)
    if tj.get("tree_hash") != tree:
        return None, f"refused {name}: measured on tree {tj.get('tree_hash')}, this tree is {tree}", None
    if not (tj.get("algorithmic_bytes_per_launch") == per_launch_bytes and tj.get("samples") == samples
            and tj.get("index_len") == index_len and bool(tj.get("combinatorial")) == combinatorial):
        return None, f"refused {name}: measured on another launch shape", None
    return tj.get("hbm_bytes_per_launch"), (f"{name} (tree {tree}): FETCH_SIZE x2 + WRITE_SIZE per launch, "
                                            f"{tj.get('traffic_over_algorithmic')}x algorithmic"), tj.get("valu")


# The chip's wave64 VALU issue rates, measured in steady state (round 6: scripts/ubench_valu.hip's deadline mode --
# every wave runs until a common s_memrealtime deadline and only instructions inside the window count, so the
# launch ramp and tail are outside; profiles/r06_ubench_valu.txt).  At 4 waves/SIMD (the tally's occupancy) and
# 2.35-2.38 GHz: VOP2-class v_and / v_add / v_lshrrev 0.42-0.49 inst/cycle/SIMD (~2 cycles each), v_bitop3 and
# v_cndmask ~3 cycles, and v_perm, v_dot4, DPP, v_ffbl, 64-bit shifts and adds, v_alignbit/byte, v_or3, v_lshl_or,
# v_bcnt, v_min and the multiplies 0.246-0.248 (4 cycles each: 600 G/s chip-wide); the tally's classify mix 0.275.
# (The round-4 figure of 647 G/s for v_and was a wall-clock rate over a launch whose waves overlapped 2.5 of 4.)
# The bound the kernel meets is the SIMDs' VALU-busy share: SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves)
# over the SIMD quad-cycles of the launch.
VALU_PEAK_G = 600.0   # 4-cycle class (v_perm, v_dot4, ... : most of the tally's VALU), 4 waves/SIMD, steady state
VALU_MIX_G = 666.2    # the tally's classify mix (v_perm, v_dot4, masks), 4 waves/SIMD, steady state
SIMD_CLOCK_GHZ = 2.35  # in-kernel shader clock under load (s_memtime / s_memrealtime, profiles/r06_ubench_valu.txt)
NUM_SIMDS = 1024


def valu_roofline(valu, per_launch_ms):
    """The kernel's second bound: VALU issue.  SQ_INSTS_VALU per launch (the same PMC file, same tree)
    over this run's measured launch time against the 4-cycle class's steady-state rate (600 G/s) and the
    classify mix's (666 G/s); simd_valu_busy = SQ_ACTIVE_INST_VALU quad-cycles over the launch's SIMD
    quad-cycles.  None without a VALU pass for this tree."""
    if not valu or not valu.get("insts_per_launch") or per_launch_ms <= 0:
        return None
    g = valu["insts_per_launch"] / (per_launch_ms / 1e3) / 1e9
    busy = None
    if valu.get("active_quad_cycles_per_launch"):  # the SIMDs' VALU-busy share of the launch
        busy = round(4.0 * valu["active_quad_cycles_per_launch"] /
                     (NUM_SIMDS * per_launch_ms * 1e-3 * SIMD_CLOCK_GHZ * 1e9), 4)
    return {"achieved": round(g, 1), "peak": VALU_PEAK_G, "unit": "G wave64 VALU inst/s",
            "frac": round(g / VALU_PEAK_G, 4), "mix_ceiling_4waves": VALU_MIX_G,
            "frac_of_mix_ceiling": round(g / VALU_MIX_G, 4), "insts_per_record": valu.get("insts_per_record"),
            "simd_valu_busy": busy}


def _gz(chunk: bytes) -> bytes:
    import gzip

    return gzip.compress(chunk, compresslevel=1)


_E2E = None


def e2e_scan(args, ns, d, n, cores):
    """The product `scan` command (frender_amd.scan.frender_scan: native inflate threads, GPU tally and
    classify, CSV writers) on the CPU baseline's own .fastq.gz files and cores: the end-to-end rate a
    user gets from compressed files (host-inflate-bound; `value` is the HBM-resident rate).  Run
    twice: the first run includes the context's creation (cold), the second is timed warm."""
    import argparse
    import contextlib
    import io

    from frender_amd import scan as S

    times = []
    for k in range(2):
        out = os.path.join(d, f"gpu{k}")
        os.mkdir(out)
        cwd = os.getcwd()
        os.chdir(out)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                t0 = time.perf_counter()
                S.frender_scan(argparse.Namespace(**vars(ns)))
                times.append(time.perf_counter() - t0)
        finally:
            os.chdir(cwd)
    def contents(sub):  # output names carry the run's minute: compare the files' bytes, not their names
        return sorted(open(os.path.join(d, sub, f), "rb").read() for f in os.listdir(os.path.join(d, sub)))

    same = contents("gpu1") == contents("out")
    return {"value": round(n / times[1] / 1e6, 3), "unit": "M reads/s", "cold_value": round(n / times[0] / 1e6, 3),
            "cores": cores, "outputs_equal_cpu_baseline": same,
            "sample": f"`scan -c {cores}` (frender_amd.scan.frender_scan: native inflate, GPU tally + classify, CSV) "
                      f"on the cpu_baseline's {cores} .fastq.gz files ({n} reads, gzip level 1); value = warm run, "
                      f"cold_value = first run incl. context creation; host-inflate-bound"}


def e2e_single(ns, d, path, n):
    """The product `scan` on the same records as ONE single-member .fastq.gz (one NovaSeq lane's shape):
    with `-c 16` every pool thread decodes the member together (fr_pinflate.h, the parallel single-member
    inflate), with `-c 1` one thread decodes it (the rate before the parallel decoder).  Each is run
    twice and timed warm; CSV contents are compared with the CPU baseline's (8-file) outputs."""
    import argparse
    import contextlib
    import io

    from frender_amd import _lib
    from frender_amd import scan as S

    out = {"unit": "M reads/s", "sample": f"{n} reads as one single-member gzip -1 .fastq.gz "
                                          f"({os.path.getsize(path)} B compressed)"}
    for cores in (16, 1):
        times = []
        for k in range(2):
            sub = os.path.join(d, f"single_c{cores}_{k}")
            os.mkdir(sub)
            cwd = os.getcwd()
            os.chdir(sub)
            before = _lib.gz_parallel_members()
            try:
                with contextlib.redirect_stdout(io.StringIO()):
                    t0 = time.perf_counter()
                    S.frender_scan(argparse.Namespace(**dict(vars(ns), c=float(cores), files=[path])))
                    times.append(time.perf_counter() - t0)
            finally:
                os.chdir(cwd)
            parallel = _lib.gz_parallel_members() > before
        same = sorted(open(os.path.join(d, sub, f), "rb").read() for f in os.listdir(os.path.join(d, sub))) == \
            sorted(open(os.path.join(d, "out", f), "rb").read() for f in os.listdir(os.path.join(d, "out")))
        out[f"c{cores}"] = {"value": round(n / times[1] / 1e6, 3), "cold_value": round(n / times[0] / 1e6, 3),
                            "cores": cores, "parallel_inflate": parallel, "outputs_equal_cpu_baseline": same}
    out["speedup_c16_over_c1"] = round(out["c16"]["value"] / out["c1"]["value"], 2)
    return out


def cpu_baseline(args, ctx, sheet, reclen):
    """The reference's CPU path, as restated by the oracle port (oracle.frender_oracle.scan: a
    Pool of `cores` workers over the input files, gzip text reader, tally, classify, CSV, exactly
    the reference's frender_scan structure, frender.py:189-193, :606-630), timed on this box's host
    cores over a bounded sample of the same workload: the first --cpu-reads SYN-v1 records
    (generated by the device generator, which the tests pin byte-identical to the host one) split
    into `cores` .fastq.gz files.  profiles/cpu_ref_vs_port.json (scripts/cpu_ref_vs_port.py, run
    where the reference is importable) calibrates this port against the reference itself."""
    import argparse
    import contextlib
    import io
    import tempfile
    from multiprocessing import Pool

    from oracle import frender_oracle as O

    n = args.cpu_reads
    cores = args.cpu_cores
    dev = ctx.device_alloc(n * reclen + 64)
    ctx.synth_device(dev, 0, n, args.read_len, 1, sheet.idx1, reads_idx2(args, sheet))
    data = ctx.copy_to_host(dev, n * reclen)
    ctx.device_free(dev)
    cuts = [n * i // cores for i in range(cores + 1)]
    with tempfile.TemporaryDirectory() as d:
        sheet.write_csv(os.path.join(d, "sheet.csv"))
        with Pool(cores) as pool:
            blobs = pool.map(_gz, [data[cuts[i] * reclen:cuts[i + 1] * reclen] for i in range(cores)])
        single = None
        if not args.no_single:  # the same records as ONE single-member .fastq.gz (gzip -1 of the whole text)
            os.mkdir(os.path.join(d, "single"))
            single = os.path.join(d, "single", "syn_L001_R1_001.fastq.gz")
            with open(single, "wb") as f:
                f.write(_gz(data))
        del data
        files = []
        for i, blob in enumerate(blobs):
            files.append(os.path.join(d, f"syn_L{i + 1:03d}_R1_001.fastq.gz"))
            with open(files[-1], "wb") as f:
                f.write(blob)
        del blobs
        out = os.path.join(d, "out")
        os.mkdir(out)
        ns = argparse.Namespace(n=args.nsubs, rc=args.rc, c=float(cores), s=None, o="cpu", p=None,
                                b=os.path.join(d, "sheet.csv"), files=files)
        cwd = os.getcwd()
        os.chdir(out)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                t0 = time.perf_counter()
                O.scan(ns)
                dt = time.perf_counter() - t0
        finally:
            os.chdir(cwd)
        e2e = e2e_scan(args, ns, d, n, cores)
        if single:
            e2e["single_member"] = e2e_single(ns, d, single, n)
    global _E2E
    _E2E = e2e
    cal = ""
    try:
        with open(os.path.join(ROOT, "profiles", "cpu_ref_vs_port.json")) as f:
            c = json.load(f)
        cal = (f"; calibration (scripts/cpu_ref_vs_port.py, build container, {c['cores']} cores, {c['reads']} reads): "
               f"reference {c['reference_scan_M_reads_per_s']} vs port {c['port_scan_M_reads_per_s']} M reads/s "
               f"(port/reference time ratio {c['port_scan_over_reference']}, outputs identical: {c['outputs_identical']})")
    except (OSError, KeyError, ValueError):
        pass
    return {"value": round(n / dt / 1e6, 4), "unit": "M reads/s", "cores": cores, "kind": "port",
            "sample": f"the reference's scan command restated (oracle.frender_oracle.scan: Pool over files, gzip, "
                      f"tally, classify, CSV) on the first {n} SYN-v1 reads of the workload ({args.samples} samples, "
                      f"{args.index_len}+{args.index_len}bp, n={args.nsubs}, R={args.read_len}) as {cores} .fastq.gz "
                      f"files (level 1), {cores} workers: {dt:.2f} s{cal}"}


def _cfg5_write(job):
    from frender_amd import synth

    path, r0, n, mate = job
    t = synth.generate_bytes(synth.make_sheet(96, 8, 8), r0, n, R=150, seed=5)
    if mate == 2:
        t = t.replace(b" 1:N:0:", b" 2:N:0:")
    synth.write_fastq_gz(path, t, level=1)
    return os.path.getsize(path)


def cfg5(args):
    """--cfg5: BASELINE config 5's shape (96 samples, 8+8 bp, n=1, paired-end R=150 per mate) end to end
    on this box -- not the headline metric (config 5 is quoted on 8 GPUs over 500M pairs).  Product: the
    scan and demux command lines (`python -m frender_amd`, each paying its Python start and GPU
    context) over --cfg5-files level-1 .fastq.gz file pairs, demux writing the reference's level-9
    gzip.  CPU baseline: the reference's scan + demux as restated by the oracle (scan: Pool of 8 over
    files; demux: one process, gzip.open writers, one write per line, frender.py:667-676, :726-814), on
    the first --cfg5-cpu-pairs pairs.  One JSON line."""
    import contextlib
    import io
    import subprocess
    import tempfile
    from concurrent.futures import ProcessPoolExecutor

    from frender_amd import synth
    from oracle import demux_oracle as D
    from oracle import frender_oracle as O

    n, fp = args.cfg5_pairs, args.cfg5_files
    per = n // fp
    cpu_n = min(args.cfg5_cpu_pairs, per)
    with tempfile.TemporaryDirectory() as d:
        sheet = synth.make_sheet(96, 8, 8)
        csv_path = os.path.join(d, "sheet.csv")
        sheet.write_csv(csv_path)
        os.mkdir(os.path.join(d, "in"))
        os.mkdir(os.path.join(d, "cpu_in"))
        jobs = [(os.path.join(d, "in", f"syn_L{p + 1:03d}_R{m}_001.fastq.gz"), p * per, per, m)
                for p in range(fp) for m in (1, 2)]
        jobs += [(os.path.join(d, "cpu_in", f"syn_L001_R{m}_001.fastq.gz"), 0, cpu_n, m) for m in (1, 2)]
        with ProcessPoolExecutor(8) as ex:
            in_bytes = sum(ex.map(_cfg5_write, jobs))
        r1 = sorted(os.path.join(d, "in", x) for x in os.listdir(os.path.join(d, "in")) if "_R1_" in x)
        allf = sorted(os.path.join(d, "in", x) for x in os.listdir(os.path.join(d, "in")))
        work = os.path.join(d, "gpu")
        os.mkdir(work)
        env = dict(os.environ, PYTHONPATH=ROOT)
        t0 = time.perf_counter()
        cores = str(max(1, min(16, len(os.sched_getaffinity(0)))))  # the box's share: 16 cores per GPU
        sp = subprocess.run([sys.executable, "-m", "frender_amd", "scan", "-n", "1", "-c", cores, "-o", "cfg5", "-b",
                             csv_path, *r1], cwd=work, env=env, capture_output=True, text=True)
        t1 = time.perf_counter()
        if sp.returncode:
            raise SystemExit(f"cfg5 scan failed: {sp.stderr[-2000:]}")
        res = [os.path.join(work, x) for x in os.listdir(work) if x.endswith(".csv")]
        dm = subprocess.run([sys.executable, "-m", "frender_amd", "demux", "-r", res[0], "-d",
                             os.path.join(work, "out"), "--stage-times", *allf], cwd=work, env=env,
                            capture_output=True, text=True)
        t2 = time.perf_counter()
        if dm.returncode:
            raise SystemExit(f"cfg5 demux failed: {dm.stderr[-2000:]}")
        stages = next((json.loads(x) for x in reversed(dm.stderr.splitlines()) if x.startswith("{")), None)
        out_bytes = sum(os.path.getsize(os.path.join(work, "out", x)) for x in os.listdir(os.path.join(work, "out")))
        # the CPU baseline on the first cpu_n pairs (one file pair)
        cwork = os.path.join(d, "cpu")
        os.mkdir(cwork)
        c1 = os.path.join(d, "cpu_in", "syn_L001_R1_001.fastq.gz")
        c2 = os.path.join(d, "cpu_in", "syn_L001_R2_001.fastq.gz")
        cwd = os.getcwd()
        os.chdir(cwork)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                u0 = time.perf_counter()
                O.scan(argparse.Namespace(n=1, rc=False, c=8.0, s=None, o="cpu", p=None, b=csv_path, files=[c1]))
                u1 = time.perf_counter()
                cres = [x for x in os.listdir(cwork) if x.endswith(".csv")][0]
                D.demux(argparse.Namespace(r=cres, d=os.path.join(cwork, "out"), o=None, no_index_hop=False,
                                           no_ambiguous=False, no_undeter=False, no_samples=False, strict_header=False,
                                           files=[c1, c2]), write_files=True)
                u2 = time.perf_counter()
        finally:
            os.chdir(cwd)
    return {"metric": "M read pairs/s scan+demux (BASELINE config 5 shape: 96 samples, 8+8bp, n=1, paired R=150)",
            "value": round(n / (t2 - t0) / 1e6, 4), "unit": "M read pairs/s", "n_gpus": 1,
            "higher_is_better": True, "data": "synthetic (SYN-v1, R=150 per mate, level-1 .fastq.gz inputs)",
            "config": {"workload": f"{n} read pairs in {fp} file pairs; scan -n 1 -c {cores}, then demux (gzip writers "
                                   f"deflated on the GPU, no larger than the reference's zlib level 9)",
                       "in_gz_bytes": in_bytes},
            "scan_s": round(t1 - t0, 3), "demux_s": round(t2 - t1, 3),
            "demux_M_pairs_per_s": round(n / (t2 - t1) / 1e6, 4), "demux_stages_s": stages,
            "out_gz_bytes": out_bytes,
            "cpu_baseline": {"value": round(cpu_n / (u2 - u0) / 1e6, 5), "unit": "M read pairs/s", "cores": 8,
                             "kind": "port", "scan_s": round(u1 - u0, 3), "demux_s": round(u2 - u1, 3),
                             "demux_M_pairs_per_s": round(cpu_n / (u2 - u1) / 1e6, 5),
                             "sample": f"oracle.frender_oracle.scan (Pool of 8 over the files) + oracle.demux_oracle."
                                       f"demux(write_files=True) (one process: the reference's demux loop has no "
                                       f"Pool) on the first {cpu_n} pairs (one file pair)"},
            "note": "two CLI processes for the product (each pays its Python/torch start and GPU context)"}


PIN_FILES = {"BASELINE config 2": "cfg2_pin.json", "BASELINE config 3 shape (384 samples, 10+10, -rc)": "cfg3_pin.json",
             "BASELINE config 4 shape (96 combinatorial, n=2)": "cfg4_pin.json"}


def pin_path(args):
    if args.pin_json:
        return args.pin_json
    f = PIN_FILES.get(config_name(args).split(" as ")[0])  # K files hold the same rows in the same order
    return os.path.join(ROOT, "tests", "golden", f) if f else None


def pin_check(args, ctx, sheet):
    """At N=1 on a pinned shape (BASELINE config 2, the config-3 and config-4 shapes at the pin's read
    count), the benchmarked table (the last timed step's), classified by the reference's own sequence
    (synth.pin_rows: process; with -rc pass A, the per-name call, the idx2 rewrite and pass B), must
    equal the reference's rows on the same records (tests/golden/cfg*_pin.json: unique codes, sha256
    over every row in order, first/last 1000 rows; with -rc also pass A's rows and every rc call).
    Outside the timed region."""
    from frender_amd import synth

    path = pin_path(args)
    with open(path) as f:
        pin = json.load(f)
    if pin.get("reads", args.reads) != args.reads:
        return None
    got = synth.pin_rows(ctx, sheet, args.nsubs, args.rc)
    bad = synth.pin_differences(got, pin)
    if bad:
        raise SystemExit(f"bench: the benchmarked table differs from the reference's rows ({path}): {bad}; "
                         f"{got['unique_codes']} vs {pin['unique_codes']} codes")
    return {"file": os.path.relpath(path, ROOT), "unique_codes": pin["unique_codes"], "rows_sha256": got["rows_sha256"],
            "equal": True, "rc_calls_equal": True if args.rc else None,
            "source": f"reference frender.py tally_barcodes + process{' (+ rc call and pass B)' if args.rc else ''} on "
                      f"the same records (imported in the build container by {pin.get('generated_by', '').split(':')[0]})"}


def rank_check(world):
    """--rank-check: the launcher's ranks meet over gloo; rank 0 prints the world size they agree on."""
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    t = torch.ones(1, dtype=torch.int64)
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"rank_check": True, "world": world, "ranks_joined": int(t.item())}), flush=True)
    dist.destroy_process_group()
    return 0


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # `bench.py --gpus N` without a launcher: one child rank per GPU, before anything touches a GPU
        from frender_amd.dist import launch_ranks
        return launch_ranks(args.gpus, sys.argv[1:], cmd=[sys.executable, os.path.abspath(__file__)])
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a measurement of "
              f"{world} GPU(s) as {args.gpus}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cfg5:
        print(json.dumps(cfg5(args)), flush=True)
        return 0
    if args.rank_check:
        return rank_check(world) if world > 1 else (print(json.dumps({"rank_check": True, "world": 1,
                                                                      "ranks_joined": 1})) or 0)
    dist = None
    if args.merge_leg and world == 1:  # a one-rank RCCL group: the merge leg's collectives on device tensors
        import socket

        import torch
        import torch.distributed as dist
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif world > 1:
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
    from frender_amd.dist import device_callbacks, gather_rows, partition_merge_device, reduce_sum, tree_merge
    from frender_amd.host import reverse_complement
    from frender_amd.scan import _sheet_names

    sheet = synth.make_sheet(args.samples, args.index_len, args.index_len,
                             combinatorial=(12, 8) if args.combinatorial else None)
    reclen = synth.record_length(args.index_len, args.index_len, args.read_len)
    n = args.reads
    nbytes = n * reclen
    # launches of up to 16 GiB: the first feed (no history) is cut into ranges <= 4 GiB that may log;
    # once a feed's commits did not log, a feed is one launch (fr_feed_device)
    tuning = {k: int(v) for k, v in (kv.split("=", 1) for kv in args.tuning.split(",") if kv)}
    ctx = _lib.Context(device=local, chunk_bytes=(args.launch_gib << 30) - (1 << 20), table_slots=1 << 22,
                       tuning=tuning or None)
    buf = ctx.device_alloc(nbytes + 64)
    # with --rc the reads of synth.CFG3_RC_NAMES carry rc(idx2) (the sheet is unchanged), so the per-name
    # call flips those samples and pass B classifies against the rewritten idx2 list (tests/golden/cfg3_pin.json)
    ctx.synth_device(buf, rank * n, n, args.read_len, 1, sheet.idx1, reads_idx2(args, sheet))
    names, nid = _sheet_names(sheet.ids)
    merge_cbs = device_callbacks(ctx)
    wire = "cpu" if args.dist_backend == "gloo" else "cuda"  # where small collectives' tensors live
    idx2rc = [reverse_complement(x) for x in sheet.idx2]

    # --files K: record cuts at multiples of 8 records (device feeds start 16-byte aligned: 8 x 74 B = 37 x 16 B)
    cuts = [(n * i // max(args.files, 1)) // 8 * 8 for i in range(max(args.files, 1))] + [n]
    tally_timing = []
    timing_on = [False]  # the step whose tally launches are timed (the last timed one) reads them back

    def step():
        ctx.reset()
        # rank r's records are the byte range [r n reclen, (r+1) n reclen) of one logical file:
        # global ordinals, so the merged first-occurrence order is the single-GPU one
        if args.files <= 1:
            ctx.begin_file(None, file_index=0, byte_base=rank * nbytes)
            ctx.feed_device(buf, nbytes)
            st = ctx.end_file()
            assert st.records == n and st.error == 0, (st.records, st.error)
        else:  # --files K: the same records as K consecutive files (per-file presence scans at each file's end)
            for i in range(args.files):
                ctx.begin_file(None, file_index=rank * args.files + i, byte_base=0)
                ctx.feed_device(buf + cuts[i] * reclen, (cuts[i + 1] - cuts[i]) * reclen)
                st = ctx.end_file()
                assert st.records == cuts[i + 1] - cuts[i] and st.error == 0, (i, st.records, st.error)
        if timing_on[0] or not tally_timing:  # the tally launches of this step (the merge resets the context)
            tally_timing[:] = [ctx.timing()]
        U, _, _ = ctx.finalize()
        classify_here = True
        if world > 1 and args.merge == "tree":  # one exchange: binary tree into rank 0 (dist.py)
            U = tree_merge(dist, "cuda", U, *merge_cbs)
            classify_here = rank == 0
        elif world > 1 or args.merge_leg:  # one exchange: all-to-all into hash partitions (dist.py)
            phase("tally")
            U = partition_merge_device(dist, "cuda", ctx)
            phase("merge")
        if classify_here:
            ctx.set_sheet(sheet.idx1, sheet.idx2, idx2rc, nid, len(names))
            ctx.classify(args.nsubs, args.rc, to_host=False)
            if args.rc:
                f, r = ctx.rc_counts()
                if world > 1 and args.merge == "a2a":  # per-name sums over all partitions
                    f, r = reduce_sum(dist, wire, list(f)), reduce_sum(dist, wire, list(r))
                use = [int(a) < int(b) for a, b in zip(f, r)]
                # pass B's idx2 and its reverse complements are selections (rc(rc(x)) = x)
                if any(use):
                    pick = [use[nid[i]] for i in range(len(sheet.idx2))]
                    idx2b = [c if u else x for u, x, c in zip(pick, sheet.idx2, idx2rc)]
                    idx2brc = [x if u else c for u, x, c in zip(pick, sheet.idx2, idx2rc)]
                else:  # no name takes rc: pass B's lists are pass A's
                    idx2b, idx2brc = sheet.idx2, idx2rc
                ctx.set_sheet(sheet.idx1, idx2b, idx2brc, nid, len(names))
                ctx.classify(args.nsubs, False, to_host=False)
            if args.merge_leg:  # the product's writer: every partition's rows to rank 0
                phase("classify")
                gather_rows(dist, "cuda", ctx.export_rows("cuda"))
                phase("gather")
        # (no stream sync here: fr_classify already waited for its error flags, and the timed loop is
        # bracketed by ctx.sync() + barrier on both sides)
        return U

    phase_ms = {}  # --merge-leg: per-phase ms of the extra steps after the timed ones (synchronised at each phase)
    phase_on = [False]
    phase_t = [0.0]

    def phase(name):
        if not phase_on[0]:
            return
        ctx.sync()
        now = time.perf_counter()
        phase_ms.setdefault(name, []).append((now - phase_t[0]) * 1e3)
        phase_t[0] = now

    def barrier():
        if world > 1:
            dist.barrier()

    # HIP timing events (fr_set_timing) only in the last timed step: its launches give the kernel's
    # duration (roofline); the other steps run as the product does, without the events' stream bubbles
    ctx.set_timing(False)
    for _ in range(args.warmup):
        step()
    barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - 1:
            ctx.set_timing(True)
            timing_on[0] = True
        U = step()
    ctx.sync()
    barrier()
    dt = time.perf_counter() - t0
    t_after = tally_timing[0]
    ms = dt / args.steps * 1e3
    merge_leg = None
    if args.merge_leg:  # three more steps, each phase synchronised and timed on the host
        for _ in range(3):
            ctx.sync()
            phase_t[0] = time.perf_counter()
            phase_on[0] = True
            step()
            phase_on[0] = False
        ctx.sync()
        med = {k: round(sorted(v)[len(v) // 2], 3) for k, v in phase_ms.items()}
        merge_leg = {"rows": int(U), "row_bytes": 24, "world": 1, "backend": "nccl (RCCL), one rank",
                     "ms_per_step_with_leg": round(ms, 4), "phase_ms": med,
                     "note": "phases timed with a device sync at each boundary; 'tally' = reset, tally and finalize, 'merge' = export, all-to-all, "
                             "rebuild and finalize of the partition (partition_merge_device), 'classify' = "
                             "set_sheet + classify, 'gather' = export + gather_rows to rank 0 (host copy)"}
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
    traffic, traffic_note, valu = load_traffic(args.traffic_json, _lib.source_tree_hash(), per_launch_bytes,
                                         args.samples, args.index_len, args.combinatorial)

    dg = ctx.diag()  # the last feed's launch-log folds (fullest sub-region of 4096 slots, overflowed entries)
    csum = table_checksum(ctx, U) if (world == 1 or args.merge == "a2a" or rank == 0) else 0
    if world > 1 and args.merge == "a2a":  # report the merged table's size (sum of the partitions)
        U, csum = (int(x) for x in reduce_sum(dist, wire, [U, csum]))
    csum &= (1 << 64) - 1
    pinned = None
    pp = pin_path(args)
    if world == 1 and pp and os.path.exists(pp) and not args.no_pin:
        pinned = pin_check(args, ctx, sheet)
    if rank == 0:
        cpu = None if (args.no_cpu or world > 1) else cpu_baseline(args, ctx, sheet, reclen)  # N=1 only
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
            "config": {"workload": f"{config_name(args)}: {n} SYN-v1 reads/GPU, {args.samples} samples, "
                                   f"{args.index_len}+{args.index_len}bp, n={args.nsubs}"
                                   f"{', -rc' if args.rc else ''}, R={args.read_len} ({reclen} B/record), "
                                   f"decoded FASTQ resident in HBM",
                       "reads_per_gpu": n, "bytes_per_record": reclen, "samples": args.samples,
                       "nsubs": args.nsubs, "rc": bool(args.rc), "unique_codes": int(U),
                       "table_checksum": f"{csum:016x}", "reference_pin": pinned, "tuning": tuning or None,
                       "parallelism": f"dp{world} (record shards) + {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} "
                                      + ("all-to-all hash-partitioned merge" if args.merge == "a2a" else "tree merge") if world > 1 else "1 GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_note,
                         "kernel": "fr::chunk_kernel", "bytes_per_launch": int(per_launch_bytes),
                         "avg_launch_ms": round(per_launch_ms, 4), "launches_per_step": int(launches),
                         "log_aggregation_ms_per_launch": round(t_after.log_ms / max(launches, 1), 4),
                         "log_fold": {"max": dg["fold_max"], "over": dg["fold_over"], "slots": 4096},
                         "valu_issue": valu_roofline(valu, per_launch_ms)},
            "cpu_baseline": cpu,
            "e2e": _E2E,
        }
        if merge_leg:
            out["merge_leg"] = merge_leg
        print(json.dumps(out), flush=True)
    ctx.device_free(buf)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
