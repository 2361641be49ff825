"""BASELINE config 5 shape, end to end on this box (one JSON line per run): paired-end .fastq.gz
inputs (96 samples, 8+8 bp dual index, R=150 per mate, level-1 gzip, `pairs` file pairs) -> the
product `scan` (n=1, native inflate + GPU tally + classify + CSV) -> the product `demux` (native
inflate, GPU routing, per-sample .fq.gz writers), both through `python -m frender_amd` like a user's
command line.  Config 5 is quoted on 8 GPUs over 500M pairs; this is its per-GPU shape at a size one
box finishes in a minute: M pairs/s for the whole scan + demux, and each stage's seconds.

usage: python scripts/e2e_cfg5.py [pairs_total] [file_pairs] [gz_level ...]
"""
import json
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from frender_amd import synth  # noqa: E402


def _write(job):
    path, r0, n, mate = job
    sheet = synth.make_sheet(96, 8, 8)
    t = synth.generate_bytes(sheet, r0, n, R=150, seed=5)
    if mate == 2:
        t = t.replace(b" 1:N:0:", b" 2:N:0:")
    synth.write_fastq_gz(path, t, level=1)
    return os.path.getsize(path)


def run(d, n, pairs, level, gpus=1):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r1 = sorted(os.path.join(d, x) for x in os.listdir(d) if "_R1_" in x)
    allf = sorted(os.path.join(d, x) for x in os.listdir(d) if x.endswith(".fastq.gz"))
    work = tempfile.mkdtemp(dir=d)
    t0 = time.perf_counter()
    s = subprocess.run([sys.executable, "-m", "frender_amd", "scan", "-n", "1", "-c", str(pairs), "-o", "cfg5",
                        "-b", os.path.join(d, "sheet.csv"), "--gpus", str(gpus), *r1],
                       cwd=work, env=env, capture_output=True, text=True)
    t1 = time.perf_counter()
    assert s.returncode == 0, s.stderr[-2000:]
    res = [os.path.join(work, x) for x in os.listdir(work) if x.endswith(".csv") and "rc-mode" not in x]
    assert len(res) == 1, os.listdir(work)
    m = subprocess.run([sys.executable, "-m", "frender_amd", "demux", "-r", res[0], "-d", os.path.join(work, "out"),
                        "--gz-level", str(level), "--gpus", str(gpus), *allf],
                       cwd=work, env=env, capture_output=True, text=True)
    t2 = time.perf_counter()
    assert m.returncode == 0, m.stderr[-2000:]
    outs = os.listdir(os.path.join(work, "out"))
    out_bytes = sum(os.path.getsize(os.path.join(work, "out", x)) for x in outs)
    return {"path": "cfg5_scan_demux", "read_pairs": n, "file_pairs": pairs, "gpus": gpus, "gz_level": level,
            "scan_s": round(t1 - t0, 3), "demux_s": round(t2 - t1, 3), "total_s": round(t2 - t0, 3),
            "M_pairs_per_s": round(n / (t2 - t0) / 1e6, 4), "demux_M_pairs_per_s": round(n / (t2 - t1) / 1e6, 4),
            "out_files": len(outs), "out_gz_bytes": out_bytes,
            "note": "two CLI processes (each pays its python/torch start and GPU context); inputs level-1 gzip"}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    levels = [int(x) for x in sys.argv[3:]] or [9, 1]
    per = n // pairs
    with tempfile.TemporaryDirectory() as d:
        sheet = synth.make_sheet(96, 8, 8)
        sheet.write_csv(os.path.join(d, "sheet.csv"))
        jobs = [(os.path.join(d, f"syn_L{p + 1:03d}_R{m}_001.fastq.gz"), p * per, per, m)
                for p in range(pairs) for m in (1, 2)]
        with ProcessPoolExecutor(min(8, len(jobs))) as ex:
            in_bytes = sum(ex.map(_write, jobs))
        for lvl in levels:
            line = run(d, per * pairs, pairs, lvl)
            line["in_gz_bytes"] = in_bytes
            print(json.dumps(line), flush=True)
