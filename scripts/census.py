"""Collective census of a multi-rank `scan`: how many collectives a scan makes, of which
kind, how long each kind blocks and how many bytes it moves, per rank.

Writes FILES level-1 .fastq.gz files of READS SYN-v1 records each (96 samples, 8+8 bp), then runs the
product command `python -m frender_amd scan -n 1 -c FILES --gpus N` with FRENDER_DIST_CENSUS=1 (and
FRENDER_DIST_BACKEND, default gloo: N ranks rehearsed on one GPU), once per N in GPUS, and prints one
JSON object: wall time per N and each rank's census (dist.CENSUS).
usage: GPUS="1 2" FILES=4 READS=1000000 python scripts/census.py
"""
import gzip
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from frender_amd import synth
    nfiles = int(os.environ.get("FILES", "4"))
    reads = int(os.environ.get("READS", "1000000"))
    gpus = [int(x) for x in os.environ.get("GPUS", "1 2").split()]
    sheet = synth.make_sheet(96, 8, 8)
    out = {"files": nfiles, "reads_per_file": reads, "backend": os.environ.get("FRENDER_DIST_BACKEND", "gloo"),
           "runs": {}}
    with tempfile.TemporaryDirectory() as d:
        sheet.write_csv(os.path.join(d, "sheet.csv"))
        files = []
        for i in range(nfiles):
            files.append(os.path.join(d, f"syn_L{i + 1:03d}_R1_001.fastq.gz"))
            with open(files[-1], "wb") as f:
                f.write(gzip.compress(synth.generate_bytes(sheet, i * reads, reads, R=8), compresslevel=1))
        for n in gpus:
            wd = os.path.join(d, f"out{n}")
            os.mkdir(wd)
            env = dict(os.environ, FRENDER_DIST_CENSUS="1", PYTHONPATH=ROOT,
                       FRENDER_DIST_BACKEND=os.environ.get("FRENDER_DIST_BACKEND", "gloo"))
            t0 = time.perf_counter()
            p = subprocess.run([sys.executable, "-m", "frender_amd", "scan", "-n", "1", "-c", str(nfiles),
                                "--gpus", str(n), "-b", os.path.join(d, "sheet.csv")] + files,
                               cwd=wd, env=env, capture_output=True, text=True, timeout=600)
            dt = time.perf_counter() - t0
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                return 1
            ranks = [json.loads(line[len("census "):]) for line in p.stderr.splitlines() if line.startswith("census ")]
            tot = {}
            for r in ranks:
                for k, v in r["collectives"].items():
                    t = tot.setdefault(k, {"calls": 0, "ms_max_rank": 0.0})
                    t["calls"] = max(t["calls"], v["calls"])
                    t["ms_max_rank"] = max(t["ms_max_rank"], round(v["ms"], 2))
            out["runs"][n] = {"wall_s": round(dt, 3), "per_kind": tot,
                              "ranks": sorted(ranks, key=lambda r: r["rank"]),
                              "csv": sorted(os.listdir(wd))}
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
