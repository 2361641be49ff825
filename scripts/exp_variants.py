"""A/B of tally-kernel build variants (scripts/build_exp.sh NAME FLAGS -> libfrender_hip_exp_NAME.so).

usage: python scripts/exp_variants.py NAME [NAME ...]     (env: READS, ROUNDS, SHAPES="96:8,384:10")
Each variant runs in its own process (one library per process), rounds interleaved (rule: perf deltas
from interleaved rounds).  Per shape: device-fed SYN-v1 records, one reset + tally + finalize per
repetition; prints the tally ms per 100M reads (median of 5), the unique count and an order-free
checksum of every (key, count, first) row, so a variant with a different table shows up at once.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys, statistics
sys.path.insert(0, ROOT)
import numpy as np
from frender_amd import _lib, synth
n = int(os.environ.get("READS", "100000000"))
out = {}
for shape in os.environ.get("SHAPES", "96:8,384:10").split(","):
    S, L = (int(x) for x in shape.split(":"))
    sheet = synth.make_sheet(S, L, L)
    reclen = synth.record_length(L, L, 8)
    ctx = _lib.Context(device=0, chunk_bytes=3900 << 20)
    buf = ctx.device_alloc(n * reclen + 64)
    ctx.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
    ms = []
    for rep in range(6):
        ctx.reset(); ctx.begin_file(None); ctx.feed_device(buf, n * reclen); ctx.end_file()
        U, NP, NE = ctx.finalize()
        t = ctx.timing()
        if rep:
            ms.append((t.scan_ms + t.log_ms) * 1e8 / n)
    k, c, f = (np.asarray(x, dtype=np.uint64) for x in ctx.unique()[:3])
    h = k * np.uint64(0x9E3779B97F4A7C15) ^ c * np.uint64(0xBF58476D1CE4E5B9) ^ f * np.uint64(0x94D049BB133111EB)
    out[shape] = {"ms_per_100M": round(statistics.median(ms), 4), "min": round(min(ms), 4), "U": int(U),
                  "tally_ms": round(t.scan_ms * 1e8 / n, 4), "log_ms": round(t.log_ms * 1e8 / n, 4),
                  "csum": int(np.bitwise_xor.reduce(h ^ (h >> np.uint64(29)))) if U else 0}
    ctx.device_free(buf); ctx.close()
print("RESULT " + json.dumps(out), flush=True)
'''


def main():
    names = sys.argv[1:]
    rounds = int(os.environ.get("ROUNDS", "2"))
    res = {nm: [] for nm in names}
    for r in range(rounds):
        for nm in names:
            base, *kv = nm.split("@")  # NAME@VAR=VALUE@...: the variant with extra environment
            lib = os.path.join(ROOT, "frender_amd", f"libfrender_hip_exp_{base}.so") if base != "main" else \
                os.path.join(ROOT, "frender_amd", "libfrender_hip.so")
            env = dict(os.environ, FRENDER_HIP_LIB=lib, **dict(x.split("=", 1) for x in kv))
            p = subprocess.run([sys.executable, "-c", "ROOT=%r\n" % ROOT + CHILD], env=env, capture_output=True,
                               text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(f"{nm}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[0][7:])
            res[nm].append(d)
            print(f"round {r} {nm}: {d}", flush=True)
    print("SUMMARY " + json.dumps({nm: v[-1] for nm, v in res.items()}))


if __name__ == "__main__":
    main()
