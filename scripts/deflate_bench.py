"""GPU deflate throughput on a demux window (fr_defl over host bytes: H2D copy + kernels + D2H of the
streams), one JSON line.  The window is `mib` MiB of routed R=150 FASTQ split into `dest` destination
ranges (destination-major, as fr_dmx_route leaves a window).  Run it under rocprofv3 --kernel-trace
--stats for the kernels' own time.

usage: python scripts/deflate_bench.py [mib=512] [dest=97] [reps=3]
"""
import json
import os
import sys
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from deflate_cases import routed_fastq  # noqa: E402
from frender_amd import _lib  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dest = int(sys.argv[2]) if len(sys.argv) > 2 else 97
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    unit = routed_fastq(60000, 150)
    n = mib << 20
    data = np.frombuffer((unit * (n // len(unit) + 1))[:n], dtype=np.uint8)
    cuts = np.sort(np.random.default_rng(1).integers(0, n, dest - 1))
    offs = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    z = _lib.Deflater(0)
    comp, crc, out = z.compress(data, offs)  # warm-up (allocations)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        comp, crc, out = z.compress(data, offs)
        ts.append(time.perf_counter() - t0)
    z.close()
    s = 20 << 20
    sample = data[:s].tobytes()
    z9 = len(zlib.compress(sample, 9)) - 6
    k = int(np.searchsorted(offs, s, side="right")) - 1
    print(json.dumps({"path": "gpu_deflate", "window_MiB": mib, "streams": dest, "reps": reps,
                      "best_s": round(min(ts), 4), "GB_per_s": round(n / min(ts) / 1e9, 3),
                      "ratio": round(n / int(comp.sum()), 4),
                      "zlib9_ratio_first_20MiB": round(s / z9, 4),
                      "note": "wall time of fr_defl_run_host + fr_defl_fetch (H2D, kernels, D2H); streams "
                              f"{k} of {dest} cover the zlib sample"}), flush=True)


if __name__ == "__main__":
    main()
