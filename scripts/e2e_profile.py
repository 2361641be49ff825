"""cProfile of one `scan` over F .fastq.gz files (where the end-to-end time goes).
usage: e2e_profile.py [reads] [files]  (default 24M reads in 8 files: the bench cpu_baseline / e2e shape)"""
import cProfile
import os
import pstats
import sys
import tempfile
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from frender_amd import synth  # noqa: E402
from frender_amd.scan import frender_scan  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 24_000_000
files = int(sys.argv[2]) if len(sys.argv) > 2 else 8
sheet = synth.make_sheet(96, 8, 8)
with tempfile.TemporaryDirectory() as d:
    paths = synth.make_dataset(d, sheet, n, n_files=files, R=8, seed=1, level=1)
    sheet.write_csv(os.path.join(d, "sheet.csv"))
    args = types.SimpleNamespace(files=paths, b=os.path.join(d, "sheet.csv"), n=1, c=files, s=None, rc=False, o=None, p=None)
    os.chdir(d)
    frender_scan(args)  # warm (context, kernels)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    frender_scan(args)
    pr.disable()
    print("scan s", round(time.perf_counter() - t0, 3))
    pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
    pstats.Stats(pr).sort_stats("tottime").print_stats(20)
