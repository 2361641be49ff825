"""Diagnostic: device-feed SYN-v1 data at several launch sizes / totals; report records."""
import sys, time
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from frender_amd import _lib, synth

sheet = synth.make_sheet(96, 8, 8)
reclen = synth.record_length(8, 8, 8)
for n in (int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000,):
    for chunk in [int(c) << 20 for c in (sys.argv[2] if len(sys.argv) > 2 else "1,16,256,512").split(",")]:
        ctx = _lib.Context(device=0, chunk_bytes=chunk, table_slots=1 << 22)
        buf = ctx.device_alloc(n * reclen + 64)
        ctx.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
        for grid_note in ("run",):
            ctx.reset(); ctx.begin_file(None)
            t = time.time(); ctx.feed_device(buf, n * reclen); st = ctx.end_file(); dt = time.time() - t
            U, NP, NE = ctx.finalize()
            tm = ctx.timing()
            print(f"n={n} chunk={chunk>>20}MiB records={st.records} lines={st.lines} err={st.error} "
                  f"erroff={st.error_offset} U={U} launches={tm.scan_launches} scan_ms={tm.scan_ms:.3f} wall={dt:.3f} {ctx.diag()}",
                  flush=True)
        ctx.device_free(buf); ctx.close()
