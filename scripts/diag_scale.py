"""Diagnostic: device-feed SYN-v1 data at several launch sizes / totals; report records."""
import sys, time
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from frender_amd import _lib, synth

S = int(os.environ.get("DIAG_S", "96"))
L = int(os.environ.get("DIAG_L", "8"))
sheet = synth.make_sheet(S, L, L)
reclen = synth.record_length(L, L, 8)
for n in (int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000,):
    for chunk in [int(c) << 20 for c in (sys.argv[2] if len(sys.argv) > 2 else "1,16,256,512").split(",")]:
        ctx = _lib.Context(device=0, chunk_bytes=chunk, table_slots=int(os.environ.get("DIAG_SLOTS", str(1 << 22))))
        buf = ctx.device_alloc(n * reclen + 64)
        ctx.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
        ctx.reset(); ctx.begin_file(None); ctx.feed_device(buf, n * reclen); ctx.end_file()  # warm: table grown
        for grid_note in ("run",):
            ctx.reset(); ctx.begin_file(None)
            t = time.time(); ctx.feed_device(buf, n * reclen); st = ctx.end_file(); dt = time.time() - t
            U, NP, NE = ctx.finalize()
            tm = ctx.timing()
            print(f"n={n} chunk={chunk>>20}MiB records={st.records} lines={st.lines} err={st.error} "
                  f"erroff={st.error_offset} U={U} launches={tm.scan_launches} scan_ms={tm.scan_ms:.3f} log_ms={tm.log_ms:.3f} wall={dt:.3f} {ctx.diag()}",
                  flush=True)
        ctx.device_free(buf); ctx.close()
