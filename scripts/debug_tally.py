"""Debug: tiny host and device feeds through the tally kernel, one step at a time (prints flush)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from frender_amd import _lib, synth  # noqa: E402

step = sys.argv[1] if len(sys.argv) > 1 else "host"
print("start", step, flush=True)
ctx = _lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16)
print("ctx ok", flush=True)
data = b"@r1 1:N:0:ACGT+TTTT\nACGT\n+\nFFFF\n" * 3
if step == "host":
    ctx.reset()
    ctx.begin_file(None)
    print("feeding", flush=True)
    ctx.feed(data)
    print("fed", flush=True)
    st = ctx.end_file()
    print("end_file", st.records, st.lines, st.error, flush=True)
    print(ctx.finalize(), flush=True)
    print(ctx.unique(), flush=True)
elif step == "device":
    sheet = synth.make_sheet(96, 8, 8)
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    host = synth.generate_bytes(sheet, 0, n, R=8, seed=1)
    p = ctx.device_alloc(len(host))
    ctx.synth_device(p, 0, n, 8, 1, sheet.idx1, sheet.idx2)
    ctx.reset()
    ctx.begin_file(None)
    t = time.time()
    ctx.feed_device(p, len(host))
    st = ctx.end_file()
    print("end_file", st.records, st.lines, st.error, time.time() - t, flush=True)
    print(ctx.finalize(), ctx.diag(), flush=True)
ctx.close()
print("done", flush=True)
