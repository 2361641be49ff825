"""Phases of the N>1 merge leg (frender_amd/dist.py partition_merge_device) on the full config-2 table, at
world 1 over a one-rank RCCL group: each phase synchronised and timed on the host."""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from frender_amd import _lib as lib, synth  # noqa: E402
from frender_amd.dist import exchange, owner_of  # noqa: E402

with socket.socket() as so:
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
sheet = synth.make_sheet(96, 8, 8)
n, reclen = 100_000_000, 74
c = lib.Context(device=0, chunk_bytes=(16 << 30) - (1 << 20), table_slots=1 << 22)
buf = c.device_alloc(n * reclen + 64)
c.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
res = {}
for it in range(4):
    c.reset()
    c.begin_file(None, file_index=0, byte_base=0)
    c.feed_device(buf, n * reclen)
    c.end_file()
    c.finalize()
    c.sync()
    t = [time.perf_counter()]

    def mark(name):
        torch.cuda.synchronize()
        c.sync()
        now = time.perf_counter()
        res.setdefault(name, []).append((now - t[0]) * 1e3)
        t[0] = now

    rows = c.export_rows("cuda")
    mark("export")
    dest = owner_of(rows[:, 0], 1)
    mark("owner_of")
    mine = exchange(dist, "cuda", rows, dest)
    mark("exchange")
    c.reset()
    mark("reset")
    c.merge_rows(mine)
    mark("merge_rows")
    u, _, _ = c.finalize()
    mark("finalize")
print({k: round(sorted(v)[len(v) // 2], 3) for k, v in res.items()}, "rows", int(u))
c.device_free(buf)
c.close()
dist.destroy_process_group()
