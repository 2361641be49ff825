"""Launch-log fold occupancy per device feed: the config-2 and config-3 shapes fed twice on
one context; prints each feed's launches and fr_get_diag's fold statistics (fold_max of AGG_LNS = 4096)."""
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from frender_amd import _lib as lib, synth  # noqa: E402

for name, S, L, rc in (("cfg2", 96, 8, False), ("cfg3", 384, 10, True)):
    sheet = synth.make_sheet(S, L, L)
    reclen = synth.record_length(L, L, 8)
    n = 100_000_000
    idx2 = synth.read_idx2(sheet, synth.CFG3_RC_NAMES) if rc else sheet.idx2
    c = lib.Context(device=0, chunk_bytes=(16 << 30) - (1 << 20), table_slots=1 << 22)
    buf = c.device_alloc(n * reclen + 64)
    try:
        c.synth_device(buf, 0, n, 8, 1, sheet.idx1, idx2)
        for step in range(3):
            c.reset()
            c.begin_file(None)
            c.feed_device(buf, n * reclen)
            c.end_file()
            d = c.diag()
            print(name, step, "launches", c.timing().scan_launches, "fold_max", d["fold_max"], "fold_over", d["fold_over"],
                  "step_bytes", d["feed_step"], "keys", d["keys"], flush=True)
    finally:
        c.device_free(buf)
        c.close()
