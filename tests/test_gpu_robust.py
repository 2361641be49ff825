"""Robustness of the tally's launch machinery (round-5 advisor findings), on the GPU through the C ABI.

* A reused context whose previous feed was low-cardinality takes one big unlogged launch; a feed of
  other data that outgrows the table inside it is rolled back and replayed in smaller ranges with the
  table grown between them (fr_feed_device) -- never FR_ERR_CAPACITY, never a different table.
* Two processes scanning host feeds on one GPU at once (and an oversubscribed grid): every chunk goes
  by ticket, so a look-back never waits on a workgroup that is not running.
* A device range over 4 GiB (one launch, chunk-relative offsets) with an exotic code, non-ASCII bytes,
  bad UTF-8 and a header without ' ' past 4 GiB: first ordinals, exotic codes and error offsets equal
  a run of the same buffer in ranges under 4 GiB.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def lib():
    from frender_amd import _lib
    return _lib


def _distinct_records(n, seed):
    rng = np.random.default_rng(seed)
    codes = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=(n, 17))]
    codes[:, 8] = ord("+")
    head = np.frombuffer(b"@r 1:N:0:", np.uint8)
    tail = np.frombuffer(b"\nA\n+\nF\n", np.uint8)
    rec = np.concatenate([np.broadcast_to(head, (n, head.size)), codes, np.broadcast_to(tail, (n, tail.size))], 1)
    return rec.tobytes()


def _feed_once(c, data):
    p = c.device_alloc(len(data) + 64)
    try:
        c.copy_to_device(p, data)
        c.reset()
        c.begin_file(None)
        c.feed_device(p, len(data))
        st = c.end_file()
    finally:
        c.device_free(p)
    c.finalize()
    keys, counts, first = c.unique()
    return st, keys, counts


def test_room_rollback_low_then_high_cardinality(lib):
    from frender_amd.synth import generate_bytes, make_sheet
    from oracle.frender_oracle import tally_text

    light = b"".join(b"@r%d 1:N:0:AAAAAAAA+CCCCCCCC\nACGT\n+\nFFFF\n" % i for i in range(300_000))
    heavy = _distinct_records(300_000, 5)
    syn = generate_bytes(make_sheet(96, 8, 8), 0, 200_000, R=8, seed=8)
    c = lib.Context(device=0, chunk_bytes=(16 << 30) - (1 << 20), table_slots=1 << 12, tuning={"ovf_cap": 1 << 16})
    try:
        for data, k in ((light, "light"), (light, "light"), (heavy, "heavy"), (syn, "syn"), (heavy, "heavy")):
            st, keys, counts = _feed_once(c, data)
            exp, recs = tally_text(data.decode())
            assert st.error == 0 and st.records == recs, k
            assert list(zip(lib.decode_keys(keys), counts.tolist())) == list(exp.items()), k
        assert c.diag()["big_rollbacks"] >= 1
    finally:
        c.close()


def test_two_host_fed_scans_at_once(tmp_path):
    """Two processes, each a host-fed scan (every chunk looks back for its exact line prefix), on the
    same GPU at the same time, one of them with a grid 4x the device's resident workgroups."""
    script = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from frender_amd import _lib, synth
grid = int(sys.argv[2])
data = synth.generate_bytes(synth.make_sheet(96, 8, 8), 0, 1_500_000, R=8, seed=17)
c = _lib.Context(device=0, chunk_bytes=8 << 20, table_slots=1 << 20, tuning={"grid": grid} if grid else None)
out = []
for _ in range(3):
    c.reset(); c.begin_file(None)
    for o in range(0, len(data), 16 << 20):
        c.feed(data[o:o + (16 << 20)])
    st = c.end_file(); c.finalize()
    k, n, f = c.unique()
    out.append([int(st.records), int(k.size), int((k ^ n ^ f).sum() & ((1 << 63) - 1))])
print(json.dumps(out))
'''
    p = tmp_path / "host_feed.py"
    p.write_text(script)
    env = dict(os.environ, PYTHONPATH=ROOT)
    procs = [subprocess.Popen([sys.executable, str(p), ROOT, str(g)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for g in (0, 4096)]
    res = []
    for q in procs:
        o, e = q.communicate(timeout=240)
        assert q.returncode == 0, e[-3000:]
        res.append(json.loads(o.strip().splitlines()[-1]))
    assert res[0] == res[1]
    assert all(r == res[0][0] for r in res[0]) and res[0][0][0] == 1_500_000


def test_range_over_4gib_rare_paths(lib):
    from frender_amd import synth

    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, 8)
    n = 60_000_000  # 4.44e9 B: one 16-GiB launch vs two of < 4 GiB
    nbytes = n * reclen
    assert nbytes > (4 << 30) + (64 << 20)
    # records past 4 GiB to patch: an exotic code, valid 2-byte UTF-8 in a qual line, an invalid byte in
    # a seq line, and a header whose ' ' became '_' (the reference's IndexError)
    at = [(4 << 30) // reclen + 1000 + 7919 * i for i in range(4)]
    hostrec = {r: bytearray(synth.generate_bytes(sheet, r, 1, R=8, seed=1)) for r in at}
    e = hostrec[at[0]]
    e[e.index(b"+", 40) + 1] = ord("x")  # idx2's first base -> 'x': exotic code
    q = hostrec[at[1]]
    q[-3:-1] = "é".encode()  # qual line: valid UTF-8
    s = hostrec[at[2]]
    s[55] = 0xFF  # seq line: invalid UTF-8
    h = hostrec[at[3]]
    h[h.index(b" ")] = ord("_")  # header without ' '
    runs = []
    for gib in (4, 16):
        c = lib.Context(device=0, chunk_bytes=(gib << 30) - (1 << 20), table_slots=1 << 22)
        buf = c.device_alloc(nbytes + 64)
        try:
            c.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
            for r, b in hostrec.items():
                c.copy_to_device(buf + r * reclen, bytes(b))
            got = None
            for step in range(2):  # the 16-GiB context's second feed is one launch
                c.reset()
                c.begin_file(None)
                c.feed_device(buf, nbytes)
                st = c.end_file()
                launches = c.timing().scan_launches
                c.finalize()
                keys, counts, first = c.unique()
                codes, ecounts, efirst, _, _ = c.exotic_table()
                got = (st.records, st.error, st.error_offset, st.utf8_bad, st.exotic, keys.tolist(), counts.tolist(),
                       first.tolist(), [x.decode() for x in codes], ecounts.tolist(), efirst.tolist())
            assert launches == (1 if gib == 16 else 2), (gib, launches)
            runs.append(got)
        finally:
            c.device_free(buf)
            c.close()
    a, b = runs
    assert a == b
    assert a[1] == 1 and a[2] == at[3] * reclen  # FR_SCAN_NO_SPACE at the patched header (past 4 GiB)
    assert a[3] == 1 and a[4] == 1
    assert a[8] == [hostrec[at[0]].split(b"\n")[0].split(b" ")[1].split(b":")[-1].decode()]
    assert a[10] == [(1 << 44) | (at[0] * reclen & ~3)]  # the exotic record's ordinal: file tag 1, byte offset (4-B floor)
