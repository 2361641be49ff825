"""GPU parity: the HIP scan path (through the C ABI) against the CPU oracle and the
reference's golden vectors.  Bit-exact everywhere: this is integer/byte work."""
import os
import random

import numpy as np
import pytest

from harness import case_names, run_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from frender_amd import _lib
    return _lib


@pytest.fixture(scope="module")
def ctx(lib):
    c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16)
    yield c
    c.close()


def gpu_tally(ctx, lib, files, sample=None, mode="host", pieces=None, rng=None):
    """Tally fast-alphabet inputs on the GPU -> ({code: count} in order, [records])."""
    ctx.reset()
    recs = []
    for data in files:
        ctx.begin_file(sample)
        if mode == "device":
            p = ctx.device_alloc(len(data) + 16)
            try:
                if data:
                    ctx.copy_to_device(p, data)
                ctx.feed_device(p, len(data))
                st = ctx.end_file()
            finally:
                ctx.device_free(p)
        else:
            pos = 0
            while pos < len(data):
                n = pieces(rng) if pieces else len(data)
                if ctx.feed(data[pos:pos + n]):
                    break
                pos += n
            st = ctx.end_file()
        assert st.error == 0 and st.exotic == 0
        recs.append(int(st.records))
    ctx.finalize()
    keys, counts, first = ctx.unique()
    assert np.all(np.diff(first.astype(np.float64)) > 0)
    return dict(zip(lib.decode_keys(keys), counts.tolist())), recs


def oracle_tally(files, sample=None):
    from oracle.frender_oracle import tally_text
    total, recs = {}, []
    for data in files:
        c, r = tally_text(data.decode(), sample)
        for k, v in c.items():
            total[k] = total.get(k, 0) + v
        recs.append(r)
    return total, recs


def assert_same(got, exp):
    assert got[1] == exp[1], ("records", got[1], exp[1])
    assert list(got[0].items()) == list(exp[0].items())


# ---------------------------------------------------------------------------------------
# golden vectors produced by the reference itself
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", case_names())
def test_golden_case_on_gpu(name):
    from frender_amd import scan
    diffs = run_case(name, scan.frender_scan)
    assert not diffs, "\n".join(diffs)


# ---------------------------------------------------------------------------------------
# synthetic generator: device == host
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("L,R", [(8, 8), (10, 150)])
def test_device_synth_matches_host(ctx, L, R):
    from frender_amd import synth
    sheet = synth.make_sheet(96, L, L)
    n, r0 = 3000, 123_456_789
    want = synth.generate_bytes(sheet, r0, n, R=R, seed=5)
    p = ctx.device_alloc(len(want))
    try:
        ctx.synth_device(p, r0, n, R, 5, sheet.idx1, sheet.idx2)
        assert ctx.copy_to_host(p, len(want)) == want
    finally:
        ctx.device_free(p)


# ---------------------------------------------------------------------------------------
# tally parity on random inputs (look-back across many tiles and launches)
# ---------------------------------------------------------------------------------------
def random_fastq(rng, n, long_every=0, styles=("\n", "\r\n", "\r"), blank_seq=False):
    out = []
    alphabet = "ACGTN"
    for i in range(n):
        nl = rng.choice(styles)
        a = "".join(rng.choice(alphabet) for _ in range(rng.randint(1, 10)))
        b = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 10)))
        code = a + "+" + b if rng.random() < 0.95 else a
        pre = "@r%d:%s" % (i, "x" * (700 if long_every and i % long_every == 0 else rng.randint(0, 30)))
        tag = rng.choice(["1:N:0:", "", "2:Y:18:", "::"])
        tail = rng.choice(["", " more:stuff", " x"])
        seq = "" if blank_seq and rng.random() < 0.2 else "ACGT" * rng.randint(0, 40)
        out.append(f"{pre} {tag}{code}{tail}{nl}{seq}{nl}+{nl}{'F' * len(seq)}{nl}")
    return "".join(out).encode()


@pytest.mark.parametrize("mode", ["host", "device"])
@pytest.mark.parametrize("seed", [1, 2])
def test_random_fastq_tally(ctx, lib, mode, seed):
    rng = random.Random(seed)
    files = [random_fastq(rng, 20000, long_every=997, blank_seq=True), random_fastq(rng, 5000, styles=("\r\n",)),
             b"", random_fastq(rng, 1)]
    got = gpu_tally(ctx, lib, files, mode=mode, pieces=lambda r: r.choice([1, 7, 4096, 70000, 1 << 20]), rng=rng)
    assert_same(got, oracle_tally(files))


@pytest.mark.parametrize("sample", [1, 3, 1000, 19999, 50000])
@pytest.mark.parametrize("mode", ["host", "device"])
def test_sample_limit(ctx, lib, sample, mode):
    rng = random.Random(sample)
    files = [random_fastq(rng, 20000), random_fastq(rng, 300)]
    got = gpu_tally(ctx, lib, files, sample=sample, mode=mode, pieces=lambda r: 65536, rng=rng)
    assert_same(got, oracle_tally(files, sample))


def test_no_trailing_newline_and_truncated(ctx, lib):
    rng = random.Random(9)
    base = random_fastq(rng, 50)
    files = [base[:-1], base + b"@last 1:N:0:ACGT+TTTT", base + b"@last 1:N:0:ACGT+TTTT\nAC\n", b"\n\n\n\n"[:0]]
    for mode in ("host", "device"):
        assert_same(gpu_tally(ctx, lib, files, mode=mode), oracle_tally(files))


@pytest.mark.parametrize("log_min", [None, "0"])
def test_speculative_commit_replay(lib, log_min):
    """A file whose chunks look like 4-line FASTQ one line off the true phase: every chunk after
    the first guesses the wrong line phase, commits at once, the launch-end check catches it and
    the feed is replayed with every chunk waiting for its exact prefix (fr_feed_device).  With
    log_min=0 the failed attempt's commits went through the launch log and its aggregation."""
    recs = ["L 1:N:0:AAAA+CCCC\n"] + [f"@r{i} 1:N:0:ACGT+ACGT\nACGT\n+\nA AC\n" for i in range(60000)]
    data = "".join(recs).encode()
    exp = oracle_tally([data])
    assert list(exp[0]) == ["AAAA+CCCC", "AC"]
    c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16,
                    tuning=None if log_min is None else {"log_min": int(log_min)})
    try:
        assert_same(gpu_tally(c, lib, [data], mode="device"), exp)
        assert c.diag()["spec_replays"] == 1
        good = "".join(f"@r{i} 1:N:0:ACGT+ACG{'ACGT'[i % 4]}\nACGT\n+\nFFFF\n" for i in range(60000)).encode()
        assert_same(gpu_tally(c, lib, [data, good], mode="device"), oracle_tally([data, good]))
        assert c.diag()["spec_replays"] == 2  # the second file (non-empty table) commits without a replay
    finally:
        c.close()


@pytest.mark.parametrize("log_min,log_hot", [("0", 4), ("0", 1 << 30), ("60", 4), ("100000000", 4)])
def test_launch_log_commits(lib, log_min, log_hot):
    """Commits of at least fr_tuning.log_min pairs go to the launch log and are aggregated after the launch
    (count / scatter / LDS reduce / round-based table inserts); smaller ones insert directly.  Every
    commit logged (0), a mix (60: these 2-wave-tile chunks commit ~30-110 pairs), and none must give the
    oracle's tally, including a table that has to grow between launches.  log_hot 2^30 logs the hot
    codes too (every pair of every commit goes through the log)."""
    from frender_amd import synth
    rng = random.Random(int(log_min) + 7)
    sheet = synth.make_sheet(384, 10, 10)
    files = [synth.generate_bytes(sheet, 0, 300000, R=8, seed=3), random_fastq(rng, 20000, blank_seq=True),
             synth.generate_bytes(sheet, 300000, 5000, R=8, seed=3)]
    exp = oracle_tally(files)
    for mode, slots in (("device", 1 << 12), ("host", 1 << 20)):
        c = lib.Context(device=0, chunk_bytes=1 << 22, table_slots=slots,
                        tuning={"log_min": int(log_min), "log_hot": log_hot})
        try:
            assert_same(gpu_tally(c, lib, files, mode=mode, pieces=lambda r: r.choice([4096, 1 << 20, 1 << 23]),
                                  rng=rng), exp)
        finally:
            c.close()


def test_launch_log_parts_full(lib):
    """A launch whose commits log more pairs than a sub-region part holds: with chunk_bytes 16 MiB the log
    has its minimum of 65 536 entries, 256 per sub-region part (fr_api.hip), while one 16-MiB launch of
    34-B records over 300 000 codes logs ~450 000 pairs, ~900 per part.  The pairs past a part's end insert
    straight into the table (commit_buffers' put) during the tally, the rest through the aggregation's
    plain-store inserts afterwards -- mixed on the same codes -- and the tally must equal the oracle's."""
    rng = random.Random(11)
    pool = ["".join(rng.choice("ACGT") for _ in range(8)) + "+" + "".join(rng.choice("ACGT") for _ in range(8))
            for _ in range(300_000)]
    files = []
    for f in range(2):
        recs = [f"@r{f} 1:N:0:{pool[rng.randrange(len(pool))]}\nA\n+\nI\n" for _ in range(480_000)]
        files.append("".join(recs).encode())
    assert all(len(d) < 16 << 20 for d in files)
    exp = oracle_tally(files)
    c = lib.Context(device=0, chunk_bytes=16 << 20, table_slots=1 << 21, tuning={"log_min": 0})
    try:
        assert_same(gpu_tally(c, lib, files, mode="device"), exp)
    finally:
        c.close()


def test_heavy_chunk_switch(lib):
    """Ramped launches switch to the heavy chunk size once at least a quarter of the chunks since the
    reset logged their commits; the device decides at the end of each launch for the next one
    (fr_kernels.hip note_commit) and fr_reset clears it.  A 6-workgroup grid makes 1 MiB launches
    ramped.  Checked: a config-3-shape pass switches in the middle (its first launch walks 5-tile chunks,
    later ones 7), a reused context's next pass over single-code data (commits never log) walks 5-tile
    chunks again, and a third pass switches again; every tally equals the oracle's."""
    from frender_amd import synth
    from oracle.frender_oracle import tally_text
    c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16,
                    tuning={"grid": 6, "log_min": 100, "chunk_tiles": 5, "chunk_tiles_heavy": 7})
    try:
        assert c.diag()["chunk_tiles"] == 5
        sheet = synth.make_sheet(384, 10, 10)
        n = 300_000
        heavy_data = synth.generate_bytes(sheet, 0, n, R=8, seed=4)
        p = c.device_alloc(len(heavy_data))
        c.synth_device(p, 0, n, 8, 4, sheet.idx1, sheet.idx2)
        light = b"".join(b"@r%d 1:N:0:AAAA+CCCC\nACGT\n+\nFFFF\n" % i for i in range(400_000))
        q = c.device_alloc(len(light))
        c.copy_to_device(q, light)
        for data, ptr, heavy in ((heavy_data, p, True), (light, q, False), (heavy_data, p, True)):
            c.reset()
            c.begin_file(None)
            c.feed_device(ptr, len(data))
            st = c.end_file()
            c.finalize()
            keys, counts, first = c.unique()
            exp, _ = tally_text(data.decode())
            assert st.error == 0 and st.records == sum(exp.values())
            assert list(zip(lib.decode_keys(keys), counts.tolist())) == list(exp.items())
            d, launches = c.diag(), c.timing().scan_launches
            if heavy:  # switched after the first launch, within this pass
                assert d["chunk_tiles"] == 7 and 0 < d["heavy_launches"] < launches, (d, launches)
            else:
                assert d["chunk_tiles"] == 5 and d["heavy_launches"] == 0, (d, launches)
        c.device_free(p)
        c.device_free(q)
    finally:
        c.close()


def test_table_growth_and_overflow(lib):
    """Start from a 1024-slot table with ~60k distinct codes: the table must grow
    between launches (overflow list absorbs in-flight inserts) and stay exact."""
    from frender_amd import synth
    c = lib.Context(device=0, chunk_bytes=1 << 18, table_slots=1024)
    try:
        rng = np.random.default_rng(3)
        n = 60000
        codes = ["".join("ACGT"[x] for x in rng.integers(0, 4, 8)) + "+" + "".join("ACGT"[x] for x in rng.integers(0, 4, 8))
                 for _ in range(n)]
        data = "".join(f"@r{i} 1:N:0:{cd}\nA\n+\nF\n" for i, cd in enumerate(codes + codes[: n // 3])).encode()
        for mode in ("host", "device"):
            assert_same(gpu_tally(c, lib, [data], mode=mode), oracle_tally([data]))
        sheet = synth.make_sheet(4, 8, 8)
        big = synth.generate_bytes(sheet, 0, 200000, R=8, seed=11)
        assert_same(gpu_tally(c, lib, [big, data], mode="device"), oracle_tally([big, data]))
    finally:
        c.close()


def test_synthetic_device_scale(lib):
    """A 2M-read SYN-v1 file generated and scanned in HBM (1 MiB launches) vs the oracle."""
    from frender_amd import synth
    from oracle.frender_oracle import tally_text
    c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 20)
    try:
        sheet = synth.make_sheet(96, 8, 8)
        n = 2_000_000
        host = synth.generate_bytes(sheet, 0, n, R=8, seed=1)
        p = c.device_alloc(len(host))
        c.synth_device(p, 0, n, 8, 1, sheet.idx1, sheet.idx2)
        c.reset()
        c.begin_file(None)
        c.feed_device(p, len(host))
        st = c.end_file()
        c.device_free(p)
        assert st.records == n and st.error == 0
        c.finalize()
        keys, counts, first = c.unique()
        got = dict(zip(lib.decode_keys(keys), counts.tolist()))
        exp, recs = tally_text(host.decode())
        assert recs == n
        assert list(got.items()) == list(exp.items())
        assert int(counts.sum()) == n
    finally:
        c.close()


# ---------------------------------------------------------------------------------------
# classification parity (packed Hamming vs the oracle's string Hamming)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("nsubs", [-1, 0, 1, 2, 3, 9])
@pytest.mark.parametrize("rc", [False, True])
def test_classify_random(ctx, lib, nsubs, rc):
    from frender_amd import synth
    from frender_amd.scan import _sheet_names
    from frender_amd.host import reverse_complement
    from oracle.frender_oracle import classify_code
    rng = random.Random(nsubs * 7 + rc)
    sheet = synth.make_sheet(24, 8, 8, seed=5, combinatorial=(6, 4) if nsubs % 2 else None)
    ids = list(sheet.ids)
    ids[5] = ids[3]  # a duplicated name
    idx1, idx2 = list(sheet.idx1), list(sheet.idx2)
    idx2[7] = idx2[7].lower()
    idx2[8] = reverse_complement(idx2[2])
    codes = []
    for _ in range(3000):
        s = rng.randrange(len(idx1))
        a = list(idx1[s].upper())
        b = list((idx2[rng.randrange(len(idx1))] if rng.random() < 0.3 else idx2[s]).upper())
        if rng.random() < 0.2:
            b = list(reverse_complement("".join(b)))
        for arr in (a, b):
            for _ in range(rng.randint(0, 3)):
                arr[rng.randrange(8)] = rng.choice("ACGTN")
        codes.append("".join(a) + "+" + "".join(b))
    codes = list(dict.fromkeys(codes))
    data = "".join(f"@r{i} 1:N:0:{c}\n\n+\n\n" for i, c in enumerate(codes)).encode()
    ctx.reset()
    ctx.begin_file(None)
    ctx.feed(data)
    ctx.end_file()
    ctx.finalize()
    keys, counts, _ = ctx.unique()
    assert lib.decode_keys(keys) == codes
    names, nid = _sheet_names(ids)
    idx2rc = [reverse_complement(x) for x in idx2]
    ctx.set_sheet(idx1, idx2, idx2rc, nid, len(names))
    out = ctx.classify(nsubs, rc)
    assert out["err_unique"] == -1
    f_exp = {n: 0 for n in names}
    r_exp = {n: 0 for n in names}
    for j, code in enumerate(codes):
        e = classify_code(code, 1, idx1, idx2, ids, nsubs, rc)
        got_t = lib.CLASS_NAMES[out["cls"][j]]
        assert got_t == e["read_type"], (code, got_t, e)
        assert (idx1[out["m1"][j]] if out["m1"][j] >= 0 else "") == e["matched_idx1"], (code, e)
        assert (idx2[out["m2"][j]] if out["m2"][j] >= 0 else "") == e["matched_idx2"]
        assert (ids[out["row"][j]] if out["row"][j] >= 0 else "") == e["sample_name"]
        if rc:
            assert (idx2rc[out["rc_m2"][j]] if out["rc_m2"][j] >= 0 else "") == e["matched_rc_idx2"], (code, e)
            assert lib.CLASS_NAMES[out["rc_cls"][j]] == e["rc_read_type"]
            assert (ids[out["rc_row"][j]] if out["rc_row"][j] >= 0 else "") == e["rc_sample_name"]
            if e["sample_name"]:
                f_exp[e["sample_name"]] += 1
            if e["rc_sample_name"]:
                r_exp[e["rc_sample_name"]] += 1
    if rc:
        f, r = ctx.rc_counts()
        assert f.tolist() == [f_exp[n] for n in names]
        assert r.tolist() == [r_exp[n] for n in names]


@pytest.mark.parametrize("nsubs", [0, 1, 2, 3])
@pytest.mark.parametrize("rc", [False, True])
def test_classify_neighbourhood_maps(lib, nsubs, rc):
    """The map path (a few probes per code) against the row scan (fr_tuning.nbr = 0) and the oracle on an
    adversarial 10+10 sheet: values 1 and 2 substitutions apart (codes near several values take the
    scan), repeated values (combinatorial rows), a lower-case and an 'x' entry, duplicated names."""
    from frender_amd.host import reverse_complement
    from frender_amd.scan import _sheet_names
    from oracle.frender_oracle import classify_code
    rng = random.Random(100 + nsubs * 2 + rc)
    base = ["".join(rng.choice("ACGT") for _ in range(10)) for _ in range(40)]
    near = []
    for k, v in enumerate(base[:8]):  # neighbours of the first values at distance 1 and 2
        w = list(v)
        for p in rng.sample(range(10), 1 + k % 2):
            w[p] = rng.choice([c for c in "ACGT" if c != w[p]])
        near.append("".join(w))
    vals1 = base + near
    vals2 = ["".join(rng.choice("ACGT") for _ in range(10)) for _ in range(20)]
    idx1 = [vals1[i % len(vals1)] for i in range(96)]
    idx2 = [vals2[(i * 7) % len(vals2)] for i in range(96)]  # (idx1, idx2) pairs repeat
    idx1[10] = idx1[10].lower()
    idx2[11] = idx2[11][:4] + "x" + idx2[11][5:]
    ids = [f"s{i % 80}" for i in range(96)]
    codes = []
    for _ in range(6000):
        s = rng.randrange(96)
        a = list(idx1[s].upper())
        b = list((idx2[rng.randrange(96)] if rng.random() < 0.3 else idx2[s]).upper())
        if rng.random() < 0.3:
            b = list(reverse_complement("".join(b)))
        for arr in (a, b):
            for _ in range(rng.randint(0, 4)):
                arr[rng.randrange(10)] = rng.choice("ACGTN")
        codes.append("".join(a).replace("X", "A") + "+" + "".join(b).replace("X", "C"))
    codes = list(dict.fromkeys(codes))
    data = "".join(f"@r{i} 1:N:0:{c}\n\n+\n\n" for i, c in enumerate(codes)).encode()
    names, nid = _sheet_names(ids)
    outs = []
    for nbr in (1, 0):
        c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16, tuning={"nbr": nbr})
        try:
            c.reset()
            c.begin_file(None)
            c.feed(data)
            c.end_file()
            c.finalize()
            assert lib.decode_keys(c.unique()[0]) == codes
            c.set_sheet(idx1, idx2, [reverse_complement(x) for x in idx2], nid, len(names))
            out = c.classify(nsubs, rc)
            keep = [k for k in out if rc or not k.startswith("rc_")]  # rc_* are left unwritten without rc
            outs.append(({k: np.asarray(out[k]).tolist() if hasattr(out[k], "__len__") else out[k] for k in keep},
                         [x.tolist() for x in c.rc_counts()] if rc else None))
        finally:
            c.close()
    assert outs[0] == outs[1]
    out = outs[0][0]
    for j in rng.sample(range(len(codes)), 400):
        e = classify_code(codes[j], 1, idx1, idx2, ids, nsubs, rc)
        assert lib.CLASS_NAMES[out["cls"][j]] == e["read_type"], (codes[j], e)
        assert (ids[out["row"][j]] if out["row"][j] >= 0 else "") == e["sample_name"]
        if rc:
            assert lib.CLASS_NAMES[out["rc_cls"][j]] == e["rc_read_type"]
            assert (ids[out["rc_row"][j]] if out["rc_row"][j] >= 0 else "") == e["rc_sample_name"]


@pytest.mark.parametrize("grid,cap,chunk", [(1, 1536, 1 << 24), (4, 0, 1 << 26), (64, 16, 1 << 26), (512, 1536, 1 << 30)])
def test_many_tiles_per_workgroup(lib, grid, cap, chunk):
    """Few workgroups walking many tiles each (look-back windows sliding past 64 tiles),
    with the LDS table capped so most codes take the direct-to-HBM path."""
    from frender_amd import synth
    from oracle.frender_oracle import tally_text
    c = lib.Context(device=0, chunk_bytes=chunk, table_slots=1 << 16, tuning={"grid": grid, "flush_at": cap})
    try:
        sheet = synth.make_sheet(96, 8, 8)
        n = 1_500_000
        host = synth.generate_bytes(sheet, 7, n, R=8, seed=2)
        p = c.device_alloc(len(host))
        c.synth_device(p, 7, n, 8, 2, sheet.idx1, sheet.idx2)
        c.reset()
        c.begin_file(None)
        c.feed_device(p, len(host))
        st = c.end_file()
        c.device_free(p)
        assert st.records == n and st.error == 0
        c.finalize()
        keys, counts, _ = c.unique()
        exp, _ = tally_text(host.decode())
        assert list(zip(lib.decode_keys(keys), counts.tolist())) == list(exp.items())
    finally:
        c.close()


# ---------------------------------------------------------------------------------------
# multi-GPU merge kernel: export one context's table, merge it into another's
# ---------------------------------------------------------------------------------------
def test_merge_unique_device(lib):
    """Shard a dataset over 3 contexts (ranks); merging their compacted tables into
    rank 0 through fr_export_unique_device / fr_merge_unique_device must equal one
    context scanning the shards as consecutive files (count = sum, first = min)."""
    from frender_amd import synth
    from frender_amd.dist import device_callbacks
    import torch
    sheet = synth.make_sheet(24, 8, 8)
    shards = [synth.generate_bytes(sheet, 50_000 * i, 50_000, R=8, seed=3) for i in range(3)]
    ref = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 12)
    ranks = [lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 12) for _ in shards]
    try:
        want = gpu_tally(ref, lib, shards, mode="device")
        kref, cref, fref = ref.unique()
        for r, c in enumerate(ranks):  # rank r scans shard r as its file r (global file index)
            gpu_tally(c, lib, [b""] * r + [shards[r]], mode="device")
        export0, merge0, refin0 = device_callbacks(ranks[0])
        for c in ranks[1:]:
            export, _, _ = device_callbacks(c)
            buf = torch.empty((3, c.U), dtype=torch.int64, device="cuda")
            export(buf, c.U)
            merge0(buf, c.U)
        refin0()
        k, cnt, f = ranks[0].unique()
        assert np.array_equal(k, kref) and np.array_equal(cnt, cref) and np.array_equal(f, fref)
        assert dict(zip(lib.decode_keys(k), cnt.tolist())) == want[0]
    finally:
        ref.close()
        for c in ranks:
            c.close()


# ---------------------------------------------------------------------------------------
# demux (row f-1): the GPU path against the reference's own outputs
# ---------------------------------------------------------------------------------------
from demux_harness import case_names as demux_case_names  # noqa: E402
from demux_harness import run_case as run_demux_case  # noqa: E402
from demux_harness import run_case_cli as run_demux_case_cli  # noqa: E402


@pytest.mark.parametrize("name", demux_case_names())
def test_demux_golden_on_gpu(name):
    from frender_amd.demux import frender_demux
    diffs = run_demux_case(name, frender_demux)
    assert not diffs, "\n".join(diffs)


@pytest.mark.parametrize("name", ["syn96_scan_csv", "syn_basic", "syn_crlf", "hand_lone_cr", "syn_missing_code",
                                  "syn_bad_type", "syn_no_undet"])
def test_demux_cli_two_ranks_golden(name):
    """`demux --gpus 2` (pairs dealt to two ranks, rank 0 concatenating the per-pair gzip parts) on the
    reference's golden demux cases: the same files' contents, stdout and errors."""
    diffs = run_demux_case_cli(name, gpus=2)
    assert not diffs, "\n".join(diffs)


@pytest.mark.parametrize("bad_pair", [None, 3])
def test_demux_cli_ranks_many_pairs(tmp_path, bad_pair):
    """Seven pairs over three ranks (gloo, one GPU) against the single-rank in-process demux: every
    writer's content, the stdout lines and, with a code missing from the results in pair 3, the
    error of the first failing pair in pair order."""
    import argparse
    import contextlib
    import gzip
    import io
    import subprocess
    import sys
    from frender_amd.demux import frender_demux
    rng = random.Random(17)
    codes = ["AAAA+CCCC", "GGGG+TTTT", "AAAA+TTTT", "ACGT+ACGT", "NNNN+CCCC"]
    kinds = {"AAAA+CCCC": ("demuxable", "S1"), "GGGG+TTTT": ("demuxable", "S2"), "AAAA+TTTT": ("index_hop", ""),
             "ACGT+ACGT": ("undetermined", ""), "NNNN+CCCC": ("ambiguous", "")}
    inp = tmp_path / "in"
    inp.mkdir()
    files = []
    for p in range(7):
        r1, r2 = [], []
        for i in range(rng.randint(500, 3000)):
            c = rng.choice(codes) if not (p == bad_pair and i == 100) else "TTTT+TTTT"
            seq = "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 40)))
            r1.append(f"@p{p}r{i} 1:N:0:{c}\n{seq}\n+\n{'F' * len(seq)}\n")
            r2.append(f"@p{p}r{i} 2:N:0:{c}\n{seq[::-1]}\n+\n{'F' * len(seq)}\n")
        for m, txt in ((1, r1), (2, r2)):
            fn = inp / f"L{p}_R{m}_001.fastq.gz"
            with gzip.open(fn, "wb") as f:
                f.write("".join(txt).encode())
            files.append(str(fn))
    with open(inp / "results.csv", "w") as f:
        f.write("idx1,idx2,reads,matched_idx1,matched_idx2,read_type,sample_name,demux_ok\r\n")
        for c, (t, s) in kinds.items():
            a, b = c.split("+")[0:2]
            f.write(f"{a},{b},1,,,{t},{s},True\r\n")
    one = tmp_path / "one"
    buf = io.StringIO()
    err = None
    with contextlib.redirect_stdout(buf):
        try:
            frender_demux(argparse.Namespace(r=str(inp / "results.csv"), d=str(one), o=None, no_index_hop=False,
                                             no_ambiguous=False, no_undeter=False, no_samples=False, files=files))
        except SystemExit as e:
            err = str(e)
    many = tmp_path / "many"
    env = dict(os.environ, FRENDER_DIST_BACKEND="gloo",
               PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-m", "frender_amd", "demux", "--gpus", "3", "-r", str(inp / "results.csv"),
                        "-d", str(many), *files], cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=240)
    assert "".join(ln for ln in r.stdout.splitlines(True) if not ln.startswith("[Gloo]")) == buf.getvalue()
    if bad_pair is None:
        assert r.returncode == 0 and err is None, r.stderr[-2000:]
    else:
        assert r.returncode != 0 and err and err in r.stderr, (err, r.stderr[-2000:])
    assert sorted(os.listdir(many)) == sorted(os.listdir(one))
    for fn in os.listdir(one):
        with gzip.open(one / fn, "rb") as a, gzip.open(many / fn, "rb") as b:
            assert a.read() == b.read(), fn


@pytest.mark.parametrize("seed,window", [(1, None), (2, None), (3, 20000), (4, 4096)])
def test_demux_random_vs_oracle(seed, window, tmp_path):
    """Random paired inputs with mixed codes, CRLF/CR, long headers and a short R2 against
    the demux oracle (content of every writer)."""
    import argparse
    import gzip
    from frender_amd.demux import frender_demux
    from oracle import demux_oracle
    rng = random.Random(seed)
    codes = ["AAAA+CCCC", "GGGG+TTTT", "AAAA+TTTT", "ACGT+ACGT", "NNNN+CCCC", "acgt+TTTT", "ACG+GT"]
    kinds = {"AAAA+CCCC": ("demuxable", "S1"), "GGGG+TTTT": ("demuxable", "S2"), "AAAA+TTTT": ("index_hop", ""),
             "ACGT+ACGT": ("undetermined", ""), "NNNN+CCCC": ("ambiguous", ""), "acgt+TTTT": ("demuxable", "S1"),
             "ACG+GT": ("undetermined", "")}
    inp = tmp_path / "in"
    inp.mkdir()
    r1, r2 = [], []
    for i in range(rng.randint(3000, 6000)):
        c = rng.choice(codes)
        nl = rng.choice(["\n"] * 8 + ["\r\n", "\r"])
        pad = "x" * (rng.randint(0, 900) if rng.random() < 0.02 else rng.randint(0, 20))
        seq = "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 60)))
        r1.append(f"@r{i}:{pad}:1:FC 1:N:0:{c}{nl}{seq}{nl}+{nl}{'F' * len(seq)}{nl}")
        r2.append(f"@r{i}:{pad}:1:FC 2:N:0:{c}{nl}{seq[::-1]}{nl}+{nl}{'F' * len(seq)}{nl}")
    t2 = "".join(r2)[:-rng.randint(1, 40)]
    with gzip.open(inp / "x_R1_001.fastq.gz", "wb") as f:
        f.write("".join(r1).encode())
    with gzip.open(inp / "x_R2_001.fastq.gz", "wb") as f:
        f.write(t2.encode())
    with open(inp / "results.csv", "w") as f:
        f.write("idx1,idx2,reads,matched_idx1,matched_idx2,read_type,sample_name,demux_ok\r\n")
        for c, (t, s) in kinds.items():
            a, b = c.split("+")[0:2]
            f.write(f"{a},{b},1,,,{t},{s},True\r\n")
    files = [str(inp / "x_R1_001.fastq.gz"), str(inp / "x_R2_001.fastq.gz")]

    def ns(d):
        return argparse.Namespace(r=str(inp / "results.csv"), d=str(d), o=None, no_index_hop=False,
                                  no_ambiguous=False, no_undeter=False, no_samples=False, files=files,
                                  window=window)

    want = demux_oracle.demux(ns(tmp_path / "o_ref"))
    frender_demux(ns(tmp_path / "o_gpu"))
    for p, data in want.items():
        q = p.replace("o_ref", "o_gpu")
        with gzip.open(q, "rb") as g:
            assert g.read() == data, q


def test_scan_then_demux_96_samples(tmp_path, monkeypatch):
    """BASELINE config 5 shape end to end on the product path: `scan` (GPU) writes its CSV, `demux`
    (GPU) routes a 96-sample paired set with that CSV (scan's own column order), and
    every writer's decoded content equals the demux oracle's fed the same CSV."""
    import argparse
    import gzip
    from frender_amd import synth
    from frender_amd.demux import frender_demux
    from frender_amd.scan import frender_scan
    from oracle import demux_oracle

    sheet = synth.make_sheet(96, 8, 8)
    inp = tmp_path / "in"
    inp.mkdir()
    sheet.write_csv(str(tmp_path / "sheet.csv"))
    r1_files = []
    for lane in range(2):
        t1 = synth.generate_bytes(sheet, lane * 150_000, 150_000, R=8, seed=3).decode()
        lines = t1.split("\n")
        t2 = "\n".join(ln.replace(" 1:N:", " 2:N:", 1) if i % 4 == 0 else (ln[::-1] if i % 4 in (1, 3) else ln)
                       for i, ln in enumerate(lines))
        for mate, text in (("R1", t1), ("R2", t2)):
            p = inp / f"syn_L{lane + 1:03d}_{mate}_001.fastq.gz"
            synth.write_fastq_gz(str(p), text.encode(), level=1)
        r1_files.append(str(inp / f"syn_L{lane + 1:03d}_R1_001.fastq.gz"))
    monkeypatch.chdir(tmp_path)
    frender_scan(argparse.Namespace(n=1, rc=False, c=2.0, s=None, o="cfg5", p=None, b=str(tmp_path / "sheet.csv"),
                                    files=r1_files))
    csvs = [f for f in tmp_path.iterdir() if f.name.startswith("frender-scan-results_")]
    assert len(csvs) == 1
    files = sorted(str(p) for p in inp.iterdir())

    def ns(d):
        return argparse.Namespace(r=str(csvs[0]), d=str(tmp_path / d), o=None, no_index_hop=False,
                                  no_ambiguous=False, no_undeter=False, no_samples=False, files=files)

    want = demux_oracle.demux(ns("o_ref"))
    frender_demux(ns("o_gpu"))
    assert len(want) >= 2 * 99
    for p, data in want.items():
        with gzip.open(p.replace("o_ref", "o_gpu"), "rb") as g:
            assert g.read() == data, p


# ---------------------------------------------------------------------------------------
# multi-GPU product path: `scan --gpus 2` rehearsed on this box's GPU (2 ranks, gloo)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["s96_n1_4files", "s96_n1_rc", "two_files_order", "sample_limit",
                                  "demux_ok_samples", "same_file_twice", "wide_codes_12", "no_space_header",
                                  # one file: every rank tallies a record-aligned part of it
                                  "comb96_n1_rc", "cfg1_10k_s4_n0", "cr_only", "mixed_newlines", "multi_member_gz",
                                  "bad_utf8", "gz_truncated", "s96_r150_n1",
                                  # the config-3 shape (384 samples, 10+10, -rc) and n=2 sharded over two ranks
                                  "s384_l10_n1_rc_dup", "s96_n2"])
def test_cli_two_ranks_match_golden(name, tmp_path):
    """`python -m frender_amd scan --gpus 2` (files sharded over two ranks, or one file's record-aligned
    parts, tables key-partitioned over the ranks) writes the reference's CSV bytes and per-file lines
    (frender.py:189-205 merge), and raises the first file's error as one GPU would."""
    import os
    import re
    import subprocess
    import sys
    from harness import build_inputs, compare

    d = str(tmp_path)
    spec = build_inputs(name, d)
    a = spec["args"]
    cmd = [sys.executable, "-m", "frender_amd", "scan", "-n", str(a["n"]), "-c", str(a["c"]), "--gpus", "2"]
    if a["rc"]:
        cmd.append("-rc")
    for flag in ("s", "o", "p", "b"):
        if a.get(flag) is not None:
            cmd += [f"-{flag}", str(a[flag])]
    cmd += a["files"]
    env = dict(os.environ, FRENDER_DIST_BACKEND="gloo",
               PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    before = set(os.listdir(d))
    r = subprocess.run(cmd, cwd=d, env=env, capture_output=True, text=True, timeout=240)
    outs = {}
    for fn in sorted(set(os.listdir(d)) - before):
        with open(os.path.join(d, fn), "rb") as f:
            outs[fn] = f.read()
    err = None
    if r.returncode:
        lines = [re.sub(r"^\[rank\d+\]: ", "", ln) for ln in r.stderr.strip().splitlines()]
        last = [ln for ln in lines if ln and not ln.startswith(" ")][-1]
        typ, _, msg = last.partition(": ")
        err = {"type": typ, "msg": msg}
    diffs = compare(name, outs, err, r.stdout)
    assert not diffs, "\n".join(diffs) + "\n" + r.stderr[-2000:]


# ---------------------------------------------------------------------------------------
# wide keys, exotic volume, universal newlines on the host feed, byte shards
# ---------------------------------------------------------------------------------------
def full_tally(c, files, mode="host", sample=None, piece=1 << 22):
    """Every code (fast, wide, exotic) through the library, in first-occurrence order."""
    from frender_amd import scan
    c.reset()
    recs = []
    for fi, data in enumerate(files):
        c.begin_file(sample, file_index=fi)
        if mode == "device":
            p = c.device_alloc(len(data) + 16)
            try:
                if data:
                    c.copy_to_device(p, data)
                c.feed_device(p, len(data))
                st = c.end_file()
            finally:
                c.device_free(p)
        else:
            for pos in range(0, len(data), piece):
                if c.feed(data[pos:pos + piece]):
                    break
            st = c.end_file()
        assert st.error == 0
        recs.append(int(st.records))
    t = scan.build_table(scan.local_table(c), [f"f{i}" for i in range(len(files))], recs)
    return dict(zip(t.codes, t.counts.tolist())), recs, t


def _records(codes, nl="\n"):
    return "".join(f"@r{i} 1:N:0:{cd}{nl}ACGT{nl}+{nl}FFFF{nl}" for i, cd in enumerate(codes)).encode()


@pytest.mark.parametrize("mode", ["host", "device"])
def test_wide_codes_12_12_and_lowercase(lib, mode):
    """12+12 dual indexes and all-lowercase codes are wide keys counted on the GPU: bit-exact vs the
    oracle, with no exotic (host) records."""
    rng = np.random.default_rng(5)
    n = 1_500_000
    idx = ["".join("ACGT"[x] for x in rng.integers(0, 4, 12)) for _ in range(300)]
    a = rng.integers(0, 300, n)
    b = rng.integers(0, 300, n)
    codes = [idx[i] + "+" + idx[j] for i, j in zip(a.tolist(), b.tolist())]
    for k in rng.integers(0, n, 5000).tolist():
        codes[k] = codes[k][:5] + "N" + codes[k][6:]
    lower = [c.lower() for c in codes[: n // 2]]
    files = [_records(codes), _records(lower)]
    c = lib.Context(device=0, chunk_bytes=64 << 20, table_slots=1 << 16)
    try:
        got, recs, t = full_tally(c, files, mode)
        assert (t.exo_idx < 0).all()  # nothing left the GPU's key forms
        assert_same((got, recs), oracle_tally(files))
    finally:
        c.close()


@pytest.mark.parametrize("mode", ["host", "device"])
def test_exotic_volume_grows_and_replays(lib, mode):
    """More exotic records (mixed case, other bytes) than the initial list holds, in single
    launches: the library replays the launch capturing exotic codes only, grows the list and
    merges natively; bit-exact vs the oracle."""
    rng = np.random.default_rng(9)
    n = 1_300_000
    base = ["AcGtAcGt+TTGGCCAA", "xyz+ACGT", "ACGT+acgt", "A.C+GT", "ÄC+GT"]
    codes = [base[k] + str(v) for k, v in zip(rng.integers(0, 5, n).tolist(), rng.integers(0, 50000, n).tolist())]
    codes[::7] = ["ACGTACGT+ACGTACGT"] * len(codes[::7])
    files = [_records(codes), _records(codes[:1000])]
    c = lib.Context(device=0, chunk_bytes=256 << 20, table_slots=1 << 16)
    try:
        got, recs, _ = full_tally(c, files, mode, piece=64 << 20)
        assert_same((got, recs), oracle_tally(files))
        assert c.diag()["exo_replays"] >= 1
    finally:
        c.close()


def test_cr_only_large_host_feed(lib):
    """Universal newlines on the host feed: a >= 8 MiB file with lone '\\r' line ends through a 1 MiB
    ring cuts at its '\\r's (a CRLF is never split)."""
    rng = random.Random(4)
    data = random_fastq(rng, 120_000, styles=("\r",))
    assert len(data) >= 8 << 20
    mixed = random_fastq(rng, 60_000, styles=("\r", "\r\n", "\n"))
    c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16)
    try:
        for piece in (1 << 20, 999_983, 4096):
            got = full_tally(c, [data, mixed], "host", piece=piece)
            assert_same(got[:2], oracle_tally([data, mixed]))
    finally:
        c.close()


def test_byte_shards_merge_to_whole_file(lib):
    """fr_begin_file_at: one file tallied as record-aligned byte shards on separate contexts and
    merged (count = sum, first = min) equals the whole file on one context, row for row (the
    bench's N-GPU record shards and their ordinals)."""
    from frender_amd import synth
    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, 8)
    n = 600_000
    data = synth.generate_bytes(sheet, 0, n, R=8, seed=2)
    whole = lib.Context(device=0, chunk_bytes=8 << 20, table_slots=1 << 16)
    merged = lib.Context(device=0, chunk_bytes=8 << 20, table_slots=1 << 16)
    shards = [lib.Context(device=0, chunk_bytes=8 << 20, table_slots=1 << 16) for _ in range(3)]
    try:
        whole.reset()
        whole.begin_file(None, file_index=2)
        whole.feed(data)
        whole.end_file()
        whole.finalize()
        want = whole.unique()
        cuts = [0, 123_457, 400_001, n]
        merged.reset()
        for k, c in enumerate(shards):
            part = data[cuts[k] * reclen:cuts[k + 1] * reclen]
            c.reset()
            c.begin_file(None, file_index=2, byte_base=cuts[k] * reclen)
            p = c.device_alloc(len(part) + 16)
            c.copy_to_device(p, part)
            c.feed_device(p, len(part))
            assert c.end_file().records == cuts[k + 1] - cuts[k]
            c.device_free(p)
            U, _, _ = c.finalize()
            bufs = [c.device_alloc(8 * U) for _ in range(3)]
            c.export_unique_device(*bufs, U)
            merged.merge_unique_device(*bufs, U)
            merged.sync()
            for b in bufs:
                c.device_free(b)
        merged.finalize()
        got = merged.unique()
        for x, y in zip(got, want):
            assert np.array_equal(x, y)
    finally:
        for c in [whole, merged] + shards:
            c.close()


def bgzf(data: bytes, block: int = 65280, pad: int = 0) -> bytes:
    """BGZF: independent gzip members of <= 64 KiB input, each with a 'BC' extra subfield holding
    its compressed size - 1, then the empty EOF member (and optional NUL padding)."""
    import struct
    import zlib
    out = []
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        body = c.compress(chunk) + c.flush()
        bsize = 18 + len(body) + 8
        out.append(b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<HBBHH", 6, 66, 67, 2, bsize - 1)
                   + body + struct.pack("<II", zlib.crc32(chunk), len(chunk) & 0xFFFFFFFF))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))  # EOF member
    return b"".join(out) + b"\x00" * pad


@pytest.mark.parametrize("corrupt", [False, True])
def test_bgzf_scan_matches_oracle(tmp_path, corrupt):
    """BGZF inputs decode member-parallel in the native inflate (fr_gz.cpp): the scan's CSVs equal
    the oracle's (Python gzip reads BGZF as multi-member gzip, as the reference does); a member with
    a bad CRC fails with the reference's exception."""
    import argparse
    import contextlib
    import io
    import os

    from frender_amd import scan, synth
    from oracle import frender_oracle

    sheet = synth.make_sheet(24, 8, 8, seed=5)
    sheet.write_csv(str(tmp_path / "sheet.csv"))
    files = []
    for f in range(3):
        raw = synth.generate_bytes(sheet, f * 120000, 120000, R=8, seed=9)
        blob = bytearray(bgzf(raw, pad=16 if f == 1 else 0))
        if corrupt and f == 2:
            blob[len(blob) // 2] ^= 0x40  # inside a member's deflate data or trailer
        p = tmp_path / f"syn_L{f + 1:03d}_R1_001.fastq.gz"
        p.write_bytes(bytes(blob))
        files.append(str(p))
    outs = {}
    for label, fn in (("gpu", scan.frender_scan), ("oracle", frender_oracle.scan)):
        sub = tmp_path / label
        sub.mkdir()
        args = argparse.Namespace(n=1, rc=False, c=3.0, s=None, o="bg", p=None, b=str(tmp_path / "sheet.csv"),
                                  files=files)
        cwd = os.getcwd()
        os.chdir(sub)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                fn(args)
            outs[label] = {x: (sub / x).read_bytes() for x in sorted(os.listdir(sub))}
        except Exception as e:  # noqa: BLE001 - compared below
            outs[label] = (type(e).__name__, str(e))
        finally:
            os.chdir(cwd)
    assert outs["gpu"] == outs["oracle"]
    if not corrupt:
        assert isinstance(outs["gpu"], dict) and outs["gpu"]


# ---------------------------------------------------------------------------------------
# first-occurrence order by binning (fr_finalize, fin_* kernels)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["host", "device"])
def test_first_occurrence_bins(lib, mode):
    """Dense bins: ~22-B records whose codes are nearly all new, so every 8-KiB bin holds hundreds of
    codes ranked inside the bin; files at non-consecutive indices and one at a large byte base (the
    bins span every file's bytes); codes repeated across files keep their first file's ordinal.
    Order, counts and records equal the oracle's."""
    rng = np.random.default_rng(17)
    alpha = np.array(list("ACGT"))
    pool = ["".join(rng.choice(alpha, 8)) + "+" + "".join(rng.choice(alpha, 8)) for _ in range(60000)]
    files = []
    for n in (40000, 25000, 30000):
        idx = rng.integers(0, len(pool), n)
        files.append("".join(f"@r 1:N:0:{pool[i]}\nA\n+\nF\n" for i in idx).encode())
    c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16)
    try:
        c.reset()
        recs = []
        for fi, base, data in zip((0, 3, 7), (0, 0, 3 << 30), files):
            c.begin_file(None, file_index=fi, byte_base=base)
            if mode == "device":
                p = c.device_alloc(len(data) + 16)
                try:
                    c.copy_to_device(p, data)
                    c.feed_device(p, len(data))
                    st = c.end_file()
                finally:
                    c.device_free(p)
            else:
                for pos in range(0, len(data), 1 << 18):
                    c.feed(data[pos:pos + (1 << 18)])
                st = c.end_file()
            assert st.error == 0 and st.exotic == 0
            recs.append(int(st.records))
        U, _, _ = c.finalize()
        keys, counts, first = c.unique()
        assert U == len(keys)
        assert np.all(np.diff(first.astype(np.float64)) > 0)
        got = dict(zip(lib.decode_keys(keys), counts.tolist()))
    finally:
        c.close()
    exp = oracle_tally(files)
    assert recs == exp[1]
    assert list(got.items()) == list(exp[0].items())


@pytest.mark.gpu
def test_timing_events_off_same_table(lib):
    """fr_set_timing(0) drops the HIP timing events only: the same table, zero timings."""
    from frender_amd import synth
    sheet = synth.make_sheet(8, 8, 8, seed=5)
    data = synth.generate_bytes(sheet, 0, 30000, R=8, seed=7)
    out = []
    for on in (True, False):
        c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16)
        c.set_timing(on)
        c.reset()
        c.begin_file(None)
        c.feed(data)
        st = c.end_file()
        U, _, _ = c.finalize()
        t = c.timing()
        out.append((st.records, U, [a.tolist() for a in c.unique()]))
        assert (t.scan_ms > 0) == on and (t.finalize_ms > 0) == on and t.scan_launches > 0
        c.close()
    assert out[0] == out[1]


@pytest.mark.parametrize("launch_gib,tuning", [(4, None), (16, None), (16, {"log_min": 4_000_000_000})])
def test_bench_geometry_pinned_to_reference(lib, launch_gib, tuning):
    """bench.py's exact workload and launch geometry (BASELINE config 2: 100M SYN-v1 records in HBM,
    one device feed cut into two 3.7 GB launches of the 1024-workgroup ramped grid -- or, with 16-GiB
    launches, two for the first feed and ONE 7.4 GB launch for the next (chunk offsets past 4 GiB; every
    commit logged and one aggregation of the launch, or direct commits with the tuning) -- 4 Mi initial slots, speculative commits, heavy-chunk switch) against the REFERENCE's own tally_barcodes +
    process on the same records (tests/golden/cfg2_pin.json, tests/golden/make_golden_cfg2.py): the
    unique-code count, every row in order (sha256) and the first/last 1000 rows verbatim.  Two steps
    on one context, as the bench runs them."""
    import json

    from frender_amd import synth
    from frender_amd.host import reverse_complement
    from frender_amd.scan import _sheet_names

    with open(os.path.join(os.path.dirname(__file__), "golden", "cfg2_pin.json")) as f:
        pin = json.load(f)
    n = pin["reads"]
    sheet = synth.make_sheet(96, 8, 8)
    reclen = synth.record_length(8, 8, 8)
    c = lib.Context(device=0, chunk_bytes=(launch_gib << 30) - (1 << 20), table_slots=1 << 22, tuning=tuning)
    buf = c.device_alloc(n * reclen + 64)
    try:
        c.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
        names, nid = _sheet_names(sheet.ids)
        for step in range(2):
            c.set_timing(step == 1)
            c.reset()
            c.begin_file(None, file_index=0, byte_base=0)
            c.feed_device(buf, n * reclen)
            st = c.end_file()
            assert st.records == pin["total_reads"] and st.error == 0
            # 16-GiB launches: one for the second feed (direct commits, or logged ones whose first-feed folds
            # had room for a whole-feed aggregation)
            assert c.timing().scan_launches == (1 if launch_gib == 16 and step == 1 else 2)
            U, _, _ = c.finalize()
            assert U == pin["unique_codes"]
            keys, counts, _ = c.unique()
            c.set_sheet(sheet.idx1, sheet.idx2, [reverse_complement(x) for x in sheet.idx2], nid, len(names))
            out = c.classify(1, False)
            digest, first, last = synth.rows_digest(lib.decode_keys(keys), counts, out, sheet.idx1, sheet.idx2,
                                                    sheet.ids)
            assert first == pin["first_rows"] and last == pin["last_rows"], step
            assert digest == pin["rows_sha256"], step
    finally:
        c.device_free(buf)
        c.close()


@pytest.mark.parametrize("cfg", [3, 4])
def test_bench_geometry_pinned_cfg34(lib, cfg):
    """bench.py's config-3 shape (384 samples, 10+10, n=1, -rc: 100M SYN-v1 records = 7.8 GB in HBM, heavy
    commits logged, launch-log split/reduce, then -rc pass A, the per-name call, the idx2 rewrite and pass
    B) and config-4 shape (96 combinatorial 12x8 dual indexes, n=2), each one launch after the first feed against the REFERENCE's own frender_scan
    sequence on the same records (tests/golden/cfg3_pin.json / cfg4_pin.json, made by
    tests/golden/make_golden_cfg34.py): unique codes, every final row in order (sha256), the first/last
    1000 rows, and for config 3 every pass-A row (with the rc columns) and every per-name rc call.  Two
    steps on one context with 16-GiB launches, as bench.py runs them."""
    import json

    from frender_amd import synth

    path = os.path.join(os.path.dirname(__file__), "golden", f"cfg{cfg}_pin.json")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated")
    with open(path) as f:
        pin = json.load(f)
    n = pin["reads"]
    L, S = (10, 384) if cfg == 3 else (8, 96)
    sheet = synth.make_sheet(S, L, L, combinatorial=(12, 8) if cfg == 4 else None)
    reclen = synth.record_length(L, L, 8)
    c = lib.Context(device=0, chunk_bytes=(16 << 30) - (1 << 20), table_slots=1 << 22)
    buf = c.device_alloc(n * reclen + 64)
    try:
        # config 3: the reads of synth.CFG3_RC_NAMES carry rc(idx2), so the per-name call flips them
        c.synth_device(buf, 0, n, 8, 1, sheet.idx1,
                       synth.read_idx2(sheet, synth.CFG3_RC_NAMES if cfg == 3 else None))
        for step in range(2):
            c.reset()
            c.begin_file(None, file_index=0, byte_base=0)
            c.feed_device(buf, n * reclen)
            st = c.end_file()
            assert st.records == pin["total_reads"] and st.error == 0
            launches = c.timing().scan_launches
            c.finalize()
            got = synth.pin_rows(c, sheet, 1 if cfg == 3 else 2, cfg == 3)
            assert synth.pin_differences(got, pin) == [], (cfg, step)
            if cfg == 3:  # pass B ran on the rewritten idx2 list
                assert sorted(r[0] for r in got["rc_calls"] if r[3]) == sorted(synth.CFG3_RC_NAMES)
        # the second feed: config 4 (no commit logs) one launch; config 3's commits log, so its ranges stay
        # <= 4 GiB (one launch-log aggregation per range: its LDS fold holds that many distinct codes)
        assert launches == (2 if cfg == 3 else 1), launches
    finally:
        c.device_free(buf)
        c.close()


@pytest.mark.parametrize("mode", ["host", "device"])
def test_per_file_counts(lib, mode):
    """fr_get_presence_counts: the reads of each code in each file (the reference's per-file tables,
    frender.py:171-177), fast, wide and exotic codes, over several files and a table that grows."""
    from oracle.frender_oracle import tally_text
    from frender_amd import synth
    rng = random.Random(11)
    sheet = synth.make_sheet(24, 8, 8)
    files = []
    for i in range(4):
        text = synth.generate_bytes(sheet, i * 50000, rng.randint(20000, 60000), R=8, seed=9).decode()
        extra = "".join(f"@x{j} 1:N:0:{rng.choice(['acgtacgt+ttttcccc', 'AcGt+TTTT', 'ACGTACGTACGT+ACGTACGTAC'])}"
                        f"\nAC\n+\nFF\n" for j in range(rng.randint(0, 300)))
        files.append((text + extra).encode())
    c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 12)
    try:
        c.reset()
        for data in files:
            c.begin_file(None)
            if mode == "device":
                p = c.device_alloc(len(data) + 16)
                c.copy_to_device(p, data)
                c.feed_device(p, len(data))
                c.end_file()
                c.device_free(p)
            else:
                c.feed(data)
                c.end_file()
        c.finalize()
        keys, _, _ = c.unique()
        pu, pf = c.presence()
        ecodes, _, _, epc, epf = c.exotic_table()
        pn, epn = c.presence_counts(len(epc))
        codes = lib.decode_keys(keys)
        got = {}
        for u, f, k in zip(pu.tolist(), pf.tolist(), pn.tolist()):
            got[(codes[u], f)] = k
        for u, f, k in zip(epc.tolist(), epf.tolist(), epn.tolist()):
            got[(ecodes[u].decode(), f)] = k
        exp = {}
        for f, data in enumerate(files):
            for code, k in tally_text(data.decode())[0].items():
                exp[(code, f)] = k
        assert got == exp
    finally:
        c.close()


FORMER_KNOBS = {  # environment variables fr_create read before round 5, each at a hostile value
    "FR_ABLATE": "128", "FR_GRID": "1", "FR_FLUSH_AT": "0", "FR_NBR": "0", "FR_COLD_CAP": "1",
    "FR_LAUNCH_BYTES": "4096", "FR_LOG": "0", "FR_LOG_MIN": "0", "FR_LOG_HOT": "1", "FR_CHUNK_TILES": "2",
    "FR_CHUNK_TILES_HEAVY": "2", "FR_RAMP": "0", "FR_RAMP_UP_S": "100", "FR_RAMP_DOWN_S": "100",
    "FR_RAMP_DOWN_PCT": "1", "FR_RAMP_DOWN_PCT_H": "1", "FR_SPEC_COMMIT": "0"}


def test_stray_env_has_no_effect(lib, monkeypatch):
    """The product library reads no tuning from the environment (the geometry comes from fr_create's
    defaults or an explicit fr_tuning; timing ablations are compile-time FR_ABLATE builds): with every
    former knob set to a hostile value, a scan gives the identical table, classification, launch count
    and geometry as without them (FR_LAUNCH_BYTES used to override the caller's chunk_bytes)."""
    from frender_amd import synth
    from frender_amd.host import reverse_complement
    from frender_amd.scan import _sheet_names

    sheet = synth.make_sheet(24, 8, 8)
    n = 300000
    data = synth.generate_bytes(sheet, 0, n, R=8, seed=4)
    names, nid = _sheet_names(sheet.ids)

    def run():
        c = lib.Context(device=0, chunk_bytes=1 << 22, table_slots=1 << 14)
        try:
            p = c.device_alloc(len(data) + 16)
            c.copy_to_device(p, data)
            c.reset()
            c.begin_file(None)
            c.feed_device(p, len(data))
            st = c.end_file()
            c.device_free(p)
            c.finalize()
            keys, counts, first = c.unique()
            c.set_sheet(sheet.idx1, sheet.idx2, [reverse_complement(x) for x in sheet.idx2], nid, len(names))
            out = c.classify(1, True)
            d = c.diag()
            return (st.records, keys.tolist(), counts.tolist(), first.tolist(),
                    {k: np.asarray(v).tolist() for k, v in out.items()}, c.timing().scan_launches,
                    d["grid"], d["chunk_tiles"], d["spec_replays"])
        finally:
            c.close()

    base = run()
    for k, v in FORMER_KNOBS.items():
        monkeypatch.setenv(k, v)
    assert run() == base
    assert base[5] == -(-len(data) // (1 << 22))  # launches of the caller's chunk_bytes


def test_tuning_struct_changes_geometry_not_results(lib):
    """fr_create_tuned: an explicit fr_tuning changes the launch geometry (grid, chunk size, logging,
    ramps, speculation) but never the table."""
    from frender_amd import synth

    sheet = synth.make_sheet(96, 8, 8)
    data = synth.generate_bytes(sheet, 0, 400000, R=8, seed=6)
    exp = oracle_tally([data])
    for tuning in (None, {"grid": 3, "chunk_tiles": 2, "ramp": 0}, {"log_min": 0, "log_hot": 1},
                   {"spec_commit": 0, "cold_cap": 1024, "flush_at": 8}, {"ramp_up_s": 7, "ramp_down_pct": 10}):
        c = lib.Context(device=0, chunk_bytes=1 << 21, table_slots=1 << 14, tuning=tuning)
        try:
            assert_same(gpu_tally(c, lib, [data], mode="device"), exp)
            if tuning and "grid" in tuning:
                assert c.diag()["grid"] == 3
        finally:
            c.close()
    with pytest.raises(ValueError):
        lib.Context(device=0, tuning={"no_such_field": 1})


@pytest.mark.parametrize("world", [2, 3])
def test_cli_ranks_bgzf_single_file(tmp_path, world):
    """`scan --gpus N` on ONE BGZF file: every rank decodes only its part (fr_gz_part_open, no prefix
    inflate), and the CSVs equal the oracle's (LF and CRLF records, -rc)."""
    import argparse
    import contextlib
    import io
    import subprocess
    import sys

    from frender_amd import synth
    from oracle import frender_oracle

    sheet = synth.make_sheet(24, 8, 8, seed=5)
    sheet.write_csv(str(tmp_path / "sheet.csv"))
    raw = synth.generate_bytes(sheet, 0, 400000, R=8, seed=21, rc_names={sheet.ids[2]})
    for name, data in (("bg_R1.fq.gz", raw), ("bgcr_R1.fq.gz", raw.replace(b"\n", b"\r\n"))):
        p = tmp_path / name
        p.write_bytes(synth.bgzf_bytes(data))
        outs = {}
        for label in ("gpu", "oracle"):
            sub = tmp_path / f"{name}_{label}"
            sub.mkdir()
            if label == "gpu":
                env = dict(os.environ, FRENDER_DIST_BACKEND="gloo",
                           PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
                r = subprocess.run([sys.executable, "-m", "frender_amd", "scan", "-n", "1", "-rc", "-c", "4", "-o", "bg",
                                    "-b", str(tmp_path / "sheet.csv"), "--gpus", str(world), str(p)], cwd=str(sub),
                                   env=env, capture_output=True, text=True, timeout=240)
                assert r.returncode == 0, r.stderr[-3000:]
            else:
                args = argparse.Namespace(n=1, rc=True, c=1.0, s=None, o="bg", p=None, b=str(tmp_path / "sheet.csv"),
                                          files=[str(p)])
                cwd = os.getcwd()
                os.chdir(sub)
                try:
                    with contextlib.redirect_stdout(io.StringIO()):
                        frender_oracle.scan(args)
                finally:
                    os.chdir(cwd)
            outs[label] = {x: (sub / x).read_bytes() for x in sorted(os.listdir(sub))}
        assert outs["gpu"] == outs["oracle"] and outs["gpu"]
