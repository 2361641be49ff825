"""GPU parity: the HIP scan path (through the C ABI) against the CPU oracle and the
reference's golden vectors.  Bit-exact everywhere: this is integer/byte work."""
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


def test_speculative_commit_replay(lib):
    """A file whose chunks look like 4-line FASTQ one line off the true phase: every chunk after
    the first guesses the wrong line phase, commits at once, the launch-end check catches it and
    the feed is replayed with every chunk waiting for its exact prefix (fr_feed_device)."""
    recs = ["L 1:N:0:AAAA+CCCC\n"] + [f"@r{i} 1:N:0:ACGT+ACGT\nACGT\n+\nA AC\n" for i in range(60000)]
    data = "".join(recs).encode()
    exp = oracle_tally([data])
    assert list(exp[0]) == ["AAAA+CCCC", "AC"]
    c = lib.Context(device=0, chunk_bytes=1 << 20, table_slots=1 << 16)
    try:
        assert_same(gpu_tally(c, lib, [data], mode="device"), exp)
        assert c.diag()["spec_replays"] == 1
        good = "".join(f"@r{i} 1:N:0:ACGT+ACG{'ACGT'[i % 4]}\nACGT\n+\nFFFF\n" for i in range(60000)).encode()
        assert_same(gpu_tally(c, lib, [data, good], mode="device"), oracle_tally([data, good]))
        assert c.diag()["spec_replays"] == 2  # the second file (non-empty table) commits without a replay
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
    ctx.set_sheet(idx1, idx2, [reverse_complement(x) for x in idx2], nid, len(names))
    out = ctx.classify(nsubs, rc)
    assert out["err_unique"] == -1
    f_exp = {n: 0 for n in names}
    r_exp = {n: 0 for n in names}
    for j, code in enumerate(codes):
        e = classify_code(code, 1, idx1, idx2, ids, nsubs, rc)
        got_t = lib.CLASS_NAMES[out["cls"][j]]
        assert got_t == e["read_type"], (code, got_t, e)
        assert (idx1[out["m1"][j]] if out["m1"][j] >= 0 else "") == e["matched_idx1"] or rc
        assert (idx2[out["m2"][j]] if out["m2"][j] >= 0 else "") == e["matched_idx2"]
        assert (ids[out["row"][j]] if out["row"][j] >= 0 else "") == e["sample_name"]
        if rc:
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


@pytest.mark.parametrize("grid,cap,chunk", [(1, 1536, 1 << 24), (4, 0, 1 << 26), (64, 16, 1 << 26), (512, 1536, 1 << 30)])
def test_many_tiles_per_workgroup(lib, monkeypatch, grid, cap, chunk):
    """Few workgroups walking many tiles each (look-back windows sliding past 64 tiles),
    with the LDS table capped so most codes take the direct-to-HBM path."""
    from frender_amd import synth
    from oracle.frender_oracle import tally_text
    monkeypatch.setenv("FR_GRID", str(grid))
    monkeypatch.setenv("FR_FLUSH_AT", str(cap))
    c = lib.Context(device=0, chunk_bytes=chunk, table_slots=1 << 16)
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


@pytest.mark.parametrize("name", demux_case_names())
def test_demux_golden_on_gpu(name):
    from frender_amd.demux import frender_demux
    diffs = run_demux_case(name, frender_demux)
    assert not diffs, "\n".join(diffs)


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
