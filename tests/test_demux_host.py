"""Host helpers of the demux window (frender_amd/demux.py): a window is a list of decoded blocks that
is never joined on the host, so the line at a record start and the bytes carried into the next window
are taken across block edges; and the packing of the results file's codes into the device table's keys."""
from frender_amd.demux import _line_at, _tail


def test_line_at_across_blocks():
    parts = [b"ab\ncd", b"ef", b"gh\nij", b"k\n", b"tail"]
    whole = b"".join(parts)
    for start in range(len(whole) + 1):
        e = whole.find(b"\n", start)
        want = whole[start:] if e < 0 else whole[start:e]
        assert _line_at(parts, start) == want, start


def test_tail_across_blocks():
    parts = [b"ab\ncd", b"", b"ef", b"gh\nij", b"k\n"]
    whole = b"".join(parts)
    for start in range(len(whole) + 2):
        assert b"".join(_tail(parts, start)) == whole[start:], start
    assert _tail(parts, 0)[0] is parts[0]  # whole blocks are kept, not copied


def test_pack_fast_matches_per_character_packing():
    """The demux's device-table keys (3 bits per character of A C G T N +, 1..21 characters); any other
    character or length leaves the code to the string path."""
    import random

    import numpy as np

    from frender_amd import _lib

    def one(c):
        if not 1 <= len(c) <= 21:
            return 0, False
        v = 0
        for j, ch in enumerate(c):
            s = "ACGTN+".find(ch)
            if s < 0:
                return 0, False
            v |= (s + 1) << (3 * j)
        return v, True

    rng = random.Random(3)
    codes = ["".join(rng.choice("ACGTN+") for _ in range(rng.randint(0, 23))) for _ in range(3000)]
    codes += ["", "A", "ACGTX", "AC\x00", "A\x00C", "é", "A" * 21, "A" * 22, "acgt", "++", "C" * 20 + "Ł"]
    keys, ok = _lib.pack_fast(codes)
    for i, c in enumerate(codes):
        v, good = one(c)
        assert bool(ok[i]) == good and int(keys[i]) == v, repr(c)
    k0, o0 = _lib.pack_fast([])
    assert k0.size == 0 and o0.size == 0 and k0.dtype == np.uint64
