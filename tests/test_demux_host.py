"""Host helpers of the demux window (frender_amd/demux.py): a window is a list of decoded blocks that
is never joined on the host, so the line at a record start and the bytes carried into the next window
are taken across block edges."""
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
