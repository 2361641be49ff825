"""The tally kernel's byte classifiers (frender_amd/csrc/fr_kernels.hip), restated on the host with
v_perm_b32's byte-select semantics and checked over every byte value:

* classify4 (three lookups) is exact for all 256 bytes: bit 0 line end ('\\n' or '\\r'), bit 1 '\\r',
  bit 2 ' ', bit 3 ':', bit 4 byte >= 0x80;
* classify4_fast (two lookups) gives exactly classify4's bits 0-3 for every ASCII byte whose class
  word lacks bit 7, and sets bit 7 only for the few ASCII bytes that read a fixed 0xFF entry
  (those wave-tiles take classify4); bytes >= 0x80 are caught by the kernel's separate bit-7 test.

The table constants are read from the kernel source, so an edit there is checked here."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = open(os.path.join(ROOT, "frender_amd", "csrc", "fr_kernels.hip")).read()


def v_perm(s0: int, s1: int, sel: int) -> int:
    """One byte of V_PERM_B32 {S0, S1} with selector byte sel (CDNA ISA): 0-7 pick a byte of the
    64-bit {S0:S1}, 8-11 replicate the sign bit of bytes 1, 3, 5, 7, 12 gives 0x00, 13-255 give 0xFF."""
    data = (s0 << 32) | s1
    if sel >= 13:
        return 0xFF
    if sel == 12:
        return 0x00
    if sel >= 8:
        return 0xFF if (data >> (15 + 16 * (sel - 8))) & 1 else 0x00
    return (data >> (8 * sel)) & 0xFF


def _tables(fn: str):
    body = SRC[SRC.index(f"u32 {fn}(u32 w)"):]
    body = body[:body.index("}")]
    num = r"(0x[0-9A-Fa-f]+|\d+)u?"
    return [(int(a, 0), int(b, 0)) for a, b in re.findall(r"perm\(" + num + ", " + num, body)]


def exact(b: int) -> int:
    c = 0
    if b in (0x0A, 0x0D):
        c |= 1
    if b == 0x0D:
        c |= 2
    if b == 0x20:
        c |= 4
    if b == 0x3A:
        c |= 8
    if b >= 0x80:
        c |= 16
    return c


def test_classify4_exact_for_every_byte():
    (lo_a, lo_b), (mid_a, mid_b), (top_a, top_b) = _tables("classify4")
    for b in range(256):
        c = v_perm(lo_a, lo_b, b & 7) & v_perm(mid_a, mid_b, (b >> 3) & 7) & v_perm(top_a, top_b, (b >> 6) & 3)
        assert c & 0x1F == exact(b), hex(b)


def test_classify4_fast_exact_or_flagged():
    (lo_a, lo_b), (hi_a, hi_b) = _tables("classify4_fast")
    flagged = []
    for b in range(128):
        c = v_perm(lo_a, lo_b, b & 7) & v_perm(hi_a, hi_b, (b >> 3) & 15)
        if c & 0x80:
            flagged.append(chr(b))
            continue
        assert c & 0x7F == exact(b), hex(b)
    # the class bytes themselves and everything a FASTQ record normally holds stay on the fast path
    for ch in "\n\r :@+ACGTN0123456789!\"#$%&'()*,-./;<=>?ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefgi":
        assert ch not in flagged, repr(ch)
    assert flagged == list("hjmprux z}".replace(" ", ""))
