"""The C-ABI library loads here (no GPU) and exports every symbol include/frender_amd.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "frender_amd.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fr_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("fr_create", "fr_feed", "fr_feed_device", "fr_end_file", "fr_finalize", "fr_classify",
                 "fr_rc_counts", "fr_merge_unique_device"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import __graft_entry__ as g
    lib = ctypes.CDLL(g.build_lib())
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_binding_covers_the_header():
    from frender_amd import _lib
    assert sorted(_lib.EXPORTED) == declared()


def test_binding_fails_loudly_without_library(tmp_path):
    import subprocess
    import sys
    env = dict(os.environ, FRENDER_HIP_LIB=str(tmp_path / "missing.so"), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", "import frender_amd._lib"], env=env, capture_output=True, text=True)
    assert r.returncode != 0 and "not built" in r.stderr


def test_key_codec_roundtrip():
    import numpy as np
    from frender_amd import _lib
    codes = ["ACGT+TTGA", "A+C", "NNNNNNNNNN+NNNNNNNNNN", "ACGTACGT+ACGTACGT+AC"]
    sym = {"A": 1, "C": 2, "G": 3, "T": 4, "N": 5, "+": 6}
    keys = np.array([sum(sym[c] << (3 * i) for i, c in enumerate(s)) for s in codes], dtype=np.uint64)
    assert _lib.decode_keys(keys) == codes
    assert _lib.pack_lower("acgtx") == 1 | 2 << 3 | 3 << 6 | 4 << 9 | 7 << 12


def test_bench_refuses_traffic_of_another_tree(tmp_path):
    """bench.py reports PMC traffic only from a file taken on this source tree and launch shape."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from frender_amd._lib import source_tree_hash
    tree = source_tree_hash()
    p = str(tmp_path / "t.json")
    valu = {"insts_per_launch": 682000000, "insts_per_record": 13.64, "peak_g_insts_per_s": 614.4}
    rec = {"tree_hash": tree, "algorithmic_bytes_per_launch": 3.7e9, "samples": 96, "index_len": 8,
           "combinatorial": False, "hbm_bytes_per_launch": 4000000000, "traffic_over_algorithmic": 1.08,
           "valu": valu}
    for change, ok in (({}, True), ({"tree_hash": "0" * 16}, False), ({"samples": 384}, False)):
        with open(p, "w") as f:
            json.dump({**rec, **change}, f)
        t, note, v = bench.load_traffic(p, tree, 3.7e9, 96, 8, False)
        assert (t == 4000000000) == ok and (note.startswith("refused") != ok), note
        assert (v == valu) == ok  # the VALU figures travel with the traffic file, under the same checks
    r = bench.valu_roofline(valu, 1.45)  # 6.82e8 instructions in 1.45 ms against the bench's peaks
    g = 6.82e8 / 1.45e-3 / 1e9
    assert r["unit"] == "G wave64 VALU inst/s" and abs(r["frac"] - g / bench.VALU_PEAK_G) < 1e-3
    assert abs(r["frac_of_mix_ceiling"] - g / bench.VALU_MIX_G) < 1e-3
    assert r["simd_valu_busy"] is None  # no active-cycle counter in this record
    r2 = bench.valu_roofline(dict(valu, active_quad_cycles_per_launch=250_000_000), 1.45)
    busy = 4 * 2.5e8 / (bench.NUM_SIMDS * 1.45e-3 * bench.SIMD_CLOCK_GHZ * 1e9)  # VALU share of the SIMD cycles
    assert abs(r2["simd_valu_busy"] - busy) < 1e-3
    assert bench.valu_roofline(None, 1.45) is None
    assert bench.load_traffic(str(tmp_path / "absent.json"), tree, 3.7e9, 96, 8, False)[0] is None
