"""The reference-shaped seam (frender_amd/seam.py): tally_barcodes / process / call_rc_mode_per_id
return the reference's data shapes (frender.py:183-207, :391-426, :354-388), so the reference's own
control flow and host code run on them unchanged.

The reference's control flow here is the oracle's restatement of frender_scan (oracle.frender_oracle.scan,
frender.py:567-642: flatten_results, report_rc_call_info, the idx2 rewrite, the second pass,
call_barcodes_correctly_distributed with its demux_ok mutation, report_analysis) with its three seam
calls replaced by frender_amd.seam's: the outputs must equal the reference's golden CSVs.

CPU: the seam over tests/fake_ctx.py's stand-in context (the mapping logic).  GPU (-m gpu): over the
HIP library, every golden case."""
from __future__ import annotations

import contextlib

import pytest

from harness import case_names, run_case

SEAM_CASES = ["s96_n1_rc", "demux_ok_samples", "same_basename_two_dirs", "three_part_code"]


@contextlib.contextmanager
def _seam_in_oracle(ctx):
    """oracle.frender_oracle.scan with tally / classify_all / rc_calls -> frender_amd.seam."""
    from oracle import frender_oracle as O

    from frender_amd import seam

    saved = (O.tally, O.classify_all, O.rc_calls)
    O.tally = lambda cores, paths, sample=None: seam.tally_barcodes(cores, paths, sample, ctx=ctx)
    O.classify_all = lambda cores, total, sheet, n, rc: seam.process(cores, total, sheet, n, rc, ctx=ctx)
    O.rc_calls = seam.call_rc_mode_per_id
    try:
        yield O.scan
    finally:
        O.tally, O.classify_all, O.rc_calls = saved


def _check_case(name, ctx):
    with _seam_in_oracle(ctx) as fn:
        diffs = run_case(name, fn)
    assert not diffs, "\n".join(diffs)


@pytest.mark.parametrize("name", SEAM_CASES + ["comb96_n1_rc", "dup_sheet_row", "lowercase", "len_mismatch",
                                               "single_index", "rc_palindrome_ambig"])
def test_seam_in_reference_flow_cpu(name):
    from fake_ctx import FakeContext

    _check_case(name, FakeContext())


def test_seam_shapes_cpu(tmp_path):
    """Key order, per-file counts (same basename: the later file wins), the per-code dict's keys in the
    reference's order, demux_ok mutation, and the rc sums from the mapping == from the flattened list."""
    from fake_ctx import FakeContext

    from frender_amd import seam, synth

    sheet = synth.make_sheet(8, 8, 8)
    sheet.write_csv(str(tmp_path / "sheet.csv"))
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    recs = {"a/x_R1.fq.gz": ["AAAA+CCCC", "GGGG+TTTT", "AAAA+CCCC"], "b/x_R1.fq.gz": ["GGGG+TTTT", "NNNN+NNNN"],
            "y_R1.fq.gz": ["GGGG+TTTT", "AAAA+CCCC", "GGGG+TTTT", "acgt+acgt", "AcGt+ACGT+GG"]}
    files = []
    for rel, codes in recs.items():
        text = "".join(f"@r{i} 1:N:0:{c}\nA\n+\nF\n" for i, c in enumerate(codes))
        synth.write_fastq_gz(str(tmp_path / rel), text.encode())
        files.append(str(tmp_path / rel))
    ctx = FakeContext()
    bc = seam.tally_barcodes(1, files, ctx=ctx)
    assert list(bc) == ["total", "x_R1.fq.gz", "y_R1.fq.gz"]
    assert dict(bc["total"]) == {"AAAA+CCCC": 3, "GGGG+TTTT": 4, "NNNN+NNNN": 1, "acgt+acgt": 1, "AcGt+ACGT+GG": 1}
    assert list(bc["total"]) == ["AAAA+CCCC", "GGGG+TTTT", "NNNN+NNNN", "acgt+acgt", "AcGt+ACGT+GG"]
    assert dict(bc["x_R1.fq.gz"]) == {"GGGG+TTTT": 1, "NNNN+NNNN": 1}  # b/ replaces a/ (frender.py:204-205)
    assert dict(bc["y_R1.fq.gz"]) == {"AAAA+CCCC": 1, "GGGG+TTTT": 2, "acgt+acgt": 1, "AcGt+ACGT+GG": 1}
    assert bc["y_R1.fq.gz"].get("NNNN+NNNN", 0) == 0 and "total" in bc and "nope" not in bc
    with pytest.raises(KeyError):
        bc["nope"]
    idx = {"id": list(sheet.ids), "idx1": ["AAAA", "GGGG", "CCCC"], "idx2": ["CCCC", "TTTT", "GGGG"]}
    idx["id"] = idx["id"][:3]
    res = seam.process(1, bc["total"], idx, 0, True, ctx=ctx)
    assert list(res) == list(bc["total"])
    r = res["AAAA+CCCC"]
    assert list(r) == ["matched_idx1", "matched_idx2", "read_type", "sample_name", "reads", "matched_rc_idx2",
                       "rc_read_type", "rc_sample_name"]
    assert (r["read_type"], r["sample_name"], r["reads"]) == ("demuxable", idx["id"][0], 3)
    res["AAAA+CCCC"]["demux_ok"] = False
    assert res["AAAA+CCCC"]["demux_ok"] is False  # kept: the reference's mark-up survives to its CSV writer
    flat = [dict(idx1=c.split("+")[0], idx2=c.split("+")[1], **res[c]) for c in res]
    assert seam.call_rc_mode_per_id(res, idx["id"]) == seam.call_rc_mode_per_id(flat, idx["id"])
    plain = seam.process(1, dict(bc["total"]), idx, 0, False, ctx=ctx)  # any {code: reads} mapping
    assert [plain[c] for c in plain] == [{k: v for k, v in seam.process(1, bc["total"], idx, 0, False, ctx=ctx)[c].items()}
                                         for c in plain]
    with pytest.raises(AssertionError):
        seam.call_rc_mode_per_id(plain, idx["id"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", case_names())
def test_seam_in_reference_flow_gpu(name):
    from frender_amd import scan

    _check_case(name, scan.default_context())
