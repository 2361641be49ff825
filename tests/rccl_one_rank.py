#!/usr/bin/env python3
"""One-rank RCCL rehearsal of the multi-GPU device paths (run by tests/test_gpu_rccl.py in a fresh
process: the `nccl` process group is the first thing that touches the GPU).

The 8-GPU scaling run is the driver's; on the one GPU a pool box gives, a world of ONE rank still runs
every collective of frender_amd/dist.py through RCCL on device tensors, and the stream hand-offs
between the library's non-blocking stream and torch's / RCCL's (stream contract):

  A. the bench's merge pieces on a finalized table: export_rows (library stream -> torch tensor),
     exchange (all_to_all_single of sizes and rows), gather_rows (all_gather + send/recv path), the
     small all-reduces, and partition_merge_device (exchange -> reset -> merge_rows -> finalize);
  B. the product: `scan` through dist.sharded_tally (dist.world_group forced to the 1-rank group),
     whose CSVs must equal the one-GPU scan's and the oracle's.

Prints one JSON line and exits 0 when every check holds.  Not a scaling measurement.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1

    from frender_amd import _lib, dist as D, scan, synth
    from frender_amd.host import reverse_complement
    from oracle import frender_oracle

    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    # ---- A: device pieces on a finalized table ----------------------------------------------------
    sheet = synth.make_sheet(96, 8, 8)
    n = 400_000
    ctx = _lib.Context(device=0, chunk_bytes=1 << 24, table_slots=1 << 16)
    buf = ctx.device_alloc(n * synth.record_length(8, 8, 8) + 64)
    ctx.synth_device(buf, 0, n, 8, 1, sheet.idx1, sheet.idx2)
    ctx.reset()
    ctx.begin_file(None)
    ctx.feed_device(buf, n * synth.record_length(8, 8, 8))
    st = ctx.end_file()
    assert st.records == n
    U, _, _ = ctx.finalize()
    keys, counts, first = ctx.unique()
    ref_rows = np.stack([keys.view(np.int64), counts.view(np.int64), first.view(np.int64)], 1)
    wire = D.wire_of(dist, ctx)
    assert wire.type == "cuda"
    rows = ctx.export_rows(wire)
    assert rows.is_cuda and np.array_equal(rows.cpu().numpy(), ref_rows)
    got = D.exchange(dist, wire, rows, D.owner_of(rows[:, 0], 1))
    assert got.is_cuda and torch.equal(got, rows.contiguous())
    g = D.gather_rows(dist, wire, rows)
    assert len(g) == 1 and np.array_equal(g[0], ref_rows)
    v = [3, -5, 7]
    assert D.reduce_sum(dist, wire, v).tolist() == v
    assert D.reduce_max(dist, wire, v).tolist() == v
    assert D.reduce_min(dist, wire, v).tolist() == v
    blobs = D.gather_bytes(dist, wire, b"exotic\x00bytes")
    assert blobs == [b"exotic\x00bytes"]
    # the library's partitioned export (the RCCL merge's send side) at world 4 on this one GPU: owner blocks in
    # rank order, each row in the block of owner_of(key), the same rows as the table
    prow, pcnt = ctx.export_partitioned(4)
    pc = pcnt.cpu().tolist()
    assert sum(pc) == U and prow.shape == (U, 3)
    own = D.owner_of(prow[:, 0], 4).cpu().numpy()
    assert np.array_equal(own, np.repeat(np.arange(4), pc))
    pr = prow.cpu().numpy()
    assert np.array_equal(pr[np.lexsort(pr.T[::-1])], ref_rows[np.lexsort(ref_rows.T[::-1])])
    U2 = D.partition_merge_device(dist, wire, ctx)
    k2, c2, f2 = ctx.unique()
    assert U2 == U and np.array_equal(k2, keys) and np.array_equal(c2, counts) and np.array_equal(f2, first)
    # the classify of the merged partition (what the bench times after the merge)
    from frender_amd.scan import _sheet_names
    names, nid = _sheet_names(sheet.ids)
    ctx.set_sheet(sheet.idx1, sheet.idx2, [reverse_complement(x) for x in sheet.idx2], nid, len(names))
    cls = ctx.classify(1, False)
    assert cls["err_unique"] == -1
    ctx.device_free(buf)
    ctx.close()
    out["A"] = {"reads": n, "unique_codes": int(U), "merged_equal": True}

    # ---- B: the product scan through sharded_tally on the 1-rank RCCL group ------------------------
    real_world_group = D.world_group
    with tempfile.TemporaryDirectory() as d:
        sheet = synth.make_sheet(24, 8, 8, seed=5)
        sheet.write_csv(os.path.join(d, "sheet.csv"))
        files = synth.make_dataset(os.path.join(d, "in"), sheet, 120_000, 3, R=8, seed=13, rc_names={sheet.ids[2]})
        outs = {}
        for label in ("rccl", "one_gpu", "oracle"):
            sub = os.path.join(d, label)
            os.mkdir(sub)
            args = argparse.Namespace(n=1, rc=True, c=2.0, s=None, o="r1", p=None, b=os.path.join(d, "sheet.csv"),
                                      files=list(files))
            D.world_group = (lambda: dist) if label == "rccl" else real_world_group
            fn = frender_oracle.scan if label == "oracle" else scan.frender_scan
            cwd = os.getcwd()
            os.chdir(sub)
            try:
                with contextlib.redirect_stdout(io.StringIO()):
                    fn(args)
            finally:
                os.chdir(cwd)
                D.world_group = real_world_group
            outs[label] = {f.split("r1_")[0]: open(os.path.join(sub, f), "rb").read() for f in sorted(os.listdir(sub))}
        assert outs["rccl"] == outs["one_gpu"] == outs["oracle"], {k: sorted(v) for k, v in outs.items()}
        out["B"] = {"files": len(files), "csvs": sorted(outs["rccl"]), "equal_one_gpu_and_oracle": True}
    out["census"] = D.CENSUS
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
