"""The multi-GPU device paths over RCCL, on the one GPU a pool box has.

A one-rank `nccl` process group runs every collective of frender_amd/dist.py on device tensors and
the stream hand-offs between the library's stream and torch's / RCCL's (tests/rccl_one_rank.py).  The
N-rank protocol itself is covered by the gloo tests (test_dist_gloo.py, test_dist_scan.py); this is
the device-tensor half that gloo cannot run.  No scaling claim is made from it."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_rccl_one_rank_device_paths():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0", PYTHONPATH=os.path.dirname(HERE))
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_one_rank.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["A"]["merged_equal"] and out["B"]["equal_one_gpu_and_oracle"]
    assert out["census"]["exchange"]["calls"] >= 3 and out["census"]["gather_rows"]["calls"] >= 3
