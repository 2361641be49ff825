"""bench.py's multi-GPU entry point: `bench.py --gpus N` runs N ranks (its own launcher when no
torchrun set WORLD_SIZE) or refuses a --gpus / WORLD_SIZE disagreement; the -m gpu rehearsal checks
that 2 ranks (gloo, one GPU) report the single-rank table for the same records."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env.update(kw)
    return env


def _json_line(out: str) -> dict:
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_flag_launches_ranks(n):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--rank-check"], capture_output=True, text=True,
                       env=_env(), timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert _json_line(p.stdout) == {"rank_check": True, "world": n, "ranks_joined": n}


def test_bench_refuses_world_mismatch():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr


@pytest.mark.gpu
def test_bench_two_gloo_ranks_match_one_rank():
    """Weak scaling: 2 ranks x 2M reads (records [0, 2M) and [2M, 4M) of one logical file) merged by the
    all-to-all must give the 1-rank table of 4M reads, row for row (order-independent checksum)."""
    common = ["--steps", "1", "--warmup", "0", "--no-cpu"]
    one = subprocess.run([sys.executable, BENCH, "--reads", "4000000", *common], capture_output=True, text=True,
                         env=_env(), timeout=300)
    assert one.returncode == 0, one.stderr[-3000:]
    two = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--reads", "2000000",
                          *common], capture_output=True, text=True, env=_env(), timeout=300)
    assert two.returncode == 0, two.stderr[-3000:]
    a, b = _json_line(one.stdout), _json_line(two.stdout)
    assert b["n_gpus"] == 2 and a["n_gpus"] == 1
    assert a["config"]["unique_codes"] == b["config"]["unique_codes"]
    assert a["config"]["table_checksum"] == b["config"]["table_checksum"]
