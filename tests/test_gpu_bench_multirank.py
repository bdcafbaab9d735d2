"""bench.py's multi-rank path (E1), rehearsed on one GPU.

The driver runs `torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
on an 8-GPU node with RCCL, one GPU per rank.  Here two ranks share the one GPU
and talk over gloo (BB_BENCH_BACKEND=gloo): the same env sharding (global env
ids, per-env terrain generators), barriers, max-over-ranks timing and rank-0
JSON line, with the weak-scaling bookkeeping the driver reads.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("terrain", ["flat", "perlin"])
def test_bench_two_ranks_over_gloo(terrain):
    env = dict(os.environ, BB_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"), "--gpus", "2",
           "--steps", "20", "--warmup", "5", "--burn-in", "20", "--envs", "512", "--terrain", terrain,
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints ONE JSON line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["total_envs"] == 1024 and line["config"]["envs_per_gpu"] == 512
    assert line["value"] > 0 and line["steps"] == 20
    assert line["value"] == pytest.approx(1024 * 20 / (line["ms_per_step"] * 20 / 1e3), rel=1e-6)
    assert "env-sharded x2" in line["config"]["parallelism"]
    # two ranks share the chip: each rank's persistent relief pair (perlin) must still have
    # finished every launch without its budget firing (bench.py would have exited non-zero)
    assert line["stats"]["pair_budget"] == 0 and line["status"] == "ok"
