"""The training entry point on more than one rank, rehearsed on one
GPU: `torch.distributed.run --nproc-per-node 2 -m ballbot_rl.training.train`, the reference's
CLI (/root/reference/ballbot_rl/training/train.py:284), with the two ranks sharing the box's GPU
over gloo (BB_TRAIN_BACKEND=gloo; the multi-GPU default is RCCL, one GPU per rank).  Each rank
steps its env shard; at the update the rollouts are gathered to rank 0 (north_star's design, the
default update_mode), which updates, evaluates and writes the run directory.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import yaml

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_train_cli_two_ranks_gather(tmp_path):
    env_cfg = {"env": {"max_allowed_tilt": 20, "max_ep_steps": 100, "max_wheel_velocity": 10.0},
               "problem": {"reward": {"type": "directional", "config": {"target_direction": [0.0, 1.0]}},
                           "terrain": {"type": "flat", "config": {}}}}
    train_cfg = {"env_config": str(tmp_path / "env.yaml"),
                 "algo": {"batch_sz": 2048, "clip_range": 0.015, "ent_coef": 0.001, "learning_rate": -1,
                          "n_epochs": 2, "n_steps": 8, "name": "ppo", "normalize_advantage": False, "target_kl": 0.3,
                          "vf_coef": 2.0, "weight_decay": 0.01},
                 "evaluation": {"freq": 8, "n_episodes": 4}, "hidden_sz": 64, "num_envs": 1024, "seed": 10,
                 "total_timesteps": 1024 * 8 * 2}
    (tmp_path / "env.yaml").write_text(yaml.safe_dump(env_cfg))
    (tmp_path / "train.yaml").write_text(yaml.safe_dump(train_cfg))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, BB_TRAIN_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2",
               PYTHONPATH=str(ROOT / "openballbot-rl_amd") + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out = tmp_path / "run"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "-m", "ballbot_rl.training.train", "--config",
           str(tmp_path / "train.yaml"), "--out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    runs = [d for d in out.iterdir() if d.is_dir()]  # the reference's <time>_<algo>_<terrain>_<reward>_seed<s> layout
    assert len(runs) == 1, runs
    out = runs[0]
    for f in ("config.yaml", "info.txt", "progress.csv", "final_model.safetensors"):
        assert (out / f).exists(), f
    info = json.loads((out / "info.txt").read_text())
    assert info["world_size"] == 2 and info["num_envs"] == 1024
    from ballbot_rl.training.logger import read_progress

    cols = read_progress(str(out / "progress.csv"))
    # rank 0 counts every rank's env-steps, and its updates' epochs (gather: it alone updates)
    last = {k: [v for v in cols[k] if v is not None][-1] for k in ("time/total_timesteps", "train/n_updates")}
    assert last["time/total_timesteps"] == 1024 * 8 * 2
    assert last["train/n_updates"] == 2  # SB3 dumps before the update: the first update's 2 epochs
