"""Train a policy from the reference's YAML configs (ballbot_rl/training/train.py:38-284).

    python -m ballbot_rl.training.train --config configs/train/ppo_directional.yaml
    torchrun --nproc-per-node 8 ... -m ballbot_rl.training.train --config ...   (one rank per GPU)

Same config keys as the reference (algo.*, hidden_sz, num_envs, total_timesteps,
seed, evaluation.*, env.*, problem.terrain/reward).  Differences, by design:
* `num_envs` envs run in ONE BallbotVecEnv per GPU (split over ranks) instead of
  a SubprocVecEnv of CPU MuJoCo processes; GPU-sized runs raise num_envs into the
  thousands and lower n_steps (configs in tools/ppo_gpu.yaml);
* the interactive overwrite/updates-per-rollout confirmations (train.py:194-266)
  become printed warnings -- a batch job cannot answer them;
* checkpoints are safetensors (no pickled SB3 zip); with a `camera` section the
  depth cameras are on, as in the reference; `frozen_cnn` names an encoder
  pretrained by ballbot_rl.encoders.pretrain (safetensors) -- the reference's
  pickled encoder files are never loaded -- else the rgbd
  branches are the Extractor's trainable CNNs.
Output directory layout as the reference: outputs/experiments/runs/
{timestamp}_{algo}_{terrain}_{reward}_seed{seed}/ with config.yaml, info.txt,
progress.csv (SB3 columns), best_model.safetensors and final_model.safetensors.
"""
from __future__ import annotations

import argparse
import json
import os
import random
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, Optional

import numpy as np
import torch
import torch.distributed as dist
import yaml

from ballbot_gym.core.config import get_component_config, load_training_config
from ballbot_rl.training.logger import CSVLogger
from ballbot_rl.training.ppo import BatchedPPO
from ballbot_rl.training.schedules import lr_schedule


def ppo_kwargs(config: Dict[str, Any]) -> Dict[str, Any]:
    """The PPO(...) arguments the reference passes (train.py:125-142, 39-56)."""
    a = config["algo"]
    lr = float(a["learning_rate"])
    h = int(config.get("hidden_sz", 128))
    return dict(ent_coef=float(a["ent_coef"]), clip_range=float(a["clip_range"]),
                target_kl=float(a["target_kl"]) if a.get("target_kl") is not None else None,
                vf_coef=float(a["vf_coef"]), learning_rate=lr if lr != -1 else lr_schedule,
                n_steps=int(a["n_steps"]), batch_size=int(a["batch_sz"]), n_epochs=int(a["n_epochs"]),
                normalize_advantage=bool(a["normalize_advantage"]), weight_decay=float(a["weight_decay"]),
                net_arch={"pi": [h] * 4, "vf": [h] * 4})


def experiment_dir(config: Dict[str, Any], out: Optional[str] = None) -> Path:
    ts = datetime.now().strftime("%Y%m%d_%H%M%S")
    terrain = config.get("problem", {}).get("terrain", {}).get("type", "unknown")
    reward = config.get("problem", {}).get("reward", {}).get("type", "unknown")
    name = f"{ts}_{config['algo']['name']}_{terrain}_{reward}_seed{config.get('seed', 'unknown')}"
    if out and out.strip():
        p = Path(out).resolve()
        return p / name if (p.is_dir() or not p.suffix) else p
    return Path("outputs/experiments/runs") / name


def make_env(config: Dict[str, Any], num_envs: int, device, seed: int, precision: str = "fp64", stream_seeds=None):
    """One rank's BallbotVecEnv.  stream_seeds None: every env on np_random(seed)."""
    from ballbot_gym.envs import BallbotVecEnv

    env_cfg = {"camera": config.get("camera", {}), "env": config.get("env", {}), "logging": config.get("logging", {})}
    # the reference trains with its depth cameras on (make_ballbot_env(disable_cams=False),
    # training/utils.py:11-20) whenever the config has a camera section
    cams = bool(config.get("camera")) and not config.get("disable_cameras", False)
    return BallbotVecEnv(num_envs, device=device, reward_config=get_component_config(config, "reward"),
                         terrain_config=get_component_config(config, "terrain"), env_config=env_cfg, seed=seed,
                         precision=precision, n_terrains=config.get("n_terrains"), disable_cameras=not cams,
                         stream_seeds=stream_seeds, shared_stream=stream_seeds is None,
                         reward_compat=str(config.get("reward_compat", "reference")))


def main(config: Dict[str, Any], seed: int, out: Optional[str] = None, total_timesteps: Optional[int] = None,
         precision: str = "fp64", update_mode: Optional[str] = None) -> BatchedPPO:
    from ballbot_gym.distributed import env_shard, shard_stream_seeds
    from ballbot_rl.evaluation import evaluate_policy

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BB_TRAIN_BACKEND=gloo: ranks sharing the box's GPUs over gloo (a one-GPU rehearsal of the
    # multi-GPU run, as bench.py's BB_BENCH_BACKEND); the multi-GPU default is RCCL ("nccl"), one
    # GPU per rank
    backend = os.environ.get("BB_TRAIN_BACKEND", "nccl")
    gpu = local if backend == "nccl" else local % max(torch.cuda.device_count(), 1)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    n_total = int(config["num_envs"])
    first, n_local = env_shard(n_total, rank, world)
    # training env g draws its terrains from np_random(seed + g): PPO(seed=seed) seeds the
    # VecEnv (env i -> seed + i) and learn()'s first reset re-seeds every env's _np_random
    # with it (train.py:126-141, ballbot_env.py:596); config terrain_streams: shared keeps
    # one np_random(seed) for every env instead
    shared = str(config.get("terrain_streams", "per_env")) == "shared"
    env = make_env(config, n_local, dev, seed, precision, shard_stream_seeds(seed, first, n_local, per_env=not shared))
    eval_cfg = config.get("evaluation", {}) or {}
    n_eval = int(eval_cfg.get("n_episodes", 8))
    # the eval VecEnv: N_ENVS envs, env i on np_random(seed + N_ENVS + i) (train.py:90-97);
    # evaluation.num_envs overrides its size for GPU-sized runs (thousands of training envs)
    n_eval_envs = int(eval_cfg.get("num_envs", n_total))
    eval_env = (make_env(config, n_eval_envs, dev, seed + n_total, precision,
                         shard_stream_seeds(seed + n_total, 0, n_eval_envs, per_env=True)) if rank == 0 else None)

    out_path = experiment_dir(config, out if out is not None else config.get("out"))
    logger = None
    if rank == 0:
        if out_path.exists() and any(out_path.iterdir()):
            print(f"warning: output directory {out_path} exists and is not empty; files will be overwritten")
        out_path.mkdir(parents=True, exist_ok=True)
        with (out_path / "config.yaml").open("w") as f:
            yaml.safe_dump(config, f)
        with (out_path / "info.txt").open("w") as f:
            json.dump({"algo": config["algo"]["name"], "num_envs": n_total, "out": str(out_path),
                       "resume": config.get("resume", ""), "seed": seed, "world_size": world}, f)
        logger = CSVLogger(str(out_path) + "/", stdout=True)
        upd = config["algo"]["n_epochs"] * n_total * config["algo"]["n_steps"] / config["algo"]["batch_sz"]
        print(f"{upd:.1f} gradient updates per rollout (n_epochs x num_envs x n_steps / batch_sz)")

    frozen = None
    fc = str(config.get("frozen_cnn") or "")
    if env.cameras and fc.endswith(".safetensors") and Path(fc).exists():
        from ballbot_rl.encoders import load_frozen_encoder

        frozen = load_frozen_encoder(fc, device=dev)  # the reference's frozen_cnn (train.py:45-47)
    elif env.cameras and fc and rank == 0:
        print(f"warning: frozen_cnn {fc!r} is not a safetensors encoder (pickled modules are not loaded); "
              "the rgbd branches train from scratch")
    model = BatchedPPO(env, seed=seed, logger=logger, frozen_encoder=frozen, update_mode=update_mode,
                       **ppo_kwargs(config))
    if config.get("resume"):
        model.load_policy(config["resume"])
    model.warm_up()  # the update graphs and first library calls, before the run (SB3's _setup_model)
    eval_freq = int(eval_cfg.get("freq", 5000))
    on_rollout = None
    if rank == 0 and eval_env is not None:
        from ballbot_rl.training.callbacks import EvalCallback

        on_rollout = EvalCallback(eval_env, n_eval_episodes=n_eval, eval_freq=eval_freq, n_total_envs=n_total,
                                  log_path=out_path / "results", best_model_save_path=out_path)

    total = int(float(total_timesteps if total_timesteps is not None else config["total_timesteps"]))
    model.learn(total_timesteps=total, rollout_callback=on_rollout)
    if rank == 0:
        model.save(str(out_path / "final_model.safetensors"))
    env.close()
    if eval_env is not None:
        eval_env.close()
    model.out_path = out_path
    return model


def cli_main() -> None:
    ap = argparse.ArgumentParser(description="Train a policy on the MI355X batched ballbot env.")
    ap.add_argument("--config", required=True, help="training YAML (reference format)")
    ap.add_argument("--total-timesteps", type=float, default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--precision", default="fp64", choices=["fp32", "fp64"])
    ap.add_argument("--update-mode", default=None, choices=["gather", "allreduce"],
                    help="multi-GPU PPO update: gather the rollouts to rank 0 (north_star; the default) or the "
                         "data-parallel all-reduce")
    args = ap.parse_args()
    cfg = load_training_config(str(Path(args.config).resolve()))
    seed = int(cfg.get("seed", 0))
    if seed != -1:
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
    main(cfg, seed, out=args.out, total_timesteps=None if args.total_timesteps is None else int(args.total_timesteps),
         precision=args.precision, update_mode=args.update_mode)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    cli_main()
