"""PPO training throughput and learning curve on the GPU env.

    python tools/bench_ppo.py --envs 4096 --n-steps 64 --timesteps 10e6 --out gpurun_out/ppo_flat

One JSON line: env-steps/s of whole PPO iterations (rollout + GAE + update),
the rollout/update time split, and the final rollout statistics; the SB3-format
progress.csv lands in --out (compare with the reference's archived
outputs/experiments/archived_models/2025-12-04_ppo-flat-directional-seed10/progress.csv:
ep_rew_mean ~8, ep_len_mean ~300 over 10M steps at ~200 env-steps/s).
Hyperparameters are the reference's (configs/train/ppo_directional.yaml) except
the rollout shape: num_envs x n_steps and batch_sz scaled for one GPU.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--n-steps", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--timesteps", type=float, default=4096 * 64 * 4)
    ap.add_argument("--terrain", default="flat")
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--lr", type=float, default=-1, help="-1: the reference's lr_schedule")
    ap.add_argument("--out", default=None)
    ap.add_argument("--seed", type=int, default=10)
    ap.add_argument("--cameras", action="store_true", help="depth cameras on (rgbd policy branch)")
    ap.add_argument("--conv-benchmark", action="store_true", help="MIOpen kernel search for the CNN")
    ap.add_argument("--frozen-encoder", action="store_true",
                    help="with --cameras: pretrain a TinyAutoencoder on GPU frames first and freeze it (reference setup)")
    ap.add_argument("--eval-freq", type=int, default=0,
                    help="EvalCallback every N vec-env steps (the reference: 5000) on an eval VecEnv of --envs envs, "
                         "env i on np_random(seed + envs + i); writes <out>/results/evaluations.npz")
    ap.add_argument("--eval-episodes", type=int, default=8)
    a = ap.parse_args()

    import torch

    if a.conv_benchmark:
        torch.backends.cudnn.benchmark = True

    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO
    from ballbot_rl.training.schedules import lr_schedule

    env = BallbotVecEnv(a.envs, device="cuda:0", precision=a.precision, seed=a.seed,
                        terrain_config={"type": a.terrain, "config": {}}, disable_cameras=not a.cameras)
    frozen, pre_s = None, 0.0
    if a.cameras and a.frozen_encoder:
        from ballbot_rl.encoders import TinyAutoencoder, collect_depth_images, train_autoencoder

        t = time.perf_counter()
        # frames from a separate env (>= 1024 envs: fast collection; the training env's terrain
        # streams stay untouched by the pretraining)
        penv = BallbotVecEnv(max(a.envs, 1024), device="cuda:0", precision=a.precision, seed=a.seed + 1,
                             terrain_config={"type": a.terrain, "config": {}}, disable_cameras=False)
        imgs = collect_depth_images(penv, 65536, seed=a.seed)
        penv.close()
        ae = TinyAutoencoder(env.cam_h, env.cam_w)
        train_autoencoder(ae, imgs, epochs=2, batch_size=256, log=lambda *_: None)
        frozen = ae.encoder.eval()
        torch.cuda.synchronize()
        pre_s = time.perf_counter() - t
        del imgs
    m = BatchedPPO(env, n_steps=a.n_steps, batch_size=a.batch, n_epochs=a.epochs, ent_coef=0.001, clip_range=0.015,
                   vf_coef=2.0, target_kl=0.3, learning_rate=lr_schedule if a.lr == -1 else a.lr,
                   normalize_advantage=False, weight_decay=0.01, seed=a.seed,
                   logger=CSVLogger(a.out, stdout=False), frozen_encoder=frozen)
    t_roll = t_upd = 0.0
    roll_times, upd_times = [], []
    orig_collect, orig_train = m.collect_rollouts, m.train

    def collect():
        nonlocal t_roll
        torch.cuda.synchronize(); t = time.perf_counter()
        orig_collect(); torch.cuda.synchronize(); roll_times.append(time.perf_counter() - t); t_roll += roll_times[-1]

    def train():
        nonlocal t_upd
        torch.cuda.synchronize(); t = time.perf_counter()
        orig_train(); torch.cuda.synchronize(); upd_times.append(time.perf_counter() - t); t_upd += upd_times[-1]

    t_setup = time.perf_counter()
    m.warm_up()  # graphs captured and primed, BLAS initialised: setup, reported apart from the run
    setup_s = time.perf_counter() - t_setup
    m.collect_rollouts, m.train = collect, train
    iters = [0]

    def cb(_m):
        iters[0] += 1
        if iters[0] % 10 == 0:
            print(f"iter {iters[0]} t={_m.num_timesteps} ep_rew={_eprew(_m):.3f}", file=sys.stderr, flush=True)
        return True

    ecb, t_eval = None, [0.0]
    if a.eval_freq:
        from ballbot_gym.distributed import shard_stream_seeds
        from ballbot_rl.training.callbacks import EvalCallback

        eenv = BallbotVecEnv(a.envs, device="cuda:0", precision=a.precision, seed=a.seed + a.envs,
                             stream_seeds=shard_stream_seeds(a.seed + a.envs, 0, a.envs),
                             terrain_config={"type": a.terrain, "config": {}}, disable_cameras=not a.cameras)
        inner = EvalCallback(eenv, n_eval_episodes=a.eval_episodes, eval_freq=a.eval_freq, n_total_envs=a.envs,
                             log_path=Path(a.out) / "results" if a.out else None)

        def ecb(_m, first, last):
            torch.cuda.synchronize(); t = time.perf_counter()
            inner(_m, first, last); torch.cuda.synchronize(); t_eval[0] += time.perf_counter() - t

    t0 = time.perf_counter()
    m.learn(total_timesteps=int(a.timesteps), callback=cb, rollout_callback=ecb)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = {"metric": "PPO env-steps/sec (rollout + GAE + update)", "value": m.num_timesteps / el,
           "unit": "env-steps/s", "timesteps": m.num_timesteps, "iterations": iters[0], "wall_s": el,
           "rollout_s": t_roll, "update_s": t_upd, "eval_s": t_eval[0], "setup_s": setup_s,
           "value_including_setup": m.num_timesteps / (el + setup_s),
           "rollout_env_steps_per_s": m.num_timesteps / max(t_roll, 1e-9),
           "rollout_times_s": [round(x, 4) for x in roll_times], "update_times_s": [round(x, 4) for x in upd_times],
           "kl_stops": getattr(m, "kl_stops", None),
           "config": {"envs": a.envs, "n_steps": a.n_steps, "batch_size": a.batch, "n_epochs": a.epochs,
                      "terrain": a.terrain, "precision": a.precision, "cameras": a.cameras,
                      "frozen_encoder": frozen is not None, "encoder_pretrain_s": pre_s},
           "ep_rew_mean": _eprew(m), "ep_len_mean": _eplen(m), "env_stats": env.stats()}
    print(json.dumps(out), flush=True)
    env.close()


def _eprew(m):
    import numpy as np
    return float(np.mean([e["r"] for e in m.ep_info_buffer])) if m.ep_info_buffer else float("nan")


def _eplen(m):
    import numpy as np
    return float(np.mean([e["l"] for e in m.ep_info_buffer])) if m.ep_info_buffer else float("nan")


if __name__ == "__main__":
    main()
