"""Encoder pretraining (reference ballbot_rl/encoders/pretrain.py:1-93, training.py:9-77,
data/collect.py:13-41).

The reference collects depth frames by running a PPO policy in SubprocVecEnv
envs that log their camera images to disk, loads them into a Dataset, splits
80/20 and trains TinyAutoencoder with Adam(lr 1e-3), MSE reconstruction, batch
64, saving the encoder at every validation improvement.  Here the frames come
straight from the GPU env's depth cameras (bb_render_depth, every rendered
frame of every env, both cameras) into one device tensor, and the training
loop runs over device-resident minibatches -- no files, no DataLoader workers.

    python -m ballbot_rl.encoders.pretrain --n_envs 1024 --n_frames 200000 \\
        --save_encoder_to outputs/encoders/encoder.safetensors [--policy model.safetensors]
"""
from __future__ import annotations

import argparse
from typing import Dict, Optional

import torch

from ballbot_rl.encoders.models import TinyAutoencoder, save_encoder


@torch.no_grad()
def collect_depth_images(env, n_frames: int, policy=None, seed: int = 0, max_steps: int = 100000) -> torch.Tensor:
    """Depth frames [n_frames, 1, H, W] from the env's cameras.

    Each step keeps the images of the envs whose cameras rendered in it
    (the reference's 6-step cadence); actions come from `policy.predict`
    (deterministic, as data/collect.py:31-33) or uniform random in [-1, 1]."""
    if not getattr(env, "cameras", False):
        raise ValueError("collect_depth_images needs BallbotVecEnv(..., disable_cameras=False)")
    g = torch.Generator(device=env.device).manual_seed(int(seed))
    obs, _ = env.reset()
    out = []
    have = 0
    steps = torch.zeros(env.num_envs, dtype=torch.int64, device=env.device)
    fresh = torch.ones(env.num_envs, dtype=torch.bool, device=env.device)  # reset frames
    for _ in range(max_steps):
        if fresh.any():
            imgs = env.depth[fresh].reshape(-1, 1, env.cam_h, env.cam_w)
            out.append(imgs.clone())
            have += imgs.shape[0]
            if have >= n_frames:
                break
        if policy is not None:
            from ballbot_rl.training.ppo import policy_obs

            cams = not policy.features_extractor._proprio_only
            a = policy.predict(policy_obs(obs, env.depth, env.rel_ts) if cams else obs)
        else:
            a = torch.rand(env.num_envs, 3, generator=g, device=env.device) * 2 - 1
        obs, _, _, _, _ = env.step(a)
        fresh = (env.rel_ts == 0)  # rendered this step (incl. auto-resets)
        steps += 1
    return torch.cat(out)[:n_frames]


def train_autoencoder(model: TinyAutoencoder, images: torch.Tensor, epochs: int = 100, lr: float = 1e-3,
                      batch_size: int = 64, val_ratio: float = 0.2, seed: int = 0,
                      save_path: Optional[str] = None, log=print) -> Dict[str, float]:
    """Adam + MSE reconstruction with a random 80/20 split (training.py:9-77);
    the encoder is saved (safetensors) whenever the validation loss improves."""
    dev = images.device
    model = model.to(dev)
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    n = images.shape[0]
    perm = torch.randperm(n, generator=g).to(dev)
    n_val = int(n * val_ratio)
    val, train = images[perm[:n_val]], images[perm[n_val:]]
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    best = float("inf")
    hist = {}
    for epoch in range(epochs):
        model.train()
        order = torch.randperm(train.shape[0], generator=g).to(dev)
        tot = torch.zeros((), device=dev)
        for s in range(0, train.shape[0], batch_size):
            x = train[order[s:s + batch_size]]
            if x.shape[0] < 2:  # BatchNorm needs more than one sample
                continue
            loss = torch.nn.functional.mse_loss(model(x), x)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            tot += loss.detach() * x.shape[0]
        model.eval()
        with torch.no_grad():
            vl = torch.zeros((), device=dev)
            for s in range(0, val.shape[0], 4096):
                x = val[s:s + 4096]
                vl += torch.nn.functional.mse_loss(model(x), x, reduction="sum") / x[0].numel()
        train_loss = float(tot) / max(train.shape[0], 1)
        val_loss = float(vl) / max(val.shape[0], 1)
        log(f"Epoch {epoch + 1}: train_loss={train_loss:.8f}, val_loss={val_loss:.8f}")
        hist = {"epoch": epoch + 1, "train_loss": train_loss, "val_loss": val_loss}
        if val_loss < best:
            best = val_loss
            hist["best_val_loss"] = best
            if save_path:
                p_sum = save_encoder(model, save_path)
                log(f"improved val loss, saving ENCODER with p_sum={p_sum}")
    hist["best_val_loss"] = best
    return hist


def cli_main() -> None:
    ap = argparse.ArgumentParser(description="Pretrain the depth encoder on GPU-rendered frames")
    ap.add_argument("--n_envs", type=int, default=1024)
    ap.add_argument("--n_frames", type=int, default=100000)
    ap.add_argument("--terrain", default="perlin")
    ap.add_argument("--policy", default="", help="optional policy weights (safetensors) to drive the robots")
    ap.add_argument("--save_encoder_to", required=True)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--batch_size", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    from ballbot_gym.envs import BallbotVecEnv

    env = BallbotVecEnv(a.n_envs, device="cuda:0", terrain_config={"type": a.terrain, "config": {}},
                        disable_cameras=False, seed=a.seed)
    policy = None
    if a.policy:
        from safetensors.torch import load_file

        from ballbot_rl.policies import ActorCriticPolicy, obs_spaces

        sd = load_file(a.policy, device="cuda:0")
        cams = any(k.startswith("features_extractor.extractors.rgbd") for k in sd)
        policy = ActorCriticPolicy(obs_spaces(cameras=cams)).to("cuda:0")
        policy.load_state_dict(sd)
        policy.eval()
    imgs = collect_depth_images(env, a.n_frames, policy=policy, seed=a.seed)
    print(f"collected {imgs.shape[0]} depth frames")
    train_autoencoder(TinyAutoencoder(env.cam_h, env.cam_w), imgs, epochs=a.epochs, batch_size=a.batch_size,
                      save_path=a.save_encoder_to, seed=a.seed)
    env.close()


if __name__ == "__main__":
    cli_main()
