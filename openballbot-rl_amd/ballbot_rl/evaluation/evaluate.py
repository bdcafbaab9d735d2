"""Deterministic policy evaluation on the batched env.

Mirrors what the reference's EvalCallback (SB3 evaluate_policy, deterministic,
ballbot_rl/training/callbacks.py:550-551: every `evaluation.freq` vec-steps,
`evaluation.n_episodes` episodes) and evaluate.py measure: the undiscounted
return and length of whole episodes.  Here one env per requested episode runs
in the same GPU launch, each counted on its first episode only.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch


@torch.no_grad()
def evaluate_policy(policy, env, n_eval_episodes: int = 8, deterministic: bool = True,
                    max_steps: int = 100000) -> Dict[str, float]:
    """Run policy on `env` (num_envs >= n_eval_episodes) until each of the first
    n_eval_episodes envs ends one episode. -> mean/std reward, mean length."""
    n = int(env.num_envs)
    if n_eval_episodes > n:
        raise ValueError(f"env has {n} envs, fewer than n_eval_episodes={n_eval_episodes}")
    obs, _ = env.reset()
    dev = obs.device
    ret = torch.zeros(n, dtype=torch.float64, device=dev)
    length = torch.zeros(n, dtype=torch.int64, device=dev)
    active = torch.zeros(n, dtype=torch.bool, device=dev)
    active[:n_eval_episodes] = True
    for _ in range(max_steps):
        a = policy.predict(obs, deterministic=deterministic)
        obs, r, term, trunc, info = env.step(a)
        flags = info.get("done_flags") if isinstance(info, dict) else None
        done = (term | trunc) if flags is None else ((flags & 1) != 0) | trunc
        ret += torch.where(active, r.double(), torch.zeros_like(ret))
        length += active.long()
        active &= ~done
        if not bool(active.any()):
            break
    rr = ret[:n_eval_episodes].cpu().numpy()
    ll = length[:n_eval_episodes].cpu().numpy()
    return {"mean_reward": float(np.mean(rr)), "std_reward": float(np.std(rr)), "mean_ep_length": float(np.mean(ll))}
