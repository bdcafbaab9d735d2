"""CPU restatement of the stable-baselines3 2.6.0 pieces the reference trains with.

TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker of bb_gae and
BatchedPPO; never by the product).  SB3 is a third-party dependency of the
reference (ballbot_rl/pyproject.toml; version 2.6.0 per the archived
checkpoints' system_info.txt), not installed here and not vendored, so its
published algorithm is restated:

* RolloutBuffer.compute_returns_and_advantage (common/buffers.py): numpy
  float32 arrays, Python-float gamma / gae_lambda, reverse loop over steps;
  next_non_terminal = 1 - dones (last step) or 1 - episode_starts[t+1];
  delta = r + gamma*V' * nnt - V; A = delta + gamma*lambda*nnt*A'; R = A + V.
  Under NumPy 2 (NEP 50) the Python floats act as float32 scalars, so the
  coefficients are f32(gamma) and f32(gamma*lambda) and the arithmetic is
  float32, left to right -- what bb_gae reproduces bit for bit.
* PPO.train loss pieces (ppo/ppo.py) in float64 for loss checks.

Parity against SB3 itself is pinned only by the known answers in
tests/test_ppo.py (lambda = 1 Monte-Carlo returns, lambda = 0 TD errors,
episode cuts), not by SB3 output: SB3 cannot run here.
"""
from __future__ import annotations

import numpy as np


def compute_gae(rewards, values, episode_starts, last_values, dones, gamma=0.99, gae_lambda=0.95):
    """rewards/values/episode_starts [T][N]; last_values/dones [N] -> (advantages, returns) float32."""
    rewards = np.asarray(rewards, np.float32)
    values = np.asarray(values, np.float32)
    starts = np.asarray(episode_starts, np.float32)
    last_values = np.asarray(last_values, np.float32)
    dones = np.asarray(dones, np.float32)
    T = rewards.shape[0]
    g = np.float32(gamma)
    gl = np.float32(gamma * gae_lambda)
    adv = np.zeros_like(rewards)
    last = np.zeros_like(last_values)
    for t in reversed(range(T)):
        if t == T - 1:
            nnt = np.float32(1.0) - dones
            nv = last_values
        else:
            nnt = np.float32(1.0) - starts[t + 1]
            nv = values[t + 1]
        delta = rewards[t] + g * nv * nnt - values[t]
        last = delta + gl * nnt * last
        adv[t] = last
    return adv, adv + values


def ppo_losses(logp, old_logp, adv, values, returns, entropy, clip, ent_coef, vf_coef):
    """PPO.train minibatch loss terms (no advantage normalisation, no value clipping)."""
    logp, old_logp, adv = (np.asarray(x, np.float64) for x in (logp, old_logp, adv))
    ratio = np.exp(logp - old_logp)
    pg = -np.mean(np.minimum(adv * ratio, adv * np.clip(ratio, 1 - clip, 1 + clip)))
    vf = np.mean((np.asarray(returns, np.float64) - np.asarray(values, np.float64)) ** 2)
    ent = -np.mean(entropy)
    lr = logp - old_logp
    kl = np.mean(np.exp(lr) - 1 - lr)
    return {"pg": pg, "vf": vf, "ent": ent, "loss": pg + ent_coef * ent + vf_coef * vf, "approx_kl": kl,
            "clip_fraction": float(np.mean(np.abs(ratio - 1) > clip))}
