"""Deterministic policy evaluation on the batched env, with SB3's semantics.

Restates stable-baselines3 2.6.0 `evaluate_policy` as the reference's
EvalCallback calls it (ballbot_rl/training/callbacks.py:607-617: deterministic,
`evaluation.n_episodes` episodes, the eval VecEnv of train.py:90-97 wrapped in
Monitor, training/utils.py:81-83):
* the VecEnv is reset at the start (every env draws its next terrain from its
  own generator, np_random(seed + N_ENVS + i));
* env i must finish (n_eval_episodes + i) // n_envs episodes; all envs step
  together until every env has -- envs that are done or have no episode to
  count keep stepping and auto-resetting (their generators advance, exactly as
  in the reference, so the next evaluation starts on the same terrains);
* an episode's return is Monitor's: the float64 sum of the float32 step
  rewards since the env's last reset, rounded to 6 decimals; its length the
  step count; episodes are listed in the order they finish (env order within a
  step), which is the row order of EvalCallback's evaluations.npz.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch


def _policy_obs(env, obs):
    from ballbot_rl.training.ppo import policy_obs

    return policy_obs(obs, env.depth, env.rel_ts) if getattr(env, "cameras", False) else obs


@torch.no_grad()
def evaluate_policy(policy, env, n_eval_episodes: int = 8, deterministic: bool = True,
                    max_steps: int = 1_000_000, return_episode_rewards: bool = False) -> Dict[str, object]:
    """SB3 evaluate_policy on a BallbotVecEnv (auto-reset on).  -> {"mean_reward",
    "std_reward", "mean_ep_length", "episode_rewards", "episode_lengths"}."""
    n = int(env.num_envs)
    targets = np.array([(n_eval_episodes + i) // n for i in range(n)], dtype=np.int64)
    counts = np.zeros(n, dtype=np.int64)
    was_training = getattr(policy, "training", False)
    if hasattr(policy, "eval"):
        policy.eval()  # SB3 predict: set_training_mode(False) (BatchNorm running statistics)
    rewards: List[float] = []
    lengths: List[int] = []
    obs, _ = env.reset()
    dev = obs.device
    ret = torch.zeros(n, dtype=torch.float64, device=dev)
    length = torch.zeros(n, dtype=torch.int64, device=dev)
    try:
        for _ in range(max_steps):
            a = policy.predict(_policy_obs(env, obs), deterministic=deterministic)
            obs, r, term, trunc, info = env.step(a)
            flags = info.get("done_flags") if isinstance(info, dict) else None
            done = (term | trunc) if flags is None else ((flags & 1) != 0) | trunc
            ret += r.double()  # Monitor: float64 sum of the float32 rewards
            length += 1
            if bool(done.any()):
                d = done.cpu().numpy()
                rr, ll = ret.cpu().numpy(), length.cpu().numpy()
                for i in np.nonzero(d)[0]:
                    if counts[i] < targets[i]:
                        rewards.append(round(float(rr[i]), 6))
                        lengths.append(int(ll[i]))
                        counts[i] += 1
                ret.masked_fill_(done, 0.0)
                length.masked_fill_(done, 0)
                if not (counts < targets).any():
                    break
    finally:
        if hasattr(policy, "train"):
            policy.train(was_training)
    out = {"mean_reward": float(np.mean(rewards)) if rewards else float("nan"),
           "std_reward": float(np.std(rewards)) if rewards else float("nan"),
           "mean_ep_length": float(np.mean(lengths)) if lengths else float("nan"),
           "episode_rewards": rewards, "episode_lengths": lengths}
    return out
