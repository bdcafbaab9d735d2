"""SB3 EvalCallback as the reference configures it (ballbot_rl/training/callbacks.py:607-617).

Every `eval_freq` vec-env steps of the training VecEnv, `n_eval_episodes`
deterministic episodes on the eval VecEnv (evaluation.evaluate_policy, SB3's
semantics), with the parameters the training rollout ran with at that step
(SB3 calls EvalCallback._on_step inside collect_rollouts; BatchedPPO.learn
calls this with the rollout's vec-step range before the update).  Per
evaluation, as SB3 writes them:
* progress.csv gets a row with eval/mean_reward, eval/mean_ep_length,
  time/total_timesteps (and the train/* values recorded by the last update,
  which SB3's logger dumps with it);
* log_path/evaluations.npz holds timesteps [n_evals], results and ep_lengths
  [n_evals][n_eval_episodes] (np.savez, loadable with allow_pickle=False);
* a new best mean reward saves best_model.safetensors.
"""
from __future__ import annotations

from pathlib import Path
from typing import List, Optional

import numpy as np


class EvalCallback:
    def __init__(self, eval_env, n_eval_episodes: int = 8, eval_freq: int = 5000, n_total_envs: int = 1,
                 log_path: Optional[Path] = None, best_model_save_path: Optional[Path] = None,
                 deterministic: bool = True):
        self.eval_env = eval_env
        self.n_eval_episodes, self.eval_freq = int(n_eval_episodes), int(eval_freq)
        self.n_total_envs = int(n_total_envs)
        self.log_path = None if log_path is None else Path(log_path)
        self.best_path = None if best_model_save_path is None else Path(best_model_save_path)
        self.deterministic = deterministic
        self.best_mean_reward = -np.inf
        self.timesteps: List[int] = []
        self.results: List[List[float]] = []
        self.ep_lengths: List[List[int]] = []

    def due(self, first: int, last: int) -> List[int]:
        """Every multiple of eval_freq in vec-env steps [first, last]: SB3 calls _on_step at
        every vec-env step, so with eval_freq < n_steps one rollout holds several evaluations."""
        k0 = max(1, -(-first // self.eval_freq))
        return [k * self.eval_freq for k in range(k0, last // self.eval_freq + 1)]

    def __call__(self, model, first: int, last: int) -> None:
        for step in self.due(first, last):  # the rollout's fixed parameters, one evaluation per multiple
            self._evaluate(model, step)

    def _evaluate(self, model, step: int) -> None:
        from ballbot_rl.evaluation import evaluate_policy

        r = evaluate_policy(model.policy, self.eval_env, n_eval_episodes=self.n_eval_episodes,
                            deterministic=self.deterministic)
        ts = step * self.n_total_envs  # SB3's num_timesteps at that step
        self.timesteps.append(ts)
        self.results.append(r["episode_rewards"])
        self.ep_lengths.append(r["episode_lengths"])
        if self.log_path is not None:
            self.log_path.mkdir(parents=True, exist_ok=True)
            np.savez(self.log_path / "evaluations.npz", timesteps=np.array(self.timesteps),
                     results=np.array(self.results), ep_lengths=np.array(self.ep_lengths))
        L = model.logger
        L.record("eval/mean_reward", float(r["mean_reward"]))
        L.record("eval/mean_ep_length", float(r["mean_ep_length"]))
        L.record("time/total_timesteps", ts)
        L.dump(step=ts)
        if r["mean_reward"] > self.best_mean_reward:
            self.best_mean_reward = r["mean_reward"]
            if self.best_path is not None:
                model.save(str(self.best_path / "best_model.safetensors"))
