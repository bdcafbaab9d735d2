"""Directional reward (reference ballbot_gym/rewards/directional.py:8-54).

r = state["vel"][-3:-1] . target_direction.  In the batched env this plugin is
fused into the step kernel (reward kind BB_REWARD_DIRECTIONAL)."""
import numpy as np

from ballbot_gym.rewards.base import BaseReward


class DirectionalReward(BaseReward):
    def __init__(self, target_direction: np.ndarray):
        self.target_direction = target_direction

    def __call__(self, state: dict) -> float:
        return state["vel"][-3:-1].dot(self.target_direction)
