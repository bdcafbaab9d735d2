"""Distance reward (reference ballbot_gym/rewards/distance.py:8-50).

r = -scale * || goal - pos2d ||.  Fused as BB_REWARD_DISTANCE in the batched
env (pos2d = xpos[base][:2] of RK stage 4)."""
from typing import Dict

import numpy as np

from ballbot_gym.rewards.base import BaseReward


class DistanceReward(BaseReward):
    def __init__(self, goal_position: np.ndarray, scale: float = 1.0):
        self.goal_position = np.array(goal_position, dtype=np.float32)
        if self.goal_position.shape != (2,):
            raise ValueError(f"goal_position must be shape (2,), got {self.goal_position.shape}")
        self.scale = float(scale)

    def __call__(self, state: Dict) -> float:
        if "pos2d" not in state:
            raise ValueError("DistanceReward requires 'pos2d' in state dictionary")
        pos = np.array(state["pos2d"], dtype=np.float32)
        return -self.scale * np.linalg.norm(self.goal_position - pos)
