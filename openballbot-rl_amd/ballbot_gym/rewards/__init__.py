"""Reward plugins; built-ins auto-register on import (rewards/__init__.py:8-9)."""
from ballbot_gym.core.registry import ComponentRegistry
from ballbot_gym.rewards.base import BaseReward
from ballbot_gym.rewards.directional import DirectionalReward
from ballbot_gym.rewards.distance import DistanceReward

for _name, _cls in (("directional", DirectionalReward), ("distance", DistanceReward)):
    if _name not in ComponentRegistry.list_rewards():
        ComponentRegistry.register_reward(_name, _cls)

__all__ = ["BaseReward", "DirectionalReward", "DistanceReward"]
