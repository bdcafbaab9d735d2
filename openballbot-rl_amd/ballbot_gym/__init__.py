"""ballbot_gym (MI355X-native): the ballbot mj_step hot path as HIP kernels
behind the reference's Gym/plugin API.

Importing registers the built-in terrains and rewards, like the reference
(ballbot_gym/__init__.py:39-40).  The env classes live in ballbot_gym.envs and
load the HIP library lazily (no CPU fallback).
"""
import ballbot_gym.terrain  # noqa: F401  (registers terrain plugins)
import ballbot_gym.rewards  # noqa: F401  (registers reward plugins)
from ballbot_gym.core import ComponentRegistry, create_policy, create_reward, create_terrain, validate_config
from ballbot_gym.registration import make, register, registry  # "ballbot-v0.1" (reference __init__.py:47-53)

__version__ = "0.1.0"

__all__ = ["ComponentRegistry", "create_reward", "create_terrain", "create_policy", "validate_config", "make",
           "register", "registry"]
