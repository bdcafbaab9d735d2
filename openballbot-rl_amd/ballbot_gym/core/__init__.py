"""Plugin registry, factories and YAML config (reference ballbot_gym/core)."""
from ballbot_gym.core.registry import ComponentRegistry
from ballbot_gym.core.factories import create_policy, create_reward, create_terrain, validate_config

__all__ = ["ComponentRegistry", "create_reward", "create_terrain", "create_policy", "validate_config"]
