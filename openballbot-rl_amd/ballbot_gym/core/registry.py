"""ComponentRegistry: name -> component plugin tables.

Same public API and error behaviour as the reference
ballbot_gym/core/registry.py:8-231 (class-level tables, ValueError on
duplicates / unknown names, rewards must subclass BaseReward).
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Type


def _lookup(table: Dict[str, Any], kind: str, plural: str, name: str):
    if name not in table:
        raise ValueError(f"Unknown {kind}: '{name}'. Available {plural}: {list(table)}")
    return table[name]


def _insert(table: Dict[str, Any], kind: str, plural: str, name: str, obj: Any) -> None:
    if name in table:
        raise ValueError(f"{kind.capitalize()} '{name}' is already registered. Available {plural}: {list(table)}")
    table[name] = obj


class ComponentRegistry:
    """Central plugin registry for rewards, terrains, policies and sensors."""

    _rewards: Dict[str, Type] = {}
    _terrains: Dict[str, Callable] = {}
    _policies: Dict[str, Type] = {}
    _sensors: Dict[str, Type] = {}

    # rewards (registry.py:35-86)
    @classmethod
    def register_reward(cls, name: str, reward_class: Type) -> None:
        from ballbot_gym.rewards.base import BaseReward

        if name in cls._rewards:
            _insert(cls._rewards, "reward", "rewards", name, reward_class)
        if not (isinstance(reward_class, type) and issubclass(reward_class, BaseReward)):
            raise ValueError(f"Reward class must inherit from BaseReward, got {reward_class}")
        cls._rewards[name] = reward_class

    @classmethod
    def get_reward(cls, name: str, **kwargs):
        return _lookup(cls._rewards, "reward", "rewards", name)(**kwargs)

    @classmethod
    def list_rewards(cls) -> List[str]:
        return list(cls._rewards)

    # terrains (registry.py:88-133)
    @classmethod
    def register_terrain(cls, name: str, terrain_fn: Callable) -> None:
        if name in cls._terrains:
            _insert(cls._terrains, "terrain", "terrains", name, terrain_fn)
        if not callable(terrain_fn):
            raise ValueError(f"Terrain must be callable, got {type(terrain_fn)}")
        cls._terrains[name] = terrain_fn

    @classmethod
    def get_terrain(cls, name: str) -> Callable:
        return _lookup(cls._terrains, "terrain", "terrains", name)

    @classmethod
    def list_terrains(cls) -> List[str]:
        return list(cls._terrains)

    # policies (registry.py:135-178)
    @classmethod
    def register_policy(cls, name: str, policy_class: Type) -> None:
        _insert(cls._policies, "policy", "policies", name, policy_class)

    @classmethod
    def get_policy(cls, name: str) -> Type:
        return _lookup(cls._policies, "policy", "policies", name)

    @classmethod
    def list_policies(cls) -> List[str]:
        return list(cls._policies)

    # sensors (registry.py:180-223)
    @classmethod
    def register_sensor(cls, name: str, sensor_class: Type) -> None:
        _insert(cls._sensors, "sensor", "sensors", name, sensor_class)

    @classmethod
    def get_sensor(cls, name: str) -> Type:
        return _lookup(cls._sensors, "sensor", "sensors", name)

    @classmethod
    def list_sensors(cls) -> List[str]:
        return list(cls._sensors)

    @classmethod
    def clear(cls) -> None:
        for t in (cls._rewards, cls._terrains, cls._policies, cls._sensors):
            t.clear()
