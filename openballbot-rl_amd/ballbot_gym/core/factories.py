"""Config -> component factories (reference ballbot_gym/core/factories.py:9-215).

Built-in rewards get their constructor arguments filtered (environment-level
coefficients scale/action_reg_coef/survival_bonus stay with the env); custom
reward types receive the whole config.  Terrain factories return a closure
that merges runtime overrides (e.g. seed) over the configured arguments.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Type

import numpy as np

from ballbot_gym.core.registry import ComponentRegistry


def _type_of(config: Any, what: str) -> str:
    if not isinstance(config, dict):
        raise ValueError(f"{what} config must be a dictionary, got {type(config)}")
    t = config.get("type")
    if t is None:
        raise ValueError(f"{what} config must have 'type' key")
    return t


def _as_f32(x):
    return np.array(x, dtype=np.float32) if isinstance(x, list) else x


def create_reward(config: Dict[str, Any]):
    rtype = _type_of(config, "Reward")
    rcfg = config.get("config", {})
    if rtype == "directional":
        if "target_direction" not in rcfg:
            raise ValueError("DirectionalReward requires 'target_direction' in config")
        kwargs = {"target_direction": _as_f32(rcfg["target_direction"])}
    elif rtype == "distance":
        if "goal_position" not in rcfg:
            raise ValueError("DistanceReward requires 'goal_position' in config")
        kwargs = {"goal_position": _as_f32(rcfg["goal_position"]), "scale": rcfg.get("scale", 1.0)}
    else:
        kwargs = rcfg
    try:
        return ComponentRegistry.get_reward(rtype, **kwargs)
    except ValueError as e:
        raise ValueError(f"Failed to create reward '{rtype}': {e}")
    except TypeError as e:
        raise TypeError(f"Failed to create reward '{rtype}' with parameters {list(kwargs)}: {e}")


def create_terrain(config: Dict[str, Any]) -> Callable:
    ttype = _type_of(config, "Terrain")
    tcfg = config.get("config", {})
    try:
        fn = ComponentRegistry.get_terrain(ttype)
    except ValueError as e:
        raise ValueError(f"Failed to get terrain '{ttype}': {e}")

    def configured_terrain(n: int, **override_kwargs) -> np.ndarray:
        return fn(n, **{**tcfg, **override_kwargs})

    return configured_terrain


def create_policy(config: Dict[str, Any]) -> Type:
    ptype = _type_of(config, "Policy")
    try:
        return ComponentRegistry.get_policy(ptype)
    except ValueError as e:
        raise ValueError(f"Failed to get policy '{ptype}': {e}")


_LISTS = {
    "reward": ComponentRegistry.list_rewards,
    "terrain": ComponentRegistry.list_terrains,
    "policy": ComponentRegistry.list_policies,
}


def validate_config(config: Dict[str, Any], component_type: str) -> bool:
    if not isinstance(config, dict):
        raise ValueError(f"Config must be a dictionary, got {type(config)}")
    if "type" not in config:
        raise ValueError(f"{component_type} config must have 'type' key")
    if component_type not in _LISTS:
        raise ValueError(f"Unknown component_type '{component_type}'. Must be one of: 'reward', 'terrain', 'policy'")
    available = _LISTS[component_type]()
    if config["type"] not in available:
        raise ValueError(f"Unknown {component_type} type '{config['type']}'. Available: {available}")
    return True
