"""Env registration: `make("ballbot-v0.1", **kwargs)`.

The reference registers its env with gymnasium (ballbot_gym/__init__.py:47-53,
id "ballbot-v0.1", entry point ballbot_gym.envs.ballbot_env:BBotSimulation)
and its callers build it with gym.make(...) (training/utils.py:64-76,
tests/unit/test_env.py).  gymnasium is not installed here, so this module
keeps a registry of its own with the same id and entry point, and also
registers with gymnasium when it is importable.
"""
from __future__ import annotations

import importlib
from typing import Any, Dict


class EnvSpec:
    def __init__(self, id: str, entry_point: str, kwargs: Dict[str, Any]):
        self.id, self.entry_point, self.kwargs = id, entry_point, dict(kwargs)

    def make(self, **kwargs):
        mod, cls = self.entry_point.split(":")
        return getattr(importlib.import_module(mod), cls)(**{**self.kwargs, **kwargs})


class _Registry:
    def __init__(self):
        self.env_specs: Dict[str, EnvSpec] = {}

    def __contains__(self, env_id: str) -> bool:
        return env_id in self.env_specs


registry = _Registry()


def register(id: str, entry_point: str, kwargs: Dict[str, Any] | None = None) -> None:
    if id in registry.env_specs:
        raise ValueError(f"Environment {id} already registered")
    registry.env_specs[id] = EnvSpec(id, entry_point, kwargs or {})
    try:  # the reference's registration, when gymnasium is present
        import gymnasium as gym

        if id not in gym.envs.registry:
            gym.register(id=id, entry_point=entry_point, kwargs=kwargs or {})
    except ImportError:
        pass


def make(env_id: str, **kwargs):
    """gym.make(env_id, **kwargs) for the envs registered here."""
    if env_id not in registry.env_specs:
        raise ValueError(f"No registered env with id: {env_id}")
    return registry.env_specs[env_id].make(**kwargs)


ENV_ID = "ballbot-v0.1"
register(ENV_ID, "ballbot_gym.envs.ballbot_env:BBotSimulation", {"xml_path": None})
