"""Observation/action spaces of the ballbot env without a gymnasium dependency.

The reference builds gymnasium spaces (ballbot_env.py:235-256,
envs/observation_spaces.py:9-100).  gymnasium is not installed in this image,
so `Box` and `Dict` restate the parts callers use: shape, dtype, bounds,
`sample()`, `contains()`, `seed()` and the sorted key order of `Dict` (what
SB3's MultiInputPolicy and the reference's Extractor iterate over).  When
gymnasium is importable, `to_gymnasium()` converts to the real classes.
"""
from __future__ import annotations

from typing import Dict as TDict, Optional, Tuple

import numpy as np


class Box:
    """gymnasium.spaces.Box(low, high, shape, dtype): a closed box in R^shape."""

    def __init__(self, low, high, shape: Optional[Tuple[int, ...]] = None, dtype=np.float32, seed=None):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.ndim(low) else np.shape(high)
        self.shape = tuple(int(s) for s in shape)
        self.low = np.broadcast_to(np.asarray(low, self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, self.dtype), self.shape).copy()
        self._rng = np.random.default_rng(seed)

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def sample(self) -> np.ndarray:
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    __contains__ = contains

    def to_gymnasium(self):
        import gymnasium as gym

        return gym.spaces.Box(self.low, self.high, shape=self.shape, dtype=self.dtype)

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class Dict:
    """gymnasium.spaces.Dict: named sub-spaces, keys kept sorted as gymnasium does."""

    def __init__(self, spaces: TDict[str, Box]):
        self.spaces = dict(sorted(spaces.items()))

    def __getitem__(self, k):
        return self.spaces[k]

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def seed(self, seed=None):
        for i, s in enumerate(self.spaces.values()):
            s.seed(None if seed is None else seed + i)
        return [seed]

    def sample(self):
        return {k: s.sample() for k, s in self.spaces.items()}

    def contains(self, x) -> bool:
        return isinstance(x, dict) and x.keys() == self.spaces.keys() and all(
            s.contains(x[k]) for k, s in self.spaces.items())

    __contains__ = contains

    def to_gymnasium(self):
        import gymnasium as gym

        return gym.spaces.Dict({k: s.to_gymnasium() for k, s in self.spaces.items()})

    def __repr__(self):
        return "Dict(" + ", ".join(f"{k}: {s}" for k, s in self.spaces.items()) + ")"


def action_space() -> Box:
    """ballbot_env.py:235-238: three normalised omniwheel commands in [-1, 1]."""
    return Box(-1.0, 1.0, shape=(3,), dtype=np.float32)


def observation_space(im_shape: TDict[str, int], num_channels: int, disable_cameras: bool) -> Dict:
    """envs/observation_spaces.py:9-100 (create_observation_space)."""
    f = np.float32
    s = {
        "orientation": Box(-np.pi, np.pi, shape=(3,), dtype=f),
        "angular_vel": Box(-2, 2, shape=(3,), dtype=f),
        "vel": Box(-2, 2, shape=(3,), dtype=f),
        "motor_state": Box(-2.0, 2.0, shape=(3,), dtype=f),
        "actions": Box(-1.0, 1.0, shape=(3,), dtype=f),
    }
    if not disable_cameras:
        img = (num_channels, int(im_shape["h"]), int(im_shape["w"]))
        s["rgbd_0"] = Box(0.0, 1.0, shape=img, dtype=f)
        s["rgbd_1"] = Box(0.0, 1.0, shape=img, dtype=f)
        s["relative_image_timestamp"] = Box(0.0, 0.1, shape=(1,), dtype=f)
    return Dict(s)
