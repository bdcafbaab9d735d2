"""Spiral terrain (reference terrain/spiral.py:7-78)."""
from typing import Optional

import numpy as np

from ballbot_gym.terrain._common import check_odd, unit_grid


def generate_spiral_terrain(n: int, spiral_tightness: float = 0.1, height_variation: float = 0.5,
                            direction: str = "cw", center_x: float = 0.5, center_y: float = 0.5,
                            seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    assert spiral_tightness > 0, "spiral_tightness must be positive"
    assert 0 <= height_variation <= 1.0, "height_variation should be between 0 and 1"
    assert direction in ["cw", "ccw"], "direction must be 'cw' or 'ccw'"
    X, Y = unit_grid(n)
    dx, dy = X - center_x, Y - center_y
    r = np.sqrt(dx ** 2 + dy ** 2)
    th = (np.arctan2(dy, dx) + 2 * np.pi) % (2 * np.pi)
    if direction == "cw":
        th = 2 * np.pi - th
    t = height_variation * np.sin(spiral_tightness * th + r)
    t = t * (1.0 - np.clip(r / (np.sqrt(2.0) / 2.0), 0.0, 1.0) * 0.3)
    return np.clip(0.5 + t * 0.5, 0.0, 1.0).flatten()
