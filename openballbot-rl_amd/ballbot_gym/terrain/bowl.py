"""Bowl depression (reference terrain/bowl.py:13-76): 1 - depth * (1 - smoothstep(r / radius))."""
from typing import Optional

import numpy as np

from ballbot_gym.terrain._common import check_odd, smoothstep, unit_grid


def generate_bowl_terrain(n: int, depth: float = 0.6, radius: float = 0.4, center_x: float = 0.5,
                          center_y: float = 0.5, smoothness: float = 0.5, seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    assert 0 <= depth <= 1.0, "depth should be between 0 and 1"
    assert 0 < radius <= 1.0, "radius should be between 0 and 1"
    assert 0 <= center_x <= 1.0, "center_x should be between 0 and 1"
    assert 0 <= center_y <= 1.0, "center_y should be between 0 and 1"
    X, Y = unit_grid(n)
    r = np.sqrt((X - center_x) ** 2 + (Y - center_y) ** 2)
    bowl = depth * (1.0 - smoothstep(0.0, 1.0, np.clip(r / radius, 0.0, 1.0)))
    return np.clip(np.ones((n, n)) - bowl, 0.0, 1.0).flatten()
