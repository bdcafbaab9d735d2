"""Sinusoidal waves (reference terrain/sinusoidal.py:6-61)."""
from typing import Optional

import numpy as np

from ballbot_gym.terrain._common import check_odd, minmax


def generate_sinusoidal_terrain(n: int, amplitude: float = 0.5, frequency: float = 0.1, direction: str = "both",
                                phase: float = 0.0, seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    assert 0 <= amplitude <= 1.0, "amplitude should be between 0 and 1"
    assert frequency > 0, "frequency must be positive"
    assert direction in ["x", "y", "both"], "direction must be 'x', 'y', or 'both'"
    g = np.linspace(0, 2 * np.pi * frequency * n, n)
    X, Y = np.meshgrid(g, g, indexing="ij")
    if direction == "x":
        t = amplitude * np.sin(X + phase)
    elif direction == "y":
        t = amplitude * np.sin(Y + phase)
    else:
        t = amplitude * (np.sin(X + phase) + np.sin(Y + phase)) / 2.0
    return minmax(t).flatten()
