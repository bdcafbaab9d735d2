"""Gradient field (reference terrain/gradient.py:7-99): linear / radial slope
of 2 tan(max_slope), min-max normalised.  The 'perlin' mode adds
snoise2(i/25, j/25, octaves=3, persistence=0.3, base=seed) * smoothness
(restated simplex noise, ballbot_gym/terrain/perlin.py; parity unpinned)."""
from typing import Optional

import numpy as np

from ballbot_gym.terrain._common import centred_grid, check_odd, minmax


def generate_gradient_terrain(n: int, max_slope: float = 20.0, gradient_type: str = "linear",
                              smoothness: float = 0.5, direction: str = "x",
                              seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    assert 0 <= max_slope <= 45, "max_slope should be between 0 and 45 degrees"
    assert gradient_type in ["linear", "radial", "perlin"], "gradient_type must be 'linear', 'radial', or 'perlin'"
    assert direction in ["x", "y"], "direction must be 'x' or 'y'"
    g = np.tan(np.radians(max_slope)) * 2.0
    X, Y = centred_grid(n)
    if gradient_type == "linear":
        t = g * ((X if direction == "x" else Y) + 1.0) / 2.0
    elif gradient_type == "radial":
        t = g * np.clip(np.sqrt(X ** 2 + Y ** 2) / np.sqrt(2.0), 0.0, 1.0)
    else:
        from ballbot_gym.terrain.perlin import snoise2_grid

        i = np.arange(n, dtype=np.float64)
        noise = snoise2_grid(i / 25.0, i / 25.0, octaves=3, persistence=0.3, lacunarity=2.0, base=0 if seed is None
                             else seed, repeat=None)
        base = ((X if direction == "x" else Y) + 1.0) / 2.0
        t = g * (base + noise * smoothness)
    return minmax(t).flatten()
