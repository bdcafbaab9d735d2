"""Gaussian hills (reference ballbot_gym/terrain/hills.py:7-103).

Hill centres come from numpy RandomState(seed or 0) with rejection of
centres closer than 2*hill_radius; heights are smoothstep-truncated
Gaussians on an (i, j)-indexed unit grid, summed and clipped to [0, 1]."""
from typing import Optional

import numpy as np


def generate_hills_terrain(n: int, num_hills: int = 5, hill_height: float = 0.7, hill_radius: float = 0.15,
                           flat_ratio: float = 0.4, seed: Optional[int] = None) -> np.ndarray:
    assert n % 2 == 1, "n should be odd for heightfield symmetry"
    assert num_hills > 0, "num_hills must be positive"
    assert 0 <= hill_height <= 1.0, "hill_height should be between 0 and 1"
    assert 0 < hill_radius <= 0.5, "hill_radius should be between 0 and 0.5"
    rng = np.random.RandomState(0 if seed is None else seed)
    centres = []
    for _ in range(num_hills * 100):
        if len(centres) >= num_hills:
            break
        x = rng.uniform(hill_radius, 1.0 - hill_radius)
        y = rng.uniform(hill_radius, 1.0 - hill_radius)
        if all(np.sqrt((x - cx) ** 2 + (y - cy) ** 2) >= 2.0 * hill_radius for cx, cy in centres):
            centres.append((x, y))
    grid = np.linspace(0, 1, n)
    X, Y = np.meshgrid(grid, grid, indexing="ij")
    sigma = hill_radius / 3.0
    out = np.zeros((n, n))
    for cx, cy in centres:
        r = np.sqrt((X - cx) ** 2 + (Y - cy) ** 2)
        bump = hill_height * np.exp(-(r ** 2) / (2 * sigma ** 2))
        t = np.clip(1.0 - (r / hill_radius), 0.0, 1.0)
        out += bump * (t * t * (3.0 - 2.0 * t))
    return np.clip(out, 0.0, 1.0).flatten()
