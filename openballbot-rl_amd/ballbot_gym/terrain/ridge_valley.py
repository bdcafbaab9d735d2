"""Ridges and valleys (reference terrain/ridge_valley.py:13-89).

cos pattern mapped to [valley_depth, ridge_height], optional k x k box
blur (edge padding, k = int(5 * smoothness) + 1) blended by smoothness,
clipped (not renormalised).  Each window is summed as one contiguous k*k
vector (numpy's pairwise order, as np.mean of the window slice) / k*k."""
from typing import Optional

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view

from ballbot_gym.terrain._common import check_odd, unit_grid


def generate_ridge_valley_terrain(n: int, ridge_height: float = 0.6, valley_depth: float = 0.4,
                                  spacing: float = 0.2, orientation: str = "x", smoothness: float = 0.3,
                                  seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    assert 0 <= ridge_height <= 1.0, "ridge_height should be between 0 and 1"
    assert 0 <= valley_depth <= 1.0, "valley_depth should be between 0 and 1"
    assert spacing > 0, "spacing must be positive"
    assert orientation in ["x", "y", "diagonal"], "orientation must be 'x', 'y', or 'diagonal'"
    X, Y = unit_grid(n)
    c = X if orientation == "x" else (Y if orientation == "y" else X + Y)
    pattern = np.cos(2 * np.pi * spacing * c)
    t = valley_depth + (ridge_height - valley_depth) * (pattern + 1.0) / 2.0
    if smoothness > 0:
        k = int(smoothness * 5) + 1
        if k > 1:
            P = np.pad(t, k // 2, mode="edge")
            win = sliding_window_view(P, (k, k))[:n, :n].reshape(n, n, k * k)
            t = t * (1.0 - smoothness) + (win.sum(-1) / (k * k)) * smoothness
    return np.clip(t, 0.0, 1.0).flatten()
