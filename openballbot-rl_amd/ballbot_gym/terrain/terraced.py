"""Terraced terrain (reference terrain/terraced.py:13-108).

Per point: terrace index int(c / w) (capped), position (c % w) / w, smoothstep
transitions into the previous / next terrace within transition_size =
w * transition_width (compared against the NORMALISED position, as the
reference does), clipped."""
from typing import Optional

import numpy as np

from ballbot_gym.terrain._common import check_odd, smoothstep, unit_grid


def generate_terraced_terrain(n: int, num_terraces: int = 5, terrace_height: float = 0.15,
                              transition_width: float = 0.1, smoothness: float = 0.7, direction: str = "x",
                              seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    assert num_terraces > 0, "num_terraces must be positive"
    assert 0 < terrace_height <= 1.0, "terrace_height should be between 0 and 1"
    assert 0 < transition_width < 1.0, "transition_width should be between 0 and 1"
    assert direction in ["x", "y"], "direction must be 'x' or 'y'"
    X, Y = unit_grid(n)
    c = X if direction == "x" else Y
    w = 1.0 / num_terraces
    ts = w * transition_width
    idx = np.minimum((c / w).astype(np.int64), num_terraces - 1)
    pos = np.mod(c, w) / w
    base = idx * terrace_height
    prev = (idx - 1) * terrace_height
    nxt = (idx + 1) * terrace_height
    up = prev + (base - prev) * smoothstep(0.0, 1.0, pos / ts)
    dn = base + (nxt - base) * smoothstep(0.0, 1.0, (pos - (1.0 - ts)) / ts)
    t = np.where(pos < ts, np.where(idx > 0, up, base),
                 np.where(pos > 1.0 - ts, np.where(idx < num_terraces - 1, dn, base), base))
    return np.clip(t.astype(np.float64), 0.0, 1.0).flatten()
