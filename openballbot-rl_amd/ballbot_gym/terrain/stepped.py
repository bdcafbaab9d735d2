"""Stepped terrain (reference terrain/stepped.py:7-67).

Step index = min(i // s + j // s, num_steps - 1) with s = n // num_steps,
then ONE in-place Gauss-Seidel smoothing sweep over the interior
(0.7 * self + 0.3 * mean of the 4 neighbours, already-updated up/left
neighbours included), then min-max normalisation.  The sweep is a true
recurrence, so it runs row by row; the neighbour mean keeps the reference's
summation order (up + down + left + right) / 4."""
from typing import Optional

import numpy as np

from ballbot_gym.terrain._common import check_odd, minmax


def generate_stepped_terrain(n: int, num_steps: int = 5, step_height: float = 0.1,
                             seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    assert num_steps > 0, "num_steps must be positive"
    assert step_height > 0, "step_height must be positive"
    s = n // num_steps
    k = np.arange(n) // s
    t = np.minimum(k[:, None] + k[None, :], num_steps - 1) * step_height
    t = t.astype(np.float64)
    for i in range(1, n - 1):
        up = t[i - 1]
        row = t[i].tolist()
        down = t[i + 1]
        ud = (up + down).tolist()  # first two terms of the neighbour sum
        left = row[0]
        for j in range(1, n - 1):
            v = 0.7 * row[j] + 0.3 * (((ud[j] + left) + row[j + 1]) / 4)
            row[j] = v
            left = v
        t[i] = row
    return minmax(t).flatten()
