"""Ramp / inclined-plane terrain (reference terrain/ramp.py:17-173).

Height = smoothstep ramp of max_height = 2 tan(angle) along x, y (single or
periodic ramps) or radially, then min-max normalised.  Vectorised; the
element formulas are the reference's."""
from typing import Optional

import numpy as np

from ballbot_gym.terrain._common import centred_grid, check_odd, minmax, smoothstep


def _ramp_1d(c, flat_ratio, num_ramps, hmax):
    if num_ramps == 1:
        fw = flat_ratio / 2.0
        r = smoothstep(0.0, 1.0, (c + fw) / (fw * 2))
        return np.where(c < -fw, 0.0, np.where(c < fw, r * hmax, hmax))
    period = 2.0 / num_ramps
    p = np.mod(c + 1.0, period) / period
    rp = smoothstep(0.0, 1.0, (p - flat_ratio / 2) / (1.0 - flat_ratio))
    return np.where(p < flat_ratio / 2, 0.0, np.where(p < 1.0 - flat_ratio / 2, rp * hmax, hmax))


def generate_ramp_terrain(n: int, ramp_angle: float = 15.0, ramp_direction: str = "x", flat_ratio: float = 0.3,
                          num_ramps: int = 1, transition_smoothness: float = 0.5,
                          seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    assert 0 <= ramp_angle <= 45, "ramp_angle should be between 0 and 45 degrees"
    assert 0 <= flat_ratio <= 1.0, "flat_ratio should be between 0 and 1"
    assert num_ramps > 0, "num_ramps must be positive"
    assert ramp_direction in ["x", "y", "radial"], "ramp_direction must be 'x', 'y', or 'radial'"
    hmax = np.tan(np.radians(ramp_angle)) * 2.0
    X, Y = centred_grid(n)
    with np.errstate(divide="ignore", invalid="ignore"):
        if ramp_direction in ("x", "y"):
            t = _ramp_1d(X if ramp_direction == "x" else Y, flat_ratio, num_ramps, hmax)
        else:
            R = np.sqrt(X ** 2 + Y ** 2)
            rmax = np.sqrt(2.0)
            fr = flat_ratio * rmax / np.sqrt(2.0)
            rr = np.clip((R - fr) / (rmax - fr), 0.0, 1.0)
            t = np.where(R < fr, 0.0, smoothstep(0.0, 1.0, rr) * hmax)
    return minmax(np.asarray(t, np.float64)).flatten()
