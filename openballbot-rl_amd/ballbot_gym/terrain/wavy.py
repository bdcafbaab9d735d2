"""Wavy terrain (reference terrain/wavy.py:7-86): sum of directional sines + 0.5, clipped."""
from typing import List, Optional

import numpy as np

from ballbot_gym.terrain._common import check_odd


def generate_wavy_terrain(n: int, wave_amplitudes: Optional[List[float]] = None,
                          wave_frequencies: Optional[List[float]] = None,
                          wave_directions: Optional[List[float]] = None, phase_offsets: Optional[List[float]] = None,
                          seed: Optional[int] = None) -> np.ndarray:
    check_odd(n)
    amps = [0.3, 0.2, 0.1] if wave_amplitudes is None else wave_amplitudes
    freqs = [0.05, 0.1, 0.2] if wave_frequencies is None else wave_frequencies
    dirs = [0.0, 45.0, 90.0] if wave_directions is None else wave_directions
    phases = [0.0, 0.5, 1.0] if phase_offsets is None else phase_offsets
    k = len(amps)
    assert len(freqs) == k, "wave_frequencies must match wave_amplitudes length"
    assert len(dirs) == k, "wave_directions must match wave_amplitudes length"
    assert len(phases) == k, "phase_offsets must match wave_amplitudes length"
    g = np.linspace(0, 2 * np.pi, n)
    X, Y = np.meshgrid(g, g, indexing="ij")
    t = np.zeros((n, n))
    for a, f, d, p in zip(amps, freqs, dirs, phases):
        r = np.radians(d)
        t += a * np.sin(f * (X * np.cos(r) + Y * np.sin(r)) + p)
    t += 0.5
    return np.clip(t, 0.0, 1.0).flatten()
