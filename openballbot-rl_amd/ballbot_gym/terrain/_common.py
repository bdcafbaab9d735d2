"""Shared helpers of the terrain plugins (reset-time, host numpy)."""
import numpy as np


def smoothstep(edge0, edge1, x):
    """Hermite step, as the reference's per-module smoothstep (e.g. ramp.py:6-14)."""
    x = np.clip((x - edge0) / (edge1 - edge0), 0.0, 1.0)
    return x * x * (3.0 - 2.0 * x)


def unit_grid(n):
    """(X, Y) on linspace(0, 1, n), 'ij' indexing (row i <-> X)."""
    g = np.linspace(0, 1, n)
    return np.meshgrid(g, g, indexing="ij")


def centred_grid(n):
    """(X, Y) = (k - n//2) / (n//2), 'ij' indexing."""
    c = n // 2
    g = (np.arange(n) - c) / c
    return np.meshgrid(g, g, indexing="ij")


def minmax(t):
    """Normalise to [0, 1]; constant fields become zeros."""
    lo, hi = t.min(), t.max()
    if hi > lo:
        return (t - lo) / (hi - lo)
    return np.zeros_like(t)


def check_odd(n):
    assert n % 2 == 1, "n should be odd for heightfield symmetry"
