"""Terrain plugins: fn(n, **cfg) -> float64[n*n] in [0, 1], row i <-> y, col j <-> x.

Registered on import like the reference (ballbot_gym/terrain/__init__.py:18-36).
The batched env evaluates them host-side once per bank slot and uploads the
heightfields with bb_set_hfield."""
import numpy as np

from ballbot_gym.core.registry import ComponentRegistry
from ballbot_gym.terrain.hills import generate_hills_terrain


def generate_flat_terrain(n: int, **kwargs) -> np.ndarray:
    """Flat terrain (terrain/__init__.py:32-34)."""
    return np.zeros(n * n)


_BUILTINS = {
    "hills": generate_hills_terrain,
    "flat": generate_flat_terrain,
}
for _name, _fn in _BUILTINS.items():
    if _name not in ComponentRegistry.list_terrains():
        ComponentRegistry.register_terrain(_name, _fn)

__all__ = ["generate_flat_terrain", "generate_hills_terrain"]
