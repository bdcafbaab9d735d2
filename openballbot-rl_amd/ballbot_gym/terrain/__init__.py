"""Terrain plugins: fn(n, **cfg) -> float64[n*n] in [0, 1], row i <-> y, col j <-> x.

Registered on import like the reference (ballbot_gym/terrain/__init__.py:18-36).
The batched env evaluates them host-side once per bank slot (reset-time work,
never on the step path) and uploads the heightfields with bb_set_hfield.
Every numpy generator is pinned bit-for-bit against the reference's outputs
in tests/golden/terrains.npz; perlin restates the `noise` library's simplex
fBm (absent here) and is property-tested only (parity unpinned)."""
import numpy as np

from ballbot_gym.core.registry import ComponentRegistry
from ballbot_gym.terrain.bowl import generate_bowl_terrain
from ballbot_gym.terrain.gradient import generate_gradient_terrain
from ballbot_gym.terrain.hills import generate_hills_terrain
from ballbot_gym.terrain.mixed import generate_mixed_terrain
from ballbot_gym.terrain.perlin import generate_perlin_terrain
from ballbot_gym.terrain.ramp import generate_ramp_terrain
from ballbot_gym.terrain.ridge_valley import generate_ridge_valley_terrain
from ballbot_gym.terrain.sinusoidal import generate_sinusoidal_terrain
from ballbot_gym.terrain.spiral import generate_spiral_terrain
from ballbot_gym.terrain.stepped import generate_stepped_terrain
from ballbot_gym.terrain.terraced import generate_terraced_terrain
from ballbot_gym.terrain.wavy import generate_wavy_terrain


def generate_flat_terrain(n: int, **kwargs) -> np.ndarray:
    """Flat terrain (terrain/__init__.py:32-34)."""
    return np.zeros(n * n)


BUILTIN_TERRAINS = {
    "perlin": generate_perlin_terrain,
    "stepped": generate_stepped_terrain,
    "ramp": generate_ramp_terrain,
    "sinusoidal": generate_sinusoidal_terrain,
    "ridge_valley": generate_ridge_valley_terrain,
    "hills": generate_hills_terrain,
    "bowl": generate_bowl_terrain,
    "gradient": generate_gradient_terrain,
    "terraced": generate_terraced_terrain,
    "wavy": generate_wavy_terrain,
    "spiral": generate_spiral_terrain,
    "mixed": generate_mixed_terrain,
    "flat": generate_flat_terrain,
}


def register_builtin_terrains() -> None:
    """(Re-)register the built-ins, skipping names already present."""
    have = set(ComponentRegistry.list_terrains())
    for name, fn in BUILTIN_TERRAINS.items():
        if name not in have:
            ComponentRegistry.register_terrain(name, fn)


register_builtin_terrains()

__all__ = ["generate_flat_terrain", "register_builtin_terrains", "BUILTIN_TERRAINS"] + [
    f.__name__ for f in BUILTIN_TERRAINS.values() if f is not generate_flat_terrain]
