"""Composite terrain (reference terrain/mixed.py:8-101): components built via
create_terrain, blended additively (normalised weights), by max, or weighted
average, then clipped."""
from typing import Any, Dict, List, Optional

import numpy as np

from ballbot_gym.terrain._common import check_odd


def generate_mixed_terrain(n: int, components: List[Dict[str, Any]], blend_mode: str = "additive",
                           seed: Optional[int] = None) -> np.ndarray:
    from ballbot_gym.core.factories import create_terrain

    check_odd(n)
    assert len(components) > 0, "components list cannot be empty"
    assert blend_mode in ["additive", "max", "weighted"], "blend_mode must be 'additive', 'max', or 'weighted'"
    gens, weights = [], []
    for comp in components:
        if not isinstance(comp, dict):
            raise ValueError(f"Component must be a dict, got {type(comp)}")
        ctype = comp.get("type")
        if ctype is None:
            raise ValueError("Component must have 'type' key")
        cfg = {"type": ctype, "config": comp.get("config", {})}
        if "seed" not in cfg["config"] and seed is not None:
            cfg["config"]["seed"] = seed
        gens.append(create_terrain(cfg))
        weights.append(comp.get("weight", 1.0))
    parts = [g(n, seed=seed).reshape(n, n) for g in gens]
    t = np.zeros((n, n))
    if blend_mode == "max":
        for p, w in zip(parts, weights):
            t = np.maximum(t, p * w)
    else:
        tw = sum(weights)
        for p, w in zip(parts, weights):
            t += p * (w / tw) if blend_mode == "additive" else p * w
        if blend_mode == "weighted":
            t = t / tw
    return np.clip(t, 0.0, 1.0).flatten()
