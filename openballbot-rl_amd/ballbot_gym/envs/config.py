"""Host-side configuration of the batched env (no GPU needed; unit-tested on CPU).

* params_from_configs: BBotSimulation kwargs / YAML (ballbot_env.py:157-231,
  configs/env/*.yaml) + reward plugin -> bb_params for the C-ABI.  Built-in
  rewards map to fused kernel ids (B2); any other BaseReward is evaluated on
  the host.
* terrain_bank: the registered terrain plugin evaluated per seed
  (ballbot_env.py:501-513) with the ramp/gradient size_z rescale (:486-495).
* np_random: gymnasium's seeding (Generator(PCG64(SeedSequence(seed))),
  ballbot_env.py:596-599), the stream terrain seeds are drawn from.
* init_offset: reset height placement (ballbot_env.py:546-563), including the
  reference's cell_size = size / nrows quirk.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .. import _native as N

HFIELD_HALF_SIZE = 5.0   # ballbot.xml:23 size 5 5 2.0 0.1
DEFAULT_SIZE_Z = 2.0
TERRAIN_SEED_HIGH = 10000  # ballbot_env.py:505-510 integers(0, 10000)


def np_random(seed: Optional[int]) -> np.random.Generator:
    """gymnasium.utils.seeding.np_random restated (seed None -> OS entropy)."""
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


def terrain_size_z(terrain_config: Dict[str, Any]) -> float:
    """hfield_size[2] for the terrain type (ballbot_env.py:486-495)."""
    ttype = terrain_config.get("type", "flat")
    tcfg = terrain_config.get("config", {}) or {}
    if ttype == "ramp":
        return float(2 * HFIELD_HALF_SIZE * np.tan(np.radians(tcfg.get("ramp_angle", 15.0))))
    if ttype == "gradient":
        return float(2 * HFIELD_HALF_SIZE * np.tan(np.radians(tcfg.get("max_slope", 20.0))))
    return DEFAULT_SIZE_Z


def terrain_bank(terrain_config: Dict[str, Any], n_terrains: Optional[int], seed: Optional[int],
                 n: int = N.HF_N) -> Tuple[List[np.ndarray], List[int], float]:
    """Heightfields (float32[n*n]) for the bank slots, the terrain seeds used and size_z.

    flat / seeded configs give one slot; otherwise `n_terrains` (default 16)
    seeds are the first draws of np_random(seed).integers(0, 10000), the
    reference's per-reset draw (ballbot_env.py:505-510)."""
    from ..core.factories import create_terrain

    ttype = terrain_config.get("type", "flat")
    tcfg = terrain_config.get("config", {}) or {}
    size_z = terrain_size_z(terrain_config)
    gen = create_terrain(terrain_config)
    if ttype == "flat" or tcfg.get("seed") is not None:
        return [np.asarray(gen(n), dtype=np.float32)], [tcfg.get("seed", -1)], size_z
    k = int(n_terrains or 16)
    if k < 1:
        raise ValueError(f"n_terrains must be >= 1, got {k}")
    seeds = [int(s) for s in np_random(seed).integers(0, TERRAIN_SEED_HIGH, size=k)]
    return [np.asarray(gen(n, seed=s), dtype=np.float32) for s in seeds], seeds, size_z


PERLIN_DEFAULTS = {"scale": 25.0, "octaves": 4, "persistence": 0.2, "lacunarity": 2.0, "amplitude": 1.0}


def gpu_perlin_plan(terrain_config: Dict[str, Any], n_terrains: Optional[int],
                    seed: Optional[int]) -> Optional[Tuple[List[int], N.PerlinCfg, float]]:
    """Seeds + generator args when the bank is generated on the GPU (bb_generate_perlin), else None.

    Perlin without a fixed config seed: the reference draws a fresh seed from
    integers(0, 10000) at every reset and regenerates (ballbot_env.py:501-513).
    With n_terrains None the bank holds that whole seed space (slot == seed,
    3.4 GB of HBM), so every reset draw the reference can make is resident; an
    explicit n_terrains keeps the first n_terrains draws of np_random(seed)."""
    if terrain_config.get("type", "flat") != "perlin":
        return None
    tcfg = dict(terrain_config.get("config", {}) or {})
    if tcfg.get("seed") is not None:
        return None
    tcfg.pop("seed", None)
    unknown = set(tcfg) - set(PERLIN_DEFAULTS)
    if unknown:  # generate_perlin_terrain() would raise TypeError on these too
        raise ValueError(f"perlin terrain: unknown config keys {sorted(unknown)}")
    args = {**PERLIN_DEFAULTS, **tcfg}
    if n_terrains is None:
        seeds = list(range(TERRAIN_SEED_HIGH))
    else:
        if int(n_terrains) < 1:
            raise ValueError(f"n_terrains must be >= 1, got {n_terrains}")
        seeds = [int(s) for s in np_random(seed).integers(0, TERRAIN_SEED_HIGH, size=int(n_terrains))]
    pc = N.PerlinCfg(float(args["scale"]), int(args["octaves"]), float(args["persistence"]),
                     float(args["lacunarity"]), float(args["amplitude"]))
    return seeds, pc, terrain_size_z(terrain_config)


def init_offset(hfield: np.ndarray, size_z: float, n: int = N.HF_N) -> float:
    """Initial height offset: max terrain height under the ball footprint + 1 cm."""
    sz = HFIELD_HALF_SIZE
    cell = sz / n                       # reference uses size/nrows, not 2*size/(nrows-1)
    r = 0.09                            # ball radius
    c = n // 2
    x0 = c - abs(int(np.floor(-r / cell)))
    x1 = c + int(np.floor(r / cell)) + 1
    H = np.asarray(hfield, dtype=np.float32).reshape(n, n)
    return float(np.float32(H[x0:x1, x0:x1].max()) * size_z + 0.01)


def params_from_configs(reward_config: Optional[Dict[str, Any]] = None, env_config: Optional[Dict[str, Any]] = None,
                        max_ep_steps: Optional[int] = None, precision: str = "fp64",
                        seed: int = 0) -> Tuple[N.BBParams, Any, Optional[Any]]:
    """-> (bb_params, reward plugin object, host reward or None)."""
    from ..core.factories import create_reward
    from ..rewards.directional import DirectionalReward
    from ..rewards.distance import DistanceReward

    if precision not in ("fp32", "fp64"):
        raise ValueError(f"precision must be 'fp32' or 'fp64', got {precision!r}")
    reward_config = reward_config or {"type": "directional", "config": {"target_direction": [0.0, 1.0]}}
    env = (env_config or {}).get("env", {}) or {}
    rcfg = reward_config.get("config", {}) or {}
    p = N.default_params()
    p.max_ep_steps = int(env.get("max_ep_steps", max_ep_steps if max_ep_steps is not None else 4000))
    p.max_allowed_tilt = float(env.get("max_allowed_tilt", 20.0))
    p.max_wheel_velocity = float(env.get("max_wheel_velocity", 10.0))
    p.reward_scale = float(rcfg.get("scale", 0.01))
    p.action_reg_coef = float(rcfg.get("action_reg_coef", -0.0001))
    p.survival_bonus = float(rcfg.get("survival_bonus", 0.02))
    reward = create_reward(reward_config)
    host = None
    if type(reward) is DirectionalReward:
        td = np.asarray(reward.target_direction, dtype=np.float32).reshape(-1)
        if td.shape != (2,):
            raise ValueError(f"target_direction must have 2 components, got {td.shape}")
        p.reward_kind = N.REWARD_DIRECTIONAL
        p.target_dir[0], p.target_dir[1] = float(td[0]), float(td[1])
    elif type(reward) is DistanceReward:
        p.reward_kind = N.REWARD_DISTANCE
        p.goal[0], p.goal[1] = float(reward.goal_position[0]), float(reward.goal_position[1])
        p.goal_scale = float(reward.scale)
    else:
        p.reward_kind = N.REWARD_NONE
        host = reward
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    p.fp64 = 1 if precision == "fp64" else 0
    return p, reward, host
