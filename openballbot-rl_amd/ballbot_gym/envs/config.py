"""Host-side configuration of the batched env (no GPU needed; unit-tested on CPU).

* params_from_configs: BBotSimulation kwargs / YAML (ballbot_env.py:157-231,
  configs/env/*.yaml) + reward plugin -> bb_params for the C-ABI.  Built-in
  rewards map to fused kernel ids (B2); any other BaseReward is evaluated on
  the host.
* terrain_plan: which terrain every reset of every env gets.  The reference
  draws r_seed = _np_random.integers(0, 10000) at each reset
  (ballbot_env.py:505-510) from a generator that eval_env=[True, seed] fixes
  at construction (:378-384); train.py:82-89 builds every training env that
  way with the same seed, so the k-th reset of EVERY training env draws the
  k-th value of np_random(seed).integers(0, 10000).  The plan holds those
  draws per stream as bank slots, plus the seeds the bank must hold.
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


def stream_draws(seed: Optional[int], k: int) -> np.ndarray:
    """The first k terrain seeds one env draws, one per reset: the values of
    _np_random.integers(0, 10000) called once per reset (ballbot_env.py:505-510)
    on np_random(seed).  One vector call gives the same values as k scalar calls
    (PCG64's 32-bit draws are buffered in the bit generator; pinned by
    tests/test_host_config.py)."""
    return np_random(seed).integers(0, TERRAIN_SEED_HIGH, size=int(k)).astype(np.int64)


# resident draws per stream when the bank holds the whole seed space (slot == seed)
FULL_BANK_DRAWS_SHARED = 1 << 16
FULL_BANK_DRAWS_PER_ENV = 1024
NUMPY_BANK_DRAWS = 128  # default for host-generated banks (hills: ~14 ms per terrain)


class TerrainPlan:
    """Bank contents and per-reset draws of the batched env.

    streams  int32[n_streams][draws]: bank slot of each stream's k-th reset
             (None: no draws -- one fixed terrain, flat or a config seed)
    env_stream int32[num_envs] or None (every env on stream 0)
    seeds    terrain seed held by each bank slot (-1: seedless, e.g. flat)
    full     True when the bank holds the whole seed space (slot == seed)
    """

    def __init__(self, seeds, streams, env_stream, full, size_z):
        self.seeds, self.streams, self.env_stream, self.full, self.size_z = seeds, streams, env_stream, full, size_z

    def seed_of_draw(self, stream: int, k: int) -> int:
        return int(self.seeds[int(self.streams[stream][k % self.streams.shape[1]])])


def terrain_plan(terrain_config: Dict[str, Any], n_terrains: Optional[int], seed: Optional[int], num_envs: int,
                 stream_seeds: Optional[List[int]] = None, full_bank: bool = False,
                 draws: Optional[np.ndarray] = None) -> TerrainPlan:
    """Draw streams and bank slots.  stream_seeds None: every env shares
    np_random(seed) (train.py:82-89); else env i draws from np_random(stream_seeds[i])
    (an eval VecEnv's seed + N_ENVS + i, train.py:90-97).  n_terrains: draws kept per
    stream (the bank holds the distinct seeds among them); full_bank: the bank is
    the whole seed space [0, 10000) and n_terrains (default 65536 shared / 1024
    per env) only sets how many draws are resident.  draws: the terrain seeds of
    one stream given explicitly (every env on it), e.g. a non-eval env's stream,
    which its first reset also advances by a permutation (ballbot_env.py:658-661)."""
    ttype = terrain_config.get("type", "flat")
    tcfg = terrain_config.get("config", {}) or {}
    size_z = terrain_size_z(terrain_config)
    if ttype == "flat" or tcfg.get("seed") is not None:
        return TerrainPlan([int(tcfg["seed"]) if tcfg.get("seed") is not None else -1], None, None, False, size_z)
    if stream_seeds is not None:
        stream_seeds = [int(x) for x in stream_seeds]
        if len(stream_seeds) != num_envs:
            raise ValueError(f"stream_seeds needs one seed per env ({num_envs}), got {len(stream_seeds)}")
        uniq = sorted(set(stream_seeds), key=stream_seeds.index)
        env_stream = np.array([uniq.index(s) for s in stream_seeds], np.int32)
    else:
        uniq, env_stream = [seed], None
    if n_terrains is not None and int(n_terrains) < 1:
        raise ValueError(f"n_terrains must be >= 1, got {n_terrains}")
    if full_bank:
        k = int(n_terrains) if n_terrains is not None else (
            FULL_BANK_DRAWS_SHARED if len(uniq) == 1 else FULL_BANK_DRAWS_PER_ENV)
    else:
        k = int(n_terrains) if n_terrains is not None else NUMPY_BANK_DRAWS
    if draws is not None:
        draws = np.asarray(draws, np.int64).reshape(1, -1)
        env_stream = None
    else:
        draws = np.stack([stream_draws(s, k) for s in uniq])
    if full_bank:
        return TerrainPlan(list(range(TERRAIN_SEED_HIGH)), draws.astype(np.int32), env_stream, True, size_z)
    seeds: List[int] = []
    slot: Dict[int, int] = {}
    for v in draws.ravel():  # distinct seeds in order of first draw
        if int(v) not in slot:
            slot[int(v)] = len(seeds)
            seeds.append(int(v))
    streams = np.vectorize(slot.__getitem__, otypes=[np.int32])(draws)
    return TerrainPlan(seeds, streams, env_stream, False, size_z)


def terrain_bank(terrain_config: Dict[str, Any], n_terrains: Optional[int], seed: Optional[int],
                 n: int = N.HF_N, num_envs: int = 1, stream_seeds: Optional[List[int]] = None
                 ) -> Tuple[List[np.ndarray], List[int], float]:
    """Heightfields (float32[n*n]) for the bank slots of terrain_plan(...), the
    seed of each slot and size_z (flat / seeded configs: one slot)."""
    plan = terrain_plan(terrain_config, n_terrains, seed, num_envs, stream_seeds)
    return bank_fields(terrain_config, plan, n), plan.seeds, plan.size_z


def bank_fields(terrain_config: Dict[str, Any], plan: TerrainPlan, n: int = N.HF_N) -> List[np.ndarray]:
    """The registered terrain plugin evaluated for every bank slot of the plan
    (ballbot_env.py:501-513: terrain_gen(nrows, seed=r_seed))."""
    from ..core.factories import create_terrain

    gen = create_terrain(terrain_config)
    if plan.streams is None:
        return [np.asarray(gen(n), dtype=np.float32)]
    return [np.asarray(gen(n, seed=s), dtype=np.float32) for s in plan.seeds]


PERLIN_DEFAULTS = {"scale": 25.0, "octaves": 4, "persistence": 0.2, "lacunarity": 2.0, "amplitude": 1.0}


def gpu_perlin_plan(terrain_config: Dict[str, Any], n_terrains: Optional[int], seed: Optional[int],
                    num_envs: int = 1, stream_seeds: Optional[List[int]] = None, draws: Optional[np.ndarray] = None
                    ) -> Optional[Tuple[TerrainPlan, N.PerlinCfg]]:
    """(plan, generator args) when the bank is generated on the GPU (bb_generate_perlin), else None.

    Perlin without a fixed config seed: the reference draws a fresh seed from
    integers(0, 10000) at every reset and regenerates (ballbot_env.py:501-513).
    With n_terrains None the bank holds that whole seed space (slot == seed,
    3.4 GB of HBM), so every reset draw the reference can make is resident; an
    explicit n_terrains keeps the first n_terrains draws per stream."""
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
    plan = terrain_plan(terrain_config, n_terrains, seed, num_envs, stream_seeds, full_bank=n_terrains is None,
                        draws=draws)
    pc = N.PerlinCfg(float(args["scale"]), int(args["octaves"]), float(args["persistence"]),
                     float(args["lacunarity"]), float(args["amplitude"]))
    return plan, pc


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
