"""Host-side configuration of the batched env (no GPU needed; unit-tested on CPU).

* params_from_configs: BBotSimulation kwargs / YAML (ballbot_env.py:157-231,
  configs/env/*.yaml) + reward plugin -> bb_params for the C-ABI.  Built-in
  rewards map to fused kernel ids (B2); any other BaseReward is evaluated on
  the host.
* terrain_plan: which terrains the bank holds and which generator every env
  draws its terrain seeds from.  The reference draws r_seed =
  _np_random.integers(0, 10000) at each reset (ballbot_env.py:505-510).  In
  training, SB3 seeds the VecEnv with the PPO seed (VecEnv.seed(seed) -> env i
  gets seed + i) and the first reset of learn() calls reset(seed=seed+i),
  which gymnasium's Env.reset turns into a new _np_random = np_random(seed+i)
  (:596, train.py:126-141; training/utils.py:42-46 says so): training env i
  draws every terrain from np_random(seed + i).  Eval env i keeps the
  np_random(seed + N_ENVS + i) fixed at construction (eval_env=[True, s],
  :378-384, train.py:90-97).  The draws run on the GPU (bb_set_terrain_rng:
  numpy's PCG64 per env, bit-exact, unbounded); the plan names each env's
  generator seed and the bank slot of every terrain seed.
* terrain_bank / bank_fields: the registered terrain plugin evaluated per seed
  (ballbot_env.py:501-513) with the ramp/gradient size_z rescale (:486-495).
* np_random / pcg64_words: gymnasium's seeding (Generator(PCG64(SeedSequence(
  seed))), ballbot_env.py:596-599) and its generator state as the device takes it.
* init_offset: reset height placement (ballbot_env.py:546-563), including the
  reference's cell_size = size / nrows quirk.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import _native as N

HFIELD_HALF_SIZE = 5.0   # ballbot.xml:23 size 5 5 2.0 0.1
DEFAULT_SIZE_Z = 2.0
TERRAIN_SEED_HIGH = 10000  # ballbot_env.py:505-510 integers(0, 10000)

# reference generators that ignore their seed argument ("unused, for API
# compatibility": terrain/{ramp,terraced,wavy,spiral,sinusoidal,ridge_valley,
# bowl}.py, gradient.py unless gradient_type is "perlin"): one bank slot serves
# every draw
SEEDLESS_TERRAINS = frozenset({"ramp", "terraced", "wavy", "spiral", "sinusoidal", "ridge_valley", "bowl"})


def np_random(seed: Optional[int]) -> np.random.Generator:
    """gymnasium.utils.seeding.np_random restated (seed None -> OS entropy)."""
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


def pcg64_words(gen_or_seed) -> np.ndarray:
    """The state of np_random(seed) (or of a Generator / PCG64 as it stands) as the
    five words bb_set_terrain_rng takes: state >> 64, state & (2^64 - 1),
    inc >> 64, inc & (2^64 - 1), (has_uint32 << 32) | uinteger."""
    if isinstance(gen_or_seed, np.random.Generator):
        bg = gen_or_seed.bit_generator
    elif isinstance(gen_or_seed, np.random.PCG64):
        bg = gen_or_seed
    else:
        bg = np.random.PCG64(np.random.SeedSequence(gen_or_seed))
    st = bg.state
    if st["bit_generator"] != "PCG64":
        raise ValueError(f"device terrain draws restate PCG64, not {st['bit_generator']}")
    m = (1 << 64) - 1
    s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
    return np.array([s >> 64, s & m, inc >> 64, inc & m, (int(st["has_uint32"]) << 32) | int(st["uinteger"])],
                    dtype=np.uint64)


# the device generator restated on the host (bb_kernels.hip: pcg64_next64 /
# pcg64_next32 / pcg64_terrain_seed): a checker for the kernel and a pin of the
# restatement against numpy (tests/test_host_config.py)
_PCG_MULT = 0x2360ED051FC65DA44385DF649FCCF645


def pcg64_terrain_draws(words: Sequence[int], k: int) -> Tuple[List[int], np.ndarray]:
    """k values of integers(0, 10000) from a generator in pcg64_words form
    -> (values, the words after them)."""
    m64, m128 = (1 << 64) - 1, (1 << 128) - 1
    st = (int(words[0]) << 64) | int(words[1])
    inc = (int(words[2]) << 64) | int(words[3])
    has, buf = int(words[4]) >> 32, int(words[4]) & 0xFFFFFFFF

    def next32():
        nonlocal st, has, buf
        if has:
            has = 0
            return buf
        st = (st * _PCG_MULT + inc) & m128
        hi, lo = st >> 64, st & m64
        rot = hi >> 58
        x = hi ^ lo
        x = ((x >> rot) | (x << ((64 - rot) & 63))) & m64
        has, buf = 1, x >> 32
        return x & 0xFFFFFFFF

    out = []
    excl = TERRAIN_SEED_HIGH
    threshold = (0xFFFFFFFF - (excl - 1)) % excl
    for _ in range(int(k)):
        mm = next32() * excl
        if (mm & 0xFFFFFFFF) < excl:
            while (mm & 0xFFFFFFFF) < threshold:
                mm = next32() * excl
        out.append(mm >> 32)
    return out, np.array([st >> 64, st & m64, inc >> 64, inc & m64, (has << 32) | buf], dtype=np.uint64)


def terrain_size_z(terrain_config: Dict[str, Any]) -> float:
    """hfield_size[2] for the terrain type (ballbot_env.py:486-495)."""
    ttype = terrain_config.get("type", "flat")
    tcfg = terrain_config.get("config", {}) or {}
    if ttype == "ramp":
        return float(2 * HFIELD_HALF_SIZE * np.tan(np.radians(tcfg.get("ramp_angle", 15.0))))
    if ttype == "gradient":
        return float(2 * HFIELD_HALF_SIZE * np.tan(np.radians(tcfg.get("max_slope", 20.0))))
    return DEFAULT_SIZE_Z


def terrain_is_seedless(terrain_config: Dict[str, Any]) -> bool:
    """The terrain does not depend on the drawn seed (SEEDLESS_TERRAINS)."""
    ttype = terrain_config.get("type", "flat")
    tcfg = terrain_config.get("config", {}) or {}
    if ttype == "gradient":
        return tcfg.get("gradient_type", "linear") != "perlin"
    return ttype in SEEDLESS_TERRAINS


def stream_draws(seed: Optional[int], k: int) -> np.ndarray:
    """The first k terrain seeds one env draws, one per reset: the values of
    _np_random.integers(0, 10000) called once per reset (ballbot_env.py:505-510)
    on np_random(seed).  One vector call gives the same values as k scalar calls
    (PCG64's 32-bit draws are buffered in the bit generator; pinned by
    tests/test_host_config.py)."""
    return np_random(seed).integers(0, TERRAIN_SEED_HIGH, size=int(k)).astype(np.int64)


def sb3_stream_seeds(seed: int, num_envs: int, first_env: int = 0) -> List[int]:
    """Terrain generator seed of each env of a VecEnv seeded the way SB3 seeds
    it: VecEnv.seed(seed) gives env i the seed seed + i, used by the first
    reset (SB3 2.x VecEnv.seed / DummyVecEnv.reset, called from PPO(seed=...)
    and learn(), ballbot_rl/training/train.py:126-141, 284); first_env offsets
    a rank's block of global env ids."""
    return [int(seed) + int(first_env) + i for i in range(int(num_envs))]


# draws per stream whose seeds a host-generated bank holds by default: shared
# stream / one generator per env; past those a draw whose seed is not resident
# is counted (stats[5]); when the draws name more than FULL_HOST_BANK distinct
# seeds the bank holds the whole seed space instead
NUMPY_BANK_DRAWS = 128
NUMPY_BANK_DRAWS_PER_ENV = 16
FULL_HOST_BANK = 2500


class TerrainPlan:
    """Bank contents and per-reset draws of the batched env.

    seeds        terrain seed held by each bank slot (-1: seedless, e.g. flat)
    stream_seeds generator seed of every env (device PCG64 draws,
                 bb_set_terrain_rng), or None: one fixed terrain / a draw table
    seed_slot    int32[10000] bank slot of each terrain seed (-1: not resident),
                 or None: slot == seed (the bank is the whole seed space)
    streams      int32[1][draws]: an explicit draw table (bank slots) that every
                 env walks (bb_set_terrain_stream), or None
    full         the bank holds the whole seed space (slot == seed)
    """

    def __init__(self, seeds, stream_seeds, seed_slot, full, size_z, streams=None, env_stream=None,
                 seedless: bool = False):
        self.seeds, self.stream_seeds, self.seed_slot = seeds, stream_seeds, seed_slot
        self.full, self.size_z, self.streams, self.env_stream = full, size_z, streams, env_stream
        self.seedless = seedless

    def rng_words(self) -> np.ndarray:
        """uint64[n][5]: every env's generator np_random(stream_seeds[e]) (bb_set_terrain_rng)."""
        cache: Dict[int, np.ndarray] = {}
        out = np.empty((len(self.stream_seeds), 5), np.uint64)
        for e, s in enumerate(self.stream_seeds):
            if s not in cache:
                cache[s] = pcg64_words(s)
            out[e] = cache[s]
        return out

    def slot_of(self, seed: int) -> int:
        """Bank slot of a terrain seed (-1: not resident)."""
        if self.full:
            return int(seed)
        if self.seed_slot is not None:
            return int(self.seed_slot[int(seed)])
        return self.seeds.index(int(seed)) if int(seed) in self.seeds else -1

    def covers(self, seeds) -> bool:
        """Every terrain seed in `seeds` is resident."""
        return self.full or self.seedless or all(self.seed_slot[int(s)] >= 0 for s in seeds)


def terrain_plan(terrain_config: Dict[str, Any], n_terrains: Optional[int], seed: Optional[int], num_envs: int,
                 stream_seeds: Optional[List[int]] = None, full_bank: bool = False,
                 draws: Optional[np.ndarray] = None, shared: bool = False) -> TerrainPlan:
    """Generators and bank slots.  stream_seeds: env i draws from
    np_random(stream_seeds[i]); None: np_random(seed + i) (SB3's seeding,
    sb3_stream_seeds), or np_random(seed) for every env with shared=True.
    n_terrains: the draws per generator whose seeds the bank holds (default
    NUMPY_BANK_DRAWS for one shared generator, NUMPY_BANK_DRAWS_PER_ENV
    otherwise); when they name more than FULL_HOST_BANK distinct seeds the bank
    holds the whole seed space instead;
    full_bank: the bank is the whole seed space [0, 10000).  draws: the terrain
    seeds of one explicit draw table that every env walks (no generator)."""
    ttype = terrain_config.get("type", "flat")
    tcfg = terrain_config.get("config", {}) or {}
    size_z = terrain_size_z(terrain_config)
    if ttype == "flat" or tcfg.get("seed") is not None:
        return TerrainPlan([int(tcfg["seed"]) if tcfg.get("seed") is not None else -1], None, None, False, size_z)
    if n_terrains is not None and int(n_terrains) < 1:
        raise ValueError(f"n_terrains must be >= 1, got {n_terrains}")
    if draws is not None:  # explicit table: the distinct seeds, in order of first draw
        draws = np.asarray(draws, np.int64).reshape(-1)
        seeds = list(dict.fromkeys(int(v) for v in draws))
        slot = {v: i for i, v in enumerate(seeds)}
        table = np.array([[slot[int(v)] for v in draws]], np.int32)
        return TerrainPlan(seeds, None, None, False, size_z, streams=table)
    if stream_seeds is None:
        stream_seeds = [int(seed)] * int(num_envs) if shared else sb3_stream_seeds(seed if seed is not None else 0,
                                                                                    num_envs)
    stream_seeds = [int(x) for x in stream_seeds]
    if len(stream_seeds) != num_envs:
        raise ValueError(f"stream_seeds needs one seed per env ({num_envs}), got {len(stream_seeds)}")
    if terrain_is_seedless(terrain_config):
        first = int(stream_draws(stream_seeds[0], 1)[0])
        return TerrainPlan([first], stream_seeds, np.zeros(TERRAIN_SEED_HIGH, np.int32), False, size_z, seedless=True)
    uniq = list(dict.fromkeys(stream_seeds))
    if not full_bank:
        k = int(n_terrains) if n_terrains is not None else (
            NUMPY_BANK_DRAWS if len(uniq) == 1 else NUMPY_BANK_DRAWS_PER_ENV)
        seen: Dict[int, None] = {}
        for s in uniq:
            for v in stream_draws(s, k):
                seen.setdefault(int(v))
            if len(seen) > FULL_HOST_BANK:
                break
        full_bank = len(seen) > FULL_HOST_BANK
    if full_bank:
        return TerrainPlan(list(range(TERRAIN_SEED_HIGH)), stream_seeds, None, True, size_z)
    seeds = list(seen)
    seed_slot = np.full(TERRAIN_SEED_HIGH, -1, np.int32)
    seed_slot[np.asarray(seeds, np.int64)] = np.arange(len(seeds), dtype=np.int32)
    return TerrainPlan(seeds, stream_seeds, seed_slot, False, size_z)


def terrain_bank(terrain_config: Dict[str, Any], n_terrains: Optional[int], seed: Optional[int],
                 n: int = N.HF_N, num_envs: int = 1, stream_seeds: Optional[List[int]] = None
                 ) -> Tuple[List[np.ndarray], List[int], float]:
    """Heightfields (float32[n*n]) for the bank slots of terrain_plan(...), the
    seed of each slot and size_z (flat / seeded configs: one slot)."""
    plan = terrain_plan(terrain_config, n_terrains, seed, num_envs, stream_seeds)
    return bank_fields(terrain_config, plan, n), plan.seeds, plan.size_z


def _gen_chunk(terrain_config: Dict[str, Any], seeds: List[int], n: int) -> List[np.ndarray]:
    from ..core.factories import create_terrain

    gen = create_terrain(terrain_config)  # seed None: the config's own (a fixed config seed, or none)
    return [np.asarray(gen(n) if s is None else gen(n, seed=s), dtype=np.float32) for s in seeds]


def _builtin_generator(terrain_config: Dict[str, Any]) -> bool:
    """The registered generator(s) are the built-ins (a fresh process registers the same)."""
    from ..core.registry import ComponentRegistry
    from ..terrain import BUILTIN_TERRAINS

    types = [terrain_config.get("type", "flat")]
    if types[0] == "mixed":
        types += [c.get("type") for c in (terrain_config.get("config", {}) or {}).get("components", [])]
    try:
        return all(t in BUILTIN_TERRAINS and ComponentRegistry.get_terrain(t) is BUILTIN_TERRAINS[t] for t in types)
    except Exception:
        return False


def bank_fields(terrain_config: Dict[str, Any], plan: TerrainPlan, n: int = N.HF_N,
                workers: Optional[int] = None) -> List[np.ndarray]:
    """The registered terrain plugin evaluated for every bank slot of the plan
    (ballbot_env.py:501-513: terrain_gen(nrows, seed=r_seed)).  Large banks of
    built-in generators (e.g. the whole seed space for per-env generators) run on
    a pool of host processes; custom plugins run in this process."""
    if plan.stream_seeds is None and plan.streams is None:
        return _gen_chunk(terrain_config, [None], n)
    seeds = list(plan.seeds)
    import os

    w = workers if workers is not None else min(16, os.cpu_count() or 1)
    if len(seeds) < 64 or w <= 1 or not _builtin_generator(terrain_config):
        return _gen_chunk(terrain_config, seeds, n)
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor

    step = -(-len(seeds) // (4 * w))
    parts = [seeds[i:i + step] for i in range(0, len(seeds), step)]
    # spawn: the workers run numpy only, never the GPU state of this process
    with ProcessPoolExecutor(w, mp_context=mp.get_context("spawn")) as ex:
        out = []
        for r in ex.map(_gen_chunk, [terrain_config] * len(parts), parts, [n] * len(parts)):
            out += r
    return out


PERLIN_DEFAULTS = {"scale": 25.0, "octaves": 4, "persistence": 0.2, "lacunarity": 2.0, "amplitude": 1.0}


def gpu_perlin_plan(terrain_config: Dict[str, Any], n_terrains: Optional[int], seed: Optional[int],
                    num_envs: int = 1, stream_seeds: Optional[List[int]] = None, draws: Optional[np.ndarray] = None,
                    shared: bool = False) -> Optional[Tuple[TerrainPlan, N.PerlinCfg]]:
    """(plan, generator args) when the bank is generated on the GPU (bb_generate_perlin), else None.

    Perlin without a fixed config seed: the reference draws a fresh seed from
    integers(0, 10000) at every reset and regenerates (ballbot_env.py:501-513).
    With n_terrains None the bank holds that whole seed space (slot == seed,
    3.4 GB of HBM), so every reset draw the reference can make is resident; an
    explicit n_terrains keeps the seeds of the first n_terrains draws per generator."""
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
                        draws=draws, shared=shared)
    return plan, perlin_cfg(terrain_config)


def perlin_cfg(terrain_config: Dict[str, Any]) -> N.PerlinCfg:
    """bb_perlin_cfg of a perlin terrain config (terrain/perlin.py:8-16 defaults)."""
    tcfg = {k: v for k, v in (terrain_config.get("config", {}) or {}).items() if k != "seed"}
    args = {**PERLIN_DEFAULTS, **tcfg}
    return N.PerlinCfg(float(args["scale"]), int(args["octaves"]), float(args["persistence"]),
                       float(args["lacunarity"]), float(args["amplitude"]))


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


DISTANCE_REWARD_ERROR = "DistanceReward requires 'pos2d' in state dictionary"  # rewards/distance.py:43-44
REWARD_COMPAT = ("reference", "fused")


def params_from_configs(reward_config: Optional[Dict[str, Any]] = None, env_config: Optional[Dict[str, Any]] = None,
                        max_ep_steps: Optional[int] = None, precision: str = "fp64",
                        seed: int = 0, reward_compat: str = "reference") -> Tuple[N.BBParams, Any, Optional[Any]]:
    """-> (bb_params, reward plugin object, host reward or None).

    reward_compat: "reference" keeps the reference env's behaviour with
    DistanceReward -- its obs dict never carries pos2d (ballbot_env.py:929
    calls reward_obj(obs)), so the first step raises ValueError
    (rewards/distance.py:43-44); "fused" computes it from the step's pos2d in
    the kernel (BB_REWARD_DISTANCE).  Check reward_error() of the result."""
    if reward_compat not in REWARD_COMPAT:
        raise ValueError(f"reward_compat must be one of {REWARD_COMPAT}, got {reward_compat!r}")
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


def reward_error(reward: Any, reward_compat: str = "reference") -> Optional[str]:
    """The error the reference env raises at its first step with this reward
    plugin, or None (see params_from_configs)."""
    from ..rewards.distance import DistanceReward

    if reward_compat == "reference" and type(reward) is DistanceReward:
        return DISTANCE_REWARD_ERROR
    return None
