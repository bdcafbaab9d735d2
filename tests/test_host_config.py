"""Host-side glue of BallbotVecEnv (no GPU): config -> bb_params, reward
plugin routing (fused kernel id vs host plugin), terrain bank, obs layout."""
import numpy as np
import pytest


def test_directional_reward_maps_to_fused_kernel(reward_config):
    from ballbot_gym import _native as N
    from ballbot_gym.envs.config import params_from_configs

    env_cfg = {"env": {"max_ep_steps": 1000, "max_allowed_tilt": 15.0, "max_wheel_velocity": 8.0}}
    cfg = {"type": "directional", "config": {"target_direction": [1.0, 0.0], "scale": 0.05,
                                             "action_reg_coef": -0.001, "survival_bonus": 0.1}}
    p, plugin, host = params_from_configs(cfg, env_cfg, precision="fp32", seed=7)
    assert host is None and p.reward_kind == N.REWARD_DIRECTIONAL
    assert (p.target_dir[0], p.target_dir[1]) == (1.0, 0.0)
    assert (p.max_ep_steps, p.max_allowed_tilt, p.max_wheel_velocity) == (1000, 15.0, 8.0)
    assert p.reward_scale == pytest.approx(0.05) and p.survival_bonus == pytest.approx(0.1)
    assert p.action_reg_coef == pytest.approx(-0.001)
    assert p.fp64 == 0
    p, _, _ = params_from_configs(reward_config)
    assert p.fp64 == 1 and p.max_ep_steps == 4000


def test_distance_and_custom_rewards():
    from ballbot_gym import ComponentRegistry
    from ballbot_gym import _native as N
    from ballbot_gym.envs.config import params_from_configs
    from ballbot_gym.rewards import BaseReward

    p, _, host = params_from_configs({"type": "distance", "config": {"goal_position": [1.0, -2.0], "scale": 3.0}})
    assert host is None and p.reward_kind == N.REWARD_DISTANCE
    assert (p.goal[0], p.goal[1], p.goal_scale) == (1.0, -2.0, 3.0)

    class Upright(BaseReward):
        def __init__(self, weight=1.0):
            self.weight = weight

        def __call__(self, state):
            return -self.weight * float(np.linalg.norm(state["orientation"]))

    if "upright_test" not in ComponentRegistry.list_rewards():
        ComponentRegistry.register_reward("upright_test", Upright)
    p, plugin, host = params_from_configs({"type": "upright_test", "config": {"weight": 2.0}})
    assert p.reward_kind == N.REWARD_NONE and host is plugin and plugin.weight == 2.0


def test_distance_reward_compat_switch():
    """The reference env never puts pos2d into the reward's state (ballbot_env.py:929
    calls reward_obj(obs)), so DistanceReward raises ValueError at the first step
    (rewards/distance.py:43-44): reward_compat="reference" (the default) keeps that;
    "fused" computes it in the kernel from the step's pos2d."""
    from ballbot_gym.envs.config import DISTANCE_REWARD_ERROR, params_from_configs, reward_error
    from ballbot_gym.rewards.distance import DistanceReward

    cfg = {"type": "distance", "config": {"goal_position": [1.0, -2.0], "scale": 3.0}}
    _, plugin, _ = params_from_configs(cfg)
    assert reward_error(plugin) == DISTANCE_REWARD_ERROR
    assert reward_error(plugin, "fused") is None
    with pytest.raises(ValueError, match="pos2d"):  # the reference plugin itself, on the reference's obs dict
        DistanceReward([1.0, -2.0])({"vel": np.zeros(3, np.float32)})
    _, d, _ = params_from_configs({"type": "directional", "config": {"target_direction": [0.0, 1.0]}})
    assert reward_error(d) is None
    with pytest.raises(ValueError, match="reward_compat"):
        params_from_configs(cfg, reward_compat="maybe")


def test_config_errors():
    from ballbot_gym.envs.config import params_from_configs

    with pytest.raises(ValueError, match="precision"):
        params_from_configs(None, precision="bf16")
    with pytest.raises(ValueError, match="target_direction"):
        params_from_configs({"type": "directional", "config": {}})
    with pytest.raises(ValueError, match="Unknown reward"):
        params_from_configs({"type": "nope", "config": {}})


def test_terrain_bank_seeds_and_size_z():
    from ballbot_gym.envs.config import np_random, terrain_bank

    hf, seeds, sz = terrain_bank({"type": "flat", "config": {}}, None, 0, n=33)
    assert len(hf) == 1 and sz == 2.0 and hf[0].dtype == np.float32 and not hf[0].any()
    hf, seeds, sz = terrain_bank({"type": "hills", "config": {}}, 4, 10, n=33)
    assert seeds == [7765, 9560, 2640, 2076]  # gymnasium np_random(10).integers(0, 10000)
    from ballbot_gym.terrain import generate_hills_terrain

    np.testing.assert_array_equal(hf[2], generate_hills_terrain(33, seed=2640).astype(np.float32))
    _, _, sz = terrain_bank({"type": "ramp", "config": {"ramp_angle": 10.0}}, 1, 0, n=33)
    assert sz == pytest.approx(10 * np.tan(np.radians(10.0)))
    _, _, sz = terrain_bank({"type": "gradient", "config": {}}, 1, 0, n=33)
    assert sz == pytest.approx(10 * np.tan(np.radians(20.0)))
    hf, seeds, _ = terrain_bank({"type": "hills", "config": {"seed": 3}}, 8, 0, n=33)
    assert len(hf) == 1 and seeds == [3]
    assert np_random(1).integers(0, 10000) == np_random(1).integers(0, 10000)


def test_obs_layout_is_sorted_keys():
    from ballbot_gym.envs import OBS_KEYS, split_obs

    assert list(OBS_KEYS) == sorted(OBS_KEYS)
    d = split_obs(np.arange(15.0))
    assert list(d) == list(OBS_KEYS)
    np.testing.assert_array_equal(d["orientation"], [9, 10, 11])


def test_fast_sin_restated():
    """noise/_noise.h fast_sin: sin(pi u) to ~1e-3, exact at the quarter points, periodic."""
    from ballbot_gym.terrain.perlin import fast_sin

    u = np.linspace(-2, 2, 4001, dtype=np.float32)
    err = np.abs(fast_sin(u) - np.sin(np.pi * u.astype(np.float64)))
    assert err.max() < 1.2e-3
    assert fast_sin(np.float32(0.5)) == 1.0 and fast_sin(np.float32(0.0)) == 0.0
    assert np.array_equal(fast_sin(u[:1000] + np.float32(2.0)), fast_sin(u[:1000]))


def test_gpu_perlin_plan():
    from ballbot_gym.envs.config import gpu_perlin_plan, stream_draws

    assert gpu_perlin_plan({"type": "hills", "config": {}}, None, 0) is None
    assert gpu_perlin_plan({"type": "perlin", "config": {"seed": 5}}, None, 0) is None  # fixed seed: host path
    plan, pc = gpu_perlin_plan({"type": "perlin", "config": {"seed": None}}, None, 0)
    assert plan.full and plan.seeds == list(range(10000)) and plan.size_z == 2.0 and plan.seed_slot is None
    assert plan.stream_seeds == [0]  # SB3 seeding: env i on np_random(seed + i)
    assert (pc.scale, pc.octaves, pc.lacunarity, pc.amplitude) == (25.0, 4, 2.0, 1.0)
    assert abs(pc.persistence - 0.2) < 1e-7
    plan, pc = gpu_perlin_plan({"type": "perlin", "config": {"octaves": 5}}, 4, 10, shared=True)
    assert plan.seeds == [7765, 9560, 2640, 2076] and pc.octaves == 5 and plan.stream_seeds == [10]
    assert [plan.slot_of(s) for s in (7765, 9560, 2640, 2076, 1)] == [0, 1, 2, 3, -1]
    plan, _ = gpu_perlin_plan({"type": "perlin", "config": {}}, 2, 10, num_envs=3)
    assert plan.stream_seeds == [10, 11, 12]
    assert plan.seeds == list(dict.fromkeys(int(v) for s in (10, 11, 12) for v in stream_draws(s, 2)))
    with pytest.raises(ValueError, match="unknown config keys"):
        gpu_perlin_plan({"type": "perlin", "config": {"octave": 3}}, 4, 0)
    with pytest.raises(ValueError):
        gpu_perlin_plan({"type": "perlin", "config": {}}, 0, 0)


def test_stream_draws_match_per_reset_scalar_calls():
    """The reference draws ONE value per reset, _np_random.integers(0, 10000)
    (ballbot_env.py:505-510); the plan draws a vector at once.  PCG64 buffers
    its 32-bit outputs in the bit generator, so both give the same stream."""
    from ballbot_gym.envs.config import np_random, stream_draws

    for seed in (0, 10, 12345):
        g = np_random(seed)
        scalar = [int(g.integers(0, 10000)) for _ in range(3000)]
        assert stream_draws(seed, 3000).tolist() == scalar
    assert stream_draws(10, 4).tolist() == [7765, 9560, 2640, 2076]  # tests/golden/seeds.json


def test_pcg64_restatement_matches_numpy():
    """The device generator (bb_kernels.hip pcg64_next64 / next32 / terrain_seed),
    restated on the host by pcg64_terrain_draws: numpy's PCG64 step + XSL-RR
    output, the bit generator's 32-bit buffer and Generator.integers' Lemire
    rejection.  Pinned against numpy itself: the values AND the generator state
    after them, from fresh seeds and from a state that holds a buffered half
    (an odd number of draws, and a permutation in between as the non-eval
    reference env's first reset does, ballbot_env.py:655-661)."""
    import string

    from ballbot_gym.envs.config import np_random, pcg64_terrain_draws, pcg64_words

    for seed in (0, 10, 2 ** 40 + 3, 987654321):
        g = np_random(seed)
        w = pcg64_words(seed)
        assert np.array_equal(w, pcg64_words(g))
        vals, w2 = pcg64_terrain_draws(w, 2001)
        assert vals == [int(g.integers(0, 10000)) for _ in range(2001)]
        assert np.array_equal(w2, pcg64_words(g)), seed  # buffered half included
        g.permutation(list(string.ascii_letters + string.digits))
        more, _ = pcg64_terrain_draws(pcg64_words(g), 50)
        assert more == [int(g.integers(0, 10000)) for _ in range(50)]


def test_pcg64_rejection_branch():
    """Lemire's rejection (a 32-bit draw u with (u * 10000) mod 2^32 < (2^32 - 10000) %
    10000 = 7296 is redrawn) hits ~2e-6 of the draws.  Force it: pick the LCG state
    after the next step so that its XSL-RR output has a low half of 0 (and, in a
    second case, a buffered half of 0), step it back through the inverse
    multiplier, and compare the restatement with numpy from that state."""
    from ballbot_gym.envs.config import _PCG_MULT, pcg64_terrain_draws, pcg64_words

    m128 = (1 << 128) - 1
    minv = pow(_PCG_MULT, -1, 1 << 128)
    rng = np.random.default_rng(5)
    for case in range(6):
        inc = (int(rng.integers(0, 2 ** 63)) << 65) | (int(rng.integers(0, 2 ** 63)) << 1) | 1
        hi = int(rng.integers(0, 2 ** 63)) << 1 | 1
        x = int(rng.integers(1, 2 ** 31)) << 32  # output: low half 0 (rejected), high half accepted
        rot = hi >> 58
        lo = hi ^ (((x << rot) | (x >> ((64 - rot) & 63))) & ((1 << 64) - 1))
        nxt = (hi << 64) | lo
        st = ((nxt - inc) * minv) & m128
        bg = np.random.PCG64()
        bg.state = {"bit_generator": "PCG64", "state": {"state": st, "inc": inc},
                    "has_uint32": case % 2, "uinteger": 0}  # odd cases: a buffered 0 is rejected first
        w = pcg64_words(bg)
        g = np.random.Generator(bg)
        vals, w2 = pcg64_terrain_draws(w, 6)
        assert vals == [int(g.integers(0, 10000)) for _ in range(6)], case
        assert np.array_equal(w2, pcg64_words(g)), case


def test_terrain_plan_generators_and_banks():
    """Which generator each env draws from, and which terrains the bank holds.
    SB3 seeding (default): env i on np_random(seed + i); shared=True: every env on
    np_random(seed); stream_seeds: explicit (the eval VecEnv's seed + N_ENVS + i,
    train.py:90-97)."""
    from ballbot_gym.envs.config import FULL_HOST_BANK, stream_draws, terrain_plan

    plan = terrain_plan({"type": "hills", "config": {}}, 32, 10, num_envs=4096, shared=True)
    d = stream_draws(10, 32)
    assert plan.stream_seeds == [10] * 4096 and not plan.full
    assert plan.seeds == list(dict.fromkeys(d.tolist()))  # distinct seeds, in order of first draw
    assert all(plan.seeds[plan.slot_of(v)] == v for v in d)
    assert (plan.seed_slot >= 0).sum() == len(plan.seeds)
    seeds = [100 + i % 3 for i in range(7)]
    plan = terrain_plan({"type": "stepped", "config": {}}, 5, 0, num_envs=7, stream_seeds=seeds)
    assert plan.stream_seeds == seeds
    assert set(plan.seeds) == {int(v) for s in (100, 101, 102) for v in stream_draws(s, 5)}
    words = plan.rng_words()
    assert words.shape == (7, 5) and np.array_equal(words[0], words[3]) and not np.array_equal(words[0], words[1])
    per_env = terrain_plan({"type": "hills", "config": {}}, 4, 7, num_envs=5)
    assert per_env.stream_seeds == [7, 8, 9, 10, 11]
    assert per_env.covers([int(v) for s in per_env.stream_seeds for v in stream_draws(s, 4)])
    # many generators name most of the seed space: the bank becomes all of it (slot == seed)
    big = terrain_plan({"type": "hills", "config": {}}, None, 0, num_envs=4096)
    assert big.full and big.seed_slot is None and len(big.seeds) == 10000 and FULL_HOST_BANK < 10000
    # seedless generators (their seed argument is unused): one slot serves every draw
    ramp = terrain_plan({"type": "ramp", "config": {}}, None, 0, num_envs=64)
    assert len(ramp.seeds) == 1 and ramp.seedless and (ramp.seed_slot == 0).all() and ramp.covers([1, 9999])
    grad = terrain_plan({"type": "gradient", "config": {"gradient_type": "perlin"}}, 3, 0, num_envs=2)
    assert not grad.seedless and len(grad.seeds) > 1
    explicit = terrain_plan({"type": "hills", "config": {}}, None, 0, 1, draws=[5, 9, 5])
    assert explicit.seeds == [5, 9] and explicit.streams.tolist() == [[0, 1, 0]] and explicit.stream_seeds is None
    assert terrain_plan({"type": "flat", "config": {}}, None, 0, 8).stream_seeds is None
    assert terrain_plan({"type": "hills", "config": {"seed": 4}}, 8, 0, 8).seeds == [4]
    with pytest.raises(ValueError, match="one seed per env"):
        terrain_plan({"type": "hills", "config": {}}, 4, 0, num_envs=3, stream_seeds=[1, 2])


class _RefLikeEnv:
    """The reference env's RNG lines restated (not the reference's code): gymnasium's
    Env.reset(seed) replaces _np_random when seed is not None, BBotSimulation.reset
    then draws r_seed = _np_random.integers(0, 10000) (ballbot_env.py:378-384,
    596-599, 505-510).  eval_env=[True, seed] fixes the generator at construction."""

    def __init__(self, seed):
        from ballbot_gym.envs.config import np_random

        self._np_random = np_random(seed)
        self.draws = []

    def reset(self, seed=None):
        from ballbot_gym.envs.config import np_random

        if seed is not None:
            self._np_random = np_random(seed)
        self.draws.append(int(self._np_random.integers(0, 10000)))


class _SB3LikeVecEnv:
    """SB3 2.x VecEnv seeding restated: seed(s) stores s + i per env; reset() passes
    them to env i's reset once, then forgets them; auto-resets in step_wait pass none."""

    def __init__(self, envs):
        self.envs, self._seeds = envs, [None] * len(envs)

    def seed(self, seed):
        self._seeds = [seed + i for i in range(len(self.envs))]
        return self._seeds

    def reset(self):
        for e, s in zip(self.envs, self._seeds):
            e.reset(seed=s)
        self._seeds = [None] * len(self.envs)

    def auto_reset(self, i):
        self.envs[i].reset()


def test_sb3_seeding_flow_gives_env_i_np_random_seed_plus_i():
    """train.py:82-89 builds N training envs with eval_env=[True, seed]; PPO(seed=seed)
    calls set_random_seed(seed) -> VecEnv.seed(seed) (train.py:126-141), and learn()
    starts with VecEnv.reset() (train.py:284): env i's terrains are the draws of
    np_random(seed + i).  The batched env's default plan names exactly those
    generators (sb3_stream_seeds), and a second VecEnv.seed(s2) + reset() moves
    env i to np_random(s2 + i) (BallbotVecEnv.seed)."""
    from ballbot_gym.envs.config import sb3_stream_seeds, stream_draws, terrain_plan

    seed, n = 10, 6
    vec = _SB3LikeVecEnv([_RefLikeEnv(seed) for _ in range(n)])
    vec.seed(seed)
    vec.reset()
    for _ in range(4):
        for i in range(n):
            vec.auto_reset(i)
    plan = terrain_plan({"type": "hills", "config": {}}, 5, seed, num_envs=n)
    assert plan.stream_seeds == sb3_stream_seeds(seed, n)
    for i, e in enumerate(vec.envs):
        assert e.draws == stream_draws(seed + i, 5).tolist()
        assert e.draws == stream_draws(plan.stream_seeds[i], 5).tolist()
    vec.seed(77)
    vec.reset()
    vec.auto_reset(2)
    for i, e in enumerate(vec.envs):
        assert e.draws[5:] == stream_draws(77 + i, 2 if i == 2 else 1).tolist()
    # a rank's block of global env ids (distributed.shard_stream_seeds)
    from ballbot_gym.distributed import shard_stream_seeds

    assert shard_stream_seeds(10, 4096, 3) == [4106, 4107, 4108]
    assert shard_stream_seeds(10, 4096, 3, per_env=False) is None


def test_spaces_and_registration():
    """Gym surface (B1): "ballbot-v0.1" registered (reference __init__.py:47-53),
    action_space Box(-1, 1, (3,)), observation_space with the reference's keys
    (envs/observation_spaces.py:9-100), sorted as gymnasium's Dict keeps them."""
    import ballbot_gym
    from ballbot_gym import spaces

    assert "ballbot-v0.1" in ballbot_gym.registry.env_specs
    assert ballbot_gym.registry.env_specs["ballbot-v0.1"].entry_point == "ballbot_gym.envs.ballbot_env:BBotSimulation"
    a = spaces.action_space()
    assert a.shape == (3,) and a.dtype == np.float32
    a.seed(0)
    for _ in range(100):
        x = a.sample()
        assert x.dtype == np.float32 and a.contains(x)
    assert not a.contains(np.array([0, 0, 1.5], np.float32))
    o = spaces.observation_space({"h": 64, "w": 64}, 1, disable_cameras=True)
    assert list(o.keys()) == ["actions", "angular_vel", "motor_state", "orientation", "vel"]
    o = spaces.observation_space({"h": 64, "w": 64}, 1, disable_cameras=False)
    assert o["rgbd_0"].shape == (1, 64, 64) and o["relative_image_timestamp"].shape == (1,)
    assert o.contains(o.sample())
    with pytest.raises(ValueError, match="No registered env"):
        ballbot_gym.make("ballbot-v9")
