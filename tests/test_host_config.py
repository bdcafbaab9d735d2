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
    from ballbot_gym.envs.config import gpu_perlin_plan

    assert gpu_perlin_plan({"type": "hills", "config": {}}, None, 0) is None
    assert gpu_perlin_plan({"type": "perlin", "config": {"seed": 5}}, None, 0) is None  # fixed seed: host path
    plan, pc = gpu_perlin_plan({"type": "perlin", "config": {"seed": None}}, None, 0)
    assert plan.full and plan.seeds == list(range(10000)) and plan.size_z == 2.0
    assert plan.streams.shape == (1, 65536)  # slot == seed: the draws themselves
    assert (pc.scale, pc.octaves, pc.lacunarity, pc.amplitude) == (25.0, 4, 2.0, 1.0)
    assert abs(pc.persistence - 0.2) < 1e-7
    plan, pc = gpu_perlin_plan({"type": "perlin", "config": {"octaves": 5}}, 4, 10)
    assert plan.seeds == [7765, 9560, 2640, 2076] and pc.octaves == 5
    assert plan.streams.tolist() == [[0, 1, 2, 3]]
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


def test_terrain_plan_shared_and_per_env_streams():
    """train.py:82-89: every training env is built with eval_env=[True, seed]
    -> all envs share one stream (reset k of every env draws value k);
    train.py:90-97: eval env i uses seed + N_ENVS + i -> its own stream."""
    from ballbot_gym.envs.config import stream_draws, terrain_plan

    plan = terrain_plan({"type": "hills", "config": {}}, 32, 10, num_envs=4096)
    d = stream_draws(10, 32)
    assert plan.env_stream is None and plan.streams.shape == (1, 32)
    assert [plan.seeds[s] for s in plan.streams[0]] == d.tolist()
    assert len(plan.seeds) == len(set(d.tolist()))  # distinct seeds only
    assert all(plan.seed_of_draw(0, k) == d[k] for k in range(32))
    seeds = [100 + i % 3 for i in range(7)]
    plan = terrain_plan({"type": "stepped", "config": {}}, 5, 0, num_envs=7, stream_seeds=seeds)
    assert plan.streams.shape == (3, 5) and plan.env_stream.tolist() == [0, 1, 2, 0, 1, 2, 0]
    for i, s in enumerate(seeds):
        assert [plan.seeds[x] for x in plan.streams[plan.env_stream[i]]] == stream_draws(s, 5).tolist()
    full = terrain_plan({"type": "perlin", "config": {}}, None, 3, num_envs=2, stream_seeds=[7, 8], full_bank=True)
    assert full.streams.shape == (2, 1024) and full.streams[1, :5].tolist() == stream_draws(8, 5).tolist()
    explicit = terrain_plan({"type": "hills", "config": {}}, None, 0, 1, draws=[5, 9, 5])
    assert explicit.seeds == [5, 9] and explicit.streams.tolist() == [[0, 1, 0]]
    assert terrain_plan({"type": "flat", "config": {}}, None, 0, 8).streams is None
    assert terrain_plan({"type": "hills", "config": {"seed": 4}}, 8, 0, 8).seeds == [4]
    with pytest.raises(ValueError, match="one seed per env"):
        terrain_plan({"type": "hills", "config": {}}, 4, 0, num_envs=3, stream_seeds=[1, 2])


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
