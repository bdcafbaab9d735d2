"""B1 / B2 on the GPU: the single-env Gym surface and custom reward plugins.

The first group restates the reference's own env tests
(/root/reference/tests/unit/test_env.py:8-90) against `ballbot_gym.make`
(gymnasium is not installed: ballbot_gym.registration keeps the
"ballbot-v0.1" registry).  The reference's reward asserts
isinstance(reward, float); the env returns the float32 value as a Python float.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _make(**kw):
    import ballbot_gym

    return ballbot_gym.make("ballbot-v0.1", GUI=False, **kw)


# --- reference tests/unit/test_env.py, restated -----------------------------
def test_environment_registration():
    import ballbot_gym

    assert "ballbot-v0.1" in ballbot_gym.registry.env_specs


def test_environment_creation():
    env = _make(terrain_type="flat")
    assert env is not None
    env.close()


def test_reset():
    env = _make(terrain_type="flat")
    obs, info = env.reset()
    assert obs is not None and isinstance(obs, dict)
    env.close()


def test_step():
    env = _make(terrain_type="flat")
    env.reset()
    obs, reward, terminated, truncated, info = env.step(env.action_space.sample())
    assert obs is not None and isinstance(reward, (int, float))
    env.close()


def test_observation_and_action_space():
    env = _make(terrain_type="flat")
    assert env.observation_space is not None
    assert env.action_space is not None and env.action_space.shape == (3,)
    env.close()


@pytest.mark.parametrize("kw", [{"terrain_type": "flat", "reward_config": {"type": "directional",
                                                                           "config": {"target_direction": [0.0, 1.0]}}},
                                {"terrain_config": {"type": "flat", "config": {}}}], ids=["reward_config",
                                                                                         "terrain_config"])
def test_environment_with_configs(kw):
    env = _make(**kw)
    env.reset()
    obs, reward, terminated, truncated, info = env.step(env.action_space.sample())
    assert isinstance(reward, float)
    env.close()


# --- values ------------------------------------------------------------------
def test_single_env_matches_oracle(oracle):
    """reset -> (obs, info) and a few steps of the single env vs the oracle from the
    reset state (flat, proprio keys, cameras off)."""
    env = _make(terrain_type="flat", disable_cameras=True)
    obs, info = env.reset(seed=0)
    assert set(obs) == {"orientation", "angular_vel", "vel", "motor_state", "actions"}
    assert all(v.dtype == np.float32 and v.shape == (3,) for v in obs.values())
    assert info == {"success": False, "failure": False, "step_counter": 0, "pos2d": info["pos2d"]}
    q, v, w = oracle.reset_state(0.01)
    sc = np.zeros(1, np.int32)
    cfg = oracle.default_cfg()
    rng = np.random.default_rng(0)
    for t in range(20):
        a = rng.uniform(-1, 1, 3).astype(np.float32)
        obs, r, term, trunc, info = env.step(a)
        o, ro, fl, p2, _ = oracle.env_step(cfg, q, v, w, sc, a, oracle.flat_hfield())
        keys = ("actions", "angular_vel", "motor_state", "orientation", "vel")
        got = np.concatenate([obs[k] for k in keys])
        assert np.abs(got - o).max() < 1e-6, t
        assert abs(r - ro) < 1e-7 and term == bool(fl & 1) and trunc is False
        assert info["step_counter"] == t + 1 and info["failure"] == bool(fl & 2)
        assert np.abs(info["pos2d"] - p2).max() < 1e-6
        if term:
            break
    env.close()


def test_cameras_in_observation():
    env = _make(terrain_type="flat")  # the reference's default: cameras on, depth only
    obs, _ = env.reset()
    assert obs["rgbd_0"].shape == (1, 64, 64) and obs["rgbd_1"].shape == (1, 64, 64)
    assert obs["relative_image_timestamp"].shape == (1,)
    assert env.observation_space.contains({k: np.clip(v, env.observation_space[k].low, env.observation_space[k].high)
                                           for k, v in obs.items()})
    for _ in range(7):
        obs, *_ = env.step(np.zeros(3, np.float32))
    assert 0.0 < float(obs["rgbd_0"].min()) <= 1.0
    env.close()


# --- B2: custom reward plugins -------------------------------------------------
class VelocityMagnitudeReward:
    """examples/02_custom_reward.py:19-45 (scale * |vel[:2]|), per-env ABI."""

    def __init__(self, scale: float = 0.1):
        self.scale = scale

    def __call__(self, state):
        return self.scale * np.linalg.norm(state["vel"][:2])


class BatchedVelocityMagnitudeReward(VelocityMagnitudeReward):
    def batched(self, state):
        return self.scale * torch.linalg.vector_norm(state["vel"][:, :2], dim=1)


def _register():
    from ballbot_gym import ComponentRegistry
    from ballbot_gym.rewards import BaseReward

    names = ComponentRegistry.list_rewards()
    if "velocity_magnitude_test" not in names:
        ComponentRegistry.register_reward("velocity_magnitude_test",
                                          type("VM", (VelocityMagnitudeReward, BaseReward), {}))
    if "velocity_magnitude_batched_test" not in names:
        ComponentRegistry.register_reward("velocity_magnitude_batched_test",
                                          type("VMB", (BatchedVelocityMagnitudeReward, BaseReward), {}))


def test_custom_reward_batched_and_per_env():
    """The reference's reward chain (ballbot_env.py:929-937, 1019-1020) in float32:
    plugin(obs) * scale + action penalty, then + survival bonus unless failed.
    The reward config's "scale" is also the env's reward_scale (ballbot_env.py:228-229),
    so the plugin's 0.1 * |vel| is scaled by 0.1 again.  The per-env host path matches
    numpy's float32 chain (atol 2e-8: the action-norm rounding, as in the parity tests);
    the batched device path (plugin.batched on torch tensors, no host sync) agrees within 1e-8."""
    from ballbot_gym.envs import BallbotVecEnv

    _register()
    n = 512
    envs = {k: BallbotVecEnv(n, device="cuda:0", seed=5, reward_config={"type": k, "config": {"scale": 0.1}})
            for k in ("velocity_magnitude_test", "velocity_magnitude_batched_test")}
    g = torch.Generator(device="cuda:0").manual_seed(1)
    f32 = np.float32
    for t in range(60):
        a = torch.rand(n, 3, generator=g, device="cuda:0") * 2 - 1
        out = {k: e.step(a) for k, e in envs.items()}
        o, r, term, trunc, info = out["velocity_magnitude_test"]
        tob = info["terminal_observation"].cpu().numpy()
        fail = info["failure"].cpu().numpy()
        ah = a.cpu().numpy()
        p = np.array([f32(0.1 * np.linalg.norm(tob[i, 12:14])) for i in range(n)], f32)
        nrm = np.sqrt((ah * ah).sum(1, dtype=f32), dtype=f32)
        exp = p * f32(0.1) + f32(-0.0001) * (nrm * nrm)
        exp = np.where(fail, exp, exp + f32(0.02)).astype(f32)
        np.testing.assert_allclose(r.cpu().numpy(), exp, rtol=0, atol=2e-8)
        rb = out["velocity_magnitude_batched_test"][1]
        assert torch.allclose(rb, r, rtol=0, atol=1e-8)
    for e in envs.values():
        e.close()


# --- A12: DistanceReward through the env -----------------------------------------
def test_distance_reward_raises_like_the_reference_and_fused_on_request():
    """reward_compat="reference" (default): construction and reset work, the first
    step raises the reference's ValueError (its obs dict lacks pos2d,
    ballbot_env.py:929, rewards/distance.py:43-44) -- batched env and gym.make alike.
    reward_compat="fused": the kernel's reward is the reference chain on the step's
    pos2d: (-scale * |goal - pos2d|) * scale + action penalty (+ survival bonus)."""
    from ballbot_gym.envs import BallbotVecEnv

    cfg = {"type": "distance", "config": {"goal_position": [1.0, -2.0], "scale": 0.5}}
    n = 128
    env = BallbotVecEnv(n, device="cuda:0", reward_config=cfg)
    env.reset()
    with pytest.raises(ValueError, match="pos2d"):
        env.step(torch.zeros(n, 3, device="cuda:0"))
    with pytest.raises(ValueError, match="pos2d"):
        env.step_multi(torch.zeros(2, n, 3, device="cuda:0"))
    env.close()
    single = _make(terrain_type="flat", reward_config=cfg, disable_cameras=True)
    single.reset()
    with pytest.raises(ValueError, match="pos2d"):
        single.step(np.zeros(3, np.float32))
    single.close()
    env = BallbotVecEnv(n, device="cuda:0", reward_config=cfg, reward_compat="fused")
    g = torch.Generator(device="cuda:0").manual_seed(3)
    f32 = np.float32
    for _ in range(30):
        a = torch.rand(n, 3, generator=g, device="cuda:0") * 2 - 1
        _, r, _, _, info = env.step(a)
        p2 = info["pos2d"].cpu().numpy()
        ah = a.cpu().numpy()
        dist = np.sqrt(((np.array([1.0, -2.0], f32) - p2) ** 2).sum(1, dtype=f32), dtype=f32)
        nrm = np.sqrt((ah * ah).sum(1, dtype=f32), dtype=f32)
        exp = (-f32(0.5) * dist) * f32(0.5) + f32(-0.0001) * (nrm * nrm)
        exp = np.where(info["failure"].cpu().numpy(), exp, exp + f32(0.02)).astype(f32)
        np.testing.assert_allclose(r.cpu().numpy(), exp, rtol=0, atol=2e-7)
    env.close()
