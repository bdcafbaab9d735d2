"""bb_rollout: a whole PPO rollout (policy, sample, clip, env step, bookkeeping)
in ONE launch, against its two references.

- The policy step: the rollout kernel's fp32 team GEMVs against
  bb_ppo_mlp_act's MFMA tiles on the same observations and noise (the two sum
  in different orders: fp32 rounding tolerance).
- The env steps and the bookkeeping: replaying the kernel's own clipped actions
  through bb_step (serial route) on a twin env must reproduce every stored
  observation, reward, episode start, finished-episode record and the final
  states bit for bit (the step code is bb_step_multi's).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _ppo(env, T, seed=4):
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO, fused_mlp_slots

    m = BatchedPPO(env, n_steps=T, batch_size=256, n_epochs=1, seed=seed, logger=CSVLogger(None, stdout=False))
    with torch.no_grad():  # a non-trivial policy: random weights, log_std away from 0
        for p in m.policy.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    slots = fused_mlp_slots(m, update=False)
    assert slots
    return m, slots


def _env(n, terrain="flat", **kw):
    from ballbot_gym.envs import BallbotVecEnv

    return BallbotVecEnv(n, device="cuda:0", seed=11, terrain_config={"type": terrain, "config": {}}, **kw)


def test_rollout_policy_matches_mlp_act():
    import ctypes as C

    from ballbot_gym import _native as N

    n = 512
    env = _env(n)
    env.step(torch.rand(n, 3, device="cuda:0") * 2 - 1)  # non-trivial observations
    m, slots = _ppo(env, 1)
    obs0 = env.obs.clone()
    m._last_obs = env.obs
    torch.manual_seed(0)
    m.gen.manual_seed(123)
    m._collect_rollout_kernel(slots)
    noise = torch.randn(1, n, 3, generator=torch.Generator(device="cuda:0").manual_seed(123), device="cuda:0")
    act = torch.empty(n, 3, device="cuda:0")
    val = torch.empty(n, device="cuda:0")
    lp = torch.empty(n, device="cuda:0")
    flat = m.optimizer.flat
    offs = (C.c_int32 * 21)(*slots)
    N.check(N.lib().bb_ppo_mlp_act(C.c_void_p(flat.data_ptr()), offs, int(flat.numel()), C.c_void_p(obs0.data_ptr()),
                                   15, C.c_void_p(noise.data_ptr()), n, None, C.c_void_p(act.data_ptr()), None,
                                   C.c_void_p(val.data_ptr()), C.c_void_p(lp.data_ptr()), None), "bb_ppo_mlp_act")
    torch.cuda.synchronize()
    b = m.buf
    assert torch.equal(b.obs[0], obs0)
    assert torch.allclose(b.actions[0], act, rtol=1e-5, atol=1e-5), (b.actions[0] - act).abs().max()
    assert torch.allclose(b.values[0], val, rtol=1e-5, atol=1e-5), (b.values[0] - val).abs().max()
    assert torch.allclose(b.log_probs[0], lp, rtol=1e-5, atol=1e-4), (b.log_probs[0] - lp).abs().max()
    env.close()


@pytest.mark.parametrize("terrain,route,park,pair,n_envs,precision", [
    ("flat", "1", "1", "1", 1024, "fp64"), ("perlin", "1", "1", "1", 256, "fp64"), ("perlin", "1", "0", "1", 256, "fp64"),
    ("perlin", "0", "1", "1", 256, "fp64"), ("perlin", "0", "1", "0", 256, "fp64"), ("perlin", "0", "1", "1", 4096, "fp64"),
    ("perlin", "0", "1", "1", 256, "fp32")])
def test_rollout_steps_replay_bit_exact(terrain, route, park, pair, n_envs, precision, monkeypatch):
    """The kernel's env steps == bb_step on the kernel's own clipped actions.  Route 1 (fast
    path, hand-over): rollout_kernel, hand-overs parked for a finish launch (BB_MULTI_PARK=1)
    or inline (0); route 0 on perlin (predictor): the relief pair with the policy in it
    (relief_pair1_kernel<T, true>, the default), or the relief work queue (BB_RELIEF_PAIR=0);
    the pair also at PPO's size, 4096 envs on per-env generators."""
    monkeypatch.setenv("BB_ROUTE", route)
    monkeypatch.setenv("BB_MULTI_PARK", park)
    monkeypatch.setenv("BB_RELIEF_PAIR", pair)
    n, T = (n_envs, 64) if terrain == "flat" else (n_envs, 96)
    kw = {"max_ep_steps": 30} if terrain == "flat" else {"n_terrains": None, "max_ep_steps": 200,
                                                          "stream_seeds": [70 + i for i in range(n)]}
    kw["precision"] = precision
    a, b = _env(n, terrain, **kw), _env(n, terrain, **kw)
    m, slots = _ppo(a, T)
    m._last_obs = a.obs
    m._last_starts.fill_(1)
    ep_r, ep_l = m._collect_rollout_kernel(slots)
    torch.cuda.synchronize()
    buf = m.buf
    obs = b.obs.clone()
    starts = torch.ones(n, dtype=torch.uint8, device="cuda:0")
    ret = torch.zeros(n, dtype=torch.float64, device="cuda:0")
    ln = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    for t in range(T):
        assert torch.equal(buf.obs[t], obs), t
        assert torch.equal(buf.starts[t], starts), t
        o, r, term, _, info = b.step(buf.actions[t].clamp(-1.0, 1.0))
        assert torch.equal(buf.rewards[t], r), t
        ret += r.double()
        ln += 1
        done = term
        er = torch.where(done, ret, torch.full_like(ret, float("nan")))
        assert torch.equal(torch.isnan(ep_r[t]), torch.isnan(er)), t
        assert torch.equal(ep_r[t][done], er[done]) and torch.equal(ep_l[t], torch.where(done, ln, 0 * ln)), t
        ret.masked_fill_(done, 0.0)
        ln.masked_fill_(done, 0)
        starts = done.to(torch.uint8)
        obs = o.clone()
    assert torch.equal(a.obs, obs) and torch.equal(m._last_starts, starts)
    assert torch.equal(m._ep_ret, ret) and torch.equal(m._ep_len, ln)
    for x, y in zip(a.get_state(), b.get_state()):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(a.env_terrain(), b.env_terrain()):
        np.testing.assert_array_equal(x, y)
    sa, sb = a.stats(), b.stats()
    assert sa == sb, (sa, sb)
    assert sa["resets"] > 0
    if terrain == "perlin":
        assert sa["slow_path"] > 0  # hand-overs to the inline full step happened
    a.close(), b.close()


def test_pair_rollout_budget_expiry_is_loud(monkeypatch):
    """The relief pair's rollout form ends on its wall-clock budget loudly, as bb_step_multi's does
    (test_gpu_multi_step.py): with BB_PAIR_BUDGET_MS=1 most of the 8x surplus teams wait out the
    budget: the rollout itself raises (on relief banks _collect_rollout_kernel checks the fault
    before GAE and the update can read the buffer), check() raises, the next rollout
    refuses, and a full reset() clears the fault."""
    monkeypatch.setenv("BB_PAIR_BUDGET_MS", "1")  # read by bb_create
    monkeypatch.setenv("BB_ROUTE", "0")
    monkeypatch.setenv("BB_RELIEF_PAIR", "1")
    n = 512
    env = _env(n, "perlin", n_terrains=None, stream_seeds=[90 + i for i in range(n)])
    m, slots = _ppo(env, 32)
    m._last_obs = env.obs
    m._last_starts.fill_(1)
    with pytest.raises(RuntimeError, match="wall-clock budget"):
        m._collect_rollout_kernel(slots)  # the rollout's own check
    with pytest.raises(RuntimeError, match="wall-clock budget"):
        env.check()
    assert env.stats()["pair_budget"] >= 1
    with pytest.raises(RuntimeError, match="wall-clock budget"):
        m._collect_rollout_kernel(slots)
    env.reset()
    env.check()
    env.close()


def test_learn_with_the_rollout_kernel(monkeypatch):
    """BatchedPPO.learn rolls out with bb_rollout by default: finite losses, episodes logged."""
    monkeypatch.delenv("BB_FUSED_ROLLOUT", raising=False)
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    env = _env(512, max_ep_steps=40)
    m = BatchedPPO(env, n_steps=32, batch_size=1024, n_epochs=2, seed=3, logger=CSVLogger(None, stdout=False))
    calls = []
    orig = m._collect_rollout_kernel
    m._collect_rollout_kernel = lambda s: calls.append(1) or orig(s)
    m.learn(total_timesteps=512 * 32 * 2)
    assert len(calls) == 2
    v = m.logger.values
    for k in ("train/policy_gradient_loss", "train/value_loss", "train/approx_kl"):
        assert np.isfinite(v[k]), k
    assert len(m.ep_info_buffer) > 0 and m.num_timesteps == 512 * 32 * 2
    env.close()


def test_rollout_rejects_bad_arguments():
    import ctypes as C

    from ballbot_gym import _native as N

    env = _env(64)
    a = N.RolloutArgs()
    assert N.lib().bb_rollout(env._h, C.byref(a), None) < 0 and "NULL argument" in N.last_error()
    env.close()
