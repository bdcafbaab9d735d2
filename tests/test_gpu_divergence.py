"""A16: divergence handling on the GPU vs the oracle's restatement of MuJoCo.

mj_step checks qpos and qvel before its first forward (mj_checkPos/Vel: NaN or
|x| > 1e10) and qacc after it (mj_checkAcc); a bad value resets the data to
qpos0 -- without the env's reset height offset -- with zero velocity, warm
start and ctrl, and the step integrates from there.  The episode goes on: the
step counter continues and nothing terminates (mj_step leaves time = 0.002,
so ballbot_env.py:897-899's time == 0 check never fires).  A NaN control is
zeroed (mjWARN_BADCTRL).  States are injected through bb_set_state; the GPU
step is compared with the oracle env-step on the same inputs.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CASES = ("ok", "nan_qpos", "big_qpos", "nan_qvel", "big_qvel", "bad_qacc", "nan_action")


def _states(oracle, n, seed):
    rng = np.random.default_rng(seed)
    qs, vs, ws, acts, kinds = [], [], [], [], []
    for i in range(n):
        kind = CASES[i % len(CASES)]
        q, v, w = oracle.reset_state(0.01)
        q = q + np.r_[rng.normal(0, 0.01, 3), 0, 0, 0, 0, rng.normal(0, 0.1, 10)]
        v = rng.normal(0, 0.1, 15)
        w = rng.normal(0, 1.0, 15)
        a = rng.uniform(-1, 1, 3).astype(np.float32)
        if kind == "nan_qpos":
            q[rng.integers(0, 17)] = np.nan
        elif kind == "big_qpos":
            q[rng.integers(0, 17)] = 2e10 * rng.choice([-1, 1])
        elif kind == "nan_qvel":
            v[rng.integers(0, 15)] = np.nan
        elif kind == "big_qvel":
            v[rng.integers(0, 15)] = 1.5e10 * rng.choice([-1, 1])
        elif kind == "bad_qacc":  # finite and < 1e10, but the wheel damping gives |qacc| >> 1e10
            v[6 + rng.integers(0, 3)] = 5e9
        elif kind == "nan_action":
            a[rng.integers(0, 3)] = np.nan
        qs.append(q); vs.append(v); ws.append(w); acts.append(a); kinds.append(kind)
    return np.array(qs), np.array(vs), np.array(ws), np.array(acts), kinds


@pytest.mark.parametrize("terrain", ["flat", "hills"])
def test_divergence_reset_matches_oracle(oracle, terrain):
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_gym.terrain import generate_hills_terrain

    n = 70
    tcfg = {"type": "flat", "config": {}} if terrain == "flat" else {"type": "hills", "config": {"seed": 7}}
    hf = oracle.flat_hfield() if terrain == "flat" else generate_hills_terrain(293, seed=7).astype(np.float32)
    env = BallbotVecEnv(n, device="cuda:0", terrain_config=tcfg, auto_reset=True)
    assert np.array_equal(env.hfield(0), hf)
    qs, vs, ws, acts, kinds = _states(oracle, n, seed=1 if terrain == "flat" else 2)
    steps = np.full(n, 57, np.int32)
    env.set_state(qs, vs, ws, steps)
    s0 = env.stats()
    obs, rew, term, trunc, info = env.step(torch.tensor(acts, device=env.device))
    q, v, w, st = env.get_state()
    obs, rew = obs.cpu().numpy(), rew.cpu().numpy()
    fl = info["done_flags"].cpu().numpy()
    cfg = oracle.default_cfg()
    n_div = 0
    for e in range(n):
        qe, ve, we, se = qs[e].copy(), vs[e].copy(), ws[e].copy(), np.array([57], np.int32)
        o, r, f, _, _ = oracle.env_step(cfg, qe, ve, we, se, acts[e], hf)
        assert (fl[e] & 7) == (f & 7), (e, kinds[e], fl[e], f)
        div = kinds[e] not in ("ok", "nan_action")
        assert bool(f & 4) == div, (e, kinds[e])
        n_div += div
        assert np.abs(q[e] - qe).max() < 1e-9, (e, kinds[e])
        assert np.abs(v[e] - ve).max() < 1e-6 * max(1.0, np.abs(ve).max()), (e, kinds[e])
        np.testing.assert_allclose(obs[e], o, rtol=0, atol=1e-6, equal_nan=True, err_msg=f"{e} {kinds[e]}")
        if np.isnan(r):
            assert np.isnan(rew[e]) and kinds[e] == "nan_action"
        else:
            assert abs(rew[e] - r) < 1e-7, (e, kinds[e])
        if div:  # from qpos0 without the height offset, episode not ended
            assert st[e] == 58 and not f & 1
    s1 = env.stats()
    assert s1["diverged"] - s0["diverged"] == n_div
    assert s1["resets"] - s0["resets"] == int(((fl & 1) != 0).sum())  # auto-resets only on termination
    # the next step runs normally from the reset state
    obs2, _, _, _, info2 = env.step(torch.zeros(n, 3, device=env.device))
    assert not (info2["done_flags"].cpu().numpy() & 4).any()
    assert torch.isfinite(obs2).all()
    env.close()


def test_nan_state_in_route_and_cameras():
    """A NaN/huge stored state on relief terrain goes through the predictor (route 0)
    and the depth cameras without forming a heightfield cell index from it (no fault);
    the step then resets it and the images of healthy envs are unaffected."""
    from ballbot_gym.envs import BallbotVecEnv

    n = 128
    env = BallbotVecEnv(n, device="cuda:0", seed=3, terrain_config={"type": "perlin", "config": {}}, n_terrains=4,
                        disable_cameras=False)
    ref = BallbotVecEnv(n, device="cuda:0", seed=3, terrain_config={"type": "perlin", "config": {}}, n_terrains=4,
                        disable_cameras=False)
    q, v, w, s = env.get_state()
    bad = np.arange(0, n, 4)
    q[bad[0::2], 0] = np.nan
    q[bad[1::2], 10] = 3e10
    env.set_state(q, v, w, s)
    d = env.render_depth(force=True).clone()
    ok = np.setdiff1d(np.arange(n), bad)
    dr = ref.render_depth(force=True)
    assert torch.equal(d[ok], dr[ok])
    assert torch.isfinite(d).all() and float(d.max()) <= 1.0
    env.step(torch.zeros(n, 3, device="cuda:0"))
    qa, va, _, _ = env.get_state()
    assert np.isfinite(qa).all() and np.isfinite(va).all()
    assert env.stats()["diverged"] == len(bad)
    env.close()
    ref.close()
