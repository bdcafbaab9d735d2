"""BASELINE configs[2] at full size: 4096 envs on relief terrain through route 0.

Route 0 (bb_step on a relief bank) = predict kernel, split kernel, the full
step kernel over the predicted list on a side stream, the fast kernel over the
rest, then the full kernel over the fast kernel's hand-overs.  At 4096 envs
the list launches use the XCD-aware permutation over up to 1024 workgroups
and toppled robots reach the per-env HBM spill block (> 32 base-tree contacts).
Checks (size-independent, every env-step of 300 steps of random actions):
the reward is the reference's float32 chain of the returned obs/action, failure
<=> tilt > 20 deg, clips hold, quaternions stay unit, nothing diverges; then a
teacher-forced fp64 step of 64 envs -- 8 from each XCD's env range plus
toppled envs the full kernel must take -- against the oracle on each env's own
terrain.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _props(o, a, r, fl):
    from scipy.spatial.transform import Rotation as Rot

    f32 = np.float32
    assert np.array_equal(o[:, 0:3], a)
    assert np.abs(o[:, 3:9]).max() <= 2 and np.abs(o[:, 12:15]).max() <= 2
    failed = (fl & 2) != 0
    vel = o[:, 12:15]
    base = (vel[:, 0] * f32(0.0) + vel[:, 1] * f32(1.0)) * f32(0.01)
    nrm = np.sqrt((a * a).sum(1, dtype=f32), dtype=f32)
    exp = base + f32(-0.0001) * (nrm * nrm)
    exp = np.where(failed, exp, exp + f32(0.02)).astype(f32)
    assert np.allclose(r, exp, rtol=0, atol=2e-8), np.abs(r - exp).max()
    tilt = np.degrees(np.arccos(np.clip(Rot.from_rotvec(o[:, 9:12].astype(np.float64)).as_matrix()[:, 2, 2], -1, 1)))
    edge = np.abs(tilt - 20.0) < 1e-4
    assert np.array_equal(failed[~edge], tilt[~edge] > 20.0)


@pytest.mark.parametrize("terrain,n_terrains", [("perlin", None), ("hills", 32)], ids=["perlin_full_bank", "hills32"])
def test_config3_full_size_route0(oracle, terrain, n_terrains, monkeypatch):
    from ballbot_gym.envs import BallbotVecEnv

    monkeypatch.setenv("BB_ROUTE", "0")
    n = 4096
    env = BallbotVecEnv(n, device="cuda:0", seed=21, terrain_config={"type": terrain, "config": {}},
                        n_terrains=n_terrains)
    assert env.launch_config()["envs_per_wave"] == 4
    g = torch.Generator(device="cuda:0").manual_seed(9)
    for t in range(300):
        a = torch.rand(n, 3, generator=g, device="cuda:0") * 2.4 - 1.2
        obs, rew, term, trunc, info = env.step(a)
        if t % 3 == 0 or t >= 290:
            _props(info["terminal_observation"].cpu().numpy(), a.cpu().numpy(), rew.cpu().numpy(),
                   info["done_flags"].cpu().numpy())
    st = env.stats()
    assert st["slow_path"] > 0 and st["diverged"] == 0 and st["resets"] > 0
    if terrain == "perlin":  # toppled robots on perlin relief: contacts past the 32 LDS slots, in HBM
        assert st["spill"] > 0, st
    q, v, w, s = env.get_state()
    assert np.allclose(np.linalg.norm(q[:, 3:7], axis=1), 1, atol=1e-9)
    assert np.allclose(np.linalg.norm(q[:, 13:17], axis=1), 1, atol=1e-9)

    # teacher-forced spot check: 8 envs from each XCD's contiguous env range (512 envs each)
    # and the 16 most tilted envs (base-tree contacts: the full kernel)
    rng = np.random.default_rng(3)
    pick = [int(x) for b in range(8) for x in rng.choice(np.arange(512 * b, 512 * (b + 1)), 8, replace=False)]
    up = 1 - 2 * (q[:, 4] ** 2 + q[:, 5] ** 2)  # R22 of the base quaternion
    pick += [int(e) for e in np.argsort(up) if int(e) not in pick][:16]
    tid, _ = env.env_terrain()
    acts = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    s0 = env.stats()["slow_path"]
    env.set_state(q, v, w, s)
    obs, rew, term, trunc, info = env.step(torch.tensor(acts, device=env.device))
    assert env.stats()["slow_path"] - s0 >= 8
    q1, v1, _, _ = env.get_state()
    o1, r1 = info["terminal_observation"].cpu().numpy(), rew.cpu().numpy()
    cfg = oracle.default_cfg()
    full = 0
    for e in pick:
        hf = env.hfield(int(tid[e]))
        size_z = float(env.terrain_plan.size_z)
        qe, ve, we, se = q[e].copy(), v[e].copy(), w[e].copy(), np.array([s[e]], np.int32)
        fo = oracle.forward(q[e], v[e], np.zeros(3), None, hf, size_z)
        full += fo.nbody > 0
        o, r, f, _, _ = oracle.env_step(cfg, qe, ve, we, se, acts[e], hf, size_z)
        if f & 1:
            continue  # auto-reset on the GPU: the stored state is the next episode's
        assert np.abs(q1[e] - qe).max() < 1e-9, e
        assert np.abs(v1[e] - ve).max() < 1e-6 * max(1.0, np.abs(ve).max()), e
        assert np.abs(o1[e] - o).max() < 1e-6 and abs(r1[e] - r) < 1e-7, e
    assert full >= 4  # base-tree contacts among the picked envs
    env.close()
