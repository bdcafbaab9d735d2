"""SURVEY.md §8 C1's physics invariants, run through the HIP kernel (bb_step /
bb_forward via the C-ABI), with the oracle as the checker.

Physics parity against MuJoCo is unpinned (MuJoCo is absent), so these pin the
kernel to physics rather than to the oracle alone:
- RK4: the kernel's step at opt.timestep h equals the oracle's at the same h,
  and its error against a fine-step reference falls 4x per halving of h -- the
  2nd-order rotation composition MuJoCo's mj_RungeKutta has for tumbling free
  bodies (tests/test_oracle.py::test_rk4_convergence_order; 16x with RKMK);
- angular and linear momentum about the system COM and straight-line COM motion
  with gravity off (BB_DSBL_GRAVITY), airborne (no contacts): both drift at RK4's
  2nd-order rotation error, checked by their 4x fall per halving of dt;
- static load: the ball alone at rest on the plane -- the kernel's forward has
  zero vertical ball acceleration there (its contact forces carry m_ball g) and
  its rest state is the oracle's, where the oracle's summed normal force is m g.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

G = 9.81


def _airborne(oracle, seed):
    """Both trees high in the air and apart (no contact can form), the base tilted
    and tumbling, the wheels spinning."""
    rng = np.random.default_rng(seed)
    q, v, _ = oracle.reset_state(0.01)
    t = np.radians(30)
    q[3:7] = [np.cos(t / 2), *(np.sin(t / 2) * np.array([0.6, 0.8, 0.0]))]
    q[0:3] = [0.0, 0.0, 2.0]
    q[10:13] = [1.5, 1.5, 2.0]
    v[:] = rng.normal(0, 1, 15)
    v[0:3] = [0.1, -0.05, 0.2]    # both trees drift up and apart: no ground, no ball-base contact
    v[9:12] = [0.3, 0.2, 0.25]
    v[3:6] = rng.normal(0, 6, 3)
    v[6:9] = rng.normal(0, 30, 3)
    return q, v


def _gpu_run(q0, v0, n_steps, h=None, disable=0, n=4):
    from ballbot_gym.envs import BallbotVecEnv

    env = BallbotVecEnv(n, device="cuda:0", auto_reset=False, opt_timestep=h, opt_disableflags=disable)
    env.set_state(q0, v0, np.zeros(15), np.zeros(n, np.int32))
    z = torch.zeros(n, 3, device="cuda:0")
    for _ in range(n_steps):
        env.step(z)
    q, v, _, _ = env.get_state()
    st = env.stats()
    env.close()
    assert st["diverged"] == 0 and st["slow_path"] == 0  # airborne: never a base-tree contact
    return q[0], v[0]


def _oracle_run(oracle, q0, v0, n_steps, h, flags):
    oracle.set_flags(flags)
    oracle.set_timestep(h)
    q, v, w = q0.copy(), v0.copy(), np.zeros(15)
    try:
        for _ in range(n_steps):
            oracle.mj_step(q, v, w, np.zeros(3))
    finally:
        oracle.set_flags(0)
        oracle.set_timestep(0.002)
    return q, v


def test_gpu_rk4_matches_oracle_and_converges(oracle):
    q0, v0 = _airborne(oracle, 5)
    T = 0.128
    hs = (0.008, 0.004, 0.002, 0.001)
    qref, _ = _oracle_run(oracle, q0, v0, int(round(T / (hs[-1] / 64))), hs[-1] / 64, oracle.DISABLE_CONTACT)
    errs = []
    for h in hs:
        n = int(round(T / h))
        qg, vg = _gpu_run(q0, v0, n, h=h)
        qo, vo = _oracle_run(oracle, q0, v0, n, h, oracle.DISABLE_CONTACT)
        assert np.abs(qg - qo).max() < 1e-10, (h, np.abs(qg - qo).max())  # same scheme, same step size
        assert np.abs(vg - vo).max() < 1e-8, (h, np.abs(vg - vo).max())
        errs.append(np.abs(qg - qref).max())
    r = np.array(errs[:-1]) / np.array(errs[1:])
    assert np.all((r > 3.8) & (r < 4.2)), r


def test_gpu_angular_momentum_conserved_without_gravity(oracle):
    """Gravity off (BB_DSBL_GRAVITY), airborne: the bodies' angular momentum about the system COM
    is conserved up to RK4's rotation error, which falls 4x per halving of dt (2 s at 2 ms and
    at 1 ms), and the COM moves on a straight line.  The kernel's trajectory is the oracle's."""
    q0, v0 = _airborne(oracle, 6)
    P0, L0, c0 = oracle.momentum(q0, v0)
    mtot = oracle.model_info()["mass"][1:].sum()
    drift, pdrift = [], []
    for h in (0.002, 0.001):
        n = int(round(2.0 / h))
        qg, vg = _gpu_run(q0, v0, n, h=h, disable=64)  # damping on: internal torques
        if h == 0.002:
            qo, vo = _oracle_run(oracle, q0, v0, n, h, oracle.DISABLE_CONTACT | oracle.DISABLE_GRAVITY)
            assert np.abs(qg - qo).max() < 1e-8 and np.abs(vg - vo).max() < 1e-6
        P1, L1, c1 = oracle.momentum(qg, vg)
        drift.append(np.abs(L1 - L0).max() / np.linalg.norm(L0))
        pdrift.append(np.abs(P1 - P0).max() / np.linalg.norm(P0))
        np.testing.assert_allclose(c1, c0 + P0 / mtot * 2.0, atol=1e-4)
    assert drift[0] < 5e-4 and 3.5 < drift[0] / drift[1] < 4.5, drift
    # linear momentum: P is a nonlinear function of the orientations (COM offsets), so RK4 in
    # MuJoCo's coordinates conserves it only up to the same 2nd-order rotation composition:
    # the oracle gives 4.46e-4, 1.11e-4, 2.79e-5, 6.97e-6 at 4, 2, 1, 0.5 ms (4.00x per halving)
    assert pdrift[0] < 2e-4 and 3.5 < pdrift[0] / pdrift[1] < 4.5, pdrift
    # the switch acts on the kernel: with gravity on, the ball falls g t^2 / 2 further in 0.2 s
    qa, _ = _gpu_run(q0, v0, 100)
    qb, _ = _gpu_run(q0, v0, 100, disable=64)
    assert abs((qb[12] - qa[12]) - G * 0.2 ** 2 / 2) < 1e-9


def test_gpu_static_ball_load(oracle):
    hf = oracle.flat_hfield()
    q, v, w = oracle.reset_state(0.01)
    q[0:3] = [2.0, 0.0, 0.3]  # the base tree falls and lies on the ground 2 m away
    q[10:13] = [0.0, 0.0, 0.14 + 0.09 + 0.001]
    for _ in range(2000):
        oracle.mj_step(q, v, w, np.zeros(3), hf)
    # the kernel continues from the oracle's rest state
    from ballbot_gym.envs import BallbotVecEnv

    n = 8
    env = BallbotVecEnv(n, device="cuda:0", auto_reset=False)
    env.set_state(q, v, w, np.zeros(n, np.int32))
    z = torch.zeros(n, 3, device="cuda:0")
    qo, vo, wo = q.copy(), v.copy(), w.copy()
    for _ in range(200):
        env.step(z)
        oracle.mj_step(qo, vo, wo, np.zeros(3), hf)
    qg, vg, wg, _ = env.get_state()
    assert np.abs(qg[0] - qo).max() < 1e-9 and np.abs(vg[0] - vo).max() < 1e-6
    assert np.abs(vg[0]).max() < 0.01  # at rest
    # the kernel's forward at its rest state: the ball's vertical acceleration is ~0, so its
    # ground contacts carry the ball's weight (qacc_z = (F_n - m g) / m); the oracle's forces
    # at the kernel's state sum to m g
    qacc, ncon = env.forward(np.zeros(3))
    assert ncon[0, 0] >= 1 and abs(qacc[0, 11]) < 0.01 * G, qacc[0, 9:12]
    fo = oracle.forward(qg[0], vg[0], np.zeros(3), wg[0], hf)
    mball = oracle.model_info()["mass"][7]
    fb = sum(fo.con_force[3 * k] for k in range(fo.ncon) if fo.con_body1[k] == 0 and fo.con_body2[k] == 7)
    assert abs(fb - mball * G) <= 0.01 * mball * G
    env.close()


def test_opt_overrides_are_validated():
    """bb_create rejects an out-of-range timestep and disable bits it does not implement."""
    from ballbot_gym.envs import BallbotVecEnv

    with pytest.raises(RuntimeError, match="opt_timestep"):
        BallbotVecEnv(4, device="cuda:0", opt_timestep=0.5)
    with pytest.raises(RuntimeError, match="opt_disableflags"):
        BallbotVecEnv(4, device="cuda:0", opt_disableflags=16)  # mjDSBL_CONTACT: not supported
