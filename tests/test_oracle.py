"""The fp64 CPU oracle (oracle/bb_oracle.c): invariants of the restated
mj_step and env glue (physics parity vs MuJoCo is UNPINNED,
so the oracle is validated by physics invariants and by the golden-pinned
pieces of the env glue).  CPU only, seconds."""
import numpy as np
import pytest

G = 9.81


@pytest.fixture(autouse=True)
def _reset_flags(oracle):
    oracle.set_flags(0)
    oracle.set_timestep(0.002)
    yield
    oracle.set_flags(0)
    oracle.set_timestep(0.002)


def test_model_constants(oracle):
    """Masses from ballbot.xml densities (cone meshes absent -> stand-in 0)."""
    mi = oracle.model_info()
    m = mi["mass"]
    np.testing.assert_allclose(m[1], 0.11 ** 2 * np.pi * 0.28 * 23.6 + 0.2 ** 3 * 400, rtol=1e-6)  # tower + ballast
    np.testing.assert_allclose(m[2:4], np.pi * 0.01 ** 2 * (0.2 + 4 / 3 * 0.01) * 1000, rtol=1e-6)  # sticks
    np.testing.assert_allclose(m[4:7], np.pi * 0.025 ** 2 * (0.04 + 4 / 3 * 0.025) * 620, rtol=1e-6)  # wheels
    np.testing.assert_allclose(m[7], 4 / 3 * np.pi * 0.09 ** 3 * 55, rtol=1e-6)  # ball
    np.testing.assert_array_equal(mi["qpos0"][[2, 12]], [0.24, 0.26])


def test_mass_matrix_spd_and_block_structure(oracle):
    rng = np.random.default_rng(0)
    for _ in range(5):
        q, v, _ = oracle.reset_state(0.01)
        rv = rng.normal(0, 0.3, 3)
        th = np.linalg.norm(rv)
        q[3:7] = [np.cos(th / 2), *(np.sin(th / 2) * rv / th)]
        q[7:10] = rng.uniform(-3, 3, 3)
        fo = oracle.forward(q, v, np.zeros(3), None, oracle.flat_hfield())
        M = np.array(fo.M).reshape(15, 15)
        np.testing.assert_allclose(M, M.T, atol=1e-14)
        assert np.linalg.eigvalsh(M).min() > 0
        assert np.abs(M[:9, 9:]).max() == 0  # base tree and ball are separate trees
        np.testing.assert_allclose(np.diag(M)[:3], oracle.model_info()["mass"][1:7].sum(), rtol=1e-12)
        np.testing.assert_allclose(np.diag(M)[9:12], oracle.model_info()["mass"][7], rtol=1e-12)


def test_free_fall_is_exact(oracle):
    """Contacts off: both trees fall with a = -g; RK4 is exact for constant acceleration."""
    oracle.set_flags(oracle.DISABLE_CONTACT)
    q, v, w = oracle.reset_state(0.01)
    z0b, z0B = q[2], q[12]
    for _ in range(200):
        oracle.mj_step(q, v, w, np.zeros(3))
    t = 200 * 0.002
    np.testing.assert_allclose([q[2], q[12]], [z0b - 0.5 * G * t * t, z0B - 0.5 * G * t * t], atol=1e-10)
    np.testing.assert_allclose([v[2], v[11]], [-G * t, -G * t], atol=1e-10)
    np.testing.assert_allclose(v[[0, 1, 3, 4, 5, 9, 10, 12, 13, 14]], 0, atol=1e-10)


def _energy(oracle, q, v):
    fo = oracle.forward(q, v, np.zeros(3), None, None)
    return fo.energy_kin + fo.energy_pot


def test_energy_conserved_without_contact_and_damping(oracle):
    oracle.set_flags(oracle.DISABLE_CONTACT | oracle.DISABLE_DAMPING)
    rng = np.random.default_rng(1)
    q, v, w = oracle.reset_state(0.01)
    v[:] = rng.normal(0, 1.0, 15)
    e0 = _energy(oracle, q, v)
    for _ in range(500):
        oracle.mj_step(q, v, w, np.zeros(3))
    assert abs(_energy(oracle, q, v) - e0) < 1e-6 * max(1.0, abs(e0))


def test_linear_momentum_conserved_without_gravity(oracle):
    oracle.set_flags(oracle.DISABLE_CONTACT | oracle.DISABLE_DAMPING | oracle.DISABLE_GRAVITY)
    rng = np.random.default_rng(2)
    q, v, w = oracle.reset_state(0.01)
    v[:] = rng.normal(0, 1.0, 15)

    def momentum():
        M = np.array(oracle.forward(q, v, np.zeros(3), None, None).M).reshape(15, 15)
        return M[0:3] @ v, M[9:12] @ v

    p0, P0 = momentum()
    for _ in range(300):
        oracle.mj_step(q, v, w, np.zeros(3))
    p1, P1 = momentum()
    np.testing.assert_allclose(p1, p0, atol=1e-9)
    np.testing.assert_allclose(P1, P0, atol=1e-9)


def _tumbling_state(oracle, seed=5):
    """The robot in the air, base tilted 30 deg, tumbling (body rates ~6 rad/s) with the
    wheels spinning (~30 rad/s): torque-free motion whose body-frame angular velocity varies."""
    rng = np.random.default_rng(seed)
    q, v, _ = oracle.reset_state(0.01)
    t = np.radians(30)
    q[3:7] = [np.cos(t / 2), *(np.sin(t / 2) * np.array([0.6, 0.8, 0.0]))]
    v[:] = rng.normal(0, 1, 15)
    v[3:6] = rng.normal(0, 6, 3)
    v[6:9] = rng.normal(0, 30, 3)
    return q, v


def _rk4_errors(oracle, q0, v0, T=0.128, hs=(0.008, 0.004, 0.002, 0.001)):
    def run(h):
        oracle.set_timestep(h)
        q, v, w = q0.copy(), v0.copy(), np.zeros(15)
        for _ in range(int(round(T / h))):
            oracle.mj_step(q, v, w, np.zeros(3))
        return q
    ref = run(hs[-1] / 64)
    return np.array([np.abs(run(h) - ref).max() for h in hs])


def test_rk4_convergence_order(oracle):
    """SURVEY.md §8 C1, RK4 order in dt (contacts and damping off, gravity on).

    With the free joints' rotations composed as Runge-Kutta-Munthe-Kaas (BBO_RKMK,
    test-only) the qpos error after 0.128 s falls 16x per halving of dt: the forward
    dynamics the integrator samples are consistent to 4th order.  MuJoCo's own
    composition -- mj_RungeKutta sums the stages' BODY-frame angular velocities and
    mj_integratePos applies q0 * exp(h * sum) -- drops the commutator of the varying
    body rates and converges at 2nd order in the rotation: 4x per halving [MJ].  The
    oracle, like MuJoCo and the kernel, steps with MuJoCo's composition."""
    q0, v0 = _tumbling_state(oracle)
    oracle.set_flags(oracle.DISABLE_CONTACT | oracle.DISABLE_DAMPING | oracle.RKMK)
    e = _rk4_errors(oracle, q0, v0)
    r = e[:-1] / e[1:]
    assert np.all((r > 15.0) & (r < 17.0)), r
    oracle.set_flags(oracle.DISABLE_CONTACT | oracle.DISABLE_DAMPING)
    e = _rk4_errors(oracle, q0, v0)
    r = e[:-1] / e[1:]
    assert np.all((r > 3.8) & (r < 4.2)), r
    assert e[2] < 1e-5  # at ballbot.xml's 2 ms: a few microns after 64 steps of tumbling


def test_angular_momentum_conserved_without_gravity(oracle):
    """with gravity and contacts off, the bodies' angular momentum about
    the system COM is conserved -- the hinge damping and motor torques are internal, so it
    holds with damping on too -- and the COM moves on a straight line.  RK4's rotation
    error drifts it by < 1e-4 relative over 2 s at 2 ms, 4x less per halving of dt."""
    q0, v0 = _tumbling_state(oracle, seed=6)
    mtot = oracle.model_info()["mass"][1:].sum()
    drift = []
    for h, damping in ((0.002, False), (0.001, False), (0.002, True)):
        oracle.set_flags(oracle.DISABLE_CONTACT | oracle.DISABLE_GRAVITY | (0 if damping else oracle.DISABLE_DAMPING))
        oracle.set_timestep(h)
        q, v, w = q0.copy(), v0.copy(), np.zeros(15)
        P0, L0, c0 = oracle.momentum(q, v)
        n = int(round(2.0 / h))
        for _ in range(n):
            oracle.mj_step(q, v, w, np.array([3.0, -2.0, 1.0]) if damping else np.zeros(3))
        P1, L1, c1 = oracle.momentum(q, v)
        drift.append(np.abs(L1 - L0).max() / np.linalg.norm(L0))
        assert drift[-1] < 1e-4, (h, damping, drift[-1])
        assert np.abs(P1 - P0).max() < 1e-4 * np.linalg.norm(P0)
        np.testing.assert_allclose(c1, c0 + P0 / mtot * n * h, atol=1e-4)
    assert 3.5 < drift[0] / drift[1] < 4.5, drift


def test_static_ball_load_equals_weight(oracle):
    """SURVEY.md §8 C1, static load: the ball alone at rest on flat ground (the base tree
    lies on the ground 2 m away) -- the summed normal forces of its terrain contacts equal
    m_ball g within 1%; so do the base tree's ground contacts with its own weight."""
    hf = oracle.flat_hfield()
    q, v, w = oracle.reset_state(0.01)
    q[0:3] = [2.0, 0.0, 0.3]
    q[10:13] = [0.0, 0.0, 0.14 + 0.09 + 0.001]  # ball centre 1 mm above the plane
    for _ in range(2000):
        oracle.mj_step(q, v, w, np.zeros(3), hf)
    assert np.abs(v).max() < 0.01
    fo = oracle.forward(q, v, np.zeros(3), w, hf)
    m = oracle.model_info()["mass"]
    ball = [k for k in range(fo.ncon) if fo.con_body1[k] == 0 and fo.con_body2[k] == 7]
    base = [k for k in range(fo.ncon) if fo.con_body1[k] == 0 and 1 <= fo.con_body2[k] <= 6]
    assert ball and base and fo.ncon == len(ball) + len(base)  # the ball-wheel pairs are apart
    fb = sum(fo.con_force[3 * k] for k in ball)
    ft = sum(fo.con_force[3 * k] for k in base)
    assert abs(fb - m[7] * G) <= 0.01 * m[7] * G, (fb, m[7] * G)
    assert abs(ft - m[1:7].sum() * G) <= 0.01 * m[1:7].sum() * G, (ft, m[1:7].sum() * G)


def test_patched_contact_frame(oracle):
    """tools/mujoco_fix.patch: the first tangent of each ball-wheel contact is
    the capsule axis orthogonalised against the normal; the frame is orthonormal
    and right-handed (mju_makeFrame)."""
    q, v, _ = oracle.reset_state(0.01)
    fo = oracle.forward(q, v, np.zeros(3), None, oracle.flat_hfield())
    a0 = np.array([-0.1532, -0.6903, -0.7071])
    a0 /= np.linalg.norm(a0)
    for k in range(3):
        F = np.array(fo.con_frame[9 * k:9 * k + 9]).reshape(3, 3)
        np.testing.assert_allclose(F @ F.T, np.eye(3), atol=1e-12)
        np.testing.assert_allclose(np.linalg.det(F), 1.0, atol=1e-12)
        body = fo.con_body2[k]
        ang = np.radians(120 * (body - 4))
        Rz = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1]])
        ax = Rz @ a0  # base upright at reset: base frame == world frame
        n = F[0]
        t = ax - ax.dot(n) * n
        assert abs(abs(F[1].dot(t / np.linalg.norm(t))) - 1) < 1e-3


def test_rotvec_formula(oracle):
    """numpy-quaternion as_rotation_vector: 2 atan2(|v|, w) v/|v|, no w >= 0 flip."""
    rng = np.random.default_rng(3)
    for _ in range(50):
        qq = rng.normal(size=4)
        qq /= np.linalg.norm(qq)
        b = np.linalg.norm(qq[1:])
        np.testing.assert_allclose(oracle.quat_to_rotvec(qq), 2 * np.arctan2(b, qq[0]) * qq[1:] / b, atol=1e-12)
    np.testing.assert_array_equal(oracle.quat_to_rotvec(np.array([1.0, 0, 0, 0])), 0)


def test_reward_chain_matches_reward_plugin(oracle):
    """env glue: reward = 0.01 * DirectionalReward(vel) + (-1e-4)|a|^2 + 0.02 in float32."""
    from ballbot_gym.rewards import DirectionalReward

    cfg = oracle.default_cfg()
    hf = oracle.flat_hfield()
    q, v, w = oracle.reset_state(oracle.init_offset(hf))
    s = np.zeros(1, np.int32)
    rng = np.random.default_rng(4)
    plugin = DirectionalReward(np.array([0.0, 1.0], np.float32))
    for _ in range(60):
        a = rng.uniform(-1, 1, 3).astype(np.float32)
        obs, r, fl, _, _ = oracle.env_step(cfg, q, v, w, s, a, hf)
        vel = obs[12:15]
        exp = np.float32(plugin({"vel": vel})) * np.float32(0.01) + np.float32(-1e-4) * np.float32(
            np.linalg.norm(a) ** 2)
        if not fl & 2:
            exp = exp + np.float32(0.02)
        assert abs(r - float(exp)) <= 2e-7
        np.testing.assert_array_equal(obs[0:3], a)
        assert np.all(np.abs(obs[3:15]) <= 2.0)


def test_init_offset_matches_host_restatement(oracle):
    from ballbot_gym.envs.config import init_offset
    from ballbot_gym.terrain import generate_hills_terrain

    hf = generate_hills_terrain(293, seed=7).astype(np.float32)
    assert abs(oracle.init_offset(hf, 2.0) - init_offset(hf, 2.0)) < 1e-6
    assert oracle.init_offset(oracle.flat_hfield(), 2.0) == pytest.approx(0.01)


def test_pid_balances_on_flat(oracle):
    """scripts/test_pid.py:22-63 behaviour: gains (20, 15, 2) keep the robot up."""
    from pid_ref import PID, rotvec_to_R

    cfg = oracle.default_cfg()
    hf = oracle.flat_hfield()
    q, v, w = oracle.reset_state(oracle.init_offset(hf))
    s = np.zeros(1, np.int32)
    pid = PID(0.002, 20, 15, 2)
    obs = np.zeros(15, np.float32)
    for _ in range(1500):
        a = pid.act(rotvec_to_R(obs[9:12])).astype(np.float32)
        obs, r, fl, _, tilt = oracle.env_step(cfg, q, v, w, s, a, hf)
        assert fl == 0
    assert np.linalg.norm(obs[9:12]) < np.radians(5)
    assert np.abs(v).max() < 1.0


def test_ball_rests_on_plane(oracle):
    """Ball alone settles on the plane: contact depth ~ m g / k-ish, no drift."""
    cfg = oracle.default_cfg()
    hf = oracle.flat_hfield()
    q, v, w = oracle.reset_state(oracle.init_offset(hf))
    for _ in range(400):
        oracle.mj_step(q, v, w, np.zeros(3), hf)
    fo = oracle.forward(q, v, np.zeros(3), w, hf)
    assert fo.nground >= 1
    ball_bottom = q[12] - 0.14 - 0.09
    assert -5e-3 < ball_bottom < 1e-3


def _rotx(deg):
    t = np.radians(deg)
    return np.array([np.cos(t / 2), np.sin(t / 2), 0.0, 0.0])


def test_no_body_contacts_when_upright(oracle):
    hf = oracle.flat_hfield()
    q, v, _ = oracle.reset_state(oracle.init_offset(hf))
    fo = oracle.forward(q, v, np.zeros(3), None, hf)
    assert fo.nbody == 0 and fo.ncon == fo.nground + 3


def test_tower_on_flat_ground_geometry(oracle):
    """Dynamic hfield x tower-cylinder pair: base rolled 90 deg and lowered
    so the tower's side is 1 cm into flat ground; interior prisms report the
    exact depth with normal +z, every contact is terrain(world) -> base tree.
    The tower lies across more prisms than MuJoCo's mjMAXCONPAIR: its pair
    keeps the first 50 and flags the cap (bit 1)."""
    hf = oracle.flat_hfield()
    q, v, _ = oracle.reset_state(0.01)
    q[3:7] = _rotx(90)
    q[2] = 0.10           # tower axis along world y at z = 0.10, radius 0.11 -> 1 cm deep
    q[10:13] = [0, 0.6, 0.5]  # ball out of the way
    fo = oracle.forward(q, v, np.zeros(3), None, hf)
    k0 = fo.ncon - fo.nbody
    ks = range(k0, k0 + fo.nbody)
    assert fo.nbody > 0
    assert all(fo.con_body1[k] == 0 for k in ks)
    tower = [k for k in ks if fo.con_body2[k] == 1]
    assert len(tower) == 50 and fo.ground_overflow & 2
    assert tower == list(range(k0, k0 + 50))  # the tower pair comes first
    up = [k for k in tower if fo.con_frame[9 * k + 2] > 0.999]
    assert up, "no face contact"
    for k in up:
        assert fo.con_dist[k] == pytest.approx(-0.01, abs=1e-9)
        assert -0.34 <= fo.con_pos[3 * k + 1] <= -0.06  # on the tower's footprint


def test_stick_dips_into_ground(oracle):
    """cam stick (capsule r 1 cm) vs flat ground: penetration = r - lowest core z."""
    hf = oracle.flat_hfield()
    q, v, _ = oracle.reset_state(0.01)
    q[10:13] = [0, 0.8, 0.5]
    best = None
    for z in np.linspace(0.20, 0.02, 40):
        q[2] = z
        q[3:7] = _rotx(35)
        fo = oracle.forward(q, v, np.zeros(3), None, hf)
        k0 = fo.ncon - fo.nbody
        sticks = [k for k in range(k0, k0 + fo.nbody) if fo.con_body2[k] in (2, 3)]
        if sticks:
            best = (z, sticks, fo)
            break
    assert best is not None
    z, sticks, fo = best
    for k in sticks:
        assert fo.con_body1[k] == 0
        assert -0.011 < fo.con_dist[k] <= 0  # just touching at the first height that produced a contact


def test_body_contacts_keep_robot_above_ground(oracle):
    """Let the robot fall over on flat ground: the base-tree geoms stop on the
    terrain (no tunnelling) and the simulation stays finite."""
    hf = oracle.flat_hfield()
    q, v, w = oracle.reset_state(oracle.init_offset(hf))
    q[3:7] = _rotx(25)
    for _ in range(1500):
        oracle.mj_step(q, v, w, np.zeros(3), hf)
    assert np.all(np.isfinite(q)) and np.all(np.isfinite(v))
    fo = oracle.forward(q, v, np.zeros(3), w, hf)
    assert fo.nbody > 0                 # lying on its side, touching the ground
    assert q[2] > 0.0 and np.abs(v[:6]).max() < 0.05  # the base came to rest (the ball may roll off)


def _cam_pose(q, cam):
    """Camera origin and camera->world rotation from qpos (ballbot.xml:44-54), numpy."""
    from scipy.spatial.transform import Rotation as Rot

    Rb = Rot.from_quat([q[4], q[5], q[6], q[3]]).as_matrix()
    Rbody = Rot.from_euler("XYZ", [180, -30 if cam == 0 else 30, 0], degrees=True).as_matrix()
    Rcam = Rot.from_euler("XYZ", [180, 0, 0], degrees=True).as_matrix()
    o = q[:3] + Rb @ np.array([0.17 if cam == 0 else -0.17, -0.01, -0.06])
    return o, Rb @ Rbody @ Rcam


@pytest.mark.parametrize("cam", [0, 1])
def test_depth_camera_flat_ground_analytic(oracle, cam):
    """Every pixel sees the analytic ground-plane depth or something nearer (a robot
    geom); most pixels see the ground; far pixels clip to 1 (sensors/rgbd.py:74)."""
    rng = np.random.default_rng(cam)
    for trial in range(4):
        q, _, _ = oracle.reset_state(0.01)
        q = q.copy()
        q[2] += rng.uniform(0, 0.6)
        q[12] += q[2] - 0.25 - 0.01
        ang = rng.uniform(-0.2, 0.2, 3)
        from scipy.spatial.transform import Rotation as Rot

        qq = Rot.from_rotvec(ang).as_quat()
        q[3:7] = [qq[3], qq[0], qq[1], qq[2]]
        d = oracle.render_depth(q, oracle.flat_hfield(), cam)
        o, R = _cam_pose(q, cam)
        H = W = 64
        j, i = np.meshgrid(np.arange(W), np.arange(H))
        xc = 2 * (j + 0.5) / W - 1
        yc = 1 - 2 * (i + 0.5) / H
        dirs = np.stack([xc, yc, -np.ones_like(xc)], -1) @ R.T
        s = -o[2] / dirs[..., 2]
        ground = np.where(s > 0, np.minimum(s, 1.0), 1.0)
        assert (d <= ground + 1e-5).all()
        same = np.abs(d - ground) < 1e-5
        assert same.mean() > 0.3, same.mean()
        assert d.max() <= 1.0 and d.min() > 0


def test_depth_camera_sees_ball_and_culls_inside(oracle):
    """The ball occludes the ground below the robot; a camera inside its own stick
    capsule does not see the capsule (back faces culled)."""
    q, _, _ = oracle.reset_state(0.01)
    d0 = oracle.render_depth(q, oracle.flat_hfield(), 0)
    d0_far = oracle.render_depth(np.r_[q[:10], q[10] + 3.0, q[11:]], oracle.flat_hfield(), 0)  # ball moved away
    assert (d0 <= d0_far + 1e-6).all() and (d0 < d0_far - 1e-3).sum() > 50
    assert d0.min() > 0.005  # the 1 cm stick capsule around the camera origin is not drawn


def test_openmp_batch_equals_serial(oracle):
    """bbo_env_step_batch_mt (the multi-core CPU baseline) == the serial batch, bit for bit."""
    n = 16
    cfg = oracle.default_cfg()
    hf = oracle.flat_hfield()
    off = oracle.init_offset(hf)
    rng = np.random.default_rng(2)
    states = []
    for threads in (1, 4):
        q = np.zeros((n, 17)); v = np.zeros((n, 15)); w = np.zeros((n, 15))
        for e in range(n):
            q[e], v[e], w[e] = oracle.reset_state(off)
        st = np.zeros(n, np.int32)
        rr = np.random.default_rng(2)
        for _ in range(5):
            oracle.env_step_batch(cfg, q, v, w, st, rr.uniform(-1, 1, (n, 3)).astype(np.float32), hf, 2.0, off,
                                  threads=threads)
        states.append((q.copy(), v.copy()))
    assert np.array_equal(states[0][0], states[1][0]) and np.array_equal(states[0][1], states[1][1])


def _step_from(oracle, q, v, w, steps, action):
    q, v, w, sc = q.copy(), v.copy(), w.copy(), np.array([steps], np.int32)
    obs, r, fl, p2, _ = oracle.env_step(oracle.default_cfg(), q, v, w, sc, np.asarray(action, np.float32),
                                        oracle.flat_hfield())
    return q, v, w, int(sc[0]), obs, r, fl


@pytest.mark.parametrize("case", ["nan_qpos", "big_qpos", "nan_qvel", "big_qvel", "bad_qacc"])
def test_divergence_reset_is_mujocos(oracle, case):
    """A16: mj_step's mj_checkPos / mj_checkVel (NaN or |x| > 1e10) and
    mj_checkAcc (after the first forward) reset the data -- qpos0 WITHOUT the
    env's height offset, zero velocity, warm start and ctrl -- and the step
    integrates from there.  The episode goes on: step_counter continues, no
    termination (mj_step leaves time = 0.002, so ballbot_env.py:897-899's
    time == 0 check never fires), done bit 2 reports the reset."""
    q0 = np.array(oracle.model_info()["qpos0"])
    rng = np.random.default_rng(4)
    q, v, w = oracle.reset_state(0.01)
    q = q + np.r_[rng.normal(0, 0.01, 3), 0, 0, 0, 0, rng.normal(0, 0.1, 10)]
    v = rng.normal(0, 0.1, 15)
    w = rng.normal(0, 1.0, 15)
    if case == "nan_qpos":
        q[5] = np.nan
    elif case == "big_qpos":
        q[11] = 2e10
    elif case == "nan_qvel":
        v[2] = np.nan
    elif case == "big_qvel":
        v[14] = -1.5e10
    else:  # finite, |qvel| < 1e10, but the wheel damping alone gives |qacc| >> 1e10
        v[7] = 5e9
    a = np.array([0.3, -0.7, 0.5], np.float32)
    qg, vg, wg, sc, obs, r, fl = _step_from(oracle, q, v, w, 57, a)
    # expected: one step from qpos0 at rest with zero ctrl (zero action), warm start 0
    qe, ve, we, _, obs_e, _, fle = _step_from(oracle, q0, np.zeros(15), np.zeros(15), 57, np.zeros(3))
    np.testing.assert_array_equal(qg, qe)
    np.testing.assert_array_equal(vg, ve)
    np.testing.assert_array_equal(obs[3:], obs_e[3:])  # physics part of the observation
    np.testing.assert_array_equal(obs[:3], a)          # "actions" echoes the command (ballbot_env.py:919)
    assert fl & 4 and not fle & 4
    assert (fl & 3) == (fle & 3) == 0 and sc == 58    # the episode goes on
    assert np.isfinite(r)


def test_nan_action_zeroes_ctrl(oracle):
    """mjWARN_BADCTRL: a NaN control zeroes every control for the step; the
    observation still echoes the action and the reward's penalty is NaN."""
    q, v, w = oracle.reset_state(0.01)
    a = np.array([np.nan, 0.5, 0.5], np.float32)
    qg, vg, _, _, obs, r, fl = _step_from(oracle, q, v, w, 3, a)
    qe, ve, _, _, _, _, _ = _step_from(oracle, q, v, w, 3, np.zeros(3))
    np.testing.assert_array_equal(qg, qe)
    np.testing.assert_array_equal(vg, ve)
    assert np.isnan(obs[0]) and np.isnan(r) and not fl & 4


def test_flop_counter_counts_the_oracle_step():
    """oracle/flopcount.cpp (the roofline's algorithmic FLOPs): counted steps
    exclude the burn-in, counts are deterministic, the Newton solve dominates a
    flat step, and an env in free fall (no contacts) costs far less."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import flops as F

    L = F.lib()
    flat = np.zeros(293 * 293, np.float32)
    a = F.count(L, flat, 2.0, 4, 6, burn_in=100)  # landed (the reset height is 4 cm)
    b = F.count(L, flat, 2.0, 4, 6, burn_in=100)
    assert a["env_steps"] == 24
    assert a["flops_per_env_step"] == b["flops_per_env_step"]
    ph = a["flops_by_phase"]
    assert max(ph, key=ph.get) == "newton_solver"
    assert 2e5 < a["flops_per_env_step"] < 3e6
    assert ph["kinematics_mass_bias"] > 4e4  # per RK4 stage: tree kinematics, CRB mass matrix, RNE bias
    # a field 1.5 m lower than the reset height computed for it: free fall, no ground contacts
    high = np.zeros(293 * 293, np.float32)
    high[140 * 293 + 140] = 0.75  # one tall cell in the footprint window, 0.29 m off: reset height 1.51 m
    c = F.count(L, high, 2.0, 4, 6, burn_in=100)
    assert c["flops_by_phase"]["constraint_assembly"] < ph["constraint_assembly"]
    assert c["flops_per_env_step"] < 0.8 * a["flops_per_env_step"]


def test_flop_replay_of_the_timed_mix():
    """bench.py's FLOP count replays its timed window (tools/flops.py count_replay): the counts
    do not depend on how the envs are split over host threads (thread-local counters), every
    env-step is counted, and an env's resets walk its own terrain row (a row that ends sooner
    than the resets repeats its last terrain and is reported)."""
    import sys
    from pathlib import Path

    import oracle_lib as O

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import flops as F
    from ballbot_gym.terrain import generate_hills_terrain

    table = np.stack([O.flat_hfield(), generate_hills_terrain(293, seed=7).astype(np.float32)])
    offs = np.array([O.init_offset(t) for t in table])
    n, T = 12, 400
    q = np.zeros((n, 17)); v = np.zeros((n, 15)); w = np.zeros((n, 15))
    for e in range(n):
        q[e], v[e], w[e] = O.reset_state(offs[e % 2])
    acts = np.random.default_rng(0).uniform(-1.5, 1.5, (T, n, 3)).astype(np.float32)
    terr = np.array([[e % 2] for e in range(n)], np.int32)  # one terrain each: every reset overruns the row
    runs = [F.count_replay(q.copy(), v.copy(), w.copy(), np.zeros(n, np.int32), acts, table, offs, terr, 2.0,
                           threads=t) for t in (1, 3)]
    assert runs[0]["env_steps"] == runs[1]["env_steps"] == n * T
    assert runs[0]["flops_per_env_step"] == runs[1]["flops_per_env_step"] > 1e5
    assert runs[0]["terrain_overrun_resets"] == runs[1]["terrain_overrun_resets"] > 0  # large actions: resets
