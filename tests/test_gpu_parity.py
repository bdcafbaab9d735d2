"""GPU parity: the HIP step (through the C-ABI) vs the fp64 CPU oracle.

Teacher-forced: every env starts each step from the oracle's state, so the
comparison measures one mj_step + glue, not chaotic drift.  Tolerances (fp32
kernel): qpos 1e-5, qvel 1e-3 absolute per step; obs 1e-4;
reward 1e-6; flags exact except tilt within 1e-3 deg of the threshold.  The fp64
kernel is held to 1e-9 / 1e-7.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = {"fp32": dict(q=1e-5, v=1e-3, obs=1e-4, r=1e-6), "fp64": dict(q=1e-9, v=1e-7, obs=1e-6, r=1e-7)}


@pytest.fixture(scope="module")
def flat_traj(oracle):
    import traj

    return traj.record(n_envs=64, n_steps=120, hfield=oracle.flat_hfield(), seed=3)


@pytest.fixture(scope="module")
def hills_traj(oracle):
    import traj
    from ballbot_gym.terrain import generate_hills_terrain

    hf = generate_hills_terrain(293, seed=7).astype(np.float32)
    return hf, traj.record(n_envs=32, n_steps=80, hfield=hf, seed=5)


def _make_env(n, precision, terrain=None):
    from ballbot_gym.envs import BallbotVecEnv

    env = BallbotVecEnv(n, device="cuda:0", precision=precision, auto_reset=False,
                        terrain_config=terrain or {"type": "flat", "config": {}})
    return env


def _teacher_forced(env, rec, tol):
    n = rec["qpos"].shape[1]
    worst = dict(q=0.0, v=0.0, obs=0.0, r=0.0)
    for t in range(rec["qpos"].shape[0]):
        env.set_state(rec["qpos"][t], rec["qvel"][t], rec["warm"][t], rec["steps"][t])
        a = torch.tensor(rec["action"][t], dtype=torch.float32, device=env.device)
        obs, rew, term, trunc, info = env.step(a)
        q, v, w, s = env.get_state()
        worst["q"] = max(worst["q"], np.abs(q - rec["qpos1"][t]).max())
        worst["v"] = max(worst["v"], np.abs(v - rec["qvel1"][t]).max())
        worst["obs"] = max(worst["obs"], np.abs(obs.cpu().numpy() - rec["obs"][t]).max())
        worst["r"] = max(worst["r"], np.abs(rew.cpu().numpy() - rec["reward"][t]).max())
        gflags = info["done_flags"].cpu().numpy() & 3
        mism = np.nonzero(gflags != (rec["flags"][t] & 3))[0]
        assert len(mism) <= 1, f"step {t}: termination flags differ for envs {mism}"
    for k in worst:
        assert worst[k] <= tol[k], f"{k}: worst {worst[k]:.3e} > tol {tol[k]:.1e} ({worst})"
    return worst


def test_native_library_loads():
    from ballbot_gym import _native

    L = _native.lib()
    assert L.bb_abi_version() == 1


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_forward_parity(oracle, flat_traj, precision):
    rec = flat_traj
    env = _make_env(rec["qpos"].shape[1], precision)
    hf = oracle.flat_hfield()
    rng = np.random.default_rng(0)
    for t in (0, 30, 60, 100):
        ctrl = rng.uniform(-10, 10, (env.num_envs, 3))
        env.set_state(rec["qpos"][t], rec["qvel"][t], rec["warm"][t])
        qacc, ncon = env.forward(ctrl)
        for e in range(env.num_envs):
            fo = oracle.forward(rec["qpos"][t][e], rec["qvel"][t][e], ctrl[e], rec["warm"][t][e], hf)
            ref = np.array(fo.qacc)
            assert ncon[e] == fo.nground
            err = np.abs(qacc[e] - ref).max() / max(1.0, np.abs(ref).max())
            assert err < (2e-4 if precision == "fp32" else 1e-9), (t, e, err)
    env.close()


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_step_parity_flat(flat_traj, precision):
    env = _make_env(flat_traj["qpos"].shape[1], precision)
    _teacher_forced(env, flat_traj, TOL[precision])
    env.close()


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_step_parity_hills(hills_traj, precision):
    hf, rec = hills_traj
    env = _make_env(rec["qpos"].shape[1], precision, terrain={"type": "hills", "config": {"seed": 7}})
    _teacher_forced(env, rec, TOL[precision])
    env.close()
