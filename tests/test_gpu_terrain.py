"""GPU terrain bank: bb_generate_perlin vs the numpy restatement.

The kernel (csrc/bb_terrain.hip) must be BIT-IDENTICAL to
ballbot_gym.terrain.perlin.generate_perlin_terrain(...).astype(float32), the
value the reference writes into hfield_data (ballbot_env.py:513), for every
seed and generator argument set; its init offsets must equal the host
restatement of ballbot_env.py:546-563.  Perlin parity against caseman/noise
itself is unpinned (the library is absent), the GPU-vs-
restatement parity here is exact.  A teacher-forced trajectory on a perlin
terrain checks the step on the generated bank against the oracle.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HARD = {"scale": 20.0, "octaves": 5, "persistence": 0.25, "lacunarity": 2.5}  # examples/terrain_examples.yaml:310-317


def _env(cfg, n_terrains, n_envs=64, seed=0):
    from ballbot_gym.envs import BallbotVecEnv

    return BallbotVecEnv(n_envs, device="cuda:0", terrain_config={"type": "perlin", "config": dict(cfg)},
                         n_terrains=n_terrains, seed=seed, auto_reset=False, shared_stream=True)


@pytest.mark.parametrize("cfg", [{}, HARD, {"amplitude": 1.7, "seed": None}], ids=["default", "hard", "amp"])
def test_perlin_bank_bit_exact(cfg):
    from ballbot_gym.envs.config import init_offset
    from ballbot_gym.terrain.perlin import generate_perlin_terrain

    env = _env(cfg, n_terrains=6, seed=10)
    assert env.n_terrains == 6
    # seeds = the reference's reset stream: np_random(10).integers(0, 10000) -> 7765, 9560, 2640, 2076, ...
    assert list(env.terrain_seeds[:4]) == [7765, 9560, 2640, 2076]
    args = {k: v for k, v in cfg.items() if k != "seed"}
    offs = env.offsets()
    for slot, s in enumerate(env.terrain_seeds):
        ref = generate_perlin_terrain(293, seed=int(s), **args).astype(np.float32)
        got = env.hfield(slot)
        nbad = int((got != ref).sum())
        assert nbad == 0, f"seed {s}: {nbad} vertices differ, max {np.abs(got - ref).max():.3e}"
        assert offs[slot] == np.float32(init_offset(ref, 2.0)), (s, offs[slot])
    env.close()


def test_perlin_full_seed_space():
    """n_terrains=None: the whole reset seed space [0, 10000) is resident, slot == seed."""
    from ballbot_gym.terrain.perlin import generate_perlin_terrain

    env = _env({}, n_terrains=None, n_envs=256, seed=3)
    assert env.n_terrains == 10000
    for s in (0, 1, 4999, 9999):
        assert np.array_equal(env.hfield(s), generate_perlin_terrain(293, seed=s).astype(np.float32)), s
    acts = torch.zeros(256, 3, device=env.device)
    for _ in range(20):
        env.step(acts)
    st = env.stats()
    assert st["diverged"] == 0
    env.close()


def test_step_parity_on_perlin(oracle):
    """Teacher-forced fp64 steps on a GPU-generated perlin terrain vs the oracle on the restated field.

    128 envs at 4 per workgroup = 32 workgroups: the relief bank takes the
    predict/split route, whose list launches use the XCD-aware workgroup
    permutation over the active list (non-trivial from 9 active workgroups)."""
    import traj
    from ballbot_gym.terrain.perlin import generate_perlin_terrain
    from test_gpu_parity import TOL, _teacher_forced

    env = _env({}, n_terrains=1, n_envs=128, seed=10)
    s = int(env.terrain_seeds[0])
    hf = generate_perlin_terrain(293, seed=s).astype(np.float32)
    assert np.array_equal(env.hfield(0), hf)
    rec = traj.record(n_envs=128, n_steps=60, hfield=hf, seed=9)
    _teacher_forced(env, rec, TOL["fp64"])
    env.close()


NUMPY_TERRAINS = ["stepped", "ramp", "sinusoidal", "ridge_valley", "bowl", "gradient", "terraced", "wavy", "spiral",
                  "mixed"]


@pytest.mark.parametrize("ttype", NUMPY_TERRAINS)
def test_step_parity_terrain_generators(oracle, ttype):
    """Teacher-forced fp64 steps on every other terrain generator of the
    registry (terrain/__init__.py:18-36) with its default config vs the oracle
    on the same field and vertical scale (ramp and gradient rescale size_z,
    ballbot_env.py:486-495).  The relief takes the predict/split route, so
    ball-terrain and base-tree contacts on each generator's shapes (steps,
    ramps, ridges, bowls, spirals) go through both step kernels."""
    import traj
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_gym.envs.config import terrain_bank
    from test_gpu_parity import TOL, _teacher_forced

    cfg = {"type": ttype, "config": {}}
    if ttype == "mixed":  # needs components (terrain/mixed.py)
        cfg["config"] = {"components": [{"type": "hills", "weight": 0.6}, {"type": "stepped", "weight": 0.4}],
                         "blend_mode": "additive"}
    hfs, seeds, size_z = terrain_bank(cfg, 1, seed=5)
    hf = np.asarray(hfs[0], np.float32).ravel()
    env = BallbotVecEnv(32, device="cuda:0", terrain_config=cfg, n_terrains=1, seed=5, auto_reset=False,
                        shared_stream=True)
    assert np.array_equal(env.hfield(0), hf)
    rec = traj.record(n_envs=32, n_steps=40, hfield=hf, size_z=size_z, seed=17)
    _teacher_forced(env, rec, TOL["fp64"])
    env.close()
