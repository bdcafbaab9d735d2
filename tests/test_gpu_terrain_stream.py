"""A14: every reset's terrain is the reference's draw, bit-exact (integer work).

The reference draws r_seed = _np_random.integers(0, 10000) at each reset
(ballbot_env.py:505-510) from a generator fixed at construction by
eval_env=[True, seed] (:378-384), and train.py:82-89 builds EVERY training env
that way with the same seed: the k-th reset of every env takes value k of
np_random(seed).integers(0, 10000).  An eval VecEnv gives env i the seed
seed + N_ENVS + i (train.py:90-97): its own stream.  The tests step 4096 envs
with short episodes (thousands of resets, auto-reset inside the step kernel)
and compare, after every step, the terrain seed of every env with the numpy
stream at that env's draw count.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _check(env, draws_of_env, seeds):
    t, k = env.env_terrain()
    exp = draws_of_env(np.arange(env.num_envs), k - 1)
    got = seeds[t]
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"envs {bad[:8]}: terrain seed {got[bad[:8]]} != stream {exp[bad[:8]]} (draw {k[bad[:8]] - 1})"
    return t, k


@pytest.mark.parametrize("terrain,n_terrains", [("perlin", 48), ("hills", 24), ("perlin", None)],
                         ids=["perlin48", "hills24", "perlin_full_bank"])
def test_shared_stream_bit_exact(terrain, n_terrains):
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_gym.envs.config import stream_draws

    n = 4096
    env = BallbotVecEnv(n, device="cuda:0", seed=10, terrain_config={"type": terrain, "config": {}},
                        n_terrains=n_terrains, max_ep_steps=60)
    K = env.terrain_plan.streams.shape[1]
    draws = stream_draws(10, K)
    assert draws[:4].tolist() == [7765, 9560, 2640, 2076]
    seeds = np.asarray(env.terrain_seeds)

    def exp(e, k):
        return draws[k % K]

    t, k = _check(env, exp, seeds)
    assert (k == 1).all() and (seeds[t] == 7765).all()  # construction reset: draw 0 for every env
    g = torch.Generator(device="cuda:0").manual_seed(0)
    distinct = 0
    for i in range(360):
        env.step(torch.rand(n, 3, generator=g, device="cuda:0") * 3 - 1.5)
        if i % 37 == 36:  # masked resets (10% of the envs) take their own next draws: the envs drift apart
            env.reset(torch.rand(n, generator=g, device="cuda:0") < 0.1)
        t, k = _check(env, exp, seeds)
        distinct = max(distinct, len(np.unique(k)))
    resets = int(k.sum()) - n
    assert resets >= 1000, resets
    assert distinct > 2  # envs sit at different points of the stream
    st = env.stats()
    assert st["resets"] <= resets  # every auto-reset (and masked reset) took exactly one draw
    assert st["stream_wraps"] == int(np.maximum(k - K, 0).sum())
    env.close()


def test_per_env_streams_and_pins():
    """Eval-style streams (env i: np_random(100 + i)) and bb_assign_terrain pins:
    a pinned env takes no draw; unpinned, it continues its own stream."""
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_gym.envs.config import stream_draws

    n = 256
    ss = [100 + i for i in range(n)]
    env = BallbotVecEnv(n, device="cuda:0", seed=0, terrain_config={"type": "perlin", "config": {}},
                        n_terrains=None, stream_seeds=ss, max_ep_steps=20)
    K = env.terrain_plan.streams.shape[1]
    table = np.stack([stream_draws(s, K) for s in ss])
    seeds = np.asarray(env.terrain_seeds)

    def exp(e, k):
        return table[e, k % K]

    _check(env, exp, seeds)
    zeros = torch.zeros(n, 3, device="cuda:0")
    for _ in range(45):
        env.step(zeros)
        _check(env, exp, seeds)
    pin = np.full(n, -1, np.int32)
    pin[:32] = 1234  # slot == seed in the full bank
    _, k_before = env.env_terrain()
    env.assign_terrain(pin)
    for _ in range(45):
        env.step(zeros)
    t, k = env.env_terrain()
    assert (seeds[t[:32]] == 1234).all() and (k[:32] == k_before[:32]).all()
    e = np.arange(32, n)
    assert (seeds[t[e]] == table[e, (k[e] - 1) % K]).all() and (k[e] > k_before[e]).all()
    env.assign_terrain(np.full(n, -1, np.int32))
    for _ in range(25):
        env.step(zeros)
    _check(env, exp, seeds)
    env.close()
