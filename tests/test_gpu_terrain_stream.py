"""A14: every reset's terrain is the reference's draw, bit-exact (integer work).

The reference draws r_seed = _np_random.integers(0, 10000) at each reset
(ballbot_env.py:505-510).  SB3 seeds training env i through VecEnv.seed(seed)
and reset(seed=seed+i), which replaces the env's _np_random with
np_random(seed + i) (ballbot_env.py:596, train.py:126-141); an eval env keeps
np_random(seed + N_ENVS + i) (:378-384, train.py:90-97).  The batched env runs
numpy's PCG64 per env on the GPU (bb_set_terrain_rng).  The tests step 4096
envs with short episodes (thousands of resets, auto-reset inside the step
kernels) and compare, after every step, the terrain seed every env drew with
numpy's stream at that env's draw count, then the device generator states
with the host restatement (pcg64_terrain_draws) and numpy's own state.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _tables(seeds, k):
    from ballbot_gym.envs.config import stream_draws

    cache = {}
    for s in seeds:
        if s not in cache:
            cache[s] = stream_draws(s, k)
    return np.stack([cache[s] for s in seeds])


def _check(env, table):
    """Every env's last drawn seed == its generator's value at its draw count; the bank slot holds it."""
    t, k = env.env_terrain()
    _, last = env.terrain_rng()
    assert (k >= 1).all() and k.max() <= table.shape[1], k.max()
    exp = table[np.arange(env.num_envs), k - 1]
    bad = np.nonzero(last != exp)[0]
    assert len(bad) == 0, f"envs {bad[:8]}: drew {last[bad[:8]]} != numpy {exp[bad[:8]]} (draw {k[bad[:8]] - 1})"
    plan = env.terrain_plan
    slots = np.array([plan.slot_of(int(s)) for s in last])
    res = slots >= 0
    assert np.array_equal(t[res], slots[res])
    assert np.array_equal(t[~res], last[~res] % env.n_terrains)  # not resident: counted, slot seed % n
    return t, k, last


def _words_match(env, seeds, k):
    """Device generators == the host restatement after k[e] draws == numpy's state."""
    from ballbot_gym.envs.config import np_random, pcg64_terrain_draws, pcg64_words

    w, _ = env.terrain_rng()
    for e in range(env.num_envs):
        _, hw = pcg64_terrain_draws(pcg64_words(seeds[e]), int(k[e]))
        assert np.array_equal(w[e], hw), e
    for e in (0, env.num_envs // 2, env.num_envs - 1):
        g = np_random(seeds[e])
        g.integers(0, 10000, size=int(k[e]))
        assert np.array_equal(w[e], pcg64_words(g)), e


def _run(env, table, steps, masked_every=37, seed=0):
    n = env.num_envs
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    distinct = 0
    for i in range(steps):
        env.step(torch.rand(n, 3, generator=g, device="cuda:0") * 3 - 1.5)
        if i % masked_every == masked_every - 1:  # masked resets (10% of the envs) take their own next draws
            env.reset(torch.rand(n, generator=g, device="cuda:0") < 0.1)
        t, k, _ = _check(env, table)
        distinct = max(distinct, len(np.unique(k)))
    return t, k, distinct


def test_sb3_seeded_generators_4096_envs_bit_exact():
    """Default seeding, configs[2]-sized: env g draws from np_random(seed + g), on the
    whole perlin seed space (slot == seed); >= 1000 auto- and masked resets."""
    from ballbot_gym.envs import BallbotVecEnv

    n, seed = 4096, 10
    env = BallbotVecEnv(n, device="cuda:0", seed=seed, terrain_config={"type": "perlin", "config": {}},
                        max_ep_steps=60)
    seeds = [seed + e for e in range(n)]
    assert env.terrain_plan.stream_seeds == seeds and env.terrain_plan.full
    table = _tables(seeds, 48)
    assert table[0, :4].tolist() == [7765, 9560, 2640, 2076]  # env 0 = np_random(10), tests/golden/seeds.json
    t, k, _ = _check(env, table)
    assert (k == 1).all() and np.array_equal(t, table[:, 0])  # the construction reset: draw 0 of each generator
    t, k, distinct = _run(env, table, 360)
    resets = int(k.sum()) - n
    assert resets >= 1000, resets
    assert distinct > 2  # envs sit at different points of their streams
    assert env.stats()["stream_wraps"] == 0  # every draw resident
    _words_match(env, seeds, k)
    env.close()


def test_multi_step_and_rollout_draw_the_same_streams():
    """bb_step_multi (parked and work-queue forms) draws inside its launch from the same
    generators: per-env seeds after 3 x 40 steps == one bb_step per step."""
    from ballbot_gym.envs import BallbotVecEnv

    n = 512
    kw = dict(device="cuda:0", seed=31, terrain_config={"type": "perlin", "config": {}}, max_ep_steps=25)
    a, b = BallbotVecEnv(n, **kw), BallbotVecEnv(n, **kw)
    g = torch.Generator(device="cuda:0").manual_seed(2)
    acts = torch.rand(120, n, 3, generator=g, device="cuda:0") * 2.4 - 1.2
    for j in range(3):
        a.step_multi(acts[40 * j:40 * (j + 1)].contiguous())
    for t in range(120):
        b.step(acts[t])
    wa, la = a.terrain_rng()
    wb, lb = b.terrain_rng()
    assert np.array_equal(wa, wb) and np.array_equal(la, lb)
    assert np.array_equal(a.env_terrain()[1], b.env_terrain()[1])
    table = _tables([31 + e for e in range(n)], 32)
    _check(a, table)
    a.close()
    b.close()


def test_host_bank_misses_are_counted():
    """A host-generated bank (hills) holds the seeds of each generator's first
    n_terrains draws; a later draw whose seed is not resident resets onto slot
    seed % n_terrains and is counted in stats[5] -- never silently."""
    from ballbot_gym.envs import BallbotVecEnv

    n = 256
    env = BallbotVecEnv(n, device="cuda:0", seed=3, terrain_config={"type": "hills", "config": {}}, n_terrains=3,
                        max_ep_steps=15)
    seeds = [3 + e for e in range(n)]
    plan = env.terrain_plan
    assert not plan.full and env.n_terrains == len(plan.seeds)
    table = _tables(seeds, 40)
    misses_before = 0
    g = torch.Generator(device="cuda:0").manual_seed(4)
    for i in range(150):
        env.step(torch.rand(n, 3, generator=g, device="cuda:0") * 3 - 1.5)
        t, k, last = _check(env, table)
    drawn = [int(table[e, j]) for e in range(n) for j in range(int(k[e]))]
    misses = sum(plan.slot_of(s) < 0 for s in drawn)
    assert misses > misses_before and env.stats()["stream_wraps"] == misses
    _words_match(env, seeds, k)
    env.close()


def test_shared_stream_and_seed_reset():
    """shared_stream=True: every env on np_random(seed) (reset k of each env draws value k).
    seed(s) then reset(): env i restarts on np_random(s + i), as SB3's VecEnv.seed +
    reset(seed=s+i) does; a masked reset does not apply pending seeds."""
    from ballbot_gym.envs import BallbotVecEnv

    n = 1024
    env = BallbotVecEnv(n, device="cuda:0", seed=10, terrain_config={"type": "perlin", "config": {}},
                        max_ep_steps=40, shared_stream=True)
    table = _tables([10] * n, 40)
    t, k, _ = _check(env, table)
    assert (t == 7765).all()
    _run(env, table, 120, seed=1)
    assert env.seed(500) == [500 + i for i in range(n)]
    env.reset(torch.zeros(n, dtype=torch.bool, device="cuda:0"))  # masked: pending seeds wait
    _check(env, table)
    env.reset()
    table2 = _tables([500 + i for i in range(n)], 40)
    t, k, _ = _check(env, table2)
    assert (k == 1).all()
    _, k, _ = _run(env, table2, 120, seed=2)
    _words_match(env, [500 + i for i in range(n)], k)
    env.close()


def test_seed_reset_on_a_host_bank_regenerates_it():
    """seed(s) on a hills bank that lacks the new generators' draws: the bank is rebuilt
    for them at the next reset, and the draws follow np_random(s + i)."""
    from ballbot_gym.envs import BallbotVecEnv

    n = 32
    env = BallbotVecEnv(n, device="cuda:0", seed=1, terrain_config={"type": "hills", "config": {}}, n_terrains=2,
                        max_ep_steps=10)
    env.seed(9000)
    env.reset()
    seeds = [9000 + i for i in range(n)]
    table = _tables(seeds, 30)
    t, k, last = _check(env, table)
    assert env.terrain_plan.covers(table[:, :2].ravel())
    from ballbot_gym.terrain import generate_hills_terrain

    e = 5
    assert np.array_equal(env.hfield(int(t[e])), generate_hills_terrain(293, seed=int(last[e])).astype(np.float32))
    env.close()


def test_explicit_draw_table_and_pins():
    """terrain_draws: one explicit seed list that every env walks (bb_set_terrain_stream),
    and bb_assign_terrain pins: a pinned env takes no draw; unpinned, it continues."""
    from ballbot_gym.envs import BallbotVecEnv

    n = 256
    draws = [5, 9, 5, 1234, 77, 9]
    env = BallbotVecEnv(n, device="cuda:0", terrain_config={"type": "perlin", "config": {}}, n_terrains=1,
                        terrain_draws=draws, max_ep_steps=10)
    seeds = np.asarray(env.terrain_seeds)
    assert seeds.tolist() == [5, 9, 1234, 77]

    def chk():
        t, k = env.env_terrain()
        assert np.array_equal(seeds[t], np.asarray(draws)[(k - 1) % len(draws)])
        return t, k

    zeros = torch.zeros(n, 3, device="cuda:0")
    for _ in range(45):
        env.step(zeros)
        chk()
    pin = np.full(n, -1, np.int32)
    pin[:32] = 2  # slot 2 = seed 1234
    _, k_before = env.env_terrain()
    env.assign_terrain(pin)
    for _ in range(45):
        env.step(zeros)
    t, k = env.env_terrain()
    assert (seeds[t[:32]] == 1234).all() and (k[:32] == k_before[:32]).all() and (k[32:] > k_before[32:]).all()
    env.assign_terrain(np.full(n, -1, np.int32))
    for _ in range(25):
        env.step(zeros)
    chk()
    assert env.stats()["stream_wraps"] > 0  # the 6-entry table wrapped (counted)
    env.close()


def test_single_env_reset_seed_reseeds_every_time():
    """BBotSimulation.reset(seed=s) replaces _np_random by np_random(s) at every
    seeded reset, in eval mode too (gymnasium Env.reset, ballbot_env.py:596), so
    evaluate.py's reset(seed=seed+test_i) gives a reproducible terrain per episode;
    unseeded resets continue the generator.  The terrain of the drawn seed is
    generated into the env's ring of bank slots."""
    import string

    import ballbot_gym
    from ballbot_gym.envs.config import np_random
    from ballbot_gym.terrain import generate_hills_terrain

    env = ballbot_gym.make("ballbot-v0.1", GUI=False, terrain_type="hills", eval_env=[True, 10],
                           disable_cameras=True)
    seen = []
    for s in (999, 999, None, 5, None):
        env.reset(seed=s)
        seen.append(int(env.last_r_seed))
    g5 = np_random(5)
    exp5 = [int(g5.integers(0, 10000)) for _ in range(2)]
    g999 = np_random(999)
    first999 = int(g999.integers(0, 10000))
    assert seen == [first999, first999, int(g999.integers(0, 10000)), exp5[0], exp5[1]]
    hf = env._env.hfield(env._env.env_terrain()[0][0])
    assert np.array_equal(hf, generate_hills_terrain(293, seed=exp5[1]).astype(np.float32))
    env.close()
    # eval mode without seeds: np_random(10) from construction (7765, 9560, 2640)
    env = ballbot_gym.make("ballbot-v0.1", GUI=False, terrain_type="perlin", eval_env=[True, 10],
                           disable_cameras=True)
    seen = []
    for _ in range(3):
        env.reset()
        seen.append(int(env.last_r_seed))
    assert seen == [7765, 9560, 2640]
    from ballbot_gym.terrain.perlin import generate_perlin_terrain

    hf = env._env.hfield(env._env.env_terrain()[0][0])
    assert np.array_equal(hf, generate_perlin_terrain(293, seed=2640).astype(np.float32))
    env.close()
    # non-eval: the first reset's generator draws the log-dir permutation after its terrain
    env = ballbot_gym.make("ballbot-v0.1", GUI=False, terrain_type="hills", disable_cameras=True)
    g = np_random(42)
    exp = [int(g.integers(0, 10000))]
    g.permutation(list(string.ascii_letters + string.digits))
    exp += [int(g.integers(0, 10000)) for _ in range(2)]
    seen = []
    for s in (42, None, None):
        env.reset(seed=s)
        seen.append(int(env.last_r_seed))
    assert seen == exp
    env.close()


def test_captured_step_follows_reseed():
    """A step captured as a HIP graph before env.seed(s) draws its later terrains from the new
    generators np_random(s + i) at replay: bb_set_terrain_rng rewrites the device record that
    the captured Dev points at, in place (the graph holds its address only).  A host-generated
    bank whose new draws are not resident would need a new handle: refused while graphs exist."""
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_gym.envs.config import stream_draws

    n = 256
    kw = dict(device="cuda:0", seed=5, terrain_config={"type": "perlin", "config": {}}, max_ep_steps=40)
    eager, graphed = BallbotVecEnv(n, **kw), BallbotVecEnv(n, **kw)
    static_a = torch.zeros(n, 3, device="cuda:0")
    graph = graphed.capture_step(static_a)
    for e in (eager, graphed):
        e.seed(77)
        e.reset()
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for t in range(130):  # 40-step episodes: every env resets at least three times after the re-seed
        a = torch.rand(n, 3, generator=g, device="cuda:0") * 2 - 1
        eager.step(a)
        static_a.copy_(a)
        graph.replay()
    torch.cuda.synchronize()
    for x, y in zip(eager.get_state(), graphed.get_state()):
        np.testing.assert_array_equal(x, y)
    w_e, s_e = eager.terrain_rng()
    w_g, s_g = graphed.terrain_rng()
    np.testing.assert_array_equal(w_e, w_g)
    _, draws = graphed.env_terrain()
    assert draws.min() >= 4
    for i in range(0, n, 37):  # the last drawn seed is np_random(77 + i)'s draw number draws[i] - 1
        assert s_g[i] == stream_draws(77 + i, int(draws[i]))[-1]
    eager.close(), graphed.close()

    env = BallbotVecEnv(64, device="cuda:0", seed=1, n_terrains=2, terrain_config={"type": "hills", "config": {}})
    env.capture_step(torch.zeros(64, 3, device="cuda:0"))
    env.seed(999)  # hills bank of 2 draws per generator: the new generators' draws are not resident
    with pytest.raises(RuntimeError, match="HIP graph"):
        env.reset()
    env.close()
