"""bb_step_multi: K env.steps in one launch == K bb_step calls, bit for bit.

Outputs of every step (obs, reward, done flags, terminal obs, pos2d), the
final states, the counters (resets, Newton iterations, full-path env-steps)
and the terrain draws of the auto-resets must be identical: the multi-step
kernel runs the same fast/full step code per env, only without a grid-wide
barrier between steps.  Flat terrain with short episodes and large actions
(many auto-resets, toppling robots), and perlin with per-env terrain streams
(base-tree contacts: the fast path hands envs over to the inline full step).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _pair(n, terrain, monkeypatch, route="1", **kw):
    from ballbot_gym.envs import BallbotVecEnv

    monkeypatch.setenv("BB_ROUTE", route)  # read by bb_create: the per-step env's route

    def mk():
        return BallbotVecEnv(n, device="cuda:0", seed=3, terrain_config={"type": terrain, "config": {}}, **kw)
    return mk(), mk()


def _compare_runs(a, b, actions, k, exact=True):
    """a: per-step bb_step; b: bb_step_multi in chunks of k."""
    T = actions.shape[0]
    outs = {"obs": [], "reward": [], "done": [], "terminal_obs": [], "pos2d": []}
    for t in range(T):
        obs, rew, _, _, info = a.step(actions[t])
        outs["obs"].append(obs.clone())
        outs["reward"].append(rew.clone())
        outs["done"].append(info["done_flags"].clone())
        outs["terminal_obs"].append(info["terminal_observation"].clone())
        outs["pos2d"].append(info["pos2d"].clone())
    ref = {key: torch.stack(v) for key, v in outs.items()}
    got = {key: [] for key in outs}
    for t0 in range(0, T, k):
        o = b.step_multi(actions[t0:t0 + k].contiguous())
        for key in got:
            got[key].append(o[key].clone())
    got = {key: torch.cat(v) for key, v in got.items()}
    if not exact:  # route 0 against route 1: rounding (test_step_routes_agree's bounds)
        assert torch.equal(ref["done"], got["done"])
        for key in ("obs", "reward", "terminal_obs", "pos2d"):
            assert torch.allclose(ref[key], got[key], rtol=1e-6, atol=1e-6), key
        qa, va, _, sa_ = a.get_state()
        qb, vb, _, sb_ = b.get_state()
        np.testing.assert_allclose(qa, qb, rtol=0, atol=1e-11)
        np.testing.assert_allclose(va, vb, rtol=1e-9, atol=1e-9)
        np.testing.assert_array_equal(sa_, sb_)
        for x, y in zip(a.env_terrain(), b.env_terrain()):
            np.testing.assert_array_equal(x, y)
        return b.stats()
    for key in ref:
        bad = (ref[key] != got[key]).reshape(T, a.num_envs, -1).any(-1).nonzero()
        assert len(bad) == 0, f"{key}: first (step, env) mismatches {bad[:6].tolist()}"
    for x, y in zip(a.get_state(), b.get_state()):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(a.env_terrain(), b.env_terrain()):
        np.testing.assert_array_equal(x, y)
    sa, sb = a.stats(), b.stats()
    assert sa == sb, (sa, sb)
    return sa


@pytest.mark.parametrize("k", [1, 7, 16])
def test_multi_step_flat_matches_single_steps(k, monkeypatch):
    n = 1024
    a, b = _pair(n, "flat", monkeypatch, max_ep_steps=25)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    actions = torch.rand(48, n, 3, generator=g, device="cuda:0") * 4 - 2  # clipped to [-1, 1]*10 inside: topples
    st = _compare_runs(a, b, actions, k)
    assert st["resets"] >= n  # every env's episode ended (step limit or tilt) and auto-reset at least once
    a.close(), b.close()


@pytest.mark.parametrize("route,park", [("1", "1"), ("1", "0"), ("0", "1")])
def test_multi_step_perlin_hand_overs_match(route, park, monkeypatch):
    """Route 1: multi_step_kernel, hand-overs parked for a second launch (BB_MULTI_PARK=1, the
    default) or inline in one launch (0); route 0: relief_multi_kernel.  Bit-exact both ways."""
    monkeypatch.setenv("BB_MULTI_PARK", park)  # read by bb_create
    n = 512
    a, b = _pair(n, "perlin", monkeypatch, route=route, n_terrains=None, stream_seeds=[50 + i for i in range(n)],
                 max_ep_steps=200)
    g = torch.Generator(device="cuda:0").manual_seed(2)
    # rough perlin: most robots fall for ~140 steps from the reset height, then land and topple
    # (base-tree contacts); episodes end by tilt or at 200 steps
    actions = torch.rand(256, n, 3, generator=g, device="cuda:0") * 2 - 1
    st = _compare_runs(a, b, actions, 32)  # route 0: relief_multi_kernel (predictor + work queue), route 1: multi_step_kernel
    assert st["slow_path"] > 0  # base-tree contacts: the inline full step ran
    assert st["resets"] > 0
    a.close(), b.close()


def test_multi_step_relief_queue_ragged_workgroups(monkeypatch):
    """200 envs: the last workgroup of the relief work queue holds 8 envs (200 = 12 x 16 + 8),
    and the cost-balanced placement is off (it needs whole workgroups); route 0 bit-exact."""
    n = 200
    a, b = _pair(n, "perlin", monkeypatch, route="0", n_terrains=None, stream_seeds=[900 + i for i in range(n)],
                 max_ep_steps=200)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    actions = torch.rand(224, n, 3, generator=g, device="cuda:0") * 2 - 1
    st = _compare_runs(a, b, actions, 32)
    assert st["slow_path"] > 0
    a.close(), b.close()


@pytest.mark.parametrize("terrain", ["hills", "perlin"])
def test_multi_step_adaptive_relief_route(terrain, monkeypatch):
    """Relief banks with no route fixed: each bb_step_multi runs the work queue (route 0) or the
    parked launches (route 1), as the device flag chose from the previous launch's full steps
    (hills: rarely any, the parked form; perlin: many, the queue).  Against one bb_step per step
    on the serial route the results agree to rounding, launch after launch."""
    from ballbot_gym.envs import BallbotVecEnv

    n = 512 if terrain == "hills" else 256
    kw = dict(device="cuda:0", seed=3, terrain_config={"type": terrain, "config": {}}, max_ep_steps=50)
    if terrain == "hills":
        kw.update(n_terrains=2)  # the seeds of two draws per generator (later draws: counted misses)
    if terrain == "perlin":
        kw.update(n_terrains=None, stream_seeds=[60 + i for i in range(n)])
    monkeypatch.setenv("BB_ROUTE", "1")
    a = BallbotVecEnv(n, **kw)
    for var in ("BB_ROUTE", "BB_MULTI_QUEUE", "BB_MULTI_ADAPT"):
        monkeypatch.delenv(var, raising=False)
    b = BallbotVecEnv(n, **kw)  # adaptive
    g = torch.Generator(device="cuda:0").manual_seed(7)
    actions = torch.rand(192, n, 3, generator=g, device="cuda:0") * 2 - 1
    st = _compare_runs(a, b, actions, 32, exact=False)
    assert st["resets"] > 0
    a.close(), b.close()


def _chunked_equal(a, b, pool, chunks, start=0):
    """a: one bb_step per step; b: bb_step_multi launches of `chunks` steps, both reading
    the cyclic action pool from slot `start` -- every output of every step (obs, reward,
    done, terminal obs, pos2d) bit for bit, chunk by chunk."""
    PS = pool.shape[0]
    j = start
    for k in chunks:
        assert j % PS + k <= PS
        acts = pool[j % PS:j % PS + k]
        out = b.step_multi(acts)
        for t in range(k):
            obs, rew, _, _, info = a.step(acts[t])
            for key, ref in (("obs", obs), ("reward", rew), ("done", info["done_flags"]),
                             ("terminal_obs", info["terminal_observation"]), ("pos2d", info["pos2d"])):
                assert torch.equal(out[key][t], ref), (key, j + t)
        j += k
    return j


@pytest.mark.parametrize("terrain,route", [("flat", "1"), ("perlin", "0")])
def test_headline_form_k512_and_driver_window(terrain, route, monkeypatch):
    """The exact form bench.py times (its defaults: a 512-slot action pool resident in HBM,
    512 steps per launch): a burn-in of 400 steps and 300 warm-up steps (launches of 512 +
    188), then the timed 500 steps as one launch (bench.launch_chunks); and the driver's
    window, one 20-step launch after the burn-in.  Against one bb_step per step, bit for bit
    (flat: 4096 envs, configs[1]; perlin: 4096 envs, configs[2] at the bench's own size, env g
    on np_random(1000 + g) over the whole seed space as bench.py seeds it, route 0: the relief
    pair -- no launch of it may end on its budget)."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    n = 4096
    kw = {} if terrain == "flat" else {"n_terrains": None, "stream_seeds": [1000 + i for i in range(n)]}
    a, b = _pair(n, terrain, monkeypatch, route=route, **kw)
    g = torch.Generator(device="cuda:0").manual_seed(1234)
    PS = M = 512
    pool = torch.rand(PS, n, 3, generator=g, device="cuda:0") * 2 - 1
    assert bench.launch_chunks(500, M, PS) == [500]
    j = _chunked_equal(a, b, pool, bench.launch_chunks(700, M, PS))  # burn-in + warm-up
    _chunked_equal(a, b, pool, bench.launch_chunks(500, M, PS), start=0)  # the timed window
    j = _chunked_equal(a, b, pool, [20], start=0)  # the driver's --steps 20 window, post burn-in
    for x, y in zip(a.get_state(), b.get_state()):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(a.terrain_rng(), b.terrain_rng()):  # (generators on perlin; None on flat), last draws
        assert (x is None and y is None) or np.array_equal(x, y)
    sa, sb = a.stats(), b.stats()
    assert sa == sb, (sa, sb)
    assert sa["resets"] > n // 2 and sb["pair_budget"] == 0
    if terrain == "perlin":
        assert sa["slow_path"] > 0 and b.pair_counters()["steps_full"] > 0  # the pair's full loop ran
    b.check()
    a.close(), b.close()


def test_relief_pair_budget_expiry_is_loud(monkeypatch):
    """A relief-pair launch that ends on its wall-clock budget must not pass silently.  With
    BB_PAIR_BUDGET_MS=1 a team that waits 1 ms for an env (teams outnumber the 512 envs 8:1, so
    most wait from the start) ends the launch: stats count it, check() raises, and every later
    step -- bb_step, bb_step_multi -- refuses until a full reset() clears the fault."""
    monkeypatch.setenv("BB_PAIR_BUDGET_MS", "1")  # read by bb_create
    monkeypatch.setenv("BB_ROUTE", "0")
    from ballbot_gym.envs import BallbotVecEnv

    n = 512
    env = BallbotVecEnv(n, device="cuda:0", seed=3, terrain_config={"type": "perlin", "config": {}},
                        stream_seeds=[80 + i for i in range(n)])
    g = torch.Generator(device="cuda:0").manual_seed(4)
    acts = torch.rand(64, n, 3, generator=g, device="cuda:0") * 2 - 1
    env.step_multi(acts)  # asynchronous: no error yet
    with pytest.raises(RuntimeError, match="wall-clock budget"):
        env.check()
    assert env.stats()["pair_budget"] >= 1
    with pytest.raises(RuntimeError, match="wall-clock budget"):
        env.step(acts[0])
    with pytest.raises(RuntimeError, match="wall-clock budget"):
        env.step_multi(acts)
    env.reset()  # a full reset gives every env a valid state: bb_reset waits for it and clears the fault
    env.step(acts[0])  # straight after the reset, no check() in between
    env.check()
    env.close()


@pytest.mark.parametrize("variant", [{"BB_PAIR_ONE": "0"}, {"BB_PAIR_SOLO": "64", "BB_PAIR_HEAVY": "100"},
                                     {"BB_PAIR_SEG": "4"}, {"BB_RELIEF_PAIR": "0"}],
                         ids=["two-launches", "solo-waves", "seg4", "work-queue"])
def test_relief_pair_forms_match(variant, monkeypatch):
    """The relief pair's other forms: two concurrent launches instead of one, solo
    waves for the heavy envs (envs above the mean cost of the last launch, from the second
    launch on), hand-overs every 4 steps, and round 3's work queue.  Each is route 0 and must
    equal one bb_step per step bit for bit, launch after launch."""
    for k, v in variant.items():
        monkeypatch.setenv(k, v)  # read by bb_create
    n = 512
    a, b = _pair(n, "perlin", monkeypatch, route="0", n_terrains=None, stream_seeds=[70 + i for i in range(n)],
                 max_ep_steps=200)
    g = torch.Generator(device="cuda:0").manual_seed(11)
    actions = torch.rand(256, n, 3, generator=g, device="cuda:0") * 2 - 1
    st = _compare_runs(a, b, actions, 32)
    assert st["slow_path"] > 0 and st["pair_budget"] == 0
    if "BB_PAIR_SOLO" in variant:
        assert b.pair_counters()["heavy"] > 0  # the last launch marked heavy envs for the solo waves
    a.close(), b.close()


def test_multi_step_rejects_bad_shapes():
    from ballbot_gym.envs import BallbotVecEnv

    env = BallbotVecEnv(64, device="cuda:0")
    with pytest.raises(ValueError):
        env.step_multi(torch.zeros(4, 32, 3, device="cuda:0"))
    with pytest.raises(ValueError):
        env.step_multi(torch.zeros(64, 3, device="cuda:0"))
    env.close()


@pytest.mark.parametrize("n", [1, 3, 17, 65])
@pytest.mark.parametrize("terrain,route", [("flat", "1"), ("perlin", "0")])
def test_ragged_env_counts(n, terrain, route, monkeypatch):
    """Env counts that fill no wave, workgroup or XCD label evenly (1: the reference's single env;
    3, 17, 65: partial teams, partial 32-env output blocks, labels without envs -- on perlin the
    relief pair's rings of the empty labels must still drain): bb_step_multi equals one bb_step
    per step bit for bit, with auto-resets."""
    kw = {"max_ep_steps": 20} if terrain == "flat" else {"n_terrains": None, "max_ep_steps": 60,
                                                         "stream_seeds": [40 + i for i in range(n)]}
    a, b = _pair(n, terrain, monkeypatch, route=route, **kw)
    g = torch.Generator(device="cuda:0").manual_seed(3 + n)
    actions = torch.rand(96, n, 3, generator=g, device="cuda:0") * 4 - 2
    st = _compare_runs(a, b, actions, 32)
    assert st["resets"] >= 1 and st["pair_budget"] == 0
    b.check()
    a.close(), b.close()
