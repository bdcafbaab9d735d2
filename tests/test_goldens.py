"""Restatements vs golden vectors generated from the reference's own modules
(tools/gen_goldens.py).  CPU only.

Pinned bit-for-bit: every numpy terrain generator (incl. mixed), the reward
plugins, gymnasium seed streams and the registry/factory error contract.
PID (torch float32 in the reference vs numpy float32 here) within 1e-5."""
import json
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden"


def _meta(name):
    return json.loads((GOLD / name).read_text())


@pytest.mark.parametrize("case", _meta("terrains.json"), ids=lambda m: m["key"])
def test_terrain_generators_match_reference(case):
    import ballbot_gym.terrain as T

    ref = np.load(GOLD / "terrains.npz")[case["key"]]
    out = T.BUILTIN_TERRAINS[case["type"]](case["n"], **json.loads(json.dumps(case["config"])))
    assert out.shape == (case["n"] ** 2,) and out.dtype == np.float64
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("case", _meta("mixed.json"), ids=lambda m: m["key"])
def test_mixed_terrain_matches_reference(case):
    import ballbot_gym.terrain as T

    ref = np.load(GOLD / "mixed.npz")[case["key"]]
    out = T.generate_mixed_terrain(case["n"], **json.loads(json.dumps(case["config"])))
    np.testing.assert_array_equal(out, ref)


def test_terrain_properties():
    """Reference test_terrains.py checks: shape, [0,1], same seed -> same field."""
    import ballbot_gym.terrain as T

    for name, fn in T.BUILTIN_TERRAINS.items():
        if name == "mixed":
            continue
        a = fn(33, seed=3)
        assert a.shape == (33 * 33,) and a.min() >= 0.0 and a.max() <= 1.0, name
        np.testing.assert_array_equal(a, fn(33, seed=3))
    with pytest.raises(AssertionError, match="odd"):
        T.generate_hills_terrain(32)


def test_rewards_match_reference():
    from ballbot_gym.rewards import DirectionalReward, DistanceReward

    g = np.load(GOLD / "rewards.npz")
    for t, tgt in enumerate(g["targets"]):
        r = DirectionalReward(tgt)
        out = np.array([r({"vel": v}) for v in g["vel"]])
        np.testing.assert_array_equal(out, g["directional"][t])
        assert isinstance(r({"vel": g["vel"][0]}), np.float32)
    for k, goal in enumerate(g["goals"]):
        r = DistanceReward(goal, scale=g["scales"][k])
        out = np.array([r({"pos2d": p}) for p in g["pos2d"]])
        np.testing.assert_array_equal(out, g["distance"][k])
    with pytest.raises(ValueError, match="pos2d"):
        DistanceReward(np.zeros(2))({"vel": np.zeros(3)})


def test_pid_matches_reference():
    from pid_ref import PID

    g = np.load(GOLD / "pid.npz")
    pid = PID(float(g["dt"]), *g["gains"])
    for t in range(len(g["R"])):
        c = pid.act(g["R"][t])
        np.testing.assert_allclose(c, g["ctrl"][t], rtol=1e-5, atol=1e-4)


def test_seed_streams_match_gymnasium():
    from ballbot_gym.envs.config import TERRAIN_SEED_HIGH, np_random

    ref = json.loads((GOLD / "seeds.json").read_text())
    for seed, draws in ref.items():
        got = np_random(int(seed)).integers(0, TERRAIN_SEED_HIGH, size=len(draws))
        assert got.tolist() == draws
    assert ref["10"][:4] == [7765, 9560, 2640, 2076]


@pytest.fixture
def clean_registry():
    from ballbot_gym.core.registry import ComponentRegistry as R

    saved = {k: dict(v) for k, v in vars(R).items() if k.startswith("_") and isinstance(v, dict)}
    R.clear()
    yield R
    for k, v in saved.items():
        getattr(R, k).clear()
        getattr(R, k).update(v)


def test_registry_and_factory_errors_match_reference(clean_registry):
    from ballbot_gym.core import factories as fac
    from ballbot_gym.rewards import DirectionalReward, DistanceReward

    R = clean_registry
    R.register_reward("directional", DirectionalReward)
    R.register_reward("distance", DistanceReward)
    R.register_terrain("flat", lambda n, **kw: np.zeros(n * n))
    R.register_policy("mlp", object)
    cases = {
        "dup_reward": lambda: R.register_reward("directional", DirectionalReward),
        "bad_reward_class": lambda: R.register_reward("x", int),
        "unknown_reward": lambda: R.get_reward("nope"),
        "dup_terrain": lambda: R.register_terrain("flat", lambda n: None),
        "noncallable_terrain": lambda: R.register_terrain("t2", 5),
        "unknown_terrain": lambda: R.get_terrain("nope"),
        "dup_policy": lambda: R.register_policy("mlp", object),
        "unknown_policy": lambda: R.get_policy("nope"),
        "unknown_sensor": lambda: R.get_sensor("nope"),
        "reward_not_dict": lambda: fac.create_reward([1]),
        "reward_no_type": lambda: fac.create_reward({}),
        "directional_no_target": lambda: fac.create_reward({"type": "directional", "config": {}}),
        "distance_no_goal": lambda: fac.create_reward({"type": "distance", "config": {}}),
        "unknown_reward_factory": lambda: fac.create_reward({"type": "zzz", "config": {}}),
        "distance_bad_shape": lambda: fac.create_reward({"type": "distance", "config": {"goal_position": [1, 2, 3]}}),
        "terrain_not_dict": lambda: fac.create_terrain("flat"),
        "terrain_no_type": lambda: fac.create_terrain({"config": {}}),
        "unknown_terrain_factory": lambda: fac.create_terrain({"type": "zzz"}),
        "policy_no_type": lambda: fac.create_policy({}),
        "unknown_policy_factory": lambda: fac.create_policy({"type": "zzz"}),
        "validate_not_dict": lambda: fac.validate_config(3, "reward"),
        "validate_no_type": lambda: fac.validate_config({}, "reward"),
        "validate_bad_component": lambda: fac.validate_config({"type": "flat"}, "widget"),
        "validate_unknown_terrain": lambda: fac.validate_config({"type": "zzz"}, "terrain"),
        "validate_unknown_reward": lambda: fac.validate_config({"type": "zzz"}, "reward"),
        "validate_unknown_policy": lambda: fac.validate_config({"type": "zzz"}, "policy"),
    }
    ref = json.loads((GOLD / "errors.json").read_text())
    for name, fn in cases.items():
        try:
            fn()
            got = None
        except Exception as e:  # noqa: BLE001
            got = {"type": type(e).__name__, "msg": str(e)}
        assert got == ref[name], name
    lists = ref["_lists"]
    assert R.list_rewards() == lists["rewards"] and R.list_terrains() == lists["terrains"]
    assert R.list_policies() == lists["policies"] and R.list_sensors() == lists["sensors"]


def test_perlin_properties():
    """Perlin parity is UNPINNED (noise.snoise2 is absent); the reference's own
    checks (test_terrains.py:22-44) plus value range and smoothness."""
    from ballbot_gym.terrain import BUILTIN_TERRAINS
    from ballbot_gym.core.factories import create_terrain

    a = BUILTIN_TERRAINS["perlin"](129, seed=42)
    assert a.shape == (129 * 129,) and a.min() >= 0.0 and a.max() <= 1.0
    np.testing.assert_array_equal(a, BUILTIN_TERRAINS["perlin"](129, seed=42))
    assert not np.allclose(a, BUILTIN_TERRAINS["perlin"](129, seed=43))
    assert 0.3 < a.mean() < 0.7 and a.std() > 0.05
    g = a.reshape(129, 129)
    assert np.abs(np.diff(g, axis=0)).max() < 0.2 and np.abs(np.diff(g, axis=1)).max() < 0.2
    t = create_terrain({"type": "perlin", "config": {"scale": 25.0, "octaves": 4, "seed": 42}})(129)
    np.testing.assert_array_equal(t, a)
    grad = BUILTIN_TERRAINS["gradient"](33, gradient_type="perlin", seed=5)
    assert grad.min() == 0.0 and grad.max() == 1.0
