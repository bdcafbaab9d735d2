"""Generate golden vectors from the reference's importable Python modules.

Run HERE (the container that has /root/reference), never on the GPU box:

    python tools/gen_goldens.py            # writes tests/golden/*.npz|json

The reference modules are imported by file path with a stub
`ballbot_gym` package so that core/registry.py, core/factories.py and
terrain/mixed.py resolve their imports.  Only their OUTPUTS are written, as
data (inputs + expected outputs); no reference source travels.

What is pinned (consumers in tests/test_goldens.py):
  terrains.npz   every numpy terrain generator at n=33/65 (default and varied
                 configs) + hills/sinusoidal at n=293, float64
  rewards.npz    DirectionalReward / DistanceReward on random states
  pid.npz        PID.act trajectories on random rotations (torch)
  seeds.json     gymnasium np_random streams (PCG64(SeedSequence(seed)))
                 .integers(0, 10000) as used by _reset_terrain
  errors.json    ComponentRegistry / factory error messages
Not pinnable here: perlin (needs `noise.snoise2`, absent) and MuJoCo itself.
"""
from __future__ import annotations

import importlib.util
import json
import sys
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference/ballbot_gym")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden"


def _load(modname: str, path: Path):
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def _stub_package():
    """Minimal ballbot_gym package tree so that registry/factories import."""
    for name in ("ballbot_gym", "ballbot_gym.core", "ballbot_gym.rewards", "ballbot_gym.terrain"):
        pkg = types.ModuleType(name)
        pkg.__path__ = []
        sys.modules[name] = pkg
    base = _load("ballbot_gym.rewards.base", REF / "rewards" / "base.py")
    reg = _load("ballbot_gym.core.registry", REF / "core" / "registry.py")
    d = _load("ballbot_gym.rewards.directional", REF / "rewards" / "directional.py")
    dist = _load("ballbot_gym.rewards.distance", REF / "rewards" / "distance.py")
    fac = _load("ballbot_gym.core.factories", REF / "core" / "factories.py")
    return base, reg, d, dist, fac


TERRAIN_CASES = [
    # (generator file, function, kwargs)
    ("stepped", "generate_stepped_terrain", {}),
    ("stepped", "generate_stepped_terrain", {"num_steps": 3, "step_height": 0.25, "seed": 4}),
    ("ramp", "generate_ramp_terrain", {}),
    ("ramp", "generate_ramp_terrain", {"ramp_direction": "y", "ramp_angle": 10.0, "flat_ratio": 0.5}),
    ("ramp", "generate_ramp_terrain", {"ramp_direction": "x", "num_ramps": 3, "flat_ratio": 0.2}),
    ("ramp", "generate_ramp_terrain", {"ramp_direction": "y", "num_ramps": 2}),
    ("ramp", "generate_ramp_terrain", {"ramp_direction": "radial", "flat_ratio": 0.4}),
    ("sinusoidal", "generate_sinusoidal_terrain", {}),
    ("sinusoidal", "generate_sinusoidal_terrain", {"direction": "x", "amplitude": 0.3, "frequency": 0.05, "phase": 0.7}),
    ("sinusoidal", "generate_sinusoidal_terrain", {"direction": "y"}),
    ("ridge_valley", "generate_ridge_valley_terrain", {}),
    ("ridge_valley", "generate_ridge_valley_terrain", {"orientation": "y", "smoothness": 0.0}),
    ("ridge_valley", "generate_ridge_valley_terrain", {"orientation": "diagonal", "smoothness": 0.9, "spacing": 1.5}),
    ("hills", "generate_hills_terrain", {}),
    ("hills", "generate_hills_terrain", {"num_hills": 9, "hill_height": 0.4, "hill_radius": 0.1, "seed": 17}),
    ("bowl", "generate_bowl_terrain", {}),
    ("bowl", "generate_bowl_terrain", {"depth": 0.9, "radius": 0.7, "center_x": 0.3, "center_y": 0.6}),
    ("gradient", "generate_gradient_terrain", {}),
    ("gradient", "generate_gradient_terrain", {"gradient_type": "linear", "direction": "y", "max_slope": 5.0}),
    ("gradient", "generate_gradient_terrain", {"gradient_type": "radial", "max_slope": 25.0}),
    ("terraced", "generate_terraced_terrain", {}),
    ("terraced", "generate_terraced_terrain", {"num_terraces": 3, "terrace_height": 0.3, "transition_width": 0.3,
                                               "direction": "y"}),
    ("wavy", "generate_wavy_terrain", {}),
    ("wavy", "generate_wavy_terrain", {"wave_amplitudes": [0.4, 0.1], "wave_frequencies": [1.0, 3.0],
                                       "wave_directions": [30.0, 120.0], "phase_offsets": [0.2, 0.0]}),
    ("spiral", "generate_spiral_terrain", {}),
    ("spiral", "generate_spiral_terrain", {"direction": "ccw", "spiral_tightness": 2.0, "height_variation": 0.8,
                                           "center_x": 0.4}),
]


def gen_terrains():
    out = {}
    meta = []
    for k, (fname, fn, kw) in enumerate(TERRAIN_CASES):
        mod = _load(f"ref_terrain_{fname}", REF / "terrain" / f"{fname}.py")
        for n in (33, 65):
            arr = getattr(mod, fn)(n, **json.loads(json.dumps(kw)))
            key = f"case{k}_n{n}"
            out[key] = np.asarray(arr, np.float64)
            meta.append({"key": key, "type": fname, "n": n, "config": kw})
    hills = _load("ref_terrain_hills", REF / "terrain" / "hills.py")
    sinus = _load("ref_terrain_sinusoidal", REF / "terrain" / "sinusoidal.py")
    for seed in (0, 7, 7765):
        key = f"hills293_seed{seed}"
        out[key] = np.asarray(hills.generate_hills_terrain(293, seed=seed), np.float64)
        meta.append({"key": key, "type": "hills", "n": 293, "config": {"seed": seed}})
    out["sinusoidal293"] = np.asarray(sinus.generate_sinusoidal_terrain(293), np.float64)
    meta.append({"key": "sinusoidal293", "type": "sinusoidal", "n": 293, "config": {}})
    np.savez_compressed(OUT / "terrains.npz", **out)
    (OUT / "terrains.json").write_text(json.dumps(meta, indent=1))


def gen_mixed(fac, reg):
    """terrain/mixed.py through the reference registry (needs create_terrain)."""
    mods = {}
    for fname, fn in (("hills", "generate_hills_terrain"), ("sinusoidal", "generate_sinusoidal_terrain"),
                      ("bowl", "generate_bowl_terrain"), ("ramp", "generate_ramp_terrain")):
        mods[fname] = getattr(_load(f"ref_terrain_{fname}", REF / "terrain" / f"{fname}.py"), fn)
    reg.ComponentRegistry.clear()
    for name, f in mods.items():
        reg.ComponentRegistry.register_terrain(name, f)
    mixed = _load("ballbot_gym.terrain.mixed", REF / "terrain" / "mixed.py")
    cases = [
        ({"components": [{"type": "hills", "weight": 0.7, "config": {"num_hills": 3}},
                         {"type": "sinusoidal", "weight": 0.3, "config": {"amplitude": 0.4}}],
          "blend_mode": "additive", "seed": 5}),
        ({"components": [{"type": "bowl", "weight": 1.0}, {"type": "ramp", "weight": 0.5,
                                                           "config": {"ramp_direction": "y"}}],
          "blend_mode": "max"}),
        ({"components": [{"type": "hills", "weight": 2.0}, {"type": "bowl", "weight": 1.0}],
          "blend_mode": "weighted", "seed": 3}),
    ]
    out, meta = {}, []
    for k, kw in enumerate(cases):
        for n in (33, 65):
            arr = mixed.generate_mixed_terrain(n, **json.loads(json.dumps(kw)))
            out[f"mixed{k}_n{n}"] = np.asarray(arr, np.float64)
            meta.append({"key": f"mixed{k}_n{n}", "n": n, "config": kw})
    np.savez_compressed(OUT / "mixed.npz", **out)
    (OUT / "mixed.json").write_text(json.dumps(meta, indent=1))


def gen_rewards(d, dist):
    rng = np.random.default_rng(0)
    n = 256
    vel = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    pos2d = rng.uniform(-3, 3, (n, 2)).astype(np.float32)
    targets = np.array([[0, 1], [1, 0], [0.6, 0.8], [-0.7071, 0.7071]], np.float32)
    goals = np.array([[0, 0], [1.5, -2.0], [-3, 0.5]], np.float32)
    scales = np.array([1.0, 0.5, 2.0])
    dirv = np.zeros((len(targets), n), np.float64)
    for t, tgt in enumerate(targets):
        r = d.DirectionalReward(tgt)
        for i in range(n):
            dirv[t, i] = r({"vel": vel[i]})
    distv = np.zeros((len(goals), n), np.float64)
    for g, goal in enumerate(goals):
        r = dist.DistanceReward(goal, scale=scales[g])
        for i in range(n):
            distv[g, i] = r({"pos2d": pos2d[i]})
    np.savez_compressed(OUT / "rewards.npz", vel=vel, pos2d=pos2d, targets=targets, goals=goals, scales=scales,
                        directional=dirv, distance=distv)


def gen_pid():
    import torch

    pid_mod = _load("ref_pid", REF / "controllers" / "pid.py")
    rng = np.random.default_rng(1)
    T = 64
    rv = rng.normal(0, 0.25, (T, 3))
    Rs = []
    for v in rv:
        th = np.linalg.norm(v)
        k = v / th
        K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        Rs.append(np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K)
    Rs = np.array(Rs, np.float32)
    pid = pid_mod.PID(0.002, 20, 15, 2)
    ctrl = np.zeros((T, 3), np.float32)
    ang = np.zeros(T)
    for t in range(T):
        c, a = pid.act(torch.tensor(Rs[t]))
        ctrl[t] = c.numpy()
        ang[t] = a
    np.savez_compressed(OUT / "pid.npz", R=Rs, ctrl=ctrl, angle=ang, dt=0.002, gains=np.array([20, 15, 2.0]))


def gen_seeds():
    out = {}
    for seed in (0, 1, 10, 42, 1234):
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        out[str(seed)] = [int(x) for x in g.integers(0, 10000, size=16)]
    (OUT / "seeds.json").write_text(json.dumps(out, indent=1))


def _msg(fn):
    try:
        fn()
    except Exception as e:  # noqa: BLE001 - we record the message
        return {"type": type(e).__name__, "msg": str(e)}
    return None


def gen_errors(base, reg, d, dist, fac):
    R = reg.ComponentRegistry
    R.clear()
    R.register_reward("directional", d.DirectionalReward)
    R.register_reward("distance", dist.DistanceReward)
    R.register_terrain("flat", lambda n, **kw: np.zeros(n * n))
    R.register_policy("mlp", object)
    cases = {
        "dup_reward": lambda: R.register_reward("directional", d.DirectionalReward),
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
    out = {k: _msg(f) for k, f in cases.items()}
    out["_lists"] = {"rewards": R.list_rewards(), "terrains": R.list_terrains(), "policies": R.list_policies(),
                     "sensors": R.list_sensors()}
    (OUT / "errors.json").write_text(json.dumps(out, indent=1))


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    base, reg, d, dist, fac = _stub_package()
    gen_terrains()
    gen_mixed(fac, reg)
    gen_rewards(d, dist)
    gen_pid()
    gen_seeds()
    gen_errors(base, reg, d, dist, fac)
    for p in sorted(OUT.iterdir()):
        print(f"{p.name:20s} {p.stat().st_size:9d} B")


if __name__ == "__main__":
    main()
