"""Algorithmic FLOPs per env-step by config, from the
op-counting build of the oracle (oracle/flopcount.cpp -> oracle/_build/libbb_flops.so).

python tools/flops.py [--envs 64] [--steps 200] [--out profiles/r03_flops.json]

Counts the restated reference algorithm (MuJoCo's mj_step for this model +
env glue) at MuJoCo's solver tolerance, under uniform random actions with
auto-reset, after an uncounted burn-in from the reset state (the same
steady-state mix of episode ages bench.py times), per terrain config: flat (configs[1]),
hills and perlin (configs[2]).  FLOP = add/sub + mul + div + sqrt +
transcendental, one each; per-phase breakdown included.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))

PHASES = ("kinematics_mass_bias", "collision", "constraint_assembly", "newton_solver", "rk4_glue")
KINDS = ("add_sub", "mul", "div", "sqrt", "transcendental", "compare")
LIB = ROOT / "oracle" / "_build" / "libbb_flops.so"


_L = None


def lib():
    global _L
    if _L is not None:
        return _L
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    L = C.CDLL(str(LIB))
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int)
    L.bbo_count_prepare.argtypes = []
    L.bbo_count_flops_replay.argtypes = [C.c_int, C.c_int, dp, dp, dp, ip, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                         dp, ip, C.c_int, C.c_double, dp, ip]
    L.bbo_count_flops_replay.restype = C.c_longlong
    L.bbo_count_prepare()
    _L = L
    L.bbo_count_flops.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float), C.c_double, C.c_double, C.c_double,
                                  C.c_uint, C.POINTER(C.c_double)]
    L.bbo_count_flops.restype = C.c_longlong
    return L


def count_replay(q, v, w, sc, actions, table, offsets, terr, size_z, threads=8) -> dict:
    """Algorithmic FLOPs of the bench's own timed mix: envs replayed from their states at the
    start of the timed window with the window's actions ([T][n][3]) and their own next terrain
    draws (terr[n][max_ep] rows into table[slots][293*293] / offsets[slots]), split over host
    threads (oracle/flopcount.cpp bbo_count_flops_replay: thread-local counters)."""
    from concurrent.futures import ThreadPoolExecutor

    L = lib()
    n = q.shape[0]
    T = actions.shape[0]
    table = np.ascontiguousarray(table, np.float32)
    offsets = np.ascontiguousarray(offsets, np.float64)
    chunks = [c for c in np.array_split(np.arange(n), max(1, min(threads, n))) if len(c)]

    def work(idx):
        qq = np.ascontiguousarray(q[idx], np.float64); vv = np.ascontiguousarray(v[idx], np.float64)
        ww = np.ascontiguousarray(w[idx], np.float64); ss = np.ascontiguousarray(sc[idx], np.int32)
        aa = np.ascontiguousarray(actions[:, idx], np.float32)
        tt = np.ascontiguousarray(terr[idx], np.int32)
        out = np.zeros(30)
        over = C.c_int(0)
        f, dp, ip = C.POINTER(C.c_float), C.POINTER(C.c_double), C.POINTER(C.c_int)
        steps = L.bbo_count_flops_replay(len(idx), T, qq.ctypes.data_as(dp), vv.ctypes.data_as(dp),
                                         ww.ctypes.data_as(dp), ss.ctypes.data_as(ip), aa.ctypes.data_as(f),
                                         table.ctypes.data_as(f), offsets.ctypes.data_as(dp), tt.ctypes.data_as(ip),
                                         tt.shape[1], float(size_z), out.ctypes.data_as(dp), C.byref(over))
        return steps, out, over.value

    t0 = time.perf_counter()
    with ThreadPoolExecutor(len(chunks)) as ex:
        res = list(ex.map(work, chunks))
    steps = sum(r[0] for r in res)
    a = sum(r[1] for r in res).reshape(5, 6) / max(steps, 1)
    flop_phase = {p: float(a[i, :5].sum()) for i, p in enumerate(PHASES)}
    return {"env_steps": int(steps), "seconds": round(time.perf_counter() - t0, 2), "threads": len(chunks),
            "flops_per_env_step": float(a[:, :5].sum()), "flops_by_phase": flop_phase,
            "terrain_overrun_resets": int(sum(r[2] for r in res))}


def count(L, hf: np.ndarray, size_z: float, n_envs: int, n_steps: int, seed: int = 1, burn_in: int = 0) -> dict:
    from ballbot_gym.envs.config import init_offset

    hf = np.ascontiguousarray(hf, np.float32).ravel()
    out = (C.c_double * 30)()
    t0 = time.perf_counter()
    steps = L.bbo_count_flops(n_envs, burn_in, n_steps, hf.ctypes.data_as(C.POINTER(C.c_float)), size_z,
                              init_offset(hf, size_z), 1.0, seed, out)
    dt = time.perf_counter() - t0
    a = np.array(out[:]).reshape(5, 6)
    per_phase = {p: {k: float(a[i, j]) for j, k in enumerate(KINDS)} for i, p in enumerate(PHASES)}
    flop_phase = {p: float(a[i, :5].sum()) for i, p in enumerate(PHASES)}
    return {"env_steps": int(steps), "seconds": round(dt, 2), "flops_per_env_step": float(a[:, :5].sum()),
            "flops_by_phase": flop_phase, "ops_by_phase": per_phase}


def configs():
    from ballbot_gym.terrain import generate_hills_terrain
    from ballbot_gym.terrain.perlin import generate_perlin_terrain

    return {"flat": (np.zeros(293 * 293, np.float32), 2.0),
            "hills_seed7": (generate_hills_terrain(293, seed=7).astype(np.float32), 2.0),
            "perlin_seed7765": (generate_perlin_terrain(293, seed=7765).astype(np.float32), 2.0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--burn-in", type=int, default=400, help="uncounted steps first (steady-state episode mix)")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r03_flops.json"))
    a = ap.parse_args()
    L = lib()
    res = {"what": "algorithmic FLOPs per env-step of the restated reference algorithm (oracle op-counter, "
                   "MuJoCo tolerance 1e-8, uniform random actions, auto-reset, "
                   "counted after an uncounted burn-in from the reset state)",
           "envs": a.envs, "burn_in": a.burn_in, "steps": a.steps, "configs": {}}
    for name, (hf, sz) in configs().items():
        res["configs"][name] = count(L, hf, sz, a.envs, a.steps, burn_in=a.burn_in)
        print(name, json.dumps({k: v for k, v in res["configs"][name].items() if k != "ops_by_phase"}), flush=True)
    Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
