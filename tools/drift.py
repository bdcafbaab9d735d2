"""Free-running drift of the GPU step vs the fp64 oracle.

    python tools/drift.py --envs 64 --steps 400 --out profiles/r01_drift.json

Both sides start from the same reset state and receive the same action
sequence (the oracle's recorded PID+noise / random actions, tests/traj.py); no
teacher forcing, so per-step differences compound through the dynamics.  Per
step: ||qpos_gpu - qpos_oracle||_2 over the envs still in their first episode
(median, p99, max), and per env the first step where it exceeds 1e-3.
Reported for the fp64 and fp32 kernels, flat and hills.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "openballbot-rl_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))


def run(precision: str, terrain: str, n: int, T: int, seed: int):
    import torch

    import oracle_lib as O
    import traj
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_gym.terrain import generate_hills_terrain

    from ballbot_gym.envs.config import np_random
    from ballbot_gym.terrain.perlin import generate_perlin_terrain

    nt = None
    if terrain == "flat":
        hf, tcfg = O.flat_hfield(), {"type": "flat", "config": {}}
    elif terrain == "hills":
        hf = generate_hills_terrain(293, seed=7).astype(np.float32)
        tcfg = {"type": "hills", "config": {"seed": 7}}
    else:  # perlin: the GPU bank's slot 0 = first seed of np_random(0)
        s0 = int(np_random(0).integers(0, 10000))
        hf = generate_perlin_terrain(293, seed=s0).astype(np.float32)
        tcfg, nt = {"type": "perlin", "config": {}}, 1
    rec = traj.record(n_envs=n, n_steps=T, hfield=hf, seed=seed)
    alive = np.cumprod((rec["flags"] & 1) == 0, axis=0).astype(bool)  # still in the first episode after step t
    env = BallbotVecEnv(n, device="cuda:0", precision=precision, terrain_config=tcfg, auto_reset=False,
                        n_terrains=nt, seed=0)
    env.set_state(rec["qpos"][0], rec["qvel"][0], rec["warm"][0], rec["steps"][0])
    err = np.full((T, n), np.nan)
    for t in range(T):
        env.step(torch.tensor(rec["action"][t], device=env.device))
        q, _, _, _ = env.get_state()
        e = np.linalg.norm(q - rec["qpos1"][t], axis=1)
        err[t] = np.where(alive[t], e, np.nan)
    env.close()
    steps = {}
    for t in (1, 10, 50, 100, 200, T - 1):
        if t < T and np.isfinite(err[t]).any():
            v = err[t][np.isfinite(err[t])]
            steps[str(t + 1)] = {"median": float(np.median(v)), "p99": float(np.percentile(v, 99)),
                                 "max": float(v.max()), "envs": int(v.size)}
    t_cross = []
    for e in range(n):
        col = err[:, e]
        over = np.nonzero(np.nan_to_num(col, nan=0.0) > 1e-3)[0]
        live = int(np.isfinite(col).sum())
        t_cross.append(int(over[0]) + 1 if len(over) else None)
        _ = live
    crossed = [x for x in t_cross if x is not None]
    return {"precision": precision, "terrain": terrain, "envs": n, "steps": T,
            "qpos_l2_by_step": steps,
            "envs_crossing_1e-3": len(crossed),
            "steps_to_1e-3_median": float(np.median(crossed)) if crossed else None,
            "mean_first_episode_len": float(alive.sum(0).mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = [run(p, t, a.envs, a.steps, a.seed) for p in ("fp64", "fp32") for t in ("flat", "perlin")]  # hills seed 7 is flat around the start
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        Path(a.out).write_text(s)


if __name__ == "__main__":
    main()
