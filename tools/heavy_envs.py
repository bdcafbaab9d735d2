"""Which envs make the perlin relief pair's chain?  Runs the bench's perlin workload
(4096 envs, per-env generators, 700 burn-in/warm-up steps), then one 500-step pair launch, and
reports for the heaviest and the median envs (by the cycles their steps took in that launch): the
tilt, the episode step count, the contact counts of a forward at the launch's end, the full-step
share and the resets in the launch (GPU box).

    python tools/heavy_envs.py [--out gpurun_out/heavy.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))


def tilt_deg(q):
    import numpy as np

    w, x, y, z = q[3], q[4], q[5], q[6]
    zz = 1 - 2 * (x * x + y * y)  # R[2][2] of the base quaternion
    return float(np.degrees(np.arccos(np.clip(zz, -1, 1))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch

    from ballbot_gym.distributed import shard_stream_seeds
    from ballbot_gym.envs import BallbotVecEnv

    n = a.envs
    env = BallbotVecEnv(n, device="cuda:0", seed=1000, terrain_config={"type": "perlin", "config": {}},
                        stream_seeds=shard_stream_seeds(1000, 0, n))
    g = torch.Generator(device="cuda:0").manual_seed(1234)
    pool = torch.rand(512, n, 3, generator=g, device="cuda:0") * 2 - 1
    env.step_multi(pool)            # 512 burn-in steps
    env.step_multi(pool[:188])      # + 188 warm-up
    st0 = env.stats()
    q0, v0, w0, s0 = env.get_state()
    out = env.step_multi(pool[:500])  # the timed form: one 500-step launch
    torch.cuda.synchronize()
    cyc, fin = env.pair_env_times()
    q1, v1, w1, s1 = env.get_state()
    done = out["done"].cpu().numpy()  # [500][n]
    qacc, ncon = env.forward(np.zeros((n, 3)))
    order = np.argsort(cyc)[::-1]
    med = order[len(order) // 2]

    def info(e):
        e = int(e)
        return {"env": e, "mcycles": float(cyc[e]) / 1e6, "resets_in_launch": int((done[:, e] & 1).sum()),
                "failures_in_launch": int((done[:, e] & 2).sum() // 2), "tilt_deg_start": tilt_deg(q0[e]),
                "tilt_deg_end": tilt_deg(q1[e]), "episode_step_end": int(s1[e]), "base_z_end": float(q1[e][2]),
                "ball_z_end": float(q1[e][12]), "speed_end": float(np.linalg.norm(v1[e][9:12])),
                "ground_contacts_end": int(ncon[e, 0]), "body_contacts_end": int(ncon[e, 1])}

    res = {"pair": env.pair_counters(), "stats_delta": {k: env.stats()[k] - st0[k] for k in st0},
           "mcycles_percentiles": {p: float(np.percentile(cyc, p)) / 1e6 for p in (0, 50, 90, 99, 100)},
           "heaviest": [info(e) for e in order[:a.top]], "median": info(med),
           "median_of_all": {"body_contacts_end": float(np.median(ncon[:, 1])),
                             "resets_in_launch": float(np.median((done & 1).sum(0)))}}
    print(json.dumps(res, indent=1))
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))
    env.check()
    env.close()


if __name__ == "__main__":
    main()
