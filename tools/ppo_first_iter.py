"""Where the first PPO iteration's extra time goes: wall time of each phase with a
device sync around it -- env and trainer construction, BatchedPPO.warm_up (when asked), then the
first three rollouts and updates.

    python tools/ppo_first_iter.py --terrain flat [--warm-up] [--out gpurun_out/x.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--n-steps", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--terrain", default="flat")
    ap.add_argument("--warm-up", action="store_true")
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--cprofile", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    t = {}

    def mark(name, t0):
        torch.cuda.synchronize()
        t[name] = round(time.perf_counter() - t0, 4)

    t0 = time.perf_counter()
    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO
    from ballbot_rl.training.schedules import lr_schedule

    kw = {} if a.terrain == "flat" else {"n_terrains": None}
    env = BallbotVecEnv(a.envs, device="cuda:0", seed=10, terrain_config={"type": a.terrain, "config": {}}, **kw)
    mark("env", t0)
    t0 = time.perf_counter()
    m = BatchedPPO(env, n_steps=a.n_steps, batch_size=a.batch, n_epochs=5, ent_coef=0.001, clip_range=0.015,
                   vf_coef=2.0, target_kl=0.3, learning_rate=lr_schedule, normalize_advantage=False, seed=10,
                   logger=CSVLogger(None, stdout=False))
    mark("ppo_ctor", t0)
    if a.warm_up:
        t0 = time.perf_counter()
        m.warm_up()
        mark("warm_up", t0)
    if a.probe:  # the first call of each piece of the first rollout, one at a time
        t0 = time.perf_counter()
        m._last_obs, _ = env.reset()
        mark("probe_reset", t0)
        t0 = time.perf_counter()
        m.policy.predict_values(torch.zeros(a.envs, 15, device="cuda:0"))
        mark("probe_predict_values", t0)
        b = m.buf
        t0 = time.perf_counter()
        m.gae_fn(b.rewards, b.values, b.starts, torch.zeros(a.envs, device="cuda:0"),
                 m._last_starts.contiguous(), m.gamma, m.gae_lambda)
        mark("probe_gae", t0)
        t0 = time.perf_counter()
        torch.randn(a.n_steps, a.envs, 3, device="cuda:0")
        mark("probe_randn", t0)
    for i in range(3):
        t0 = time.perf_counter()
        m.collect_rollouts()
        mark(f"rollout{i}", t0)
        t0 = time.perf_counter()
        if a.cprofile and i == 0:  # host-side breakdown of the first update
            import cProfile
            import pstats

            pr = cProfile.Profile()
            pr.enable()
            m.train()
            torch.cuda.synchronize()
            pr.disable()
            pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(30)
        else:
            m.train()
        mark(f"update{i}", t0)
    print(json.dumps({"terrain": a.terrain, "warm_up": a.warm_up, "times_s": t}), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(t))
    env.close()


if __name__ == "__main__":
    main()
