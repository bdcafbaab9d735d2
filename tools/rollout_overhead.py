"""Where the PPO rollout's wall time goes (GPU box): the env step alone, the
fused rollout (policy + env + bookkeeping), and the host time per step with
the GPU kept idle (a sync after every step).  One JSON line."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))


def main():
    import torch

    from ballbot_gym.envs import BallbotVecEnv
    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO

    env = BallbotVecEnv(4096, device="cuda:0", seed=10)
    m = BatchedPPO(env, n_steps=64, batch_size=8192, n_epochs=5, seed=10, logger=CSVLogger(None, stdout=False))
    a = torch.zeros(4096, 3, device="cuda:0")
    out = {}
    for _ in range(2):
        m.collect_rollouts()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(64):
        env.step_flags(a)
    torch.cuda.synchronize()
    out["env_step_ms"] = (time.perf_counter() - t) / 64 * 1e3
    t = time.perf_counter()
    for _ in range(4):
        m.collect_rollouts()
    torch.cuda.synchronize()
    out["collect_ms_per_step"] = (time.perf_counter() - t) / 256 * 1e3
    m.n_steps_saved = m.n_steps
    # host cost of the rollout loop body with the GPU drained after each step
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host, gpu = 0.0, 0.0
    orig = env.step_flags

    def timed_step(x):
        nonlocal host, gpu
        torch.cuda.synchronize()
        ev0.record()
        r = orig(x)
        ev1.record()
        torch.cuda.synchronize()
        gpu += ev0.elapsed_time(ev1)
        return r

    env.step_flags = timed_step
    t = time.perf_counter()
    m.collect_rollouts()
    torch.cuda.synchronize()
    out["collect_synced_ms_per_step"] = (time.perf_counter() - t) / 64 * 1e3
    out["env_step_gpu_ms_synced"] = gpu / 64
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
