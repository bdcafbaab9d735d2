"""Host-side cost of enqueueing one bb_step_multi launch from Python (diagnostic, GPU box).

The driver's 20-step window is one launch: the GPU idles while the host enqueues it, so that
time is part of the line.  Times, per call: the six tensor slices bench.py makes, the stream
lookup, the C call with precomputed arguments, and the whole step_multi_raw.

  python tools/launch_overhead.py [--envs 4096] [--reps 200]
"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))

import torch  # noqa: E402

from ballbot_gym import _native as N  # noqa: E402
from ballbot_gym.envs import BallbotVecEnv  # noqa: E402


def per_call(fn, reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = (time.perf_counter() - t) / reps * 1e6
    torch.cuda.synchronize()
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    env = BallbotVecEnv(a.envs, device=dev)
    env.reset()
    n, K = a.envs, 1
    pool = torch.rand(8, n, 3, device=dev) * 2 - 1
    mo = torch.empty(8, n, 15, device=dev)
    mr = torch.empty(8, n, device=dev)
    md = torch.empty(8, n, dtype=torch.uint8, device=dev)
    mt = torch.empty(8, n, 15, device=dev)
    mp = torch.empty(8, n, 2, device=dev)
    for _ in range(20):  # warm: code objects loaded, queues created
        env.step_multi_raw(pool[:K], mo[:K], mr[:K], md[:K], mt[:K], mp[:K])
    torch.cuda.synchronize()
    out = {}
    out["slices_us"] = per_call(lambda: (pool[0:K], mo[:K], mr[:K], md[:K], mt[:K], mp[:K]), a.reps)
    out["stream_us"] = per_call(env._stream, a.reps)
    args = (env._h, C.c_void_p(pool.data_ptr()), K, C.c_void_p(mo.data_ptr()), C.c_void_p(mr.data_ptr()),
            C.c_void_p(md.data_ptr()), C.c_void_p(mt.data_ptr()), C.c_void_p(mp.data_ptr()), int(env.auto_reset),
            env._stream())
    f = N.lib().bb_step_multi
    out["c_call_us"] = per_call(lambda: f(*args), a.reps)
    out["step_multi_raw_us"] = per_call(lambda: env.step_multi_raw(pool[:K], mo[:K], mr[:K], md[:K], mt[:K], mp[:K]),
                                        a.reps)
    env.time_kernel(a.reps)
    out["c_call_timed_events_us"] = per_call(lambda: f(*args), a.reps)
    ev = torch.cuda.Event(enable_timing=True)
    out["torch_event_record_us"] = per_call(ev.record, a.reps)
    # the bench's case: the first launch after a synchronize (the GPU idle while it is enqueued)
    ts, tc = [], []
    for _ in range(50):
        torch.cuda.synchronize()
        t = time.perf_counter()
        env.step_multi_raw(pool[:K], mo[:K], mr[:K], md[:K], mt[:K], mp[:K])
        ts.append(time.perf_counter() - t)
    for _ in range(50):
        torch.cuda.synchronize()
        t = time.perf_counter()
        f(*args)
        tc.append(time.perf_counter() - t)
    ts.sort(); tc.sort()
    out["after_sync_step_multi_raw_us_median"] = ts[len(ts) // 2] * 1e6
    out["after_sync_step_multi_raw_us_max"] = ts[-1] * 1e6
    out["after_sync_c_call_us_median"] = tc[len(tc) // 2] * 1e6
    out["after_sync_c_call_us_max"] = tc[-1] * 1e6
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()
