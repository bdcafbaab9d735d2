"""A/B timing of variant builds of csrc/bb_kernels.hip (diagnostic, GPU box).

  python tools/lib_bench.py --variant NAME:-DFLAG[,-DFLAG2] ... [--precision fp64]

Each variant is compiled into tools/_build/libbb_<NAME>.so (hipcc gfx950),
loaded in a fresh process and timed on the bench workload (4096 envs, flat,
random actions); prints one JSON line per variant.
"""
import argparse
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))


def build(name, flags):
    """tools/_build/libbb_<name>.so from csrc/bb_kernels.hip with extra flags (python tools/lib_bench.py --build-only)."""
    out = ROOT / "tools" / "_build" / f"libbb_{name}.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    from ballbot_gym import _native

    # one object per source with the product's per-source flags, then one link
    objs = []
    for f in _native.HIP_SOURCES:
        o = out.parent / f"{name}_{f[:-4]}.o"
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *flags,
                        *_native.SOURCE_FLAGS.get(f, []), "-c", "-o", str(o),
                        str(ROOT / "openballbot-rl_amd" / "csrc" / f)], check=True)
        objs.append(str(o))
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(out), *objs], check=True)
    return out


def run_one(lib, precision, terrain, steps, warmup, multi=0, rollout=False):
    import torch
    from ballbot_gym import _native
    from ballbot_gym.envs import BallbotVecEnv

    _native.use_diagnostic_library(lib)
    env = BallbotVecEnv(4096, device="cuda:0", precision=precision, terrain_config={"type": terrain, "config": {}},
                        n_terrains=None if terrain == "perlin" else 16)
    pool = torch.rand(64, 4096, 3, device="cuda:0") * 2 - 1
    if rollout:  # PPO collect_rollouts (4096 envs x 64 steps), BB_FUSED_ROLLOUT picks bb_rollout or per-step
        from ballbot_rl.training.logger import CSVLogger
        from ballbot_rl.training.ppo import BatchedPPO

        m = BatchedPPO(env, n_steps=64, batch_size=8192, n_epochs=1, seed=1, logger=CSVLogger(None, stdout=False))
        for _ in range(3):
            m.collect_rollouts()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = max(1, steps // 64)
        for _ in range(reps):
            m.collect_rollouts()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / (reps * 64)
        return {"ms": dt * 1e3, "env_steps_per_s": 4096 / dt, "rollout": True, "stats": env.stats()}
    if multi:  # bb_step_multi: `multi` steps per launch
        assert 64 % multi == 0
        o = torch.empty(multi, 4096, 15, device="cuda:0")
        r = torch.empty(multi, 4096, device="cuda:0")
        dn = torch.empty(multi, 4096, dtype=torch.uint8, device="cuda:0")
        for i in range(0, warmup, multi):
            env.step_multi_raw(pool[i % 64:i % 64 + multi], o, r, dn)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(0, steps, multi):
            env.step_multi_raw(pool[i % 64:i % 64 + multi], o, r, dn)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / (steps // multi * multi)
        return {"ms": dt * 1e3, "env_steps_per_s": 4096 / dt, "multi": multi, "stats": env.stats()}
    for i in range(warmup):
        env.step_async_raw(pool[i % 64])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        env.step_async_raw(pool[i % 64])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"ms": dt * 1e3, "env_steps_per_s": 4096 / dt, "stats": env.stats()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", default=[], help="NAME:-DFLAG,-DFLAG2 (empty flags allowed)")
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--terrain", default="flat")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--child", default=None)
    ap.add_argument("--multi", type=int, default=0, help="steps per bb_step_multi launch (0: bb_step per step)")
    ap.add_argument("--rollout", action="store_true", help="time PPO collect_rollouts instead of env steps")
    ap.add_argument("--no-build", action="store_true", help="use the prebuilt tools/_build/libbb_<NAME>.so")
    ap.add_argument("--build-only", action="store_true", help="compile the variants (here, on the CPU) and exit")
    a = ap.parse_args()
    if a.build_only:
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(8) as ex:
            list(ex.map(lambda v: build(v.partition(":")[0], [f for f in v.partition(":")[2].split(",") if f]), a.variant))
        return
    if a.child:
        print(json.dumps(run_one(a.child, a.precision, a.terrain, a.steps, a.warmup, a.multi, a.rollout)))
        return
    for v in a.variant:
        name, _, fl = v.partition(":")
        lib = (ROOT / "tools" / "_build" / f"libbb_{name}.so") if a.no_build else build(name, [f for f in fl.split(",") if f])
        r = subprocess.run([sys.executable, __file__, "--child", str(lib), "--precision", a.precision,
                            "--terrain", a.terrain, "--steps", str(a.steps), "--warmup", str(a.warmup),
                            "--multi", str(a.multi)] + (["--rollout"] if a.rollout else []),
                           capture_output=True, text=True, timeout=600)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-2000:]
        print(json.dumps({"variant": name, "flags": fl, "precision": a.precision, "terrain": a.terrain, "multi": a.multi,
                          "result": json.loads(line) if r.returncode == 0 else line}), flush=True)


if __name__ == "__main__":
    main()
