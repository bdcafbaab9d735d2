"""bench.py -- env-steps/sec of the batched ballbot hot path on MI355X.

One "step" = one env.step of every env (one fused HIP launch: RK4 mj_step +
obs + reward + termination + auto-reset) over a batch of synthetic random
actions already resident in HBM.  Workload = BASELINE.json configs[1]:
4096 envs per GPU, flat terrain, random actions.  Multi-GPU: one process per
GPU (torchrun), envs sharded with no data-path collective (weak scaling);
the MAX elapsed time over ranks is used.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import platform
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT / "openballbot-rl_amd", ROOT / "tests"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X spec: half the 157.3 TF FP32 vector rate (MI355X_MICROARCH.md)
# the yardstick of roofline.achieved: the oracle's op count (oracle/flopcount.cpp) of MuJoCo's solver
# as restated since round 5 (PrimalSearch line search, warm-start choice); rounds before 5 counted
# the kernel-borrowed search (825,731 FLOP per flat env-step in round 4 against 942,434 now)
FLOP_BASIS = "oracle-PrimalSearch-r5"


def algorithmic_bytes(precision: str, steps_per_launch: float = 1, relief: bool = False) -> float:
    """HBM bytes one env-step must move: action in, obs/reward/done/terminal
    obs/pos2d out, and the env's state (qpos, qvel, qacc_warmstart, step
    counter, terrain id) read and written once per launch -- every step with one
    bb_step launch per step, once per K steps with bb_step_multi (the state
    stays on chip between its steps).  relief: + the heightfield vertices under
    the ball's AABB, 7 x 7 float32 per forward read once per env-step (SURVEY.md
    §8 D4: +196 B on uneven terrain)."""
    es = 8 if precision == "fp64" else 4
    state = (17 + 15 + 15) * es      # qpos, qvel, qacc_warmstart
    per_launch = 2 * state + 8 + 4   # r/w state, step counter r/w, terrain id
    out = 60 + 4 + 1 + 60 + 8        # obs, reward, done, terminal obs, pos2d
    return per_launch / steps_per_launch + 12 + out + (196 if relief else 0)


def profile_entry(path: Path, precision: str, terrain: str, envs: int, spl: float) -> dict:
    """The rocprofv3 summary (profiles/traffic.json, written by tools/prof_summary.py) of exactly
    this launch shape: precision, terrain, envs per GPU and steps per launch must all match, else
    {} -- a 512-step profile says nothing about a 20-step launch."""
    try:
        tab = json.loads(path.read_text())
    except Exception:
        return {}
    for e in tab.values():
        if (e.get("precision") == precision and e.get("terrain", "flat") == terrain and e.get("envs") == envs
                and abs(float(e.get("steps_per_launch", -1)) - spl) < 1e-9):
            return e
    return {}


def committed_flops(terrain: str):
    """The timed-mix FLOP count committed for this terrain (profiles/flops.json, tools/flops.py)."""
    try:
        e = json.loads((ROOT / "profiles" / "flops.json").read_text()).get(terrain)
        return dict(e, source="profiles/flops.json") if e else None
    except Exception:
        return None


def launch_chunks(count: int, m: int, pool_slots: int) -> list:
    """bb_step_multi launch sizes for `count` steps from action-pool slot 0 on: up
    to m steps each, none crossing the end of the pool (actions are reused
    cyclically from a pool of `pool_slots` steps)."""
    out, j = [], 0
    while j < count:
        out.append(min(m, count - j, pool_slots - j % pool_slots))
        j += out[-1]
    return out


def bench_fields(env, terrain: str, n_fields: int = 4):
    """The terrains a CPU leg samples for this line's workload: flat, or the first-drawn
    terrains of the first n_fields per-env generators of the line's bank (host copies of the
    bank slots, with their vertical scale) -> ([(hfield f32, size_z)], description)."""
    from ballbot_gym.envs.config import stream_draws

    plan = env.terrain_plan
    if plan.stream_seeds is None:
        return [(env.hfield(0), float(plan.size_z))], f"the '{terrain}' terrain"
    firsts = [int(stream_draws(s, 1)[0]) for s in list(dict.fromkeys(plan.stream_seeds))[:n_fields]]
    slots = list(dict.fromkeys(max(plan.slot_of(x), 0) for x in firsts))
    return ([(env.hfield(sl), float(plan.size_z)) for sl in slots],
            f"{len(slots)} terrain(s) of the '{terrain}' bank (seeds {[int(plan.seeds[sl]) for sl in slots]})")


def cpu_baseline(seconds: float = 12.0, threads: int = 1, fields=None, fields_desc: str = "flat") -> dict:
    """The fp64 oracle (a port of the reference step semantics, not MuJoCo) on
    `threads` host cores (one env per OpenMP thread), random actions, on the line's
    terrain: a group of envs per sampled terrain (bench_fields), auto-reset onto it."""
    import numpy as np

    import oracle_lib as O

    O.build()
    n = 32 * threads
    cfg = O.default_cfg()
    if fields is None:
        fields = [(O.flat_hfield(), 2.0)]
    groups = []
    for hf, size_z in fields:
        off = O.init_offset(hf, size_z)
        q = np.zeros((n, 17)); v = np.zeros((n, 15)); w = np.zeros((n, 15))
        for e in range(n):
            q[e], v[e], w[e] = O.reset_state(off)
        groups.append((np.ascontiguousarray(hf, np.float32), size_z, off, q, v, w, np.zeros(n, np.int32)))
    rng = np.random.default_rng(0)
    done_steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for hf, size_z, off, q, v, w, steps in groups:
            a = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
            O.env_step_batch(cfg, q, v, w, steps, a, hf, size_z, off, threads=threads)
            done_steps += n
    dt = time.perf_counter() - t0
    cpu = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": done_steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{len(groups)} x {n} envs x {done_steps // (n * len(groups))} steps on {fields_desc}, random "
                      f"actions, auto-reset, {threads} thread(s) on '{cpu}' (fp64 oracle restating the reference "
                      f"step; MuJoCo itself is not available)"}


def mix_snapshot(env, pool, steps: int, sample: int = 512, max_ep: int = 12) -> dict:
    """The timed window's mix, for flop_count: `sample` envs spread over the env ids, their
    states at the start of the window, the window's actions for them (step t reads pool slot
    t % P, as run() does), and each env's current terrain plus the next max_ep - 1 its device
    generator will draw (a seed the bank lacks resets onto slot seed % n_terrains, as the
    kernel does).  Taken before the timed region (it synchronises)."""
    import numpy as np
    import torch

    from ballbot_gym.envs.config import pcg64_terrain_draws

    n = env.num_envs
    idx = np.unique(np.linspace(0, n - 1, min(sample, n)).round().astype(np.int64))
    q, v, w, sc = env.get_state()
    slots, _ = env.env_terrain()
    words, _ = env.terrain_rng()
    P = pool.shape[0]
    it = torch.as_tensor(idx, device=pool.device)
    acts = torch.stack([pool[t % P].index_select(0, it) for t in range(steps)]).cpu().numpy()
    plan = env.terrain_plan
    rows = np.zeros((len(idx), max_ep), np.int64)
    for j, e in enumerate(idx):
        row = [int(slots[e])]
        if words is not None:
            for x in pcg64_terrain_draws([int(u) for u in words[e]], max_ep - 1)[0]:
                sl = plan.slot_of(int(x))
                row.append(sl if sl >= 0 else int(x) % env.n_terrains)
        else:  # one fixed terrain, or a shared / tabled stream: the env stays on its terrain
            row += [row[0]] * (max_ep - 1)
        rows[j] = row
    uniq, inv = np.unique(rows, return_inverse=True)
    offs = env.offsets()
    return {"q": q[idx], "v": v[idx], "w": w[idx], "sc": sc[idx].astype(np.int32), "actions": acts,
            "table": np.stack([env.hfield(int(u)) for u in uniq]), "offsets": offs[uniq].astype(np.float64),
            "terr": inv.reshape(rows.shape).astype(np.int32), "size_z": float(plan.size_z), "envs": len(idx),
            "terrains": len(uniq), "per_env_draws": words is not None}


def flop_count(mix: dict, terrain: str) -> dict:
    """Algorithmic FLOPs per env-step of the restated reference algorithm on THIS line's timed
    mix (oracle/flopcount.cpp: the oracle compiled over a counting double, MuJoCo's solver
    settings; the checker's build, in the CPU leg): the sampled envs of mix_snapshot replayed
    from their window-start states with the window's actions and their own terrain draws, on
    host threads.  The oracle's trajectories drift from the kernel's after falls (chaos), so the
    mix is the window's in distribution, not step for step."""
    sys.path.insert(0, str(ROOT / "tools"))
    import flops as F

    thr = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    r = F.count_replay(mix["q"].copy(), mix["v"].copy(), mix["w"].copy(), mix["sc"].copy(), mix["actions"],
                       mix["table"], mix["offsets"], mix["terr"], mix["size_z"], threads=thr)
    r["sample"] = (f"{mix['envs']} envs (spread over the env ids) x {mix['actions'].shape[0]} steps: the timed "
                   f"window's own start states, actions and {'per-env terrain draws' if mix['per_env_draws'] else 'terrain'}"
                   f" ({mix['terrains']} '{terrain}' terrains), auto-reset; MuJoCo solver settings (tolerance 1e-8, "
                   "PrimalSearch ls_tolerance 0.01 / 50 evaluations)")
    return r


def parity_probe(env, n_probe: int = 64) -> dict:
    """BASELINE.json's 'per-step qpos L2' next to the throughput: the first
    n_probe envs' current (post-benchmark) states take one teacher-forced step
    on the GPU and in the fp64 oracle (the checker, as in tests/); reported are
    the L2 norms of the qpos / qvel differences.  Envs that terminate in the
    probe step (the GPU auto-resets them) are skipped.  Flat terrain only."""
    import numpy as np
    import torch

    import oracle_lib as O

    O.build()
    q, v, w, st = env.get_state()
    a = np.random.default_rng(7).uniform(-1, 1, (env.num_envs, 3)).astype(np.float32)
    env.step(torch.tensor(a, device=env.device))
    q1, v1, _, _ = env.get_state()
    cfg, hf = O.default_cfg(), O.flat_hfield()
    eq, ev = [], []
    for e in range(min(n_probe, env.num_envs)):
        qe, ve, we, se = q[e].copy(), v[e].copy(), w[e].copy(), np.array([st[e]], np.int32)
        _, _, fl, _, _ = O.env_step(cfg, qe, ve, we, se, a[e], hf)
        if fl & 1:  # terminated: reset on the GPU
            continue
        eq.append(float(np.linalg.norm(q1[e] - qe)))
        ev.append(float(np.linalg.norm(v1[e] - ve)))
    return {"envs": len(eq), "qpos_l2_max": max(eq, default=None), "qpos_l2_median": float(np.median(eq)) if eq else None,
            "qvel_l2_max": max(ev, default=None), "reference": "fp64 oracle (tests/oracle_lib), teacher-forced one step"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--burn-in", type=int, default=400,
                    help="untimed steps before the warmup that bring the envs from the common reset state into the "
                         "steady-state mix of episode ages (drop/settle, balancing, falls and auto-resets), so that a "
                         "short --warmup does not time the 4 cm free fall every env starts in")
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--precision", default="fp64", choices=["fp32", "fp64"])
    ap.add_argument("--terrain", default="flat")
    ap.add_argument("--n-terrains", type=int, default=None,
                    help="draws per generator whose terrains the bank holds (default: the whole 10^4 seed space for "
                         "per-env generators -- perlin generated on the GPU, others on a host process pool)")
    ap.add_argument("--cameras", action="store_true", help="also render the depth cameras (F2) every 6 steps")
    ap.add_argument("--shared-stream", action="store_true",
                    help="all envs on one terrain seed generator np_random(1000) instead of np_random(1000 + env id)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one HIP graph (kernel_ms is then timed on eager steps after the run)")
    ap.add_argument("--multi-step", type=int, default=512,
                    help="M steps per launch (bb_step_multi: the benchmark's random actions are known in advance, so "
                         "each env runs its M steps back to back, bit-identical to M bb_step calls); 0: one bb_step "
                         "launch per step.  With M > 0 the line also reports the per-launch form under 'per_step'")
    ap.add_argument("--action-pool", type=int, default=512,
                    help="steps of random actions resident in HBM ([P][n][3], reused cyclically); a launch never "
                         "crosses the pool's end")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-step", action="store_true",
                    help="skip the one-launch-per-step comparison run (profiler counter passes)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "traffic.json"))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BB_BENCH_BACKEND=gloo + ranks sharing one device rehearse the N>1 path on a
    # one-GPU box; the driver's multi-GPU runs use RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("BB_BENCH_BACKEND", "nccl")
    gpu = local % max(torch.cuda.device_count(), 1) if backend != "nccl" else local
    # BB_BENCH_FORCE_PG=1: the process group (and its barriers / max-over-ranks all-reduce) at
    # world size 1 too -- runs the RCCL path of the driver's multi-GPU line on a one-GPU box
    use_pg = world > 1 or os.environ.get("BB_BENCH_FORCE_PG", "0") == "1"
    if use_pg:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    from ballbot_gym.distributed import env_shard, max_over_ranks, shard_stream_seeds
    from ballbot_gym.envs import BallbotVecEnv

    # weak scaling: every rank owns a contiguous block of `--envs` global env ids
    first_env, n = env_shard(args.envs * world, rank, world)
    # terrain draws: global env g draws its terrain seeds from np_random(1000 + g) on the GPU
    # (SB3's seeding of a training VecEnv, train.py:126-141), so 4096 envs sample 4096
    # terrain sequences -- configs[2]'s "random uneven heightfield"; --shared-stream puts
    # every env on np_random(1000) (all envs start on the same terrain)
    per_env = not args.shared_stream
    env = BallbotVecEnv(n, device=dev, precision=args.precision, seed=1000,
                        terrain_config={"type": args.terrain, "config": {}}, n_terrains=args.n_terrains,
                        disable_cameras=not args.cameras, shared_stream=not per_env,
                        stream_seeds=shard_stream_seeds(1000, first_env, n) if per_env else None)

    static_a = torch.zeros(n, 3, device=dev)
    graph = env.capture_step(static_a) if args.graph else None  # one rollout step = one HIP graph

    def step(a):
        if graph is not None:
            static_a.copy_(a)
            graph.replay()
            return
        env.step_async_raw(a, full_outputs=True)
        if args.cameras:
            env._render(force=False)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    PS = max(1, args.action_pool)  # action pool slots: random actions resident in HBM, reused cyclically
    pool = torch.rand(PS, n, 3, generator=g, device=dev) * 2 - 1
    M = args.multi_step
    if M and (args.cameras or args.graph or not 1 <= M <= PS):
        M = 0  # the cameras render between steps; a captured graph holds one bb_step
    if M:  # every output of the step: obs, reward, done, terminal obs and pos2d (A11's info)
        mo = torch.empty(M, n, 15, device=dev)
        mr = torch.empty(M, n, device=dev)
        md = torch.empty(M, n, dtype=torch.uint8, device=dev)
        mt = torch.empty(M, n, 15, device=dev)
        mp = torch.empty(M, n, 2, device=dev)

    def chunks(count, m):
        return launch_chunks(count, m, PS)

    def run(count, m):  # `count` steps from pool slot 0 on, m per launch (0: one bb_step per step)
        if m:
            j = 0
            for k in chunks(count, m):
                env.step_multi_raw(pool[j % PS:j % PS + k], mo[:k], mr[:k], md[:k], mt[:k], mp[:k])
                j += k
        else:
            for i in range(count):
                step(pool[i % PS])

    def timed(m):
        """args.steps steps, m per launch, bracketed by barrier + synchronize; the MAX over ranks."""
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(), ev1.record()  # torch creates an event at its first record: not inside the window
        env.time_kernel(len(chunks(args.steps, m)) if m else args.steps)  # HIP events around each launch, on its stream
        st0 = env.stats()
        gc.disable()  # no garbage-collector pass inside the window (it would land between launches)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record()
        t_ev = time.perf_counter() - t0
        run(args.steps, m)
        enq = time.perf_counter() - t0  # host time to enqueue the timed launches
        ev1.record()
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        gc.enable()
        step_ms = ev0.elapsed_time(ev1) / args.steps  # whole step sequence per step, torch's stream
        st1 = env.stats()
        if graph is not None:  # graph replays carry no per-kernel events: time eager steps of the same kernels
            env.time_kernel(min(args.steps, 100))
            for i in range(min(args.steps, 100)):
                env.step_async_raw(pool[i % PS])
            torch.cuda.synchronize()
        ktimes, kern_n = env.kernel_times()  # fast (or multi-step), predicted-full (side stream), hand-over full
        timed.enqueue_ms = enq * 1e3
        timed.event_record_ms = t_ev * 1e3
        return max_over_ranks(elapsed, device=dev), step_ms, ktimes, kern_n, st0, st1

    run(args.burn_in + args.warmup, M)
    # the CPU leg's FLOP count replays the timed window's own mix: snapshot it before the window
    mix = mix_snapshot(env, pool, args.steps) if (world == 1 and not args.no_cpu_baseline) else None
    elapsed, step_ms, ktimes, kern_n, st0, st1 = timed(M)
    enqueue_ms = {"all": timed.enqueue_ms, "torch_event_record": timed.event_record_ms}  # (timed() runs again below)
    pair = env.pair_counters() if (M and env.relief) else None  # the last timed launch (relief pair)
    if pair is not None and pair["claims_fast"] + pair["claims_full"] > 0:
        import numpy as np

        cyc, fin = env.pair_env_times()  # per env: cycles stepped, wall tick (100 MHz) of its last step
        c = cyc.astype(np.float64) / 1e6
        f = (fin.astype(np.float64) - float(fin.max())) / 1e5
        pair["env_mcycles"] = {q: float(np.percentile(c, p)) for q, p in (("p0", 0), ("p50", 50), ("p90", 90),
                                                                          ("p99", 99), ("p100", 100))}
        pair["env_mcycles"]["mean"] = float(c.mean())
        pair["env_finish_ms_before_last"] = {q: float(np.percentile(f, p)) for q, p in (("p0", 0), ("p10", 10),
                                                                                       ("p50", 50), ("p90", 90))}
        pair["corr_cycles_finish"] = float(np.corrcoef(c, f)[0, 1])
        # the launch is its slowest env's chain: how far the slowest env is from the median one
        pair["chain_p100_over_p50"] = pair["env_mcycles"]["p100"] / max(pair["env_mcycles"]["p50"], 1e-9)
    per_step = None
    if M and not args.no_per_step:  # the same steps with one bb_step launch per step (what a closed-loop rollout uses)
        run(args.warmup, 0)
        per_step = timed(0)
    stats = env.stats()
    # Launch status: every launch returned 0 (step_multi_raw / step_async_raw raise otherwise);
    # bb_check waits for the stream and raises if a relief-pair launch ended on its wall-clock
    # budget (stale outputs and a fast number); and no env diverged in the timed window.
    env.check()
    problems = []
    if stats["pair_budget"]:
        problems.append(f"{stats['pair_budget']} relief-pair launch(es) ended on the wall-clock budget")
    if st1["diverged"] != st0["diverged"]:
        problems.append(f"{st1['diverged'] - st0['diverged']} env-steps diverged in the timed window")
    if problems:
        raise SystemExit(f"bench.py rank {rank}: " + "; ".join(problems))
    # envs per launch of each kernel over the timed steps: the full kernel stepped
    # slow_path env-steps (predicted + handed over), the fast kernel the rest
    full_per_step = (st1["slow_path"] - st0["slow_path"]) / args.steps
    launch = env.launch_config()

    if rank == 0:
        total_steps = n * world * args.steps
        value = total_steps / elapsed
        # the dominant kernel: on flat banks the fast kernel; on relief banks the longer of
        # the fast kernel and the concurrent predicted full kernel (the critical path)
        dom = "fast" if ktimes["fast"] >= ktimes["predicted_full"] else "predicted_full"
        kern_ms = ktimes[dom]
        envs_dom = (n - full_per_step) if dom == "fast" else full_per_step
        spl = 1
        if M:  # one launch = up to M steps of every env (hand-overs included)
            envs_dom = n * args.steps / kern_n
            spl = args.steps / kern_n
        abytes = algorithmic_bytes(args.precision, spl, env.relief) * envs_dom
        achieved_gbs = abytes / (kern_ms * 1e-3) / 1e9
        prof = profile_entry(Path(args.traffic_json), args.precision, args.terrain, n, spl)
        relief_form = ("relief_multi_kernel<T> (work queue)" if os.environ.get("BB_RELIEF_PAIR", "1") == "0" else
                       "relief_pair1_kernel<T> (the relief pair, one launch)" if os.environ.get("BB_PAIR_ONE", "1") != "0"
                       else "relief_pair_kernel<T,false> + <T,true> (the relief pair, two concurrent launches)")
        kernel = ((f"{relief_form} or the parked multi_step_kernel<T,*> "
                   f"launches, chosen per launch from the last one's full steps ({M} steps per "
                   "launch)" if env.relief and "BB_MULTI_QUEUE" not in os.environ and
                   "BB_ROUTE" not in os.environ and os.environ.get("BB_MULTI_ADAPT", "1") != "0"
                   else f"{relief_form} ({M} steps per launch)" if env.relief
                   and os.environ.get("BB_MULTI_QUEUE", "1") != "0" and
                   os.environ.get("BB_ROUTE", "0") == "0"
                   else f"multi_step_kernel<T,false> ({M} steps per launch; hand-overs parked "
                        "for multi_step_kernel<T,true>)" if os.environ.get("BB_MULTI_PARK", "1") != "0"
                   else f"multi_step_kernel<T,true> ({M} steps per launch, hand-overs inline)") if M else
                  "step_kernel<T,false> (fast path)" if dom == "fast"
                  else "step_kernel<T,true> (predicted full kernel, side stream)")
        # the compute side: algorithmic FP64 FLOPs of the reference algorithm per env-step on this
        # workload (the oracle over a counting double, CPU leg) -- live when the CPU leg runs,
        # else the committed count for this terrain (profiles/flops.json)
        fl = None
        if mix is not None:
            try:
                fl = flop_count(mix, args.terrain)
            except Exception as e:  # the counting build needs g++ (present here and on the box)
                fl = {"error": repr(e)}
        if fl is None or "error" in fl:
            fl = committed_flops(args.terrain) or fl
        if fl and "error" not in fl:
            fl.setdefault("basis", FLOP_BASIS)
        fpe = (fl or {}).get("flops_per_env_step")
        tf = fpe * envs_dom / (kern_ms * 1e-3) / 1e12 if fpe else None
        roof = {
            # the roof that binds: FP64 vector issue and the latency of dependent solves
            "bound": "valu", "achieved": tf, "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": tf / FP64_VECTOR_PEAK_TFLOPS if tf else None,
            # HBM bytes per launch from rocprofv3 PMC passes of THIS launch shape (steps per launch,
            # envs, terrain, precision), or null (profiles/traffic.json, tools/prof_summary.py)
            "traffic": prof.get("bytes_per_launch"),
            "traffic_algorithmic_bytes": abytes,
            "issue_frac": prof.get("issue_frac"),
            "profile": prof.get("source"),
            "kernel": kernel, "kernel_ms": kern_ms, "envs_per_launch": envs_dom, "steps_per_launch": spl,
            "kernel_ms_all": ktimes, "full_kernel_envs_per_step": full_per_step,
            "kernel_launches_timed": kern_n, "step_ms_hip_events": step_ms,
            "host_enqueue_ms": enqueue_ms,
            "flops": fl,
            # the secondary roof, as BASELINE.json asks: algorithmic HBM bytes per launch over the
            # kernel's duration against the 8 TB/s peak
            "hbm": {"achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS,
                    "algorithmic_bytes_per_env_step": algorithmic_bytes(args.precision, spl, env.relief),
                    "traffic_bytes_per_env_step": (prof["bytes_per_launch"] / envs_dom
                                                   if prof.get("bytes_per_launch") else None),
                    # HBM writes per env-step (same-shape profile) against the 133 B of outputs the
                    # step stores (obs 60, reward 4, done 1, terminal obs 60, pos2d 8)
                    "write_bytes_per_env_step": (prof["write_bytes_per_launch"] / envs_dom
                                                 if prof.get("write_bytes_per_launch") else None),
                    "write_over_outputs": (prof["write_bytes_per_launch"] / envs_dom / 133.0
                                           if prof.get("write_bytes_per_launch") else None),
                    "note": "algorithmic I/O: state once per launch of the line's steps, action and all five "
                            "outputs every step" + (", 7x7 hfield vertices per step" if env.relief else "")},
        }
        if prof.get("fp64_flop_executed_per_launch"):
            ex = prof["fp64_flop_executed_per_launch"]
            roof["valu_fp64_executed"] = {"flop_per_launch_upper_bound": ex,
                                          "tflops_upper_bound": ex / (kern_ms * 1e-3) / 1e12,
                                          "executed_over_counted": ex / (fpe * envs_dom) if fpe else None}
            act = prof.get("fp64_flop_active_lanes_per_launch")
            if act:  # the FP64 FLOPs of the lanes that were active (SQ_INSTS_VALU_FLOPS_FP64)
                roof["valu_fp64_executed"].update({"flop_per_launch_active_lanes": act,
                                                   "active_over_counted": act / (fpe * envs_dom) if fpe else None})
                # the hardware's view on the same peak: the executed FP64 of the active lanes (same-shape
                # profile) over this run's kernel time -- independent of the FLOP-count basis
                roof["frac_executed"] = act / (kern_ms * 1e-3) / 1e12 / FP64_VECTOR_PEAK_TFLOPS
        line = {
            "metric": f"env-steps/sec at {n} envs per GPU ({args.terrain} terrain, random actions)",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.precision == "fp64" else "f32",
            "data": "synthetic (uniform random actions in [-1,1], resident in HBM; "
                    f"{args.burn_in} untimed burn-in steps into the steady-state episode mix before the warmup"
                    + (f"; stepped {M} per launch with bb_step_multi, bit-identical to one bb_step per step)" if M
                       else ")"),
            "config": {"workload": f"{n} envs/GPU, {args.terrain} terrain, random actions "
                                   f"(BASELINE configs[{1 if args.terrain == 'flat' else 2}])",
                       "terrain": args.terrain, "n_terrains": env.n_terrains, "depth_cameras": bool(args.cameras),
                       "terrain_streams": "per env (seed 1000 + env id)" if per_env else "shared (seed 1000)",
                       "hip_graph": graph is not None, "burn_in_steps": args.burn_in,
                       "multi_step": M, "steps_per_launch": spl,
                       "envs_per_gpu": n, "total_envs": n * world, "precision": args.precision,
                       "parallelism": f"env-sharded x{world} (no collective on the step path)",
                       "process_group": dist.get_backend() if use_pg else None,
                       "launch": launch},
            "roofline": roof,
            "stats": stats,
            "status": "ok",
        }
        if pair is not None and pair["claims_fast"] + pair["claims_full"] > 0:
            line["pair"] = pair
        if per_step is not None:
            pe, pms, pk, pn, _, _ = per_step
            line["per_step"] = {
                "value": n * world * args.steps / pe, "ms_per_step": pe / args.steps * 1e3,
                "step_ms_hip_events": pms, "kernel_ms_all": pk, "kernel_launches_timed": pn,
                "note": "the same steps with one bb_step launch per step, the form a closed-loop (policy) rollout "
                        "uses: every step waits for the slowest env of the GPU"}
        if world == 1 and not args.no_cpu_baseline:
            if args.terrain == "flat":
                line["parity"] = parity_probe(env)
            fields, desc = bench_fields(env, args.terrain)
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, fields=fields, fields_desc=desc)
            # all host cores granted to this job (OMP_NUM_THREADS; 16 on the GPU box)
            thr = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
            if thr > 1:
                line["cpu_baseline_multicore"] = cpu_baseline(args.cpu_seconds / 2, threads=thr, fields=fields,
                                                              fields_desc=desc)
        print(json.dumps(line), flush=True)
    env.close()
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
