"""Per-phase GPU cycle breakdown of the step kernel (diagnostic, GPU box).

Builds csrc/bb_kernels.hip with -DBB_PHASE_CLOCKS into tools/_build, runs the
bench workload (4096 envs, flat, random actions) and prints s_memtime cycles
per phase summed over teams, normalised per forward and per Newton iteration.
"""
import argparse
import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))
LIB = ROOT / "tools" / "_build" / "libbb_phase.so"
NAMES = ["contact_pass", "reduce", "gradient", "hessian", "cholesky", "direction", "line_search", "exit",
         "kin_mass_bias_wheel", "collide", "forwards"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--terrain", default="flat")
    ap.add_argument("--lib", default=None, help="a prebuilt -DBB_PHASE_CLOCKS library (e.g. under tools/variants)")
    a = ap.parse_args()
    global LIB
    if a.lib:
        LIB = Path(a.lib)
    from ballbot_gym import _native
    if a.build or not LIB.exists():
        LIB.parent.mkdir(parents=True, exist_ok=True)
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-DBB_PHASE_CLOCKS",
                        "-o", str(LIB)] + [str(ROOT / "openballbot-rl_amd" / "csrc" / f) for f in _native.HIP_SOURCES],
                       check=True)
    import torch
    from ballbot_gym import _native
    _native.use_diagnostic_library(LIB)
    L = _native.lib()
    L.bb_debug_phase_cycles.argtypes = [C.POINTER(C.c_ulonglong)]
    from ballbot_gym.envs import BallbotVecEnv
    env = BallbotVecEnv(4096, device="cuda:0", precision=a.precision, terrain_config={"type": a.terrain, "config": {}})
    pool = torch.rand(64, 4096, 3, device="cuda:0") * 2 - 1
    out = (C.c_ulonglong * 100)()
    for i in range(a.warmup):
        env.step_async_raw(pool[i % 64])
    torch.cuda.synchronize()
    L.bb_debug_phase_cycles(out)
    s0 = env.stats()
    for i in range(a.steps):
        env.step_async_raw(pool[i % 64])
    torch.cuda.synchronize()
    L.bb_debug_phase_cycles(out)
    s1 = env.stats()
    iters = s1["solver_iters"] - s0["solver_iters"]
    fw = out[10]
    res = {"precision": a.precision, "forwards": fw, "newton_iters": iters,
           "cycles_per_forward": {NAMES[k]: out[k] / fw for k in range(10)},
           "cycles_per_newton_iter": {NAMES[k]: out[k] / max(iters, 1) for k in range(8)}}
    res["total_cycles_per_forward"] = (sum(out[k] for k in range(10)) + out[32] + out[33]) / fw
    # the line-search phase split: setup (M s, s'Ms, per-contact terms) and the evaluation loop
    res["cycles_per_forward"]["line_search_setup"] = out[32] / fw
    res["cycles_per_forward"]["line_search_loop"] = out[33] / fw
    res["line_search_evals_per_newton_iter"] = out[11] / max(iters, 1)
    res["newton_iters_per_forward_max"] = out[21]
    res["newton_iters_per_forward_hist"] = {f"{2 * b}-{2 * b + 1}" if b < 9 else ">=18": out[22 + b] for b in range(10)}
    if out[12]:
        res["full_kernel"] = {"forwards": out[12], "body_contacts_per_forward": out[13] / out[12],
                              "body_collide_cycles_per_forward": out[14] / out[12],
                              "solve_cycles_per_forward": out[15] / out[12],
                              "newton_iters_per_forward": out[20] / out[12],
                              "geoms_in_prism_loop_per_forward": out[16] / out[12],
                              "prisms_per_forward": out[17] / out[12],
                              "prism_rounds_per_forward": out[18] / out[12],
                              "sat_runs_per_forward": out[19] / out[12]}
    for name, k in (("full", 34), ("fast", 37)):  # per-env step durations (s_memtime cycles)
        if out[k + 2]:
            res[f"{name}_env_step_cycles"] = {"max": out[k], "mean": out[k + 1] / out[k + 2], "count": out[k + 2]}
    if out[12]:  # the full kernel's solve by phase (slots 80-89), per full forward and per Newton iteration
        ph = {NAMES[k]: out[80 + k] for k in range(8)}
        ph["line_search_setup"], ph["line_search_loop"] = out[88], out[89]
        res["full_kernel"]["solve_phase_cycles_per_forward"] = {k: v / out[12] for k, v in ph.items()}
        res["full_kernel"]["solve_phase_cycles_per_newton_iter"] = {k: v / max(out[20], 1) for k, v in ph.items()}
    if out[12]:  # full kernel: per-env step duration histogram, bins of 2^20 cycles
        res["full_env_step_hist"] = [{"bin_Mcyc": b * 1.048576, "envs": out[40 + b],
                                      "body_contacts_per_step": out[50 + b] / max(out[40 + b], 1),
                                      "max_body_contacts_per_step": out[70 + b],
                                      "newton_iters_per_step": out[60 + b] / max(out[40 + b], 1)} for b in range(10)]
    if out[90]:  # the full kernel's exact-SAT rounds (slots 90-99): lanes per path, rounds per path
        r = out[90]
        res["sat_rounds"] = {"rounds": r, "rounds_per_full_forward": r / max(out[12], 1),
                             "lanes_per_round": out[91] / r,
                             "lanes": {"cylinder": out[92], "capsule_face_early_out": out[93],
                                       "capsule_intersecting": out[94], "capsule_apart": out[95],
                                       "capsule_apart_hits": out[96]},
                             "rounds_running_apart": out[97] / r, "rounds_running_cylinder_or_intersecting": out[98] / r,
                             "cycles_per_round": out[99] / r,
                             "cycles_per_full_forward": out[99] / max(out[12], 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
