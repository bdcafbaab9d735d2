"""Kernel solver vs the MuJoCo-form oracle, teacher-forced, on the CPU.

The host build of the product's per-env templates (tests/hostcheck: the kernel's
forward, its Newton solve with its own line search, RK4, glue) and the oracle
(MuJoCo's PrimalSearch, warm-start choice, improvement/gradient stop) step the
same recorded pre-step states; reported per env-step are max |dqpos|, max
|dqvel| and the share within the parity tests' stated fp64 tolerance (qpos 1e-9,
qvel 1e-6).  The residual is where the two line searches end an iteration at
different points and MuJoCo's improvement test then stops one Newton iteration
apart.

  python tools/solver_parity.py [--envs 64] [--steps 120] [--terrain flat|hills|both] [--warm-only]
                                [--out profiles/r05_solver_parity.json]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "tests", ROOT / "openballbot-rl_amd"):
    sys.path.insert(0, str(p))

import hostcheck_lib as HC  # noqa: E402
import oracle_lib as O  # noqa: E402
import traj  # noqa: E402


def measure(hf, n_envs, n_steps, seed, size_z=2.0):
    rec = traj.record(n_envs=n_envs, n_steps=n_steps, hfield=hf, size_z=size_z, seed=seed)
    cfg = HC.default_cfg()
    dq, dv = [], []
    for t in range(n_steps):
        for e in range(n_envs):
            q, v, w = rec["qpos"][t][e].copy(), rec["qvel"][t][e].copy(), rec["warm"][t][e].copy()
            st = np.array([rec["steps"][t][e]], np.int32)
            HC.env_step(cfg, q, v, w, st, rec["action"][t][e], hf, size_z)
            dq.append(float(np.abs(q - rec["qpos1"][t][e]).max()))
            dv.append(float(np.abs(v - rec["qvel1"][t][e]).max()))
    dq, dv = np.array(dq), np.array(dv)
    ok = (dq <= 1e-9) & (dv <= 1e-6)
    worst = np.argsort(-dv)[:5]
    # each outlier's pre-state stepped again by the oracle with the kernel's start (qacc_warmstart,
    # no comparison against qacc_smooth): how far the kernel is from THAT oracle step
    attrib = []
    for i in np.flatnonzero(~ok):
        t, e = divmod(int(i), n_envs)
        q, v, w = rec["qpos"][t][e].copy(), rec["qvel"][t][e].copy(), rec["warm"][t][e].copy()
        qk, vk, wk = q.copy(), v.copy(), w.copy()
        HC.env_step(cfg, qk, vk, wk, np.array([rec["steps"][t][e]], np.int32), rec["action"][t][e], hf, size_z)
        flags = O.lib().bbo_get_flags() if hasattr(O.lib(), "bbo_get_flags") else None
        O.set_flags(O.WARM_ONLY)
        O.env_step(O.default_cfg(), q, v, w, np.array([rec["steps"][t][e]], np.int32), rec["action"][t][e], hf, size_z)
        O.set_flags(0 if flags is None else flags)
        attrib.append({"t": t, "env": e, "qvel_vs_oracle": float(dv[i]),
                       "qvel_vs_warm_start_oracle": float(np.abs(vk - v).max()),
                       "qpos_vs_warm_start_oracle": float(np.abs(qk - q).max())})
    return {"env_steps": int(len(dq)), "within_q1e-9_v1e-6": float(ok.mean()), "outliers": int((~ok).sum()),
            "outlier_attribution": attrib,
            "qpos_max": float(dq.max()), "qvel_max": float(dv.max()),
            "qpos_p50": float(np.median(dq)), "qvel_p50": float(np.median(dv)),
            "qpos_p999": float(np.quantile(dq, 0.999)), "qvel_p999": float(np.quantile(dv, 0.999)),
            "worst_qvel": [float(dv[i]) for i in worst]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--terrain", default="both")
    ap.add_argument("--out", default=None)
    ap.add_argument("--warm-only", action="store_true",
                    help="oracle starts every solve from qacc_warmstart, as the kernel does (no comparison "
                         "against qacc_smooth): separates the warm-start choice from the line search")
    a = ap.parse_args()
    O.build()
    HC.build()
    O.set_flags(O.WARM_ONLY if a.warm_only else 0)
    res = {}
    if a.terrain in ("flat", "both"):
        res["flat"] = measure(O.flat_hfield(), a.envs, a.steps, seed=3)
        print("flat", json.dumps(res["flat"]), flush=True)
    if a.terrain in ("hills", "both"):
        from ballbot_gym.terrain import generate_hills_terrain

        hf = generate_hills_terrain(293, seed=7).astype(np.float32)
        res["hills"] = measure(hf, a.envs // 2, a.steps * 2 // 3, seed=5)
        print("hills", json.dumps(res["hills"]), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps({"what": "hostcheck (kernel templates, host build) vs MuJoCo-form oracle, "
                                                   "teacher-forced one step per recorded state",
                                        "oracle_warm_start": "qacc_warmstart always" if a.warm_only else "MuJoCo's choice",
                                        **res}, indent=1))


if __name__ == "__main__":
    main()
