"""Compare an EvalCallback evaluations.npz with the reference's archived one (CPU, this container).

  python tools/compare_evals.py gpurun_out/ppo_cfg5_eval/results/evaluations.npz \
      [--ref /root/reference/outputs/experiments/archived_models/2025-12-03_ppo-perlin-directional-5.2M-steps/results/evaluations.npz] \
      [--out profiles/r04_cfg5_eval_compare.json]

Both files are read with numpy.load(allow_pickle=False): plain arrays only
(timesteps [E], results [E][8], ep_lengths [E][8]).  Prints one JSON object: the
evaluation grid of each, the mean return and length per evaluation, and
summaries over the first, middle and last thirds of training.
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path

import numpy as np

REF = ("/root/reference/outputs/experiments/archived_models/2025-12-03_ppo-perlin-directional-5.2M-steps/"
       "results/evaluations.npz")


def summary(path: str) -> dict:
    z = np.load(path, allow_pickle=False)
    t, r, ln = z["timesteps"], z["results"], z["ep_lengths"]
    e = len(t)
    thirds = [slice(0, e // 3), slice(e // 3, 2 * e // 3), slice(2 * e // 3, e)]
    return {
        "path": str(path), "evaluations": int(e), "episodes_per_eval": int(r.shape[1]),
        "timesteps_first_last": [int(t[0]), int(t[-1])], "timestep_interval": int(t[1] - t[0]) if e > 1 else None,
        "mean_return_per_eval": [round(float(x), 4) for x in r.mean(1)],
        "mean_length_per_eval": [round(float(x), 2) for x in ln.mean(1)],
        "return_by_third": [round(float(r[s].mean()), 4) for s in thirds],
        "length_by_third": [round(float(ln[s].mean()), 2) for s in thirds],
        "return_all": round(float(r.mean()), 4), "return_std_all": round(float(r.std()), 4),
        "best_eval_mean_return": round(float(r.mean(1).max()), 4),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ours")
    ap.add_argument("--ref", default=REF)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {"ours": summary(a.ours), "reference": summary(a.ref)}
    o, r = res["ours"], res["reference"]
    res["same_grid"] = o["evaluations"] == r["evaluations"] and o["timesteps_first_last"] == r["timesteps_first_last"]
    res["return_ratio_by_third"] = [round(x / y, 3) if y else None for x, y in zip(o["return_by_third"],
                                                                                  r["return_by_third"])]
    txt = json.dumps(res, indent=1)
    if a.out:
        Path(a.out).write_text(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
