"""Fit tools/traffic_sweep.sh output: bytes per launch = fixed + per_env * envs.

  python tools/traffic_fit.py gpurun_out/traffic_sweep [--out profiles/r01_traffic_sweep.json]

FETCH_SIZE / WRITE_SIZE (KiB) are averaged over the last 20 fast step_kernel
dispatches of each run and least-squares fitted against the env count.  Both
the raw FETCH_SIZE and the x2 gfx950 correction (MI355X_MICROARCH.md, which
calibrates it for 16-B-per-lane streaming loads only) are reported.
"""
import argparse
import json
import re
from pathlib import Path

import numpy as np

from prof_summary import counters


def fit(x, y):
    A = np.stack([np.ones_like(x), x], 1)
    (c0, c1), *_ = np.linalg.lstsq(A, y, rcond=None)
    return float(c0), float(c1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    src = Path(a.src)
    runs = {}
    for d in sorted(src.glob("*_fetch")):
        m = re.match(r"(fp\d+)_(\d+)_fetch", d.name)
        if not m:
            continue
        prec, envs = m.group(1), int(m.group(2))
        fcsv = next(d.rglob("*counter_collection.csv"))
        wcsv = next((src / f"{prec}_{envs}_write").rglob("*counter_collection.csv"))
        f, nf = counters(fcsv, ["FETCH_SIZE"], 20)
        w, nw = counters(wcsv, ["WRITE_SIZE"], 20)
        runs.setdefault(prec, []).append({"envs": envs, "fetch_raw_bytes": f["FETCH_SIZE"] * 1024,
                                          "write_bytes": w["WRITE_SIZE"] * 1024, "dispatches": min(nf, nw)})
    out = {}
    for prec, rs in runs.items():
        rs.sort(key=lambda r: r["envs"])
        x = np.array([r["envs"] for r in rs], float)
        fr = np.array([r["fetch_raw_bytes"] for r in rs])
        wr = np.array([r["write_bytes"] for r in rs])
        f0, f1 = fit(x, fr)
        w0, w1 = fit(x, wr)
        out[prec] = {"runs": rs,
                     "fetch_raw": {"fixed_bytes_per_launch": f0, "bytes_per_env_step": f1},
                     "fetch_x2": {"fixed_bytes_per_launch": 2 * f0, "bytes_per_env_step": 2 * f1},
                     "write": {"fixed_bytes_per_launch": w0, "bytes_per_env_step": w1}}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        Path(a.out).write_text(s + "\n")


if __name__ == "__main__":
    main()
