#!/bin/bash
# Fused PPO minibatch (bb_ppo_mlp_step): GPU PPO tests, then 3M-step flat PPO
# runs with the autograd update (BB_PPO_FUSED=0) and the fused one, and a
# rocprofv3 kernel summary of a short fused run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py -x -v -k "fused or graph" --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_ppo.log 2>&1 || { tail -60 gpurun_out/pytest_ppo.log; exit 1; }
tail -3 gpurun_out/pytest_ppo.log
for r in f0 f1 f0b f1b; do
  case $r in f0*) F=0;; *) F=1;; esac
  BB_PPO_FUSED=$F timeout -k 10 200 python -u tools/bench_ppo.py --timesteps 3e6 --out gpurun_out/ppo_$r \
    > gpurun_out/ppo_$r.json 2>gpurun_out/ppo_$r.err || { tail gpurun_out/ppo_$r.err; exit 1; }
done
python - <<'PY'
import json
for f in ("f0", "f1", "f0b", "f1b"):
    d = json.load(open(f"gpurun_out/ppo_{f}.json"))
    print(f, round(d["value"]), "rollout_s", round(d["rollout_s"], 2), "update_s", round(d["update_s"], 2),
          "ep_rew", round(d["ep_rew_mean"], 2), "ep_len", round(d.get("ep_len_mean", 0), 1))
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run --output-format csv -- \
  python -u tools/bench_ppo.py --timesteps 1e6 > gpurun_out/prof_fused.log 2>&1 || { tail gpurun_out/prof_fused.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_fused/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.1f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:90]}")
print("total ms", tot / 1e6)
PY
