#!/bin/bash
# PPO trainer check on the GPU box: the PPO GPU tests, then 10M flat steps
# (bench line + SB3 progress.csv) and a 3M-step split-K A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_ppo.log 2>&1 || { tail -40 gpurun_out/pytest_ppo.log; exit 1; }
tail -1 gpurun_out/pytest_ppo.log
timeout -k 10 300 python -u tools/bench_ppo.py --timesteps 10e6 --out gpurun_out/ppo_flat10M > gpurun_out/ppo_flat10M.json 2> gpurun_out/ppo_flat10M.err || exit 1
BB_SPLITK_ROWS=512 timeout -k 10 200 python -u tools/bench_ppo.py --timesteps 3e6 --out gpurun_out/ppo_s16 > gpurun_out/ppo_s16.json 2>/dev/null || exit 1
timeout -k 10 200 python -u tools/bench_ppo.py --timesteps 3e6 --out gpurun_out/ppo_s128 > gpurun_out/ppo_s128.json 2>/dev/null || exit 1
python - <<'PY'
import json
for f in ("ppo_flat10M", "ppo_s16", "ppo_s128"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, round(d["value"]), "rollout_s", round(d["rollout_s"], 2), "update_s", round(d["update_s"], 2),
          "ep_rew", round(d["ep_rew_mean"], 2), "ep_len", round(d["ep_len_mean"], 1))
PY
