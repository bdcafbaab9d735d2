#!/bin/bash
# PPO GPU tests, then a warm-up run and two 3M-step flat PPO runs (bench lines).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_ppo.log 2>&1 || { tail -40 gpurun_out/pytest_ppo.log; exit 1; }
tail -1 gpurun_out/pytest_ppo.log
for r in warm a b; do
  timeout -k 10 200 python -u tools/bench_ppo.py --timesteps 3e6 --out gpurun_out/ppo_q_$r > gpurun_out/ppo_q_$r.json 2>gpurun_out/ppo_q_$r.err || { tail gpurun_out/ppo_q_$r.err; exit 1; }
done
python - <<'PY'
import json
for f in ("warm", "a", "b"):
    d = json.load(open(f"gpurun_out/ppo_q_{f}.json"))
    print(f, round(d["value"]), "rollout_s", round(d["rollout_s"], 2), "update_s", round(d["update_s"], 2),
          "rollout env-steps/s", round(d["rollout_env_steps_per_s"]), "ep_rew", round(d["ep_rew_mean"], 2))
PY
