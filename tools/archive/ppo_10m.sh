#!/bin/bash
# 10M-step flat PPO bench line + SB3 progress.csv, after a short warm-up process
# (the first process on a fresh box pays one-time library/JIT costs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_ppo.py --timesteps 1e6 --out gpurun_out/ppo_warm > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_ppo.py --timesteps 10e6 --out gpurun_out/ppo_flat10M > gpurun_out/ppo_flat10M.json 2> gpurun_out/ppo_flat10M.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/ppo_flat10M.json'))
print(round(d['value']), 'rollout_s', round(d['rollout_s'], 2), 'update_s', round(d['update_s'], 2), 'ep_rew', round(d['ep_rew_mean'], 2), 'ep_len', round(d['ep_len_mean'], 1))"
