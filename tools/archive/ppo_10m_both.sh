#!/bin/bash
# 10M-step PPO bench lines + SB3 progress.csv on flat and perlin terrain
# (fused rollout/update path), after a short warm-up process.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_ppo.py --timesteps 1e6 --out gpurun_out/ppo_warm > /dev/null 2>&1 || exit 1
for t in flat perlin; do
  timeout -k 10 400 python -u tools/bench_ppo.py --timesteps 10e6 --terrain $t --out gpurun_out/ppo_${t}10M \
    > gpurun_out/ppo_${t}10M.json 2> gpurun_out/ppo_${t}10M.err || { tail gpurun_out/ppo_${t}10M.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ppo_${t}10M.json'))
print('$t', round(d['value']), 'rollout_s', round(d['rollout_s'], 2), 'update_s', round(d['update_s'], 2), 'ep_rew', round(d['ep_rew_mean'], 2), 'ep_len', round(d['ep_len_mean'], 1))"
done
