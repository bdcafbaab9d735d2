#!/bin/bash
# Round-4 GPU pass U: PPO throughput on the final build (4096 envs x 64 steps, 10M steps; flat
# and perlin), SB3-format progress.csv under gpurun_out/u.
set -o pipefail
mkdir -p gpurun_out/u
for t in flat perlin; do
  timeout -k 10 400 python -u tools/bench_ppo.py --terrain $t --timesteps 10e6 --out gpurun_out/u/ppo_$t > gpurun_out/u/ppo_$t.json 2> gpurun_out/u/ppo_$t.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/u/ppo_$t.json').read().splitlines()[-1]);print('$t', round(d['value']/1e6,3), 'M', round(d['rollout_s'],2), round(d['update_s'],2), round(d['ep_rew_mean'],3), round(d['ep_len_mean'],1))"
done
