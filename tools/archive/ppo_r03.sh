#!/bin/bash
# Round-3 PPO bench lines: 10M steps flat and perlin (proprio policy, fused rollout kernel),
# after a short warm-up process; SB3-format progress.csv per run.
set -o pipefail
O=gpurun_out/ppo_r03
mkdir -p $O
timeout -k 10 200 python -u tools/bench_ppo.py --timesteps 1e6 --out $O/warm > /dev/null 2>&1 || exit 1
for t in flat perlin; do
  timeout -k 10 400 python -u tools/bench_ppo.py --timesteps 10e6 --terrain $t --out $O/$t > $O/$t.json 2> $O/$t.err || { tail $O/$t.err; exit 1; }
  python -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], round(d['value']), 'rollout_s', round(d['rollout_s'], 2), 'update_s', round(d['update_s'], 2), 'ep_rew', round(d['ep_rew_mean'], 2), 'ep_len', round(d['ep_len_mean'], 1))" $O/$t.json $t
done
ls $O
