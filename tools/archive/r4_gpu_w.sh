#!/bin/bash
# Round-4 GPU pass W: PPO update-time check (flat, 3M steps twice, update-graph debug lines).
set -o pipefail
mkdir -p gpurun_out/w
for rep in 1 2; do
  timeout -k 10 300 python -u tools/bench_ppo.py --terrain flat --timesteps 3e6 > gpurun_out/w/ppo_$rep.json 2> gpurun_out/w/ppo_$rep.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/w/ppo_$rep.json').read().splitlines()[-1]);print($rep, round(d['value']/1e6,3), round(d['rollout_s'],3), round(d['update_s'],3), d['iterations'])"
done
