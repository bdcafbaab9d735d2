#!/bin/bash
# Round-4 GPU pass V: PPO rollout (bb_rollout) with FMA contraction per expression (the product)
# against the compiler default (BB_FP_CONTRACT_FAST), flat and perlin; and the bench's perlin
# PPO with a shared terrain stream (round 3's workload).
set -o pipefail
mkdir -p gpurun_out/v
for t in flat perlin; do
  timeout -k 10 300 python -u tools/lib_bench.py --variant prod: --variant cffast: --no-build --rollout --terrain $t --steps 640 --warmup 320 > gpurun_out/v/rollout_$t.txt 2>&1 || { tail -20 gpurun_out/v/rollout_$t.txt; exit 1; }
  grep -h "env_steps" gpurun_out/v/rollout_$t.txt | python -c "
import sys, json
for l in sys.stdin:
    try: d=json.loads(l); print('$t', d.get('variant'), round(d['env_steps_per_s']/1e6,3))
    except Exception: pass"
done
