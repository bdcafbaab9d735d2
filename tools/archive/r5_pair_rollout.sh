#!/bin/bash
# Round-5: PPO rollouts on relief banks through the relief pair (relief_pair1_kernel<T, true>)
# against the work queue (BB_RELIEF_PAIR=0): parity tests, then collect_rollouts throughput
# (4096 perlin envs on per-env generators, 64 steps per rollout) and PPO end to end.
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
L=openballbot-rl_amd/ballbot_gym/_lib/libbb_mi355x.so
for p in 1 0; do
  BB_FUSED_ROLLOUT=1 BB_RELIEF_PAIR=$p timeout -k 10 300 python -u tools/lib_bench.py --child $L --terrain perlin --rollout --steps 640 > $O/roll_perlin_pair$p.json 2> $O/roll_perlin_pair$p.log || { tail $O/roll_perlin_pair$p.log; exit 1; }
  cat $O/roll_perlin_pair$p.json
done
timeout -k 10 300 python -u tools/lib_bench.py --child $L --terrain perlin --rollout --steps 640 > $O/roll_perlin_graph.json 2> $O/roll_perlin_graph.log || { tail $O/roll_perlin_graph.log; exit 1; }
cat $O/roll_perlin_graph.json
for f in 1 0; do
  BB_FUSED_ROLLOUT=$f timeout -k 10 400 python -u tools/bench_ppo.py --terrain perlin --timesteps 5e6 > $O/ppo_perlin_fused$f.json 2> $O/ppo_perlin_fused$f.log || { tail $O/ppo_perlin_fused$f.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[1], round(d['value']/1e6,3), 'rollout', round(d['rollout_s'],3), 'update', round(d['update_s'],3), 'roll/s', round(d['rollout_env_steps_per_s']/1e6,3))" $O/ppo_perlin_fused$f.json
done
echo PAIR_ROLLOUT_DONE
