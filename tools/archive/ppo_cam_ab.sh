#!/bin/bash
# Camera PPO with the frozen pretrained encoder (the reference's setup), 4M steps:
# the fused encoder (bb_depth_encoder) and the torch/MIOpen module (BB_FUSED_ENCODER=0).
set -o pipefail
mkdir -p gpurun_out
for r in fused torch; do
  case $r in fused) F=1;; *) F=0;; esac
  BB_FUSED_ENCODER=$F timeout -k 10 400 python -u tools/bench_ppo.py --cameras --frozen-encoder --timesteps 4e6 \
    --out gpurun_out/ppo_cam_$r > gpurun_out/ppo_cam_$r.json 2> gpurun_out/ppo_cam_$r.err || { tail gpurun_out/ppo_cam_$r.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ppo_cam_$r.json'))
print('$r', round(d['value']), 'rollout_s', round(d['rollout_s'], 2), 'update_s', round(d['update_s'], 2), 'ep_rew', round(d['ep_rew_mean'], 2), 'ep_len', round(d['ep_len_mean'], 1))"
done
