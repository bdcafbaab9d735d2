#!/bin/bash
# Fused encoder: serialized encoder/camera GPU tests, then a 4M-step camera PPO run.
set -o pipefail
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -x -v -p no:randomly -k "encoder or camera or fused or graph" \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1 || { tail -40 gpurun_out/pytest_enc.log; exit 1; }
tail -2 gpurun_out/pytest_enc.log
timeout -k 10 400 python -u tools/bench_ppo.py --cameras --frozen-encoder --timesteps 4e6 --out gpurun_out/ppo_cam_fused \
  > gpurun_out/ppo_cam_fused.json 2> gpurun_out/ppo_cam_fused.err || { tail gpurun_out/ppo_cam_fused.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/ppo_cam_fused.json'))
print('fused', round(d['value']), 'rollout_s', round(d['rollout_s'], 2), 'update_s', round(d['update_s'], 2), 'ep_rew', round(d['ep_rew_mean'], 2), 'ep_len', round(d['ep_len_mean'], 1))"
bash tools/ppo_cam_prof.sh
