#!/bin/bash
# Fused PPO (bb_ppo_mlp_step / bb_ppo_mlp_act): GPU PPO tests with serialized
# kernels (a fault names its launch), one 3M-step flat PPO run, and a rocprofv3
# kernel summary of a 1M-step run.
set -o pipefail
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -x -v -p no:randomly --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_ppo.log 2>&1 || { tail -60 gpurun_out/pytest_ppo.log; exit 1; }
tail -3 gpurun_out/pytest_ppo.log
timeout -k 10 200 python -u tools/bench_ppo.py --timesteps 3e6 --out gpurun_out/ppo_f1 > gpurun_out/ppo_f1.json 2>gpurun_out/ppo_f1.err || { tail gpurun_out/ppo_f1.err; exit 1; }
cat gpurun_out/ppo_f1.json
bash tools/ppo_prof_fused.sh
