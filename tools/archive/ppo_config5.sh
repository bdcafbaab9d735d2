#!/bin/bash
# Config-5 evidence on one GPU (BASELINE configs[4]: PPO on randomized perlin terrain with the
# depth cameras and a frozen encoder, the reference's coefficients):
#   A: 4096 envs x 64 steps, batch 8192 (throughput geometry), 5.3M steps
#   B: the reference's geometry, 10 envs x 2048 steps, batch 256, 5.3M steps
#      (outputs/experiments/archived_models/2025-12-03_ppo-perlin-directional-5.2M-steps/config.yaml)
# Each run pretrains the TinyAutoencoder on its own GPU-rendered frames and freezes it (the
# reference's encoder is a pickle we do not load).  progress.csv files land in gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
A="--terrain perlin --cameras --frozen-encoder --timesteps 5.3e6 --seed 10"
timeout -k 10 600 python -u tools/bench_ppo.py $A --envs 4096 --n-steps 64 --batch 8192 \
  --out gpurun_out/ppo_cfg5_4096 > gpurun_out/ppo_cfg5_4096.json 2> gpurun_out/ppo_cfg5_4096.err || exit $?
timeout -k 10 1000 python -u tools/bench_ppo.py $A --envs 10 --n-steps 2048 --batch 256 \
  --out gpurun_out/ppo_cfg5_ref10 > gpurun_out/ppo_cfg5_ref10.json 2> gpurun_out/ppo_cfg5_ref10.err || exit $?
