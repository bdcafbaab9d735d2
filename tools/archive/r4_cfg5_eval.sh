#!/bin/bash
# Config-5 learning curve with the reference's evaluation (BASELINE configs[4], one GPU): PPO on
# randomized perlin terrain with depth cameras and a frozen encoder, the reference's geometry
# (10 envs x 2048 steps, batch 256, seed 10, 5.2M steps) and EvalCallback every 5000 vec-env
# steps, 8 deterministic episodes on a 10-env eval VecEnv (env i on np_random(seed + 10 + i)).
# Writes progress.csv (eval/* rows) and results/evaluations.npz under gpurun_out/ppo_cfg5_eval.
set -o pipefail
mkdir -p gpurun_out/ppo_cfg5_eval
timeout -k 10 1130 python -u tools/bench_ppo.py --terrain perlin --cameras --frozen-encoder --timesteps 5.2e6 \
  --seed 10 --envs 10 --n-steps 2048 --batch 256 --eval-freq 5000 --eval-episodes 8 \
  --out gpurun_out/ppo_cfg5_eval > gpurun_out/ppo_cfg5_eval/bench.json 2> gpurun_out/ppo_cfg5_eval/bench.err
