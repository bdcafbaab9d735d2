#!/bin/bash
# Round-4 GPU pass A: the suite, the flat and perlin bench lines, the driver window,
# the memset-in-graph diagnostic and a short config-5 smoke with evaluations.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/suite_r4e.txt 2>&1
rc=$?
tail -6 gpurun_out/suite_r4e.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u bench.py --terrain perlin --no-cpu-baseline > gpurun_out/bench_r4e_perlin.json 2> gpurun_out/bench_r4e_perlin.err || exit $?
BB_RELIEF_PAIR=0 timeout -k 10 200 python -u bench.py --terrain perlin --no-cpu-baseline > gpurun_out/bench_r4e_perlin_queue.json 2> gpurun_out/bench_r4e_perlin_queue.err || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r4e_flat_driver.json 2> gpurun_out/bench_r4e_flat_driver.err || exit $?
timeout -k 10 120 python -u tools/graph_memset_order.py > gpurun_out/graph_memset_order.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_ppo.py --terrain perlin --cameras --frozen-encoder --timesteps 2e5 --seed 10 \
  --envs 10 --n-steps 2048 --batch 256 --eval-freq 5000 --eval-episodes 8 --out gpurun_out/ppo_cfg5_smoke \
  > gpurun_out/ppo_cfg5_smoke.json 2> gpurun_out/ppo_cfg5_smoke.err || exit $?
exit $rc
