#!/bin/bash
# Round-4 GPU pass E: relief pair on ticket rings -- multi-step parity, then counters at seg 4/16/64
# (perlin, 4096 envs, per-env generators), and the MachineLICM-off build on perlin.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_step.py tests/test_gpu_terrain_stream.py -x -v --timeout 120 --timeout-method thread > gpurun_out/suite_r4h_multi.txt 2>&1 || { tail -30 gpurun_out/suite_r4h_multi.txt; exit 1; }
tail -2 gpurun_out/suite_r4h_multi.txt
show() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), d['stats'].get('pair_budget'), d.get('pair'))"; }
P="--terrain perlin --no-cpu-baseline"
for v in "S4" "S16" "S64"; do
  env BB_PAIR_SEG=${v#S} timeout -k 10 200 python -u bench.py $P > gpurun_out/paire_$v.json 2> gpurun_out/paire_$v.err || exit $?
  show gpurun_out/paire_$v.json $v
done
BB_PAIR_SEG=64 timeout -k 10 200 python -u tools/bench_with_lib.py tools/_build/libbb_nolicm.so $P > gpurun_out/perlin_nolicm.json 2> gpurun_out/perlin_nolicm.err || exit $?
show gpurun_out/perlin_nolicm.json perlin_nolicm_S64
