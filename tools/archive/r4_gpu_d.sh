#!/bin/bash
# Round-4 GPU pass D: relief pair counters at seg 4/16/64 (perlin, 4096 envs, per-env generators);
# the MachineLICM-off variant build on flat and perlin.
set -o pipefail
mkdir -p gpurun_out
show() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), d['stats'].get('pair_budget'), d.get('pair'))"; }
P="--terrain perlin --no-cpu-baseline"
for v in "S4" "S16" "S64"; do
  env BB_PAIR_SEG=${v#S} timeout -k 10 200 python -u bench.py $P > gpurun_out/paird_$v.json 2> gpurun_out/paird_$v.err || exit $?
  show gpurun_out/paird_$v.json $v
done
timeout -k 10 200 python -u tools/bench_with_lib.py tools/_build/libbb_nolicm.so --no-cpu-baseline > gpurun_out/flat_nolicm.json 2> gpurun_out/flat_nolicm.err || exit $?
show gpurun_out/flat_nolicm.json flat_nolicm
timeout -k 10 200 python -u tools/bench_with_lib.py tools/_build/libbb_nolicm.so $P > gpurun_out/perlin_nolicm.json 2> gpurun_out/perlin_nolicm.err || exit $?
show gpurun_out/perlin_nolicm.json perlin_nolicm
