#!/bin/bash
# Round-4 GPU pass F: per-env chain times of the relief pair (perlin, 4096 envs, per-env generators).
set -o pipefail
mkdir -p gpurun_out
show() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), d['stats'].get('pair_budget'), json.dumps(d.get('pair')))"; }
P="--terrain perlin --no-cpu-baseline"
for v in "S16"; do
  env BB_PAIR_SEG=${v#S} timeout -k 10 200 python -u bench.py $P > gpurun_out/pairf_$v.json 2> gpurun_out/pairf_$v.err || exit $?
  show gpurun_out/pairf_$v.json $v
done
