#!/bin/bash
# Round-4 GPU pass G: steps per launch 256 vs 512 (one launch for the 500 timed steps) on perlin
# and flat, then the rocprofv3 evidence for the perlin line (relief pair).
set -o pipefail
mkdir -p gpurun_out
show() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), d['roofline']['kernel_launches_timed'], d['stats'].get('pair_budget'))"; }
for t in perlin flat; do
  for m in 256 512; do
    timeout -k 10 200 python -u bench.py --terrain $t --multi-step $m --no-cpu-baseline > gpurun_out/k_${t}_$m.json 2> gpurun_out/k_${t}_$m.err || exit $?
    show gpurun_out/k_${t}_$m.json ${t}_$m
  done
done
bash tools/r4_prof_perlin.sh
