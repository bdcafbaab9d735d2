#!/bin/bash
# Round-4 GPU pass O: like-for-like lines against round 3 (shared terrain stream: hills, perlin)
# and the perlin driver window.
set -o pipefail
mkdir -p gpurun_out/o
O=gpurun_out/o
line() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), r['kernel'][:40], d['stats'].get('pair_budget'))"; }
for v in "hills --shared-stream" "perlin --shared-stream" "perlin --steps 20 --warmup 5"; do
  tag=$(echo $v | tr ' -' '__')
  timeout -k 10 300 python -u bench.py --terrain $v --no-cpu-baseline > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  line $O/b_$tag.json "$v"
done
