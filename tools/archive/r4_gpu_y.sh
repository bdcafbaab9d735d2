#!/bin/bash
# Round-4 GPU pass Y: relief pair segment length A/B on perlin, three runs each.
set -o pipefail
mkdir -p gpurun_out/y
for rep in 1 2 3; do
for sg in 16 64; do
  BB_PAIR_SEG=$sg timeout -k 10 200 python -u bench.py --terrain perlin --no-cpu-baseline --no-per-step > gpurun_out/y/s${sg}_$rep.json 2> gpurun_out/y/s${sg}_$rep.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/y/s${sg}_$rep.json').read().splitlines()[-1]);print('seg$sg', round(d['value']/1e6,3))"
done
done
