#!/bin/bash
# perlin / hills bench lines for the full kernel's envs per wave (BB_EPW_FULL) and the step route (BB_ROUTE)
set -o pipefail
mkdir -p gpurun_out
for cfg in "4 0" "2 0" "1 0" "4 1"; do
  set -- $cfg
  BB_EPW_FULL=$1 BB_ROUTE=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --terrain perlin --steps 300 > gpurun_out/epwf_$1_$2.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/epwf_$1_$2.json')); print('perlin epw_full=$1 route=$2', round(d['value']), round(d['ms_per_step'],3), d['stats']['slow_path'])"
done
