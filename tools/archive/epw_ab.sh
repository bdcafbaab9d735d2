#!/bin/bash
# flat bench lines for the fast kernel's envs per wave (BB_EPW: 4 = one 4-env wave per SIMD at 4096 envs)
set -o pipefail
mkdir -p gpurun_out
for e in 4 2 1; do
  BB_EPW=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 300 > gpurun_out/epw_$e.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/epw_$e.json')); print('flat epw=$e', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"
done
