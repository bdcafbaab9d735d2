#!/bin/bash
# Round-4 rocprofv3 evidence for the perlin bench line (relief pair, 256 steps per launch):
# trace + FETCH/WRITE + SQ + FP64 passes (tools/profile.sh).  BB_PAIR_BUDGET_MS bounds a pair
# launch should the profiler serialise its two kernels (then stats.pair_budget > 0 says so).
set -o pipefail
export BB_PAIR_BUDGET_MS=3000
TAG=r04 PREC=fp64 TERRAIN=perlin MULTI=256 F64=1 bash tools/profile.sh || exit $?
for f in gpurun_out/prof_r04_fp64_perlin_multi256/bench_*.json; do
  python -c "import json,sys;d=json.loads(open('$f').read().splitlines()[-1]);print('$f', round(d['value']/1e6,3), d['stats']['pair_budget'], d.get('pair',{}).get('claims_full'))"
done
