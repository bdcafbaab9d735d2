#!/bin/bash
# Round-4 GPU pass P: team_sync as a compiler barrier (no s_waitcnt lgkmcnt(0) per sync) --
# the whole GPU suite, then flat (default and driver window) and perlin lines.
set -o pipefail
mkdir -p gpurun_out/p
O=gpurun_out/p
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/suite.txt 2>&1
rc=$?; tail -2 $O/suite.txt; grep FAILED $O/suite.txt | head
[ $rc = 0 ] || exit $rc
line() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), r.get('kernel_ms'), d['stats'].get('pair_budget'))"; }
for v in "flat" "flat --steps 20 --warmup 5" "perlin"; do
  tag=$(echo $v | tr ' -' '__')
  timeout -k 10 300 python -u bench.py --terrain $v --no-cpu-baseline > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  line $O/b_$tag.json "$v"
done
