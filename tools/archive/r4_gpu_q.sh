#!/bin/bash
# Round-4 GPU pass Q: flat A/B -- product vs MachineLICM off vs LICM off + the mass-matrix row in
# registers across Newton iterations (BB_HROW_REG), default window and driver window, twice each.
set -o pipefail
mkdir -p gpurun_out/q
O=gpurun_out/q
line() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2', round(d['value']/1e6,3), 'M', round(d['roofline']['kernel_ms'],2))"; }
for rep in 1 2; do
for v in prod nolicm hrow_nolicm; do
  if [ $v = prod ]; then C="bench.py"; else C="tools/bench_with_lib.py tools/_build/libbb_$v.so"; fi
  timeout -k 10 200 python -u $C --no-cpu-baseline > $O/f_${v}_$rep.json 2> $O/f_${v}_$rep.err || exit $?
  line $O/f_${v}_$rep.json "flat $v"
  timeout -k 10 200 python -u $C --no-cpu-baseline --steps 20 --warmup 5 > $O/d_${v}_$rep.json 2> $O/d_${v}_$rep.err || exit $?
  line $O/d_${v}_$rep.json "driver $v"
done
done
