#!/bin/bash
# Round-4 GPU pass S: scheduling variants -- the max-ILP machine scheduler for every kernel
# (-mllvm -amdgpu-sched-strategy=max-ilp) and one wave per EU declared on the multi-step kernel
# (BB_WPE1) -- against the product: flat (500-step line and driver window), perlin.
set -o pipefail
mkdir -p gpurun_out/s
O=gpurun_out/s
line() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2', round(d['value']/1e6,3), 'M', round(d['roofline']['kernel_ms'],2))"; }
for rep in 1 2; do
for v in prod maxilp wpe1; do
  if [ $v = prod ]; then C="bench.py"; else C="tools/bench_with_lib.py tools/_build/libbb_$v.so"; fi
  timeout -k 10 200 python -u $C --no-cpu-baseline > $O/f_${v}_$rep.json 2> $O/f_${v}_$rep.err || exit $?
  line $O/f_${v}_$rep.json "flat $v"
  timeout -k 10 200 python -u $C --no-cpu-baseline --steps 20 --warmup 5 > $O/d_${v}_$rep.json 2> $O/d_${v}_$rep.err || exit $?
  line $O/d_${v}_$rep.json "driver $v"
done
done
for v in prod maxilp; do
  if [ $v = prod ]; then C="bench.py"; else C="tools/bench_with_lib.py tools/_build/libbb_$v.so"; fi
  timeout -k 10 200 python -u $C --terrain perlin --no-cpu-baseline > $O/p_${v}.json 2> $O/p_${v}.err || exit $?
  line $O/p_${v}.json "perlin $v"
done
