#!/bin/bash
# Round-5 A/B of variant builds (tools/variants/libbb_<name>.so, built here by
# tools/lib_bench.py --build-only) on the flat bench line and the driver's window, alternating
# base and variant.  VARIANTS="base ls3" ROUNDS=2 bash tools/archive/r5_ab.sh
set -o pipefail
O=gpurun_out/r05ab; mkdir -p $O
B="--no-cpu-baseline --no-per-step"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base ls3}; do
    for w in flat driver; do
      X=""; [ $w = driver ] && X="--steps 20 --warmup 5"
      [ -n "$PERLIN" ] && [ $w = driver ] && X="--terrain perlin"
      timeout -k 10 300 python -u tools/bench_with_lib.py tools/variants/libbb_$v.so $B $X > $O/${v}_${w}_$r.json 2> $O/${v}_${w}_$r.log || { tail $O/${v}_${w}_$r.log; exit 1; }
      python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],2))" $O/${v}_${w}_$r.json "$v $w $r"
    done
  done
done
echo AB_DONE
