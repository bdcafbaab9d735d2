#!/bin/bash
# A/B of variant libraries on the GPU box (from the repo root): bench.py through each library,
# the product first and last.  LIBS: variant names (tools/variants/libbb_<name>.so); ARGS: bench
# arguments (default: the flat 500-step line without the CPU leg); OUT: gpurun_out subdirectory.
#   LIBS="dupls dupchol" OUT=ab1 bash tools/ab_run.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-ab}
mkdir -p $OUT
ARGS=${ARGS:-"--no-cpu-baseline --no-per-step"}
show() {
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], round(d['value']/1e6,3), 'M', 'kernel_ms', round(r['kernel_ms'],3), 'iters', d['stats']['solver_iters'])" "$1" "$2"
}
run() {  # name lib
  if [ "$2" = product ]; then
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/$1.json 2> $OUT/$1.log || { tail -5 $OUT/$1.log; exit 1; }
  else
    timeout -k 10 200 python -u tools/bench_with_lib.py tools/variants/libbb_$2.so $ARGS > $OUT/$1.json 2> $OUT/$1.log || { tail -5 $OUT/$1.log; exit 1; }
  fi
  show $OUT/$1.json $1
}
run product_a product
for v in $LIBS; do run $v $v; done
run product_b product
echo AB_DONE
