#!/bin/bash
# A/B of environment-variable variants of the product library on the GPU box (repo root): bench.py
# once per "NAME:VAR=VAL,VAR=VAL" entry of VARIANTS (NAME:- for the product defaults).
#   VARIANTS="base:- pair:BB_ROUTE=0" ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-per-step" OUT=x bash tools/ab_env.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-abenv}
mkdir -p $OUT
ARGS=${ARGS:-"--no-cpu-baseline --no-per-step"}
for v in $VARIANTS; do
  name=${v%%:*}; vars=${v#*:}
  envs=""
  [ "$vars" != "-" ] && envs=$(echo $vars | tr ',' ' ')
  env $envs timeout -k 10 200 python -u bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.log || { tail -5 $OUT/$name.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], round(d['value']/1e6,3), 'M', 'kernel_ms', round(r['kernel_ms'],3), 'launches', r['kernel_launches_timed'], 'iters', d['stats']['solver_iters'])" $OUT/$name.json "$v"
done
echo ABENV_DONE
