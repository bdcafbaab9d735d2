#!/bin/bash
# bench sweep over lanes-per-env team sizes (GPU box); results -> gpurun_out/sweep.jsonl
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep.jsonl
: > $out
for prec in ${PRECS:-fp64 fp32}; do
  for L in ${TEAMS:-8 16 32}; do
    echo "== $prec team $L" >&2
    BB_TEAM=$L timeout -k 10 240 python bench.py --steps ${STEPS:-200} --warmup ${WARM:-300} --precision $prec \
      --no-cpu-baseline > gpurun_out/sweep_tmp.json || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/sweep_tmp.json')); print(json.dumps({'prec':'$prec','team':$L,'value':d['value'],'ms':d['ms_per_step'],'launch':d['config']['launch'],'iters':d['stats']}))" | tee -a $out
  done
done
