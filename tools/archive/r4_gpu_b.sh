#!/bin/bash
# Round-4 GPU pass B: relief pair split/segment sweep on perlin (4096 envs, per-env generators),
# and the GPU suite with the captured hand-over count reset by hipMemsetAsync.
set -o pipefail
mkdir -p gpurun_out
P="--terrain perlin --no-cpu-baseline"
for v in "A" "F50" "F62" "F75" "F62S64" "A_S64" "A_S4"; do
  case $v in
    A) E="";; F50) E="BB_PAIR_ADAPT=0 BB_PAIR_FULL=50";; F62) E="BB_PAIR_ADAPT=0 BB_PAIR_FULL=62";;
    F75) E="BB_PAIR_ADAPT=0 BB_PAIR_FULL=75";; F62S64) E="BB_PAIR_ADAPT=0 BB_PAIR_FULL=62 BB_PAIR_SEG=64";;
    A_S64) E="BB_PAIR_SEG=64";; A_S4) E="BB_PAIR_SEG=4";;
  esac
  env $E timeout -k 10 200 python -u bench.py $P > gpurun_out/pair_$v.json 2> gpurun_out/pair_$v.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/pair_$v.json').read().splitlines()[-1]);print('$v', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), d['stats']['pair_budget'])"
done
BB_COUNT_MEMSET=1 timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/suite_r4f_memset.txt 2>&1
rc=$?
tail -4 gpurun_out/suite_r4f_memset.txt
exit $rc
