#!/bin/bash
# Round-4 GPU pass I: FMA contraction fixed per source expression -- the whole GPU suite, then
# flat/perlin throughput (default, one-launch pair, solo waves).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/suite_r4j.txt 2>&1
rc=$?; tail -5 gpurun_out/suite_r4j.txt; grep FAILED gpurun_out/suite_r4j.txt | head
show() { python -c "
import json;d=json.loads(open('$1').read().splitlines()[-1]);p=d.get('pair',{})
print('$2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), d['stats'].get('pair_budget'), 'heavy', p.get('heavy'), 'env_mcyc', {k: round(v) for k, v in p.get('env_mcycles', {}).items()}, 'fin', {k: round(v) for k, v in p.get('env_finish_ms_before_last', {}).items()})"; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/pairi_flat.json 2> gpurun_out/pairi_flat.err || exit $?
show gpurun_out/pairi_flat.json flat
P="--terrain perlin --no-cpu-baseline"
for v in "base" "one" "solo64" "one_solo64"; do
  case $v in
    base) E="";; one) E="BB_PAIR_ONE=1";; solo64) E="BB_PAIR_SOLO=64";; one_solo64) E="BB_PAIR_ONE=1 BB_PAIR_SOLO=64";;
  esac
  env $E timeout -k 10 200 python -u bench.py $P > gpurun_out/pairi_$v.json 2> gpurun_out/pairi_$v.err || exit $?
  show gpurun_out/pairi_$v.json $v
done
exit $rc
