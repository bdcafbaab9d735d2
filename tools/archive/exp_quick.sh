#!/bin/bash
# quick GPU pass: selected GPU tests ($TESTS) then bench lines (flat fp64 short and long forms)
set -o pipefail
mkdir -p gpurun_out/q
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/q/pytest.log 2>&1 || { tail -30 gpurun_out/q/pytest.log; exit 1; }
  tail -2 gpurun_out/q/pytest.log
fi
for s in "--steps 20 --warmup 5" "--steps 512 --warmup 256"; do
  timeout -k 10 200 python -u bench.py $s --no-cpu-baseline $BENCH_ARGS > gpurun_out/q/b.json 2>gpurun_out/q/err.log || { tail gpurun_out/q/err.log; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['value']/1e6,3),'M',round(d['ms_per_step'],4),'ms', d['stats'], 'per_step', round(d.get('per_step',{}).get('value',0)/1e6,3))" gpurun_out/q/b.json "$s"
done
