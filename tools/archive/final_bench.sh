#!/bin/bash
# Round-end GPU pass: gpu tests, smoke, bench lines (flat fp64 default, driver short form,
# flat fp32, perlin and hills relief banks), each step under its own time limit.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log | tail -1
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['value']/1e6,3),'M',round(d['ms_per_step'],4),'ms')" $O/$name.json $name
}
run bench_flat_fp64
run bench_flat_fp64_short --steps 20 --warmup 5 --no-cpu-baseline
run bench_flat_fp32 --precision fp32 --no-cpu-baseline
run bench_perlin --terrain perlin --no-cpu-baseline
run bench_hills --terrain hills --no-cpu-baseline
if [ "${QUEUE_AB:-0}" = "1" ]; then  # relief banks through the parked multi-step kernels instead of the work queue
  BB_MULTI_QUEUE=0 run bench_hills_noqueue --terrain hills --no-cpu-baseline
  BB_MULTI_QUEUE=0 run bench_perlin_noqueue --terrain perlin --no-cpu-baseline
fi
