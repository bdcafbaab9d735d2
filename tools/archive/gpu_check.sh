#!/bin/bash
# One GPU-box pass: gpu parity tests, smoke, bench lines (fp64 default, fp32), rocprof trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/bench_fp64.json 2> gpurun_out/bench_fp64.err || { tail gpurun_out/bench_fp64.err; exit 1; }
cat gpurun_out/bench_fp64.json
timeout -k 10 300 python -u bench.py --precision fp32 --no-cpu-baseline > gpurun_out/bench_fp32.json 2> gpurun_out/bench_fp32.err || exit 1
cat gpurun_out/bench_fp32.json
# the driver's own short form (steady state comes from the burn-in, not the warmup)
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err || exit 1
cat gpurun_out/bench_short.json
