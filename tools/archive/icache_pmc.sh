#!/bin/bash
# Instruction-cache counters of the step kernels (diagnostic, GPU box): which
# SQC/SQ instruction-fetch counters gfx950 exposes, then one --pmc pass per
# counter group on a short bench run (flat and perlin).
set -o pipefail
mkdir -p gpurun_out/icache
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/icache/avail.txt 2>&1; cd $GRAFT_REPO_ROOT
grep -i -E "ICACHE|IFETCH|INST_LEVEL|SQC_" gpurun_out/icache/avail.txt | head -40
for t in flat perlin; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/icache/$t -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --terrain $t --steps 30 --warmup 10 --burn-in 100 > gpurun_out/icache/$t.json 2> gpurun_out/icache/$t.err || { tail -5 gpurun_out/icache/$t.err; exit 1; }
done
