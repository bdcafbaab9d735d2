#!/bin/bash
# rocprofv3 kernel trace of the perlin bench (route 0: predict, split, full kernel on the side
# stream, fast kernel, full kernel over the hand-overs)
set -o pipefail
OUT=gpurun_out/prof_${TAG:-r02}_perlin
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --no-cpu-baseline --terrain perlin --steps 200 --warmup 100 > $OUT/bench_trace.json || exit $?
ls $OUT/trace
