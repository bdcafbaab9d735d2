#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   trace  : --kernel-trace --stats  (per-kernel average duration)
#   fetch  : --pmc FETCH_SIZE GRBM_GUI_ACTIVE (HBM read bytes, x2 on gfx950 per MI355X_MICROARCH.md;
#            busy cycles summed over the 8 XCDs -> effective clock)
#   write  : --pmc WRITE_SIZE
#   sq     : SQ instruction / wait counters
# Each pass is its own process (counters never combined with traces).
set -o pipefail
TAG=${TAG:-r01}
PREC=${PREC:-fp64}
OUT=gpurun_out/prof_${TAG}_${PREC}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --precision $PREC --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $B --steps 300 --warmup 300 > $OUT/bench_trace.json || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/fetch -o run -- \
  python3 $B --steps 20 --warmup 300 > $OUT/bench_fetch.json || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $B --steps 20 --warmup 300 > $OUT/bench_write.json || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/sq -o run -- python3 $B --steps 20 --warmup 300 > $OUT/bench_sq.json || exit $?
find $OUT -name "*.csv" | head -50
