#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   trace  : --kernel-trace --stats  (per-kernel average duration)
#   fetch  : --pmc FETCH_SIZE GRBM_GUI_ACTIVE (HBM read bytes, x2 on gfx950 per MI355X_MICROARCH.md;
#            busy cycles summed over the 8 XCDs -> effective clock)
#   write  : --pmc WRITE_SIZE
#   sq     : SQ instruction / wait counters
#   sq64   : FP64 VALU instruction counters (F64=1)
# Each pass is its own process (counters never combined with traces).
# TERRAIN=perlin profiles configs[2] (the bench's per-env terrain streams).
set -o pipefail
TAG=${TAG:-r01}
PREC=${PREC:-fp64}
TERRAIN=${TERRAIN:-flat}
OUT=gpurun_out/prof_${TAG}_${PREC}_${TERRAIN}
mkdir -p $OUT
export TMPDIR=/tmp
# MULTI=M: bench.py's bb_step_multi mode (M steps per launch); default 0 = one bb_step per step
MULTI=${MULTI:-0}
B="bench.py --precision $PREC --terrain $TERRAIN --no-cpu-baseline --multi-step $MULTI"
# PMC passes: a few launches of the timed shape (multi: whole 64-step launches only)
S="--steps 20 --warmup 300"
if [ "$MULTI" != "0" ]; then OUT=${OUT}_multi$MULTI; mkdir -p $OUT; S="--steps $((2 * MULTI)) --burn-in $((2 * MULTI)) --warmup $((2 * MULTI)) --no-per-step"; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $B --steps 512 --warmup 256 > $OUT/bench_trace.json || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/fetch -o run -- \
  python3 $B $S > $OUT/bench_fetch.json || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $B $S > $OUT/bench_write.json || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/sq -o run -- python3 $B $S > $OUT/bench_sq.json || exit $?
if [ "${F64:-0}" = "1" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
    --output-format csv -d $OUT/sq64 -o run -- python3 $B $S > $OUT/bench_sq64.json || exit $?
fi
find $OUT -name "*.csv" | head -50
