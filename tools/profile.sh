#!/bin/bash
# rocprofv3 evidence for one bench.py line (run on the GPU box from the repo root).  Every pass
# runs the line's OWN command (ARGS: its bench.py arguments; the CPU leg and the per-step
# comparison are left out, they launch nothing the summary reads), so the timed launch -- the last
# dispatch of the dominant kernel -- has exactly the line's shape (steps per launch, envs,
# terrain, precision):
#   trace  : --kernel-trace --stats  (per-kernel average duration)
#   fetch  : --pmc FETCH_SIZE GRBM_GUI_ACTIVE (HBM read bytes, x2 on gfx950 per MI355X_MICROARCH.md;
#            busy cycles summed over the 8 XCDs -> effective clock)
#   write  : --pmc WRITE_SIZE
#   sq     : SQ instruction / wait counters
#   sq64   : FP64 VALU instruction counters (F64=1)
#   lanes  : SQ_INSTS_VALU_FLOPS_FP64(_TRANS) (FP64 FLOPs of the active lanes) and VALU thread-cycles
#            against VALU busy cycles (LANES=1): how much of the 64-lane upper bound is masked lanes
# Each pass is its own process (counters never combined with traces).
#   TAG=r05 NAME=flat ARGS="--terrain flat" bash tools/profile.sh
#   -> gpurun_out/prof_${TAG}_${NAME}/{trace,fetch,write,sq,sq64}; summarise with tools/prof_summary.py
set -o pipefail
TAG=${TAG:-r05}
NAME=${NAME:-flat}
OUT=gpurun_out/prof_${TAG}_${NAME}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py $ARGS --no-cpu-baseline --no-per-step"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $B > $OUT/bench_trace.json || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/fetch -o run -- \
  python3 $B > $OUT/bench_fetch.json || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $B > $OUT/bench_write.json || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/bench_sq.json || exit $?
if [ "${F64:-1}" = "1" ]; then
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
    --output-format csv -d $OUT/sq64 -o run -- python3 $B > $OUT/bench_sq64.json || exit $?
fi
if [ "${LANES:-1}" = "1" ]; then  # lane activity: FP64 FLOPs counted per active lane, VALU thread-cycles
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU \
    --output-format csv -d $OUT/lanes -o run -- python3 $B > $OUT/bench_lanes.json || exit $?
fi
echo "profile: $OUT"
