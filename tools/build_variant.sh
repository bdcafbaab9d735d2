#!/bin/bash
# A variant build of the HIP library for A/B runs (CPU, this container): one source recompiled with
# extra flags, linked with the product's other objects (openballbot-rl_amd/ballbot_gym/_lib/obj).
#   bash tools/build_variant.sh NAME SOURCE "FLAGS"     e.g.  bash tools/build_variant.sh dupls bb_kernels.hip "-DBB_EXP_DUP_LS"
# -> tools/variants/libbb_NAME.so (travels to the GPU box; run it with tools/bench_with_lib.py or
# tools/variant_test.py).  bb_pair.hip keeps its product flag (-mllvm -disable-machine-licm).
set -e -o pipefail
NAME=$1; SRC=$2; FLAGS=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/openballbot-rl_amd/ballbot_gym/_lib/obj
OUT=$ROOT/tools/variants
mkdir -p $OUT/obj_$NAME
EXTRA=""
[ "$SRC" = "bb_pair.hip" ] && EXTRA="-mllvm -disable-machine-licm"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $EXTRA $FLAGS -c -o $OUT/obj_$NAME/${SRC%.hip}.o \
  $ROOT/openballbot-rl_amd/csrc/$SRC
OBJS=""
for o in $OBJ/*.o; do
  b=$(basename $o)
  if [ "$b" = "${SRC%.hip}.o" ]; then OBJS="$OBJS $OUT/obj_$NAME/$b"; else OBJS="$OBJS $o"; fi
done
hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libbb_$NAME.so $OBJS
echo "built $OUT/libbb_$NAME.so"
