#!/bin/bash
# Round-5 diagnostic: which of the relief pair's output stores make its write-backs.  WRITE_SIZE of
# the timed perlin launch with the product library and with variants that drop some output stores
# (-DBB_OUT_SKIP: 22 = reward/done/pos2d, 9 = obs/terminal obs, 31 = all five; outputs invalid).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
B="--terrain perlin --no-cpu-baseline --no-per-step"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_base -o run -- python3 bench.py $B > $O/base.json || exit 1
for v in skip_small skip_obs skip_all; do
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$v -o run -- \
    python3 tools/bench_with_lib.py tools/variants/libbb_$v.so $B > $O/$v.json || exit 1
done
echo OUTSKIP_DONE
