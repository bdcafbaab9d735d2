#!/bin/bash
# HBM-traffic attribution for the fast step kernel (run on the GPU box from the repo root).
# FETCH_SIZE / WRITE_SIZE per launch at several env counts: the slope is the
# per-env-step traffic, the intercept the per-launch fixed part (code object
# fetched into each XCD's L2, the shared terrain, kernel arguments).  Each pass
# is its own rocprofv3 process (counters never combined with traces).
#   tools/traffic_sweep.sh ; python tools/traffic_fit.py gpurun_out/traffic_sweep
set -o pipefail
PREC=${PREC:-fp64}
OUT=gpurun_out/traffic_sweep
mkdir -p $OUT
export TMPDIR=/tmp
for E in ${ENVS:-1024 4096 16384}; do
  B="bench.py --precision $PREC --no-cpu-baseline --envs $E --steps 20 --warmup 200"
  echo "envs=$E fetch"
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${PREC}_${E}_fetch -o run -- \
    python3 $B > $OUT/${PREC}_${E}_fetch.json || exit $?
  echo "envs=$E write"
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${PREC}_${E}_write -o run -- \
    python3 $B > $OUT/${PREC}_${E}_write.json || exit $?
done
