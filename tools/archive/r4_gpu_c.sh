#!/bin/bash
# Round-4 GPU pass C: relief pair with device-coherent hand-over (no L2 flush):
# multi-step parity first, then the segment sweep on perlin (4096 envs, per-env generators),
# then the MachineLICM-off variant build on flat and perlin.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_step.py tests/test_gpu_terrain_stream.py -x -v --timeout 120 --timeout-method thread > gpurun_out/suite_r4g_multi.txt 2>&1 || { tail -30 gpurun_out/suite_r4g_multi.txt; exit 1; }
tail -2 gpurun_out/suite_r4g_multi.txt
show() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), d['stats'].get('pair_budget'))"; }
P="--terrain perlin --no-cpu-baseline"
for v in "A" "A_S4" "A_S64" "Q"; do
  case $v in
    A) E="";; A_S4) E="BB_PAIR_SEG=4";; A_S64) E="BB_PAIR_SEG=64";; Q) E="BB_RELIEF_PAIR=0";;
  esac
  env $E timeout -k 10 200 python -u bench.py $P > gpurun_out/pairc_$v.json 2> gpurun_out/pairc_$v.err || exit $?
  show gpurun_out/pairc_$v.json $v
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/flat_base.json 2> gpurun_out/flat_base.err || exit $?
show gpurun_out/flat_base.json flat_base
timeout -k 10 200 python -u tools/bench_with_lib.py tools/_build/libbb_nolicm.so --no-cpu-baseline > gpurun_out/flat_nolicm.json 2> gpurun_out/flat_nolicm.err || exit $?
show gpurun_out/flat_nolicm.json flat_nolicm
timeout -k 10 200 python -u tools/bench_with_lib.py tools/_build/libbb_nolicm.so $P > gpurun_out/perlin_nolicm.json 2> gpurun_out/perlin_nolicm.err || exit $?
show gpurun_out/perlin_nolicm.json perlin_nolicm
