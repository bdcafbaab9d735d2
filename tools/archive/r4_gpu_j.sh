#!/bin/bash
# Round-4 GPU pass J: the one-launch relief pair's parity, the driver's flat window, and the
# rocprofv3 evidence for the perlin line on the one-launch pair (one dispatch per launch, so the
# per-dispatch counters see the whole pair).
set -o pipefail
mkdir -p gpurun_out
BB_PAIR_ONE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_multi_step.py tests/test_gpu_terrain_stream.py -q --timeout 120 --timeout-method thread > gpurun_out/suite_r4k_one.txt 2>&1 || { tail -30 gpurun_out/suite_r4k_one.txt; exit 1; }
tail -1 gpurun_out/suite_r4k_one.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/driver_flat.json 2> gpurun_out/driver_flat.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/driver_flat.json').read().splitlines()[-1]);print('driver flat', round(d['value']/1e6,3), d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline'].get('valu_fp64',{}).get('frac'))"
for v in nolicm cfoff; do
  timeout -k 10 200 python -u tools/bench_with_lib.py tools/_build/libbb_$v.so --no-cpu-baseline > gpurun_out/flat_$v.json 2> gpurun_out/flat_$v.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/flat_$v.json').read().splitlines()[-1]);print('flat $v', round(d['value']/1e6,3), d['roofline']['kernel_ms'])"
done
for v in base dup_sat dup_bodycol dup_solve_full; do
  if [ $v = base ]; then C="bench.py"; else C="tools/bench_with_lib.py tools/_build/libbb_$v.so"; fi
  timeout -k 10 200 python -u $C --terrain perlin --no-cpu-baseline > gpurun_out/perlin_$v.json 2> gpurun_out/perlin_$v.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/perlin_$v.json').read().splitlines()[-1]);p=d.get('pair',{});print('perlin $v', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), p.get('env_mcycles',{}).get('p100'), p.get('env_mcycles',{}).get('mean'))"
done
export BB_PAIR_ONE=1
bash tools/r4_prof_perlin.sh
