#!/bin/bash
# Round-4 GPU pass L: the relief pair in its own LICM-off unit -- parity, perlin/flat/hills lines
# (hills at 256 and 512 steps per launch), and the perlin pair's counters.
set -o pipefail
mkdir -p gpurun_out/l
O=gpurun_out/l
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_step.py tests/test_gpu_terrain_stream.py tests/test_gpu_bench_multirank.py -q --timeout 120 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -1 $O/suite.txt
line() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), r.get('kernel_ms'), d['stats'].get('pair_budget'))"; }
for v in "perlin" "flat" "hills --multi-step 512" "hills --multi-step 256"; do
  tag=$(echo $v | tr ' -' '__')
  timeout -k 10 300 python -u bench.py --terrain $v --no-cpu-baseline > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  line $O/b_$tag.json "$v"
done
BB_PAIR_BUDGET_MS=3000 TAG=r04l PREC=fp64 TERRAIN=perlin MULTI=512 F64=1 bash tools/profile.sh > $O/prof_perlin.txt 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof_r04l_fp64_perlin_multi512 $O/r04_perlin_pair1_multi512_nolicm --kernel pair --f64 --timed 1 --pmc-last 2 > $O/sum_perlin.txt 2>&1 || exit $?
python -c "import json;d=json.load(open('$O/r04_perlin_pair1_multi512_nolicm_summary.json'));print(d['avg_ms_rocprof'], d['pmc']['hbm_bytes_per_launch']/1e9, d['pmc']['FETCH_SIZE_kib_raw']*2048/1e9, d['pmc']['WRITE_SIZE_kib']*1024/1e9, d['derived']['issue_frac'], d['scratch'])"
