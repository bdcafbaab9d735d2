#!/bin/bash
# Round-4 GPU pass N: the relief pair with XCD-sharded rings (and the per-env hand-over record) --
# multi-step parity, perlin throughput at seg 16 / 64, and the pair's HBM traffic.
set -o pipefail
mkdir -p gpurun_out/n
O=gpurun_out/n
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_step.py tests/test_gpu_terrain_stream.py -q --timeout 120 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -1 $O/suite.txt
line() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), r.get('kernel_ms'), d['stats'].get('pair_budget'))"; }
for sg in 16 64; do
  BB_PAIR_SEG=$sg timeout -k 10 300 python -u bench.py --terrain perlin --no-cpu-baseline > $O/b_perlin_$sg.json 2> $O/b_perlin_$sg.err || exit $?
  line $O/b_perlin_$sg.json perlin_seg$sg
done
BB_PAIR_BUDGET_MS=3000 TAG=r04n PREC=fp64 TERRAIN=perlin MULTI=512 F64=1 bash tools/profile.sh > $O/prof_perlin.txt 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof_r04n_fp64_perlin_multi512 $O/r04_perlin_pair1_multi512_xcd --kernel pair --f64 --timed 1 --pmc-last 2 > $O/sum_perlin.txt 2>&1 || exit $?
python -c "import json;d=json.load(open('$O/r04_perlin_pair1_multi512_xcd_summary.json'));print(d['avg_ms_rocprof'], d['pmc']['hbm_bytes_per_launch']/1e9, d['pmc']['FETCH_SIZE_kib_raw']*2048/1e9, d['pmc']['WRITE_SIZE_kib']*1024/1e9, d['derived']['issue_frac'], d['scratch'])"
