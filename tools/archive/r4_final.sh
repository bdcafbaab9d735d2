#!/bin/bash
# Round-4 closing GPU pass: suite, smoke, rocprofv3 evidence of the flat multi-step kernel and the
# perlin relief pair (summarised here so the bench lines read their traffic), then the bench lines
# (flat / driver window / perlin / fp32 / hills).
set -o pipefail
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/suite.txt 2>&1 || { tail -20 $O/suite.txt; exit 1; }
tail -1 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
TAG=r04 PREC=fp64 TERRAIN=flat MULTI=512 F64=1 bash tools/profile.sh > $O/prof_flat.txt 2>&1 || exit $?
BB_PAIR_BUDGET_MS=3000 TAG=r04 PREC=fp64 TERRAIN=perlin MULTI=512 F64=1 bash tools/profile.sh > $O/prof_perlin.txt 2>&1 || exit $?
cp profiles/traffic.json $O/traffic.json
python tools/prof_summary.py gpurun_out/prof_r04_fp64_flat_multi512 $O/r04_fp64_multi512 --kernel multi --f64 --traffic --timed 1 --pmc-last 2 > $O/sum_flat.txt 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof_r04_fp64_perlin_multi512 $O/r04_perlin_pair1_multi512 --kernel pair --f64 --traffic --timed 1 --pmc-last 2 > $O/sum_perlin.txt 2>&1 || exit $?
T="--traffic-json $O/traffic.json"
line() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), r.get('frac'), r.get('traffic'), r.get('issue_frac'), (r.get('valu_fp64') or {}).get('frac'))"; }
timeout -k 10 400 python -u bench.py $T > $O/bench_flat.json 2> $O/bench_flat.err || exit $?
line $O/bench_flat.json flat
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 $T > $O/bench_flat_short.json 2> $O/bench_flat_short.err || exit $?
line $O/bench_flat_short.json flat_driver
timeout -k 10 400 python -u bench.py --terrain perlin $T > $O/bench_perlin.json 2> $O/bench_perlin.err || exit $?
line $O/bench_perlin.json perlin
timeout -k 10 300 python -u bench.py --precision fp32 --no-cpu-baseline $T > $O/bench_flat_fp32.json 2> $O/bench_flat_fp32.err || exit $?
line $O/bench_flat_fp32.json flat_fp32
timeout -k 10 300 python -u bench.py --terrain hills --no-cpu-baseline $T > $O/bench_hills.json 2> $O/bench_hills.err || exit $?
line $O/bench_hills.json hills
echo FINAL_DONE
# hills at 256 steps per launch (the adaptive route's parked form needs a launch without full steps)
timeout -k 10 300 python -u bench.py --terrain hills --multi-step 256 --no-cpu-baseline $T > $O/bench_hills256.json 2> $O/bench_hills256.err || exit $?
line $O/bench_hills256.json hills256
