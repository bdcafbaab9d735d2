#!/bin/bash
# One parameterised GPU session (run on the GPU box from the repo root, e.g.
#   gpurun --timeout 1200 -- 'TAG=r05 STEPS="suite smoke flat driver perlin" bash tools/gpu_session.sh').
# Every step runs under its own time limit; the first failure ends the session.
#
#   suite            pytest -m gpu (whole GPU suite)
#   tests            pytest -m gpu -k "$K" (a subset; K is a pytest -k expression)
#   smoke            __graft_entry__.smoke()
#   flat driver perlin hills fp32
#                    bench.py lines: configs[1] flat fp64 (500 timed steps), the driver's window
#                    (--steps 20 --warmup 5), configs[2] perlin and hills, flat fp32.
#                    BENCH_ARGS is appended to every bench command line.
#   prof_flat prof_perlin
#                    tools/profile.sh (rocprofv3 kernel trace + separate --pmc passes) of the line's
#                    own command, summarised into profiles/${TAG}_* by tools/prof_summary.py, with
#                    profiles/traffic.json updated for the bench line's roofline.traffic.
#   prof_driver      the same for the driver's 20-step flat launch (its own traffic entry).
#   ppo_flat ppo_perlin
#                    tools/bench_ppo.py: PPO end to end, flat 10M and perlin 5M steps (4096 x 64).
# Run the prof_* steps BEFORE the bench steps: a line reads the traffic entry of its own shape.
# Output: gpurun_out/$TAG/ (bench lines as <step>.json, logs as <step>.log).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r05}
O=gpurun_out/$TAG
mkdir -p $O
STEPS=${STEPS:-"suite smoke flat driver perlin"}
T="--traffic-json profiles/traffic.json"

line() {  # summary of a bench line: value, ms/step, roofline fields
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];x=r.get('valu_fp64_executed') or {};print(sys.argv[2], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms', 'valu_frac', r.get('frac'), 'traffic', r.get('traffic'), 'issue', r.get('issue_frac'), 'exec/counted', x.get('executed_over_counted'), 'status', d.get('status'))" "$1" "$2"
}
bench() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py "$@" $T $BENCH_ARGS > $O/$name.json 2> $O/$name.log || { tail -20 $O/$name.log; exit 1; }
  line $O/$name.json $name
}
prof() {  # name, summary kind, profile.sh env...
  local name=$1 kind=$2; shift 2
  env "$@" TAG=$TAG bash tools/profile.sh > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
}

for s in $STEPS; do
  case $s in
    suite) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
           tail -1 $O/suite.log ;;
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
           tail -1 $O/tests.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
           tail -1 $O/smoke.log ;;
    flat)   bench flat 400 ;;
    driver) bench driver 300 --steps 20 --warmup 5 ;;
    perlin) bench perlin 400 --terrain perlin ;;
    hills)  bench hills 300 --terrain hills --no-cpu-baseline ;;
    fp32)   bench fp32 300 --precision fp32 --no-cpu-baseline ;;
    prof_flat)
      prof prof_flat multi NAME=flat ARGS="--terrain flat"
      python tools/prof_summary.py gpurun_out/prof_${TAG}_flat profiles/${TAG}_flat_multi --kernel multi --f64 --traffic > $O/sum_flat.log 2>&1 || { tail $O/sum_flat.log; exit 1; }
      tail -3 $O/sum_flat.log ;;
    prof_driver)
      prof prof_driver multi NAME=driver ARGS="--terrain flat --steps 20 --warmup 5"
      python tools/prof_summary.py gpurun_out/prof_${TAG}_driver profiles/${TAG}_driver_multi --kernel multi --f64 --traffic > $O/sum_driver.log 2>&1 || { tail $O/sum_driver.log; exit 1; }
      tail -3 $O/sum_driver.log ;;
    prof_perlin)
      prof prof_perlin pair BB_PAIR_BUDGET_MS=3000 NAME=perlin ARGS="--terrain perlin"
      python tools/prof_summary.py gpurun_out/prof_${TAG}_perlin profiles/${TAG}_perlin_pair --kernel pair --f64 --traffic > $O/sum_perlin.log 2>&1 || { tail $O/sum_perlin.log; exit 1; }
      tail -3 $O/sum_perlin.log ;;
    ppo_flat)   timeout -k 10 240 python -u tools/bench_ppo.py --timesteps 10e6 --out $O/ppo_flat > $O/ppo_flat.json 2> $O/ppo_flat.log || { tail -20 $O/ppo_flat.log; exit 1; }
                python -c "import json;d=json.load(open('$O/ppo_flat.json'));print('ppo_flat', round(d['value']/1e6,3), 'M end to end, setup', round(d['setup_s'],3), 's')" ;;
    ppo_perlin) timeout -k 10 240 python -u tools/bench_ppo.py --timesteps 5e6 --terrain perlin --out $O/ppo_perlin > $O/ppo_perlin.json 2> $O/ppo_perlin.log || { tail -20 $O/ppo_perlin.log; exit 1; }
                python -c "import json;d=json.load(open('$O/ppo_perlin.json'));print('ppo_perlin', round(d['value']/1e6,3), 'M end to end, setup', round(d['setup_s'],3), 's')" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
# the summaries prof_summary wrote under profiles/ travel back with gpurun_out/ (copy them into profiles/ here)
mkdir -p $O/profiles && cp profiles/traffic.json profiles/${TAG}_* $O/profiles/ 2>/dev/null
echo SESSION_DONE
