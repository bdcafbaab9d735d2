#!/bin/bash
# Round-5 A/B: solo waves for the heavy envs' full steps (BB_PAIR_SOLO workgroups of one team,
# BB_PAIR_HEAVY: % of the mean env's cycles that marks an env heavy) on the perlin line.
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
B="--terrain perlin --no-cpu-baseline --no-per-step"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py $B > $O/$name.json 2> $O/$name.log || { tail $O/$name.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);p=d.get('pair') or {};print(sys.argv[2], round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), p.get('env_mcycles',{}).get('p100'), p.get('env_mcycles',{}).get('p50'))" $O/$name.json $name
}
run base BB_PAIR_SOLO=0
run solo120 BB_PAIR_SOLO=120
run solo120_h130 BB_PAIR_SOLO=120 BB_PAIR_HEAVY=130
run solo96 BB_PAIR_SOLO=96
run base2 BB_PAIR_SOLO=0
echo SOLO_DONE
