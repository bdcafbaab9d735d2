#!/bin/bash
# Round-5 A/B: nontemporal output stores (tools/variants/libbb_nt.so, -DBB_OUT_NT) on perlin and
# flat (speed + WRITE_SIZE of the timed launch), and two envs per wave on flat (BB_EPW=2).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
B="--no-cpu-baseline --no-per-step"
v() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2],round(d['value']/1e6,3),'M')" $1 $2; }
for t in perlin flat; do
  timeout -k 10 200 python -u bench.py --terrain $t $B > $O/${t}_base.json 2> $O/${t}_base.log || exit 1; v $O/${t}_base.json ${t}_base
  timeout -k 10 200 python -u tools/bench_with_lib.py tools/variants/libbb_nt.so --terrain $t $B > $O/${t}_nt.json 2> $O/${t}_nt.log || exit 1; v $O/${t}_nt.json ${t}_nt
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_${t}_base -o run -- python3 bench.py --terrain $t $B > /dev/null || exit 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_${t}_nt -o run -- python3 tools/bench_with_lib.py tools/variants/libbb_nt.so --terrain $t $B > /dev/null || exit 1
done
for e in 2 4; do
  BB_EPW=$e timeout -k 10 200 python -u bench.py $B > $O/flat_epw$e.json 2> $O/flat_epw$e.log || exit 1; v $O/flat_epw$e.json flat_epw$e
  BB_EPW=$e timeout -k 10 200 python -u bench.py $B --steps 20 --warmup 5 > $O/drv_epw$e.json 2> $O/drv_epw$e.log || exit 1; v $O/drv_epw$e.json drv_epw$e
done
echo AB_DONE
