#!/bin/bash
# Round-4 last check on the tree as it ends the round: suite, smoke, the default bench line.
set -o pipefail
mkdir -p gpurun_out/x
O=gpurun_out/x
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/suite.txt 2>&1 || { tail -20 $O/suite.txt; exit 1; }
tail -1 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print(round(d['value']/1e6,3), d['roofline']['traffic'], d['cpu_baseline']['value'])"
