#!/bin/bash
# Round-4 GPU pass T2: sanity after the last build change -- suite, smoke, perlin line.
set -o pipefail
mkdir -p gpurun_out/t2
O=gpurun_out/t2
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/suite.txt 2>&1 || { tail -20 $O/suite.txt; exit 1; }
tail -1 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py --terrain perlin --no-cpu-baseline > $O/perlin.json 2> $O/perlin.err || exit $?
python -c "import json;d=json.loads(open('$O/perlin.json').read().splitlines()[-1]);print('perlin', round(d['value']/1e6,3), d['stats']['pair_budget'])"
