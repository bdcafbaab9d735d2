#!/bin/bash
# Step routing A/B on flat terrain: predicted concurrent route (default) vs the
# serial fast-then-full route (BB_ROUTE=1), three runs each, bench lines only.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/r0_$i.json || exit 1
  BB_ROUTE=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/r1_$i.json || exit 1
done
python - <<'PY'
import json
for r in ("r0", "r1"):
    v = [json.load(open(f"gpurun_out/{r}_{i}.json")) for i in (1, 2, 3)]
    print(r, [round(d["value"]) for d in v], [round(d["ms_per_step"], 4) for d in v], [round(d["roofline"]["kernel_ms"], 4) for d in v])
PY
