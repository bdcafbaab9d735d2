#!/bin/bash
# Envs-per-GPU sweep (flat, fp64, 200 timed steps): env-steps/s per size.
set -o pipefail
mkdir -p gpurun_out
for n in 1024 2048 4096 8192 16384 32768 65536; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --envs $n --steps 200 --warmup 100 > gpurun_out/sweep_$n.json || exit 1
done
python - <<'PY'
import json
for n in (1024, 2048, 4096, 8192, 16384, 32768, 65536):
    d = json.load(open(f"gpurun_out/sweep_{n}.json"))
    print(n, round(d["value"]), round(d["ms_per_step"], 3))
PY
