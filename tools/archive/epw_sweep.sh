#!/bin/bash
# Envs-per-wave sweep on the GPU box: the full kernel's (BB_EPW_FULL) on perlin
# and hills, the fast kernel's (BB_EPW) on flat.  Bench lines under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
for e in 1 2 4; do
  BB_EPW_FULL=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline --terrain perlin > gpurun_out/e_perlin_$e.json || exit 1
  BB_EPW_FULL=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline --terrain hills --n-terrains 64 > gpurun_out/e_hills_$e.json || exit 1
done
for e in 1 2; do
  BB_EPW=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/e_flat_$e.json || exit 1
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/e_*.json")):
    d = json.load(open(f))
    print(f, round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["kernel_ms"], 3))
PY
