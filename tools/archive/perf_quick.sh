#!/bin/bash
# Quick perf loop on the GPU box: step parity tests, then flat / perlin / hills
# bench lines (no CPU baseline) and the perlin phase clocks.  Writes under
# gpurun_out/ and prints one summary line per bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_terrain.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -1 gpurun_out/pytest_quick.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --terrain perlin > gpurun_out/q_perlin.json &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --terrain hills --n-terrains 64 > gpurun_out/q_hills.json &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/q_flat.json || exit 1
if [ -f tools/_build/libbb_phase.so ]; then
  timeout -k 10 300 python -u tools/phase_clocks.py --terrain perlin > gpurun_out/q_pc_perlin.json || exit 1
fi
python - <<'PY'
import json, os
for f in ("flat", "perlin", "hills"):
    d = json.load(open(f"gpurun_out/q_{f}.json"))
    print(f, round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["kernel_ms"], 3))
if os.path.exists("gpurun_out/q_pc_perlin.json"):
    d = json.load(open("gpurun_out/q_pc_perlin.json"))
    print({k: round(v, 1) for k, v in d.get("full_kernel", {}).items()})
    print("fast collide", round(d["cycles_per_forward"]["collide"]), "total", round(d["total_cycles_per_forward"]))
PY
