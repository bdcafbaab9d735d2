#!/bin/bash
# PPO 3M-step runs, interleaved A/B (first run is a warm-up): step routing auto
# (serial on flat banks) vs predicted (BB_ROUTE=0), and split-K 64-row vs 512-row slices.
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 200 env $2 python -u tools/bench_ppo.py --timesteps 3e6 --out gpurun_out/ppo_$1 > gpurun_out/ppo_$1.json 2>/dev/null; }
run warm "BB_ROUTE=0" || exit 1
run r0_a "BB_ROUTE=0" && run auto_a "X=1" && run s16_a "BB_SPLITK_ROWS=512" && \
run r0_b "BB_ROUTE=0" && run auto_b "X=1" && run s16_b "BB_SPLITK_ROWS=512" || exit 1
python - <<'PY'
import json
for f in ("warm", "r0_a", "auto_a", "s16_a", "r0_b", "auto_b", "s16_b"):
    d = json.load(open(f"gpurun_out/ppo_{f}.json"))
    print(f, round(d["value"]), "rollout_s", round(d["rollout_s"], 2), "update_s", round(d["update_s"], 2))
PY
