#!/bin/bash
# rocprofv3 kernel summary of a short fused-update PPO run (1M steps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run --output-format csv -- \
  python -u tools/bench_ppo.py --timesteps 1e6 > gpurun_out/prof_fused.log 2>&1 || { tail gpurun_out/prof_fused.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_fused/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.1f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:100]}")
print("total ms", tot / 1e6)
PY
