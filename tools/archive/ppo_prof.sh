#!/bin/bash
# rocprofv3 kernel statistics of a short PPO run (diagnostic, GPU box); the
# per-dispatch trace is summarised on the box and dropped (too big to copy back).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ppo -o run -- \
  python3 tools/bench_ppo.py --timesteps 2e6 --out /tmp/ppo_prof > gpurun_out/ppo_prof.json 2> gpurun_out/ppo_prof.err || exit 1
f=$(find /tmp/prof_ppo -name "run_kernel_stats.csv" | head -1)
cp "$f" gpurun_out/ppo_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/ppo_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", round(tot / 1e6, 1))
for r in rows[:25]:
    print("%8.1f ms %5.1f%% n=%6s avg=%7.1f us  %s" % (float(r["TotalDurationNs"]) / 1e6, 100 * float(r["TotalDurationNs"]) / tot,
                                                   r["Calls"], float(r["AverageNs"]) / 1e3, r["Name"][:100]))
PY
