#!/bin/bash
# MFMA / LDS counters of the fused PPO kernels (diagnostic, GPU box): the
# available SQ counter names, then one --pmc pass per group over a short
# fused PPO run (proprio policy, 0.5M steps).
set -o pipefail
mkdir -p gpurun_out/mfma
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/mfma/avail.txt 2>&1; cd $GRAFT_REPO_ROOT
grep -o -E "SQ_[A-Z0-9_]*(MFMA|LDS|VALU_MFMA|BUSY)[A-Z0-9_]*" gpurun_out/mfma/avail.txt | sort -u | head -40
i=0
for grp in "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d gpurun_out/mfma/p$i -o run --output-format csv -- \
    python3 tools/bench_ppo.py --timesteps 5e5 > gpurun_out/mfma/p$i.log 2>&1 || { tail -5 gpurun_out/mfma/p$i.log; echo "pass $i failed"; }
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/mfma/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if "mlp_" not in name and "conv2" not in name:
            continue
        acc[name[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(f, k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
