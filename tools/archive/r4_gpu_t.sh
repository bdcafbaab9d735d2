set -o pipefail
mkdir -p gpurun_out
for v in "" "BB_PAIR_SOLO=64" "BB_PAIR_ONE=1"; do
  env $v timeout -k 10 200 python -u -m pytest tests/test_gpu_multi_step.py -q --timeout 120 --timeout-method thread -k "hand_overs or headline or adaptive" > gpurun_out/t_$RANDOM.txt 2>&1; echo "[$v] rc=$?"
done
grep -h "passed\|failed" gpurun_out/t_*.txt
