set -o pipefail
for v in base dupfbody dupls duptrsv duphess; do
  timeout -k 10 120 python tools/full_forward_bench.py --lib tools/_build/libbb_$v.so --states toppled >> gpurun_out/ffb.jsonl || exit 1
  timeout -k 10 120 python tools/full_forward_bench.py --lib tools/_build/libbb_$v.so --states mixed >> gpurun_out/ffb.jsonl || exit 1
done
