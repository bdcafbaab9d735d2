set -o pipefail
mkdir -p gpurun_out/exp1
for r in 1 0; do
 for s in "--steps 20 --warmup 5" "--steps 512 --warmup 256"; do
  BB_ROUTE=$r timeout -k 10 200 python -u bench.py $s --no-cpu-baseline > gpurun_out/exp1/r${r}_${s// /_}.json 2>gpurun_out/exp1/err.log || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value'],d['ms_per_step'],d['roofline']['kernel'])" gpurun_out/exp1/r${r}_${s// /_}.json
 done
done
