set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_ksweep; mkdir -p $O
for K in 1 2 5 10 20 40 80 160; do
  timeout -k 10 200 python -u bench.py --steps $K --warmup 5 --no-cpu-baseline --no-per-step > $O/k$K.json 2> $O/k$K.log || exit 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], round(d['value']/1e6,3), 'M kernel_ms', round(r['kernel_ms'],4), 'per step', round(r['kernel_ms']/int(sys.argv[2]),4))" $O/k$K.json $K
done
