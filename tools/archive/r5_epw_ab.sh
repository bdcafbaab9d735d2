set -o pipefail
mkdir -p gpurun_out/r05f
for e in 4 2; do
  BB_EPW=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-per-step > gpurun_out/r05f/flat_epw$e.json 2> gpurun_out/r05f/flat_epw$e.log || exit 1
  BB_EPW=$e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-per-step --steps 20 --warmup 5 > gpurun_out/r05f/drv_epw$e.json 2> gpurun_out/r05f/drv_epw$e.log || exit 1
  python -c "import json;[print('$e',f,round(json.loads(open('gpurun_out/r05f/%s_epw$e.json'%f).read().splitlines()[-1])['value']/1e6,3)) for f in ('flat','drv')]"
done
