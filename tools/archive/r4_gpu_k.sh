#!/bin/bash
# Round-4 GPU pass K: capsule_prism_apart by value (no stack frame) -- GPU suite, flat/perlin
# throughput (two-launch and one-launch pair, LICM-off variant), full-kernel solve phase clocks.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/suite_r4l.txt 2>&1
rc=$?; tail -2 gpurun_out/suite_r4l.txt; grep FAILED gpurun_out/suite_r4l.txt | head
[ $rc = 0 ] || exit $rc
show() { python -c "
import json;d=json.loads(open('$1').read().splitlines()[-1]);p=d.get('pair',{})
print('$2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],1), d['stats'].get('pair_budget'), 'env_mcyc', {k: round(v) for k, v in p.get('env_mcycles', {}).items()})"; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/pk_flat.json 2> gpurun_out/pk_flat.err || exit $?
show gpurun_out/pk_flat.json flat
for v in base one nolicm_one; do
  case $v in base) E=""; C=bench.py;; one) E="BB_PAIR_ONE=1"; C=bench.py;;
    nolicm_one) E="BB_PAIR_ONE=1"; C="tools/bench_with_lib.py tools/_build/libbb_nolicm.so";; esac
  env $E timeout -k 10 200 python -u $C --terrain perlin --no-cpu-baseline > gpurun_out/pk_$v.json 2> gpurun_out/pk_$v.err || exit $?
  show gpurun_out/pk_$v.json $v
done
timeout -k 10 300 python -u tools/phase_clocks.py --terrain perlin --steps 100 --warmup 300 > gpurun_out/phase_perlin2.json 2> gpurun_out/phase_perlin2.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/phase_perlin2.json'));f=d['full_kernel'];print({k: round(v) for k,v in f['solve_phase_cycles_per_newton_iter'].items()}); print({k: round(v) for k,v in f['solve_phase_cycles_per_forward'].items()}); print(round(f['solve_cycles_per_forward']), round(f['body_collide_cycles_per_forward']), f['newton_iters_per_forward'])"
