#!/bin/bash
# BASELINE configs[3] ("32768 envs sharded across 8 x MI355X, RCCL gather of rollouts into the PPO
# update") on the one GPU a session has (GPU box, repo root).  Not the 8-GPU measurement: it shows
# what one MI355X does with the whole 32768-env workload, and runs the 8-rank command line itself.
#   envs32k_flat / envs32k_perlin  bench.py --envs 32768 on one GPU (one process, 32768 envs)
#   ranks8_gloo                    torch.distributed.run --nproc-per-node 8 bench.py --gpus 8: eight ranks
#                                  of 4096 envs SHARING the GPU over gloo (the driver's N=8 command
#                                  line; the value is one GPU's, not a scaling point)
#   ppo32k                         tools/bench_ppo.py with 32768 envs x 64 steps (2.1M samples per update)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06c4}
mkdir -p $O
STEPS=${STEPS:-"envs32k_flat envs32k_perlin ranks8_gloo ppo32k"}
for s in $STEPS; do
  case $s in
    envs32k_flat)   timeout -k 10 300 python -u bench.py --envs 32768 --steps 200 --warmup 100 --no-per-step --cpu-seconds 4 > $O/$s.json 2> $O/$s.log || { tail -5 $O/$s.log; exit 1; } ;;
    envs32k_perlin) timeout -k 10 300 python -u bench.py --envs 32768 --terrain perlin --steps 200 --warmup 100 --no-per-step --no-cpu-baseline > $O/$s.json 2> $O/$s.log || { tail -5 $O/$s.log; exit 1; } ;;
    ranks8_gloo)    BB_BENCH_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
                      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline --no-per-step \
                      > $O/$s.json 2> $O/$s.log || { tail -5 $O/$s.log; exit 1; } ;;
    ppo32k)         timeout -k 10 400 python -u tools/bench_ppo.py --envs 32768 --n-steps 64 --batch 16384 --timesteps 21e6 --out $O/ppo32k > $O/$s.json 2> $O/$s.log || { tail -5 $O/$s.log; exit 1; } ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], round(d['value']/1e6,3), 'M', d.get('n_gpus'), d.get('config',{}).get('total_envs', d.get('config',{}).get('envs')))" $O/$s.json $s
done
echo C4_DONE
