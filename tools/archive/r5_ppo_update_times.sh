set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
for i in 1 2; do timeout -k 10 300 python -u tools/bench_ppo.py --timesteps 3e6 > $O/ppo3m_$i.json 2> $O/ppo3m_$i.log || exit 1; done
timeout -k 10 300 python -u tools/bench_ppo.py --timesteps 10e6 > $O/ppo10m.json 2> $O/ppo10m.log || exit 1
echo PPO_DONE
