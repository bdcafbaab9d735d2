"""RCCL executed on the hardware at hand.

The driver's 8-GPU runs use a "nccl" (RCCL) process group, one GPU per rank.
A one-GPU box can still run that code: an RCCL group of ONE rank executes every
collective (all-reduce, barrier) through RCCL, and BatchedPPO runs its
collectives whenever the group is RCCL, whatever its size.  So the captured
data-parallel update graphs -- RCCL all-reduce nodes between the fused
minibatch's backward and its clip + AdamW step -- replay here, and must equal
the eager data-parallel loop and the collective-free update.  bench.py's
multi-rank path (barriers, max-over-ranks all-reduce) runs under
torch.distributed.run with the RCCL group forced at world size 1.
Reference: /root/reference/ballbot_rl/training/train.py:126-141 (the VecEnv
sharding the ranks restate).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_update_worker(port, fused, q):
    """One rank, RCCL group on cuda:0: three models on the same rollout -- data-parallel with the
    captured graphs (RCCL nodes inside), data-parallel eager (RCCL between backward and step),
    and the collective-free update -- then a short learn() on the GPU env in allreduce mode."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      BB_PPO_FUSED=fused)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        from test_gpu_ppo import _gpu_fake

        from ballbot_rl.training.logger import CSVLogger
        from ballbot_rl.training.ppo import BatchedPPO

        out = {"backend": dist.get_backend()}
        models = []
        for mode, graphs in (("allreduce", True), ("allreduce", False), ("gather", True)):
            m = BatchedPPO(_gpu_fake(), n_steps=16, batch_size=512, n_epochs=3, learning_rate=3e-4,
                           target_kl=None, normalize_advantage=True, seed=4, use_graphs=graphs, update_mode=mode,
                           logger=CSVLogger(None, stdout=False))
            m.collect_rollouts()
            models.append(m)
        out["rccl"] = [m._rccl for m in models]
        out["dp"] = [m._dp for m in models]
        d0 = models[0].buf.flat()
        # count the collectives the dp graph replays: wrap dist.all_reduce while it is captured
        calls = {"n": 0}
        real = dist.all_reduce

        def counting(t, *a, **k):
            calls["n"] += 1
            return real(t, *a, **k)

        dist.all_reduce = counting
        try:
            for m in models:
                m.shuffle_gen.manual_seed(99)
                m._update({k: v.clone() for k, v in d0.items()}, dp=m._dp)
        finally:
            dist.all_reduce = real
        g = models[0]._graphs
        out["graph"] = {"dp": bool(g.dp), "fused": bool(g.fused), "epoch_graph": g.graph_epoch is not None}
        out["allreduce_calls"] = calls["n"]
        out["n_updates"] = [m._n_updates for m in models]
        keys = ("train/policy_gradient_loss", "train/value_loss", "train/approx_kl", "train/clip_fraction")
        out["logs"] = [[float(m.logger.values[k]) for k in keys] for m in models]
        out["params"] = [torch.nn.utils.parameters_to_vector(m.policy.parameters()).detach().cpu().numpy()
                         for m in models]
        # the GPU env end to end in allreduce mode (rollout kernel, GAE, captured dp update)
        from ballbot_gym.envs import BallbotVecEnv

        env = BallbotVecEnv(256, device="cuda:0", seed=3, max_ep_steps=40)
        m = BatchedPPO(env, n_steps=16, batch_size=1024, n_epochs=2, seed=5, update_mode="allreduce",
                       logger=CSVLogger(None, stdout=False))
        m.learn(total_timesteps=256 * 16 * 2)
        out["learn"] = {"n_updates": m._n_updates, "value_loss": float(m.logger.values["train/value_loss"]),
                        "graphs_dp": bool(m._graphs is not None and m._graphs.dp)}
        env.close()
        torch.cuda.synchronize()
        dist.destroy_process_group()
        q.put(("ok", out))
    except Exception as e:  # the parent reports it
        import traceback

        q.put(("error", traceback.format_exc()[-4000:] + repr(e)))


@pytest.mark.parametrize("rep", [0, 1])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_rccl_captured_data_parallel_update_one_rank(fused, rep):
    """The data-parallel update graphs with RCCL all-reduce nodes captured, replayed on one rank:
    equal to the eager data-parallel loop (RCCL calls between backward and step) and to the
    collective-free update, to the fp32 reduction-order tolerance of the one-rank graph test.
    Twice per form (fresh processes): round 6 found a timing-dependent capture invalidation here
    (the process group's watchdog polling the warm-up collectives' events during a global-mode
    capture), fixed by capturing the update graphs in thread-local mode."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_update_worker, args=(_port(), fused, q))
    p.start()
    status, out = q.get(timeout=200)
    p.join(timeout=60)
    assert status == "ok", out
    assert p.exitcode == 0
    assert out["backend"] == "nccl" and out["rccl"] == [True, True, True]
    assert out["dp"] == [True, True, False]
    assert out["graph"]["dp"] and out["graph"]["fused"] == (fused == "1")
    # the eager dp loop calls RCCL per minibatch; the graph build captures its nodes once
    assert out["allreduce_calls"] > 0
    assert out["n_updates"] == [3, 3, 3]
    la = out["logs"][0]
    for lb in out["logs"][1:]:
        for a, b in zip(la, lb):
            assert a == pytest.approx(b, rel=5e-3, abs=1e-6)
    for ref in out["params"][1:]:
        diff = np.abs(out["params"][0] - ref)
        assert float((diff > 1e-5).mean()) < 1e-2, float(diff.max())
    lr = out["learn"]
    assert lr["graphs_dp"] and lr["n_updates"] == 4 and np.isfinite(lr["value_loss"])


def test_bench_under_torchrun_with_rccl_group():
    """bench.py as the driver launches it (torch.distributed.run), one rank, with the RCCL group
    forced (BB_BENCH_FORCE_PG=1): RCCL barriers around the timed window and the max-over-ranks
    all-reduce execute, and the line is the same contract."""
    env = dict(os.environ, BB_BENCH_FORCE_PG="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("BB_BENCH_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"), "--gpus", "1",
           "--steps", "20", "--warmup", "5", "--burn-in", "20", "--envs", "1024", "--no-cpu-baseline",
           "--no-per-step"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["config"]["process_group"] == "nccl"
    assert line["n_gpus"] == 1 and line["status"] == "ok" and line["value"] > 0
    assert line["value"] == pytest.approx(1024 * 20 / (line["ms_per_step"] * 20 / 1e3), rel=1e-6)


def test_dp_local_minibatch_below_256_takes_the_autograd_graph(monkeypatch):
    """the data-parallel update's LOCAL minibatch (batch_size / world) decides the
    fused path.  A 128-row local minibatch (the reference's batch_sz 256 on two ranks) builds
    the autograd update graph instead of failing in bb_ppo_mlp_step."""
    from test_gpu_ppo import _gpu_fake

    from ballbot_rl.training.logger import CSVLogger
    from ballbot_rl.training.ppo import BatchedPPO, fused_mlp_slots

    m = BatchedPPO(_gpu_fake(), n_steps=16, batch_size=256, n_epochs=2, seed=4, update_mode="allreduce",
                   logger=CSVLogger(None, stdout=False))
    m._force_dp = True
    assert fused_mlp_slots(m) is not None and fused_mlp_slots(m, B=128) is None
    m.collect_rollouts()
    d = m.buf.flat()
    n = d["obs"].shape[0]
    g = m._graphs_for(n, 128)
    assert g is not None and g.dp and not g.fused and g.B == 128
    log = g.run(m, {k: v.clone() for k, v in d.items()}, 0.2)
    assert log.shape == (2 * n // 128, 6) and np.isfinite(log).all()
