"""Sharding / collectives of the N>1 path on CPU with gloo, world_size 2."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_env_shard_partitions():
    from ballbot_gym.distributed import env_shard

    for total, world in ((32768, 8), (4096, 1), (10, 3), (7, 7)):
        spans = [env_shard(total, r, world) for r in range(world)]
        assert spans[0][0] == 0
        assert sum(c for _, c in spans) == total
        for (s0, c0), (s1, _) in zip(spans, spans[1:]):
            assert s0 + c0 == s1
    with pytest.raises(ValueError):
        env_shard(3, 0, 4)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ballbot_gym.distributed import env_shard, gather_rollouts, max_over_ranks, shard_stream_seeds

    start, count = env_shard(10, rank, world)
    t = max_over_ranks(1.0 + rank)
    # a rollout buffer [T=3, n_local, 4] tagged with global env ids
    buf = torch.arange(start, start + count, dtype=torch.float32).view(1, count, 1).expand(3, count, 4).contiguous()
    out = gather_rollouts(buf)
    if rank == 0:
        q.put((t, out[0, :, 0].tolist(), (shard_stream_seeds(5, start, count, per_env=False), shard_stream_seeds(5, start, count))))
    dist.destroy_process_group()


def test_gloo_world2_gather_and_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    t, ids, seed0 = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0
    assert ids == [float(i) for i in range(10)]
    assert seed0 == (None, [5, 6, 7, 8, 9])  # shared stream on request; per-env generators from the global id


def _ppo_worker(rank, world, port, q, mode="gather"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fake_env import FakeEnv
    from test_ppo import _ppo

    torch.manual_seed(100 + rank)  # different local init: the broadcast must align them
    env = FakeEnv(8, seed=rank, ep_len=4)
    m = _ppo(env, n_steps=4, batch_size=16, n_epochs=1, **({} if mode == "default" else {"update_mode": mode}))
    m.learn(total_timesteps=2 * 8 * 4 * world)
    vec = torch.nn.utils.parameters_to_vector(m.policy.parameters()).detach()
    q.put((rank, m.num_timesteps, m._n_updates, vec.numpy(), len(m.ep_info_buffer), m.update_mode))
    dist.destroy_process_group()


def test_gloo_world2_ppo_update_boundary():
    """Rollouts gathered to rank 0 (64 samples per update), one update there,
    parameters broadcast: both ranks end with identical policies."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ppo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, t0, u0, v0, e0, _), (_, t1, u1, v1, e1, _) = res
    assert t0 == t1 == 2 * 8 * 4 * 2        # timesteps count every rank's envs
    assert u0 == 2 and u1 == 0             # SB3 counts epochs: 1 epoch x 2 iterations, on rank 0 only
    assert (v0 == v1).all()
    assert e0 == e1 > 0                    # episode stats gathered from both ranks


def test_gloo_world2_default_update_is_gather():
    """With more than one rank and no update_mode given, the update is north_star's gather
    (rollouts to rank 0, one update there, parameters broadcast); the data-parallel update is
    opt-in (update_mode="allreduce")."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ppo_worker, args=(r, 2, port, q, "default")) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, t0, u0, v0, e0, m0), (_, t1, u1, v1, e1, m1) = res
    assert m0 == m1 == "gather"
    assert t0 == t1 == 2 * 8 * 4 * 2 and u0 == 2 and u1 == 0
    assert (v0 == v1).all()


def _dp_worker(rank, world, port, q, target_kl):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fake_env import FakeEnv
    from test_ppo import _ppo

    torch.manual_seed(100 + rank)  # different local init: the constructor's broadcast aligns them
    env = FakeEnv(8, seed=5, ep_len=4)  # the same data on both ranks (see the single-process twin)
    m = _ppo(env, n_steps=4, batch_size=16, n_epochs=2, update_mode="allreduce", target_kl=target_kl)
    m.gen.manual_seed(77)
    m.learn(total_timesteps=2 * 8 * 4 * world)
    vec = torch.nn.utils.parameters_to_vector(m.policy.parameters()).detach()
    q.put((rank, m._n_updates, vec.numpy(), m.logger.values.get("train/approx_kl")))
    dist.destroy_process_group()


@pytest.mark.parametrize("target_kl", [None, 1e-4])
def test_gloo_world2_data_parallel_update(target_kl):
    """update_mode="allreduce": every rank updates on its own shard with batch_size/world rows
    per minibatch and the gradients averaged over the ranks.  Both ranks holding the same
    data makes the averaged gradient each rank's own, so the result must equal one process
    updating that data with batch_size/world (KL early stop on the ranks' mean approx_kl)."""
    from fake_env import FakeEnv
    from test_ppo import _ppo

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q, target_kl)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, u0, v0, kl0), (_, u1, v1, kl1) = res
    assert (v0 == v1).all() and u0 == u1  # no parameter broadcast after the update: they stay equal
    torch.manual_seed(100)  # rank 0's initial parameters
    m = _ppo(FakeEnv(8, seed=5, ep_len=4), n_steps=4, batch_size=8, n_epochs=2, target_kl=target_kl)
    m.gen.manual_seed(77)
    m.learn(total_timesteps=2 * 8 * 4)
    ref = torch.nn.utils.parameters_to_vector(m.policy.parameters()).detach().numpy()
    assert m._n_updates == u0
    np.testing.assert_allclose(v0, ref, rtol=1e-6, atol=1e-7)
    if target_kl is not None:
        assert kl0 == pytest.approx(m.logger.values.get("train/approx_kl"), rel=1e-6)


def _dp_norm_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fake_env import FakeEnv
    from test_ppo import _ppo

    env = FakeEnv(8, seed=5 + 11 * rank, ep_len=3 + rank)  # different data on the two ranks
    m = _ppo(env, n_steps=4, batch_size=16, n_epochs=2, update_mode="allreduce", normalize_advantage=True)
    seen = []
    m._dp_adv_hook = lambda raw, out: seen.append((raw.detach().numpy().copy(), out.detach().numpy().copy()))
    m.learn(total_timesteps=2 * 8 * 4 * world)
    q.put((rank, seen))
    dist.destroy_process_group()


def test_gloo_world2_data_parallel_global_advantage_normalisation():
    """update_mode="allreduce" normalises each minibatch's advantages as SB3 does --
    (adv - mean) / (std + 1e-8), unbiased std -- over the GLOBAL minibatch, the union of
    the ranks' local minibatches (one all-reduce of count, sum and sum of squares), not
    per local minibatch.  Ranks hold different data; every minibatch's normalised
    advantages are checked against the statistics of the two ranks' raw slices."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_norm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = res[0], res[1]
    assert len(a) == len(b) > 0  # the same number of minibatches on both ranks
    local_differs = False
    for (ra, na), (rb, nb) in zip(a, b):
        raw = np.concatenate([ra, rb]).astype(np.float64)
        mean, std = raw.mean(), raw.std(ddof=1)
        np.testing.assert_allclose(na, (ra - mean) / (std + 1e-8), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(nb, (rb - mean) / (std + 1e-8), rtol=1e-5, atol=1e-6)
        union = np.concatenate([na, nb]).astype(np.float64)
        assert abs(union.mean()) < 1e-5 and abs(union.std(ddof=1) - 1) < 1e-4
        local = (ra - ra.mean()) / (ra.std(ddof=1) + 1e-8)
        local_differs |= not np.allclose(local, na, atol=1e-3)
    assert local_differs  # the global statistics are not each rank's own


def _uneven_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fake_env import FakeEnv
    from test_ppo import _ppo

    try:
        _ppo(FakeEnv(8 + rank), n_steps=4, batch_size=16, update_mode="allreduce")
        q.put((rank, "built"))
    except ValueError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_gloo_world2_allreduce_rejects_uneven_shards():
    """9 + 8 envs (env_shard of an odd total): the data-parallel update would run a
    different number of minibatch all-reduces per rank and deadlock; both ranks raise."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uneven_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all("same number of envs" in v for v in res.values()), res


def test_data_parallel_needs_divisible_batch():
    from fake_env import FakeEnv
    from test_ppo import _ppo

    with pytest.raises(ValueError):
        _ppo(FakeEnv(8), update_mode="sideways")
