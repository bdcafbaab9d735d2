"""Sharding / collectives of the N>1 path on CPU with gloo, world_size 2."""
import os
import socket

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
    from ballbot_gym.distributed import env_shard, gather_rollouts, max_over_ranks, rank_seed

    start, count = env_shard(10, rank, world)
    t = max_over_ranks(1.0 + rank)
    # a rollout buffer [T=3, n_local, 4] tagged with global env ids
    buf = torch.arange(start, start + count, dtype=torch.float32).view(1, count, 1).expand(3, count, 4).contiguous()
    out = gather_rollouts(buf)
    if rank == 0:
        q.put((t, out[0, :, 0].tolist(), rank_seed(5, start)))
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
    assert seed0 == 5
