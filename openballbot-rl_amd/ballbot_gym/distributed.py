"""Multi-GPU layout of the batched env.

Envs are independent: N_total envs are split into contiguous blocks, one per
rank (one process per GPU), with no collective on the step path.  The global
env id fixes the seed stream, so a rollout is the same whatever the world
size.  Collectives exist only at boundaries: the max-over-ranks timing of the
benchmark and the gather of rollout buffers at a PPO update.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def env_shard(num_envs_total: int, rank: int, world: int) -> Tuple[int, int]:
    """(first global env id, count) of `rank`'s block; blocks differ by at most 1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    if num_envs_total < world:
        raise ValueError(f"{num_envs_total} envs cannot be split over {world} ranks")
    base, extra = divmod(num_envs_total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def shard_stream_seeds(seed: int, first_env: int, count: int, per_env: bool = True) -> Optional[List[int]]:
    """Terrain generator seeds of a rank's env block (BallbotVecEnv stream_seeds).

    per_env (default): global env g draws from np_random(seed + g) -- SB3 seeds
    training env g with reset(seed=seed+g) (VecEnv.seed, train.py:126-141;
    ballbot_env.py:596), and the eval VecEnv gives env i seed + N_ENVS + i
    (train.py:90-97, with seed the eval base).  per_env=False: None, every
    local env on the one generator np_random(seed) (BallbotVecEnv(...,
    shared_stream=True); the convention an unseeded PPO would leave)."""
    if not per_env:
        return None
    from .envs.config import sb3_stream_seeds

    return sb3_stream_seeds(seed, count, first_env)


def max_over_ranks(value: float, device=None) -> float:
    """All-reduce MAX of a scalar (elapsed time); identity without a process group (an RCCL
    group of one rank still runs the all-reduce: the driver's multi-GPU path, rehearsed)."""
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    if dist.get_world_size() == 1 and dist.get_backend() != "nccl":
        return float(value)
    if dist.get_backend() == "gloo":  # host tensors on gloo (rehearsals sharing one GPU)
        device = None
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rollouts(buf: torch.Tensor, dst: int = 0):
    """Gather equally-shaped per-rank rollout buffers [T, n_local, ...] onto `dst`
    (concatenated along the env axis); other ranks get None."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return buf
    world = dist.get_world_size()
    # gloo gathers host tensors only: device buffers (ranks sharing a GPU over gloo, the one-GPU
    # rehearsal of the RCCL path) go through host memory; RCCL gathers them in place
    host = dist.get_backend() == "gloo" and buf.device.type != "cpu"
    src = buf.detach().cpu() if host else buf.contiguous()
    parts = [torch.empty_like(src) for _ in range(world)] if dist.get_rank() == dst else None
    dist.gather(src.contiguous(), parts, dst=dst)
    if parts is None:
        return None
    out = torch.cat(parts, dim=1)
    return out.to(buf.device) if host else out
