"""Multi-GPU instance sharding: one process per GPU, RCCL (torch "nccl") only for the final gather.

The instances are independent (SURVEY §8 e): rank r owns the contiguous global id range
``[r*B/G, (r+1)*B/G)`` and generates its own inputs on device from (seed, global id), so
nothing is scattered.  The only collectives are the final gather of u0* and/or an all-reduce
of the per-motor u0* histogram (c5).  The reference has no distributed path at all.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable


@dataclass
class Shard:
    rank: int
    world: int
    start: int      # first global instance id
    count: int      # instances on this rank

    @property
    def stop(self) -> int:
        return self.start + self.count


def shard_range(global_batch: int, rank: int, world: int) -> Shard:
    """Contiguous, balanced split (the first ``global_batch % world`` ranks get one extra)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f'rank {rank} of world {world}')
    base, extra = divmod(int(global_batch), world)
    start = rank * base + min(rank, extra)
    return Shard(rank, world, start, base + (1 if rank < extra else 0))


def env_rank_world():
    return int(os.environ.get('RANK', '0')), int(os.environ.get('WORLD_SIZE', '1'))


def gather_u0(u0, shard: Shard, global_batch: int, group=None):
    """All-gather every rank's u0* [count, nu] into [global_batch, nu] (global id order).

    Equal shards use one ``all_gather_into_tensor``; ragged shards pad to the largest shard.
    """
    import torch
    import torch.distributed as dist
    world = shard.world
    if world == 1:
        return u0
    base, extra = divmod(global_batch, world)
    mx = base + (1 if extra else 0)
    if u0.shape[0] != mx:
        pad = torch.zeros((mx - u0.shape[0],) + tuple(u0.shape[1:]), dtype=u0.dtype, device=u0.device)
        u0 = torch.cat([u0, pad], dim=0)
    out = torch.empty((world * mx,) + tuple(u0.shape[1:]), dtype=u0.dtype, device=u0.device)
    dist.all_gather_into_tensor(out, u0.contiguous(), group=group)
    if extra == 0:
        return out
    parts = [out[r * mx: r * mx + shard_range(global_batch, r, world).count] for r in range(world)]
    return torch.cat(parts, dim=0)


def allreduce_histogram(counts, group=None, async_op: bool = False):
    """Sum the per-rank int64 [nu, nbins] histograms (c5: 64 bins per motor over [0, 65]).
    ``async_op``: return the collective's work handle (None on one rank) instead of the counts."""
    import torch.distributed as dist
    work = None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        work = dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
    return work if async_op else counts


def run_sharded(solve_fn: Callable, make_inputs_fn: Callable, global_batch: int, rank: int,
                world: int, gather: bool = True):
    """Driver shared by bench.py and the tests: inputs for this rank's ids -> solve -> gather.

    ``make_inputs_fn(start, count)`` returns the solver's keyword inputs for those global ids;
    ``solve_fn(**inputs)`` returns u0 [count, nu] (a torch tensor on the rank's device).
    """
    sh = shard_range(global_batch, rank, world)
    inputs = make_inputs_fn(sh.start, sh.count)
    u0 = solve_fn(**inputs)
    if gather:
        return sh, gather_u0(u0, sh, global_batch)
    return sh, u0
