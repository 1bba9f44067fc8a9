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


class StepPipeline:
    """The timed step of ``bench.py``: solve this rank's batch, then the one collective.

    ``solve(out)`` writes the rank's outputs into ``out`` = (u0 [B, nu], X|None, U|None, status)
    on the current stream.  Per step the rank then either all-gathers u0 into [world*B, nu]
    (c2-c4, ``mode='gather'``) or reduces u0 to a per-motor int64 histogram with
    ``histogram(u0, counts)`` and all-reduces it (c5, ``mode='histogram'``).  With several ranks
    the collective is issued asynchronously (RCCL runs it on the process group's own stream) and
    the outputs are double-buffered: step i's collective overlaps step i+1's solve, and an output
    set is written again only after its collective has been waited on.  The gloo test
    (tests/test_dist_gloo.py) drives this same class with a CPU solve.
    """

    def __init__(self, make_outputs: Callable, mode: str, world: int, histogram: Callable | None = None,
                 nbins: int = 64, group=None):
        import torch
        if mode not in ('gather', 'histogram'):
            raise ValueError(f'mode {mode!r}')
        if mode == 'histogram' and histogram is None:
            raise ValueError('histogram mode needs the histogram function')
        self.mode, self.world, self.group = mode, int(world), group
        self.histogram = histogram
        self.nbuf = 2 if self.world > 1 else 1
        self.outs = [make_outputs() for _ in range(self.nbuf)]
        u0 = self.outs[0][0]
        self.gathered = ([torch.empty((self.world * u0.shape[0],) + tuple(u0.shape[1:]), dtype=u0.dtype,
                                      device=u0.device) for _ in range(self.nbuf)]
                         if (mode == 'gather' and self.world > 1) else None)
        self.counts = [torch.zeros((u0.shape[1], nbins), dtype=torch.int64, device=u0.device)
                       for _ in range(self.nbuf)] if mode == 'histogram' else None
        self.pending = [None] * self.nbuf
        self.it = 0
        self.last = 0

    def step(self, solve: Callable, before: Callable | None = None, after: Callable | None = None):
        """One step; ``before`` / ``after`` run around the solve (e.g. HIP event records)."""
        import torch.distributed as dist
        i = self.it % self.nbuf
        self.it += 1
        self.last = i
        if self.pending[i] is not None:
            self.pending[i].wait()
            self.pending[i] = None
        o = self.outs[i]
        if before is not None:
            before()
        solve(o)
        if after is not None:
            after()
        if self.mode == 'histogram':
            self.counts[i].zero_()
            self.histogram(o[0], self.counts[i])
            if self.world > 1:
                self.pending[i] = dist.all_reduce(self.counts[i], op=dist.ReduceOp.SUM,
                                                  group=self.group, async_op=True)
        elif self.world > 1:
            self.pending[i] = dist.all_gather_into_tensor(self.gathered[i], o[0], group=self.group,
                                                          async_op=True)

    def drain(self):
        for i in range(self.nbuf):
            if self.pending[i] is not None:
                self.pending[i].wait()
                self.pending[i] = None

    def result(self, i: int | None = None):
        """After ``drain()``: the gathered u0 [world*B, nu] (gather; this rank's u0 on one rank)
        or the all-reduced histogram [nu, nbins] of the output set ``i`` (default: the last)."""
        i = self.last if i is None else i
        if self.mode == 'histogram':
            return self.counts[i]
        return self.gathered[i] if self.gathered is not None else self.outs[i][0]

    def bad_status(self) -> int:
        return int(sum(int((o[3] != 0).sum()) for o in self.outs))
