"""Multi-process (world_size 2, gloo, CPU) tests of the sharded driver: shard ranges, per-shard
input generation, the u0* gather and the histogram all-reduce reproduce the unsharded result.
The solver inside the driver is the CPU oracle here (the HIP solve is covered by -m gpu)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpc_blaster_amd.dist import shard_range


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for B in (0, 1, 7, 4096, 262144, 1048577):
        for G in (1, 2, 3, 4, 8):
            sh = [shard_range(B, r, G) for r in range(G)]
            assert sh[0].start == 0 and sh[-1].stop == B
            assert all(a.stop == b.start for a, b in zip(sh, sh[1:]))
            assert max(s.count for s in sh) - min(s.count for s in sh) <= 1


def _worker(rank, world, port, B, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from mpc_blaster_amd.dist import allreduce_histogram, run_sharded
        from oracle.inputs import make_inputs
        from oracle.ocp import OcpSpec, mpc_solve
        spec = OcpSpec(N=10)

        def mk(start, count):
            inp = make_inputs('c2', ids=np.arange(start, start + count, dtype=np.uint64), N=10)
            return dict(x0=inp['x0'], xref=inp['xref'], uref=inp['uref'])

        def solve(x0, xref, uref):
            return torch.from_numpy(mpc_solve(x0, xref, uref, spec)['u0'])

        sh, u0 = run_sharded(solve, mk, B, rank, world)
        u_local = solve(**mk(sh.start, sh.count))
        counts = torch.zeros((4, 64), dtype=torch.int64)
        v = np.clip(u_local.numpy(), 0.0, 65.0 - 1e-9)
        for m in range(4):
            counts[m] += torch.from_numpy(np.histogram(v[:, m], bins=64, range=(0, 65))[0])
        allreduce_histogram(counts)
        out_q.put((rank, u0.numpy(), counts.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('B', [64, 37])
def test_world2_gather_matches_unsharded(B):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec, mpc_solve
    inp = make_inputs('c2', ids=np.arange(B, dtype=np.uint64), N=10)
    ref = mpc_solve(inp['x0'], inp['xref'], inp['uref'], OcpSpec(N=10))['u0']
    hist = np.stack([np.histogram(np.clip(ref[:, m], 0, 65 - 1e-9), bins=64, range=(0, 65))[0] for m in range(4)])
    for rank, u0, counts in res:
        assert u0.shape == (B, 4)
        assert np.array_equal(u0, ref)          # shard-invariant, bit for bit
        assert np.array_equal(counts, hist)     # all-reduced histogram = global histogram


def _host_hist(u0, counts, lo=0.0, hi=65.0):
    """The device histogram kernel's binning (mpcb_aux.hip histogram_kernel), on the host."""
    nb = counts.shape[1]
    v = u0.double().numpy()
    b = np.clip(np.floor((v - lo) * (nb / (hi - lo))), 0, nb - 1).astype(np.int64)
    for m in range(v.shape[1]):
        counts[m] += torch.from_numpy(np.bincount(b[:, m], minlength=nb))


def _pipeline_worker(rank, world, port, per_rank, mode, steps, out_q):
    """bench.py's timed loop (dist.StepPipeline: double-buffered outputs, async collective of
    step i overlapping step i+1's solve) with the CPU oracle standing in for the HIP solve."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from mpc_blaster_amd.dist import StepPipeline, shard_range
        from oracle.inputs import make_inputs
        from oracle.ocp import OcpSpec, mpc_solve
        cfg = 'c5' if mode == 'histogram' else 'c4'
        N = 30 if cfg == 'c4' else 10     # c4's horizon (at N = 10 its boxes need ~100 iterations)
        sh = shard_range(per_rank * world, rank, world)
        spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0)) if cfg == 'c4' else OcpSpec(N=N)
        inp = make_inputs(cfg, ids=np.arange(sh.start, sh.stop, dtype=np.uint64), N=N)
        calls = []

        def solve(o):
            step = len(calls)
            calls.append(step)
            r = mpc_solve(inp['x0'] + 0.01 * step, inp['xref'], inp['uref'], spec, wind=inp['wind'])
            o[0].copy_(torch.from_numpy(r['u0']))
            o[3].copy_(torch.from_numpy(r['status']))

        def make_outs():
            return (torch.empty((sh.count, 4), dtype=torch.float64), None, None,
                    torch.zeros((sh.count,), dtype=torch.int32))

        pipe = StepPipeline(make_outs, mode, world, histogram=_host_hist)
        results = []
        for i in range(steps):
            pipe.step(solve)
            if i >= 1:   # the previous step's collective may still be in flight: wait on it
                j = (i - 1) % pipe.nbuf
                if pipe.pending[j] is not None:
                    pipe.pending[j].wait()
                    pipe.pending[j] = None
                results.append(pipe.result(j).clone())
        pipe.drain()
        results.append(pipe.result().clone())
        out_q.put((rank, [r.numpy() for r in results], pipe.bad_status(), pipe.nbuf))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('mode', ['gather', 'histogram'])
def test_world2_step_pipeline_matches_unsharded(mode):
    """The c4 u0 all-gather and the c5 histogram all-reduce through the exact code bench.py
    times, over 3 double-buffered steps with step-dependent inputs."""
    world, per_rank, steps = 2, 24, 3
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, per_rank, mode, steps, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec, mpc_solve
    cfg = 'c5' if mode == 'histogram' else 'c4'
    B, N = world * per_rank, (30 if cfg == 'c4' else 10)
    spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0)) if cfg == 'c4' else OcpSpec(N=N)
    inp = make_inputs(cfg, ids=np.arange(B, dtype=np.uint64), N=N)
    for rank, results, bad, nbuf in res:
        assert nbuf == 2 and bad == 0 and len(results) == steps
        for step, got in enumerate(results):
            ref = mpc_solve(inp['x0'] + 0.01 * step, inp['xref'], inp['uref'], spec, wind=inp['wind'])['u0']
            if mode == 'gather':
                assert got.shape == (B, 4) and np.array_equal(got, ref)
            else:
                c = torch.zeros((4, 64), dtype=torch.int64)
                _host_hist(torch.from_numpy(ref), c)
                assert np.array_equal(got, c.numpy())
