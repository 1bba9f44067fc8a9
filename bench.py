#!/usr/bin/env python3
"""Batched BLASTER MPC benchmark (BASELINE.json metric: MPC solves/sec, N=20, nx=12, nu=4).

A "step" = one fused SQP_RTI solve (RK4 rollout + sensitivities + Riccati QP + forward pass)
over this rank's batch of synthetic instances already resident in HBM, producing u0* [B,4],
X [B,N+1,12] and U [B,N,4]; for N>1 ranks the step also all-gathers u0* over RCCL (the
north_star's only collective).  Weak scaling: every rank owns its own slice of global
instance ids (inputs generated on device from (seed, global id)).

Default workload = BASELINE configs[1] (c2): B=4096 per GPU, N=20, fp64, random x0 + hover ref.
``--workload c3`` = configs[2]: B=65536, N=20, fp32, sinusoidal references.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FLOP_PER_INTERVAL = 34785          # dense algorithmic flops per shooting interval
PEAK_TFLOPS = {'f64': 78.6, 'f32': 157.3}   # MI355X dense vector/matrix peaks (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0

WORKLOADS = {
    'c2': dict(batch=4096, N=20, dtype='f64', ref='hover', box=False, wind=False, seed=1002),
    'c3': dict(batch=65536, N=20, dtype='f32', ref='sine', box=False, wind=False, seed=1003),
    'c4': dict(batch=65536, N=30, dtype='f32', ref='hover', box=True, wind=False, seed=1004),
    'c5': dict(batch=131072, N=40, dtype='f32', ref='hover', box=False, wind=True, seed=1005),
}


def compulsory_bytes(w) -> int:
    """Compulsory HBM bytes per solve: inputs x0 (+ per-instance refs / wind), outputs u0, X, U."""
    s = 8 if w['dtype'] == 'f64' else 4
    N = w['N']
    b = 12 * s + 4 * s + (N + 1) * 12 * s + N * 4 * s + 4   # x0, u0, X, U, status
    if w['ref'] == 'sine':
        b += (N + 1) * 12 * s
    if w['wind']:
        b += 3 * s
    return b


def cpu_baseline(w, budget_s=15.0):
    """Oracle (NumPy fp64, batch-vectorised) on this host, bounded sample of the same workload."""
    os.environ.setdefault('OMP_NUM_THREADS', '1')
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec, mpc_solve
    cfg = {'c2': 'c2', 'c3': 'c3', 'c4': 'c4', 'c5': 'c5'}[w['name']]
    spec = OcpSpec(N=w['N'], lbu=np.zeros(4) if w['box'] else None,
                   ubu=np.full(4, 65.0) if w['box'] else None)
    chunk = 512
    done, t_used, start_id = 0, 0.0, 0
    while t_used < budget_s:
        inp = make_inputs(cfg, ids=np.arange(start_id, start_id + chunk, dtype=np.uint64), N=w['N'])
        t0 = time.perf_counter()
        mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, wind=inp['wind'])
        t_used += time.perf_counter() - t0
        done += chunk
        start_id += chunk
    return dict(value=done / t_used, unit='solves/s', cores=1, kind='port',
                sample=f'{done} instances of {w["name"]} (N={w["N"]}, fp64 NumPy oracle, '
                       f'batch-vectorised, 1 thread) in {t_used:.1f} s')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--workload', default='c2', choices=sorted(WORKLOADS))
    ap.add_argument('--batch', type=int, default=None, help='override per-GPU batch')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-budget', type=float, default=15.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    w = dict(WORKLOADS[args.workload])
    w['name'] = args.workload
    if args.batch:
        w['batch'] = args.batch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device(f'cuda:{local}'))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    from mpc_blaster_amd import BatchedMPC, MPCConfig
    B, N = w['batch'], w['N']
    cfg = MPCConfig(N=N, dtype=w['dtype'], lbu=np.zeros(4) if w['box'] else None,
                    ubu=np.full(4, 65.0) if w['box'] else None)
    mpc = BatchedMPC(cfg, max_batch=B, device=dev)
    inp = mpc.gen_inputs(B, seed=w['seed'], id_offset=rank * B, ref=w['ref'], wind=w['wind'])
    torch.cuda.synchronize()
    tdt = cfg.torch_dtype
    outs = (torch.empty((B, 4), dtype=tdt, device=dev), torch.empty((B, N + 1, 12), dtype=tdt, device=dev),
            torch.empty((B, N, 4), dtype=tdt, device=dev), torch.empty((B,), dtype=torch.int32, device=dev))
    gathered = torch.empty((world * B, 4), dtype=tdt, device=dev) if world > 1 else None
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        mpc.solve(inp['x0'], inp['xref'], inp['uref'], wind=inp['wind'], out=outs)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            dist.all_gather_into_tensor(gathered, outs[0])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    st = outs[3]
    bad = int((st != 0).sum().item())
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        b = torch.tensor([bad], dtype=torch.int64, device=dev)
        dist.all_reduce(b)
        bad = int(b.item())

    if rank == 0:
        total = B * world * args.steps
        value = total / elapsed
        flops_launch = FLOP_PER_INTERVAL * N * B
        achieved_tf = flops_launch / (kern_ms * 1e-3) / 1e12
        peak = PEAK_TFLOPS[w['dtype']]
        hbm_gbs = compulsory_bytes(w) * B / (kern_ms * 1e-3) / 1e9
        line = {
            'metric': 'MPC solves/sec (N=%d, nx=12, nu=4)' % N,
            'value': value,
            'unit': 'solves/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': w['dtype'],
            'data': 'synthetic (Philox4x32-10 inputs generated on device, SURVEY §8d)',
            'config': {'workload': f'{w["name"]}: batch {B}/GPU, N={N}, nx=12, nu=4, {w["dtype"]}, '
                                   f'ref={w["ref"]}' + (', input box [0,65]' if w['box'] else '')
                                   + (', wind' if w['wind'] else ''),
                       'global_batch': B * world, 'horizon': N,
                       'parallelism': f'instance-sharded x{world}' + (' + RCCL all_gather(u0)' if world > 1 else '')},
            'roofline': {'bound': 'mfma', 'achieved': achieved_tf, 'peak': peak, 'unit': 'TFLOP/s',
                         'frac': achieved_tf / peak, 'traffic': None,
                         'note': ('compute-bound path (SURVEY §8d, ~300-700 flop/B); algorithmic flops = '
                                  f'{FLOP_PER_INTERVAL} x N x B per launch over the solve kernel time; '
                                  'peak = dense fp64/fp32 rate (VALU and MFMA peaks are equal on gfx950)'),
                         'hbm_compulsory_GBs': hbm_gbs, 'hbm_frac': hbm_gbs / HBM_PEAK_GBS,
                         'kernel_ms': kern_ms},
            'bad_status': bad,
        }
        if not args.no_cpu_baseline and world == 1:
            line['cpu_baseline'] = cpu_baseline(w, args.cpu_budget)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
