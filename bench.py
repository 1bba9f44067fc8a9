#!/usr/bin/env python3
"""Batched BLASTER MPC benchmark (BASELINE.json metric: MPC solves/sec, N=20, nx=12, nu=4).

A "step" = one SQP_RTI solve (RK4 rollout + sensitivities + Gauss-Newton QP by Riccati +
forward pass) over this rank's batch of synthetic instances already resident in HBM, producing
u0* [B,4], X [B,N+1,12] and U [B,N,4]; with N>1 ranks the step also all-gathers u0* over
RCCL (the north_star's only collective).  c5 instead reduces u0* to a 64-bin per-motor
histogram and all-reduces it.  Weak scaling: each rank owns its own slice of global instance
ids; inputs are generated on device from (seed, global id) before the timed region.

Default workload = BASELINE configs[1] (c2): B=4096 per GPU, N=20, fp64, random x0 + hover
reference.  The line also carries a ``secondary`` measurement of configs[2] (c3: B=65536,
N=20, fp32, sinusoidal references) at N=1.

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

# dense algorithmic flops per shooting interval: per phase kernel in kernel_flops
PEAK_TFLOPS = {'f64': 78.6, 'f32': 157.3}   # MI355X dense vector (= matrix) peaks, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0

WORKLOADS = {
    'c2': dict(batch=4096, N=20, dtype='f64', ref='hover', box=False, wind=False, seed=1002, hist=False),
    'c3': dict(batch=65536, N=20, dtype='f32', ref='sine', box=False, wind=False, seed=1003, hist=False),
    'c4': dict(batch=65536, N=30, dtype='f32', ref='hover', box=True, wind=False, seed=1004, hist=False),
    'c5': dict(batch=131072, N=40, dtype='f32', ref='hover', box=False, wind=True, seed=1005, hist=True),
}


def compulsory_bytes(w) -> int:
    """Compulsory HBM bytes per solve: x0 (+ per-instance refs / wind) in; u0 (+ X, U) out."""
    s = 8 if w['dtype'] == 'f64' else 4
    N = w['N']
    b = 12 * s + 4 * s + 4                                 # x0, u0, status
    if not w['hist']:
        b += (N + 1) * 12 * s + N * 4 * s                  # X, U
    if w['ref'] == 'sine':
        b += (N + 1) * 12 * s
    if w['wind']:
        b += 3 * s
    return b


def cpu_baseline(w, budget_s=12.0):
    """The oracle timed on this host's cores on a bounded sample of the same workload: the plain-C
    restatement (oracle/c, OpenMP over instances, all cores this process may use) -- the
    unconstrained path, the input box by its primal-dual active set (c4), the wind force (c5) --
    and, on a quarter of the budget, the same port on one thread (SURVEY §8 d: both figures)."""
    from oracle import c_oracle
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec
    spec = OcpSpec(N=w['N'], lbu=np.zeros(4) if w['box'] else None,
                   ubu=np.full(4, 65.0) if w['box'] else None, max_as_iter=w.get('max_as_iter', 200))
    # the GPU box exposes the whole machine's CPUs but grants this job a share; OMP_NUM_THREADS
    # carries that share there (16), so it wins over the affinity mask
    cores = int(os.environ.get('OMP_NUM_THREADS') or 0) or (
        len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else os.cpu_count())
    c_oracle.load()
    def timed(nthreads, chunk, budget):
        done, t_used, start = 0, 0.0, 0
        while t_used < budget:
            inp = make_inputs(w['name'], ids=np.arange(start, start + chunk, dtype=np.uint64), N=w['N'])
            t0 = time.perf_counter()
            c_oracle.solve(inp['x0'], inp['xref'], inp['uref'][:1], spec, nthreads=nthreads,
                           want_traj=not w['hist'], wind=inp['wind'])
            t_used += time.perf_counter() - t0
            done += chunk
            start += chunk
        return done, t_used
    done, t_used = timed(cores, 4096 if not w['box'] else 2048, 0.75 * budget_s)
    done1, t1 = timed(1, 256, 0.25 * budget_s)
    what = 'input-box active set' if w['box'] else ('wind' if w['wind'] else 'unconstrained')
    out = dict(value=done / t_used, unit='solves/s', cores=cores, kind='port',
               value_1thread=done1 / t1,
               sample=f'{done} instances of {w["name"]} (N={w["N"]}, fp64, plain-C oracle oracle/c, '
                      f'{what}, OpenMP) in {t_used:.1f} s; 1 thread: {done1} in {t1:.1f} s')
    if w['name'] == 'c2':
        out['c1_latency_ms'] = c1_latency()
    return out


def c1_latency(reps=2000):
    """SURVEY §8d's CPU figure at the c1 shape (BASELINE configs[0]: 1 instance, N=10, fp64,
    hover reference): per-instance latency of the plain-C port on ONE thread, each solve timed
    inside C (oracle/c mpc_oracle_latency_b1), over 256 seeded x0 draws cycled ``reps`` times --
    the per-control-step cost the reference's loop (simulation_blaster.py:56-107) pays, next to
    the GPU's ``latency_b1``."""
    from oracle import c_oracle
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec
    inp = make_inputs('c1', ids=np.arange(256, dtype=np.uint64), N=10)
    ms = c_oracle.latency_b1(inp['x0'], inp['xref'], inp['uref'], OcpSpec(N=10), reps=reps)
    return dict(median=float(np.median(ms)), p99=float(np.percentile(ms, 99)), mean=float(ms.mean()),
                threads=1, reps=int(reps), N=10,
                sample='c1 shape: 1 instance per solve, N=10, fp64, hover ref, 256 seeded x0 (seed 1001)')


class _DeviceClock:
    """Device time of the timed region: HIP events on the launch stream (GPU ranks) or the host
    clock (the CPU solver stub of the launcher test, tests/bench_stub.py)."""

    def __init__(self, cuda: bool):
        import torch
        self.cuda = cuda
        self.t = [0.0, 0.0]
        if cuda:
            self.stream = torch.cuda.current_stream()
            self.ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]

    def sync(self):
        if self.cuda:
            import torch
            torch.cuda.synchronize()

    def mark(self, i):
        if self.cuda:
            self.ev[i].record(self.stream)
        else:
            self.t[i] = time.perf_counter()

    def elapsed_ms(self):
        return self.ev[0].elapsed_time(self.ev[1]) if self.cuda else (self.t[1] - self.t[0]) * 1e3


def make_solver(w, B, dev, stub=None):
    """The batched solver of one rank: the HIP library (BatchedMPC) or, for the launcher test
    only, a CPU stand-in module with the same methods (``--solver-stub``)."""
    box = w['box']
    if stub:
        import importlib
        return importlib.import_module(stub).make_solver(w, B)
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    cfg = MPCConfig(N=w['N'], dtype=w['dtype'], lbu=np.zeros(4) if box else None,
                    ubu=np.full(4, 65.0) if box else None, max_as_iter=w.get('max_as_iter', 200))
    return BatchedMPC(cfg, max_batch=B, device=dev)


def run(w, world, rank, dev, steps, warmup, stub=None, dump_gather=None):
    import torch
    import torch.distributed as dist

    from mpc_blaster_amd.dist import StepPipeline
    B, N = w['batch'], w['N']
    cuda = stub is None
    mpc = make_solver(w, B, dev, stub)
    clock = _DeviceClock(cuda)
    inp = mpc.gen_inputs(B, seed=w['seed'], id_offset=rank * B, ref=w['ref'], wind=w['wind'])
    clock.sync()
    tdt = mpc.dtype
    odev = dev if cuda else 'cpu'
    traj = not w['hist']

    def make_outs():
        return (torch.empty((B, 4), dtype=tdt, device=odev),
                torch.empty((B, N + 1, 12), dtype=tdt, device=odev) if traj else None,
                torch.empty((B, N, 4), dtype=tdt, device=odev) if traj else None,
                torch.zeros((B,), dtype=torch.int32, device=odev))
    pipe = StepPipeline(make_outs, 'histogram' if w['hist'] else 'gather', world,
                        histogram=lambda u0, counts: mpc.histogram(u0, 0.0, 65.0, 64, counts=counts))

    def solve(o):
        mpc.solve(inp['x0'], inp['xref'], inp['uref'], wind=inp['wind'], want_traj=traj, out=o)

    def step():
        pipe.step(solve)

    drain = pipe.drain

    for _ in range(warmup):
        step()
    drain()
    clock.sync()
    # one event pair around the K solves on the launch stream (an event record between the
    # steps costs ~18 us of device time per step at c2: tools/host_overhead.py)
    if world > 1:
        dist.barrier()
    clock.sync()
    t0 = time.perf_counter()
    clock.mark(0)
    for i in range(steps):
        step()
    clock.mark(1)
    drain()
    clock.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = clock.elapsed_ms() / steps   # device time per solve (collectives excluded at N=1)
    bad = pipe.bad_status()
    if dump_gather and rank == 0:   # the gathered u0 [world*B, 4] (or histogram) of the last step
        np.save(dump_gather, pipe.result().cpu().numpy())
    # per-phase device time (HIP events the library records on the launch stream around each
    # kernel); a separate pass so that reading the events does not serialise the timed region
    mpc.set_timing(True)
    phases = []
    for _ in range(steps):
        step()
        phases.append(mpc.last_timing())
    drain()
    mpc.set_timing(False)
    phase_ms = {k: float(np.mean([p[k] for p in phases])) for k in phases[0]}
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=odev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        bb = torch.tensor([bad], dtype=torch.int64, device=odev)
        dist.all_reduce(bb)
        bad = int(bb.item())
        ph = torch.tensor([phase_ms[k] for k in sorted(phase_ms)], dtype=torch.float64, device=odev)
        dist.all_reduce(ph, op=dist.ReduceOp.MAX)
        phase_ms = dict(zip(sorted(phase_ms), ph.tolist()))
    qp = None
    if w['box']:   # active-set work of the last solve: forward passes, masked backward stages
        st = mpc.qp_stats(B).double().cpu().numpy()
        qp = dict(fwd_passes=float(st[:, 0].sum()), bwd_stages=float(st[:, 1].sum()),
                  mean_iters=float(st[:, 0].mean()), max_iters=int(st[:, 0].max()))
        if cuda and w['dtype'] == 'f32' and hasattr(getattr(mpc, 'lib', None), 'mpcb_debug_ref_list'):
            # instances the fp32 refinement kernel took (last chunk): its sweeps are counted in
            # fwd_passes / bwd_stages and its time in the phase, next to as_kernel's own
            import ctypes
            rl = (ctypes.c_int32 * 2)()
            if mpc.lib.mpcb_debug_ref_list(mpc._h, rl) == 0:
                qp['refined_last_chunk'] = int(rl[0])
        if world > 1:
            t = torch.tensor([qp['fwd_passes'], qp['bwd_stages']], dtype=torch.float64, device=odev)
            dist.all_reduce(t)
            qp['fwd_passes'], qp['bwd_stages'] = float(t[0]) / world, float(t[1]) / world
    # the kernels the timed solves launched, as rocprof names them (mpcb_last_kernels), checked
    # against the device-free plan of the same config (mpcb_plan_kernels) that the CPU tests pin
    # to the committed PMC summaries
    kernels = mpc.last_kernels()
    if cuda:
        plan = mpc.plan_kernels(B, want_traj=traj)
        if plan != kernels:
            raise SystemExit(f'launched kernels {kernels} differ from the plan {plan}')
    path = ' + '.join(kernels[k] for k in ('nominal', 'riccati', 'linearise', 'forward') if k in kernels)
    split = mpc.path == 'split'
    mpc.close()
    return dict(elapsed=elapsed, kern_ms=kern_ms, bad=bad, path=path, phase_ms=phase_ms,
                kernels=kernels, split=split, qp=qp, cuda=cuda)


def phase_kernels(w):
    """{phase: rocprof kernel name} of the solve this workload times: the library's own plan for
    the bench's handle (mpcb_plan_kernels: the selection code of mpcb_create / mpcb_solve, run
    without a device), so the roofline names exactly the dispatch rocprof and the PMC summary
    record (run() also checks the plan against what the timed solves launched)."""
    from mpc_blaster_amd import MPCConfig, _lib
    box = w['box']
    cfg = MPCConfig(N=w['N'], dtype=w['dtype'], lbu=np.zeros(4) if box else None,
                    ubu=np.full(4, 65.0) if box else None, max_as_iter=w.get('max_as_iter', 200))
    return _lib.plan_kernels(cfg.to_c(), w['batch'], w['batch'], want_traj=not w['hist'])


def kernel_flops(w, r, phase, kernel):
    """Dense algorithmic flops (per shooting interval) of one phase's kernel:
      nominal_row_kernel<T, ITER, DJ, true>  the RK4 rollout with its sensitivities, 21,996
      other rollouts (nominal_*)             4 f evaluations, 4 x 300 = 1,200
      row_riccati_kernel                     the rollout with sensitivities AND the Riccati
                                             backward of the same quad, 21,996 + 12,309 = 34,305
      riccati_kernel_*<E, ITER, true>        the Riccati backward over the rollout's [A|B], 12,309
      riccati_kernel_* (captured scalars)    the sensitivities minus the rollout's 4 f evaluations
                                             plus the Riccati backward, 21,996 - 1,200 + 12,309 = 33,105
      as_kernel_*                            the active set (c4): per masked backward stage
                                             recomputed 12,309, per forward stage 480 + the
                                             multipliers mu = G_u (dx, du) + h_u (136), counted from
                                             the kernel's own statistics (mpcb_qp_stats)
      fwd_rm_kernel / forward_kernel         du = K dx + k, dx' = [A|B] (dx, du) (+ gap): 480
    """
    B, N = w['batch'], w['N']
    name = kernel.split('::')[-1]
    base, targs = (name.split('<', 1) + [''])[:2]
    last_true = targs.rstrip('>').split(',')[-1].strip() == 'true'
    if base == 'nominal_row_kernel':
        per = 21996 if last_true else 1200
    elif base.startswith('nominal'):
        per = 1200
    elif base == 'row_riccati_kernel':
        per = 21996 + 12309
    elif base.startswith('riccati_kernel') or base == 'riccati':   # ('riccati': the CPU stub's)
        per = 12309 if last_true else 21996 - 1200 + 12309
    elif base.startswith('as_kernel'):
        q = r['qp']
        return 12309 * q['bwd_stages'] + (480 + 136) * N * q['fwd_passes']
    elif base in ('fwd_rm_kernel', 'forward_kernel', 'forward'):
        per = 480
    else:
        raise SystemExit(f'no flop count for kernel {kernel} (phase {phase})')
    return per * N * B


def dispatches_per_phase(B: int) -> int:
    """Launches of each split-path phase per solve of B instances (mpcb_capi.hip: chunks of
    65536, or MPCB_CHUNK)."""
    chunk = max(64, int(os.environ.get('MPCB_CHUNK') or 65536))
    return -(-int(B) // chunk)


def kernel_bytes(w, r, phase):
    """Algorithmic HBM bytes of the active-set kernel (c4, the only phase whose binding resource
    is memory): per forward stage the variable columns of [A|B] (12 x 10), K and k (4 x 13) and
    (xbar, ubar) (16); per recomputed backward stage the [A|B] columns (120), K and k (52) and the
    value-function snapshot for restarts (P by symmetry and p: 78 + 12): 188 and 262 elements,
    counted from the kernel's own statistics (mpcb_qp_stats).  (The Hessian rows of the fixed
    components, written and read only where a component is fixed, are not counted.)"""
    esz = 8 if w['dtype'] == 'f64' else 4
    q = r['qp']
    return esz * (188 * w['N'] * q['fwd_passes'] + 262 * q['bwd_stages'])


def pmc_kernel(workload: str, kernel: str):
    """Counter-derived figures of one kernel from the committed PMC summary (tools/pmc_summary.py).
    A committed summary without an entry for the kernel is an error, not a null: the roofline
    would cite a profile of some other kernel."""
    p = os.path.join(REPO, 'profiles', f'pmc_{workload}.json')
    if not os.path.exists(p):
        return None
    per = json.load(open(p)).get('per_kernel', {})
    if kernel not in per:
        raise SystemExit(f'{p} has no entry for the dominant kernel {kernel} (it holds {sorted(per)}): '
                         're-collect it (tools/collect_profiles.sh)')
    return per[kernel]


def summarize(w, r, world, steps):
    B, N = w['batch'], w['N']
    value = B * world * steps / r['elapsed']
    peak = PEAK_TFLOPS[w['dtype']]
    ph = r['phase_ms']
    if not r['split']:
        raise RuntimeError('bench expects the split path')
    names = r['kernels']
    # the dominant kernel by device time (HIP events on its launch stream)
    dom = max(names, key=lambda k: ph.get(k, 0.0))
    flop = kernel_flops(w, r, dom, names[dom])
    achieved_tf = flop / (ph[dom] * 1e-3) / 1e12
    solve_flop = sum(kernel_flops(w, r, k, names[k]) for k in names)
    solve_tf = solve_flop / (r['kern_ms'] * 1e-3) / 1e12
    hbm_gbs = compulsory_bytes(w) * B / (r['kern_ms'] * 1e-3) / 1e9
    pk = (pmc_kernel(w['name'], names[dom]) if r['cuda'] else None) or {}
    # the library launches each phase once per chunk of instances (mpcb_capi.hip mpcb_create:
    # 65536, MPCB_CHUNK); the PMC summary is per dispatch, the phase time and the flop count per
    # phase, so the counter figures are scaled to the phase (c5: 131072 = 2 dispatches)
    disp = dispatches_per_phase(B)
    ex = pk.get('executed_flops_per_launch')
    ex = ex * disp if ex else None
    tr = pk.get('hbm_bytes_per_launch')
    tr = tr * disp if tr else None
    roof = {'bound': 'valu', 'achieved': achieved_tf, 'peak': peak, 'unit': 'TFLOP/s',
            'frac': achieved_tf / peak, 'traffic': tr,
            'valu_frac': achieved_tf / peak,
            'kernel': names[dom], 'kernel_ms': ph[dom], 'dispatches_per_phase': disp,
            'flop_per_phase': flop, 'executed_flop_per_phase': ex,
            'executed_frac': (ex / (ph[dom] * 1e-3) / 1e12 / peak) if ex else None,
            'phase_ms': ph, 'phase_kernels': names,
            'phase_frac': {k: kernel_flops(w, r, k, names[k]) / (ph[k] * 1e-3) / 1e12 / peak
                           for k in names if ph.get(k, 0) > 0},
            'solve_ms': r['kern_ms'],
            'solve_achieved': solve_tf,
            'solve_frac': solve_tf / peak,
            'hbm_compulsory_GBs': hbm_gbs,
            'hbm_frac': hbm_gbs / HBM_PEAK_GBS,
            'note': ('compute-bound path (SURVEY §8d: ~300-700 flop per compulsory byte), executed '
                     'on the vector ALUs (fp64: DPP row-broadcast v_fmac_f64; fp32: VALU plus '
                     'v_mfma_f32_16x16x1_4b outer products; on gfx950 the fp32/fp64 VALU and MFMA '
                     'peaks are equal). kernel = the launch with the most device time (HIP events '
                     'on its launch stream); achieved = its dense algorithmic flops (bench.py '
                     'phase_kernels docstring) / that time. executed_frac = counter-executed flops '
                     '(64 x SQ_INSTS_VALU_FLOPS_FP32/FP64 + 512 x SQ_INSTS_VALU_MFMA_MOPS_F32, '
                     'profiles/pmc_<workload>.json) over the same time (c4: the active-set kernel is '
                     'memory-bound, so bound = hbm, achieved = its algorithmic bytes, bench.py '
                     'kernel_bytes, over its time; valu_frac keeps the flop view). traffic = HBM bytes per '
                     'phase of that kernel (per-dispatch PMC x dispatches_per_phase), '
                     '(2 x FETCH_SIZE + WRITE_SIZE) from the same PMC run '
                     '(gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md). solve_* = every kernel '
                     'of the solve over the whole solve time.')}
    if r.get('qp'):
        roof['active_set'] = r['qp']
    if w['box'] and dom == 'forward':
        # the active-set kernel re-streams its exported rows every pass (PMC: 2.9 TB/s, 47 % of
        # the wave time waiting): its binding resource is HBM, so that is the roofline it reports
        byt = kernel_bytes(w, r, dom)
        gbs = byt / (ph[dom] * 1e-3) / 1e9
        roof.update(bound='hbm', achieved=gbs, peak=HBM_PEAK_GBS, unit='GB/s', frac=gbs / HBM_PEAK_GBS,
                    bytes_per_phase=byt,
                    phase_note=('the forward phase (HIP events around it) holds as_kernel plus the '
                                'input-box hand-overs launched after it on the same stream: the '
                                'interior-point fallback (as_ipm_kernel) and the fp32 refinement '
                                '(as_ref_kernel_f32, active_set.refined_last_chunk instances); '
                                'their passes are in active_set.fwd_passes / bwd_stages, and '
                                'traffic / executed flops are as_kernel\'s own PMC entry'),
                    traffic_frac=(tr / (ph[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS) if tr else None)
    return value, roof


def launch_ranks(nproc: int, argv: list[str]) -> int:
    """``bench.py --gpus N`` without an outer launcher: start N ranks of this same script under
    ``torch.distributed.run`` (one process per GPU, rendezvous on 127.0.0.1) as CHILD processes
    and return their worst exit code.  The parent imports nothing that touches the GPU (no torch
    at all) and never execs: every HIP context lives in a child."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={nproc}',
           '--master-addr=127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + argv
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0', OMP_NUM_THREADS=os.environ.get('OMP_NUM_THREADS', '1'))
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--workload', default='c2', choices=sorted(WORKLOADS))
    ap.add_argument('--batch', type=int, default=None, help='override the per-GPU batch')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-secondary', action='store_true')
    ap.add_argument('--no-latency', action='store_true', help='skip the B=1 per-step latency block')
    ap.add_argument('--cpu-budget', type=float, default=12.0)
    ap.add_argument('--max-as-iter', type=int, default=200, help='active-set cap (box workload)')
    ap.add_argument('--secondary-batch', type=int, default=None,
                    help='per-GPU batch of the secondary workload (default: its BASELINE size)')
    ap.add_argument('--init-timeout', type=float, default=120.0,
                    help='seconds a rank waits for the others to join the process group')
    # launcher test only (tests/test_bench_launch.py): gloo ranks on the CPU with a stand-in solver
    ap.add_argument('--backend', default='nccl', choices=('nccl', 'gloo'), help=argparse.SUPPRESS)
    ap.add_argument('--solver-stub', default=None, help=argparse.SUPPRESS)
    ap.add_argument('--dump-gather', default=None, help=argparse.SUPPRESS)
    # rehearsal of the multi-rank path on a box with fewer GPUs than ranks: rank r binds
    # cuda:(LOCAL_RANK % device_count) (the driver's scaling runs have one GPU per rank)
    ap.add_argument('--share-gpus', action='store_true', help=argparse.SUPPRESS)
    args = ap.parse_args()

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        # no outer launcher: spawn the N ranks ourselves, before anything initialises a GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    w = dict(WORKLOADS[args.workload], name=args.workload)
    if args.batch:
        w['batch'] = args.batch
    w['max_as_iter'] = args.max_as_iter
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if 'WORLD_SIZE' in os.environ and args.gpus != world:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}')
    cuda = args.solver_stub is None
    if cuda and args.backend != 'nccl' and not args.share_gpus:
        raise SystemExit('--backend gloo is for the CPU solver stub and the --share-gpus rehearsal only')
    if cuda:
        gpu = local % torch.cuda.device_count() if args.share_gpus else local
        torch.cuda.set_device(gpu)
        dev = torch.cuda.current_device()
    else:
        dev = 'cpu'
    if args.solver_stub:   # imported before the rendezvous (the launcher test's stalled-rank case)
        import importlib
        importlib.import_module(args.solver_stub)
    if world > 1:
        # a rank that never joins makes the others fail within init_timeout (non-zero exit, and
        # torch.distributed.run then stops the remaining ranks) instead of hanging to the
        # driver's limit with no JSON line
        from datetime import timedelta
        tmo = timedelta(seconds=args.init_timeout)
        if cuda and args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device(f'cuda:{gpu}'), timeout=tmo)
        else:
            dist.init_process_group('gloo', timeout=tmo)

    r = run(w, world, rank, dev, args.steps, args.warmup, stub=args.solver_stub,
            dump_gather=args.dump_gather)
    # the secondary line: the BASELINE config quoted at this GPU count, so that the driver's
    # 1/4/8-GPU runs each time the config named for that count -- c3 (configs[2], 1 GPU), c4
    # (configs[3]: 262144 instances sharded over 4 GPUs, input box) and c5 (configs[4]: 1048576
    # over 8 GPUs, RCCL all_reduce of the u0* histogram)
    sec = None
    sec_name = {1: 'c3', 4: 'c4', 8: 'c5'}.get(world)
    if sec_name and args.workload == 'c2' and not args.no_secondary and (cuda or world > 1):
        ws = dict(WORKLOADS[sec_name], name=sec_name, max_as_iter=args.max_as_iter)
        if args.secondary_batch:
            ws['batch'] = args.secondary_batch
        rs = run(ws, world, rank, dev, args.steps, args.warmup, stub=args.solver_stub,
                 dump_gather=(args.dump_gather + '.secondary.npy') if args.dump_gather else None)
        if rank == 0:
            vs, roofs = summarize(ws, rs, world, args.steps)
            roofs.pop('note')
            desc = {'c3': 'BASELINE configs[2]: N=20, fp32, sinusoidal refs',
                    'c4': 'BASELINE configs[3]: N=30, fp32, input box [0,65] N, instance-sharded',
                    'c5': 'BASELINE configs[4]: N=40, fp32, wind sweep, u0* histogram all_reduce'}[sec_name]
            sec = {'workload': f'{sec_name}: batch {ws["batch"]}/GPU ({desc})',
                   'global_batch': ws['batch'] * world, 'n_gpus': world,
                   'value': vs, 'unit': 'solves/s', 'ms_per_step': rs['elapsed'] / args.steps * 1e3,
                   'dtype': ws['dtype'], 'path': rs['path'], 'roofline': roofs, 'bad_status': rs['bad']}

    if rank == 0:
        coll = 'RCCL' if args.backend == 'nccl' else 'gloo'
        value, roof = summarize(w, r, world, args.steps)
        B, N = w['batch'], w['N']
        line = {
            'metric': 'MPC solves/sec (N=%d, nx=12, nu=4)' % N,
            'value': value,
            'unit': 'solves/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': r['elapsed'] / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': w['dtype'],
            'data': 'synthetic (Philox4x32-10 inputs generated on device from (seed, global id), SURVEY §8d)',
            'config': {'workload': f'{w["name"]}: batch {B}/GPU, N={N}, nx=12, nu=4, {w["dtype"]}, '
                                   f'ref={w["ref"]}' + (', input box [0,65] N' if w['box'] else '')
                                   + (', wind sweep, u0 histogram' if w['wind'] else ''),
                       'global_batch': B * world, 'horizon': N, 'path': r['path'],
                       'parallelism': f'instance-sharded x{world}'
                                      + ((f' + {coll} all_reduce(histogram)' if w['hist'] else f' + {coll} all_gather(u0)')
                                         if world > 1 else '')
                                      + (' (ranks sharing GPUs: rehearsal)' if args.share_gpus else '')},
            'roofline': roof,
            'bad_status': r['bad'],
        }
        if not cuda:
            line['data'] += f'; CPU solver stub {args.solver_stub} over {args.backend} (launcher test)'
        if sec is not None:
            line['secondary'] = sec
        if world == 1 and cuda and args.workload == 'c2' and not args.no_latency:
            from mpc_blaster_amd.latency import measure_b1
            line['latency_b1'] = measure_b1(device=dev)
        if not args.no_cpu_baseline and world == 1:
            line['cpu_baseline'] = cpu_baseline(w, args.cpu_budget)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
