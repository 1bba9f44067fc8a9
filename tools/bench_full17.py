#!/usr/bin/env python3
"""Throughput of the full 17/6 model path on the reference's own OCP
(acados_ocp_blasterModel.json: N = 60, Tf = 2, W = diag(Q17, R6), W_e = 10 Q17, T_blast =
21.582): B instances, random x0 around hover, random per-instance POC Jacobian parameters,
hover + POC_x = 0.2 reference (simulation_blaster.py:48).  Not a BASELINE config: the
BASELINE metric is on the 12/4 slice (bench.py).  Prints one JSON line.

    python tools/bench_full17.py [--batch 4096] [--N 60] [--dtype f64] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=4096)
    ap.add_argument('--N', type=int, default=60)
    ap.add_argument('--dtype', default='f64')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--bounds', default='none', choices=['none', 'input', 'all'],
                    help="the reference's controlBound (input) and statesBound (all) by the interior point")
    ap.add_argument('--dump', default=None, help='save per-instance status and QP statistics (npz)')
    args = ap.parse_args()
    import torch
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    B, N = args.batch, args.N
    rng = np.random.default_rng(1017)
    x0 = np.zeros((B, 17))
    x0[:, 0:3] = rng.uniform(-1, 1, (B, 3))
    x0[:, 2] += 3.5
    x0[:, 3:6] = rng.uniform(-0.17, 0.17, (B, 3))
    x0[:, 6:9] = rng.uniform(-0.5, 0.5, (B, 3))
    x0[:, 9:12] = rng.uniform(-0.087, 0.087, (B, 3))
    xref = np.zeros((1, N + 1, 17))
    xref[..., 2], xref[..., 14] = 3.5, 0.2
    uref = np.zeros((1, N, 6))
    uref[..., :4] = 22.0725
    p = np.zeros((B, 25))
    p[:, :24] = rng.uniform(-0.5, 0.5, (B, 24))
    p[:, 24] = 2.2 * 9.81
    lbu = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])     # simulation_blaster.py:28-30
    ubu = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
    lbx = np.array([-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0, -0.0872665,
                    -0.0872665, -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5])
    kw = {}
    if args.bounds != 'none':
        kw.update(lbu=lbu, ubu=ubu)
    if args.bounds == 'all':
        kw.update(lbx=lbx, ubx=-lbx)
        kw['ubx'][[2, 12]] = 5.0, 1.22173
        x0 = np.clip(x0, 0.5 * lbx, 0.5 * kw['ubx'])
        x0[:, 2] = 3.5 + rng.uniform(-0.5, 0.5, B)
    cfg = MPCConfig.full(N=N, dtype=args.dtype, **kw)
    m = BatchedMPC(cfg, max_batch=B)
    dt = cfg.torch_dtype
    dev = 'cuda:0'
    x0t, xrt, urt, pt = (torch.as_tensor(a, dtype=dt, device=dev) for a in (x0, xref, uref, p))
    m.set_params(pt)
    outs = (torch.empty((B, 6), dtype=dt, device=dev), torch.empty((B, N + 1, 17), dtype=dt, device=dev),
            torch.empty((B, N, 6), dtype=dt, device=dev), torch.empty((B,), dtype=torch.int32, device=dev))
    for _ in range(args.warmup):
        m.solve(x0t, xrt, urt, out=outs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m.solve(x0t, xrt, urt, out=outs)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    bad = int((outs[3] != 0).sum().item())
    status_counts = np.bincount(outs[3].cpu().numpy(), minlength=5).tolist()   # OK, NAN, MAXITER, MINSTEP, QP_FAIL
    m.set_timing(True)                     # one more solve with per-phase HIP events
    m.solve(x0t, xrt, urt, out=outs)
    ph = m.last_timing()
    m.set_timing(False)
    # riccati17 algorithmic flops per stage (dense counts, nx = 17, nu = 6, nz = 23): P[A|B]
    # 2 nx^2 nz, [A|B]' P [A|B] 2 nz^2 nx, Cholesky nu^3/3 + K, k solves 2 nu^2 (nx + 1),
    # P update 2 nx^2 nu, vector terms 2 nx^2 + 2 nz nx + 2 (nx^2 + nu^2) + 2 nx nu, and the
    # forward pass 2 nu nx + 2 nx nz
    nx_, nu_, nz_ = 17, 6, 23
    fwd = 2 * nu_ * nx_ + 2 * nx_ * nz_
    fl = (2 * nx_ * nx_ * nz_ + 2 * nz_ * nz_ * nx_ + nu_ ** 3 / 3 + 2 * nu_ * nu_ * (nx_ + 1) + 2 * nx_ * nx_ * nu_
          + 2 * nx_ * nx_ + 2 * nz_ * nx_ + 2 * (nx_ * nx_ + nu_ * nu_) + 2 * nx_ * nu_ + fwd)
    peak = 78.6 if args.dtype == 'f64' else 157.3
    box = args.bounds != 'none'
    meh = args.bounds == 'input' and args.dtype == 'f64'
    # the interior-point / Riccati dispatch as rocprof names it, from the library's launch log
    # (mpcb_last_kernels), checked against its device-free plan
    kname = m.last_kernels()['riccati']
    assert m.last_kernels() == m.plan_kernels(B), (m.last_kernels(), m.plan_kernels(B))
    # interior point (boxes): per iteration one Riccati backward with the row terms and one forward
    # step (fl per stage), plus the rows' step-length and update arithmetic (~12 flop per row and
    # pass: rows = nu + nx with the state box); Mehrotra adds its affine step and a vector-only
    # corrector pass (the h_u, k, p' recursion over the stored factor: 2 nz nx + 2 nu^2 + 2 nx nu
    # + 2 nu nx) and the corrector's forward.  The polish pass (state box) is one backward +
    # forward + a row pass.  Iterations and polish passes are counted per instance by the kernel
    # (mpcb_qp_stats), so the count is the work each instance needed, not the wave's lock-step.
    rows = nu_ + (nx_ if args.bounds == 'all' else 0)
    it_fl = fl + 2 * 12 * rows + ((2 * nz_ * nx_ + 2 * nu_ * nu_ + 4 * nx_ * nu_ + fwd) if meh else 0)
    pol_fl = fl + 12 * rows
    qp = None
    if args.dump:
        np.savez(args.dump, status=outs[3].cpu().numpy(),
                 qp_stats=m.qp_stats(B).cpu().numpy() if box else np.zeros((B, 2), np.int32))
    if box:
        st = m.qp_stats(B).double().cpu().numpy()
        qp = dict(mean_iters=float(st[:, 0].mean()), max_iters=int(st[:, 0].max()),
                  mean_polish=float(st[:, 1].mean()), max_polish=int(st[:, 1].max()),
                  iters_total=float(st[:, 0].sum()), polish_total=float(st[:, 1].sum()))
        flop = (it_fl * qp['iters_total'] + pol_fl * qp['polish_total']) * N
    else:
        flop = fl * N * B
    ach = flop / (ph['riccati'] * 1e-3) / 1e12
    # executed flops from the committed PMC summary (profiles/pmc_full17*.json, per dispatch = one
    # launch here: 64 x SQ_INSTS_VALU_FLOPS_FP64) at the profiled configuration
    ex = None
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pj = os.path.join(root, 'profiles', 'pmc_full17.json' if not box else f'pmc_full17_{args.bounds}.json')
    pk = None
    if os.path.exists(pj) and args.dtype == 'f64' and B == 4096 and N == 60:
        per = json.load(open(pj)).get('per_kernel', {})
        if kname not in per:   # a committed summary of some other kernel: re-collect, do not cite it
            raise SystemExit(f'{pj} has no entry for {kname} (it holds {sorted(per)})')
        pk = per[kname]
        e = pk.get('executed_flops_per_launch')
        ex = e / (ph['riccati'] * 1e-3) / 1e12 / peak if e else None
    # HBM view.  Algorithmic bytes per instance-stage of one interior-point iteration (fp64): the
    # backward reads the 16 dense [A|B] columns and the 5 nonzeros of the shear column (277) and
    # writes K, k (108); the Newton-step forward reads the same rows (277) and K, k (108): 770
    # doubles; Mehrotra adds the corrector's vector pass (277 + 108 + the factor 21, gradients 24,
    # row terms 48, k 6) and its forward (385): 1639 doubles.  A polish pass is a plain iteration.
    # The unconstrained pass: one backward + forward (770).  traffic = the PMC's HBM bytes per
    # launch (profiles/pmc_full17*.json, (2 FETCH_SIZE + WRITE_SIZE) KiB) at the profiled size.
    esz = 8 if args.dtype == 'f64' else 4
    it_b = (770 + (869 if meh else 0)) * esz
    if box:
        byt = (it_b * qp['iters_total'] + 770 * esz * qp['polish_total']) * N
    else:
        byt = 770 * esz * N * B
    tr = pk.get('hbm_bytes_per_launch') if pk else None
    hbm = {'achieved': byt / (ph['riccati'] * 1e-3) / 1e9, 'peak': 8000.0, 'unit': 'GB/s',
           'bytes_per_launch': byt, 'bytes_per_iteration_stage': it_b, 'traffic': tr,
           'traffic_GBs': tr / (ph['riccati'] * 1e-3) / 1e9 if tr else None}
    hbm['frac'] = hbm['achieved'] / hbm['peak']
    hbm['traffic_frac'] = hbm['traffic_GBs'] / hbm['peak'] if tr else None
    # the boxed kernels stream their [A|B] and gains every iteration: their binding resource is
    # memory (B = 1024 -> 4096 at the same iteration count: 10.1 -> 17.1 ms, profiles/r03), the
    # unconstrained pass is issue-bound (VALU)
    roof = {'bound': 'hbm' if box else 'valu', 'kernel': kname, 'kernel_ms': ph['riccati'],
            'valu': {'achieved': ach, 'peak': peak, 'unit': 'TFLOP/s', 'frac': ach / peak,
                     'executed_frac': ex, 'flop_per_stage': fl, 'flop_per_launch': flop},
            'hbm': hbm}
    main = hbm if box else roof['valu']
    roof.update(achieved=main['achieved'], peak=main['peak'], unit=main['unit'], frac=main['frac'],
                traffic=tr, executed_frac=ex)
    if qp:
        roof.update(interior_point=qp, flop_per_iteration_stage=it_fl, flop_per_polish_stage=pol_fl)
    print(json.dumps({'metric': f'MPC solves/sec (full 17/6 model, N={N})', 'value': B * args.steps / el,
                      'unit': 'solves/s', 'ms_per_step': el / args.steps * 1e3, 'batch': B,
                      'dtype': args.dtype, 'bad_status': bad, 'status_counts': status_counts,
                      'bounds': args.bounds,
                      'phase_ms': ph, 'roofline': roof,
                      'config': 'reference OCP (acados_ocp_blasterModel.json), random x0 + POC params'}))


if __name__ == '__main__':
    main()
