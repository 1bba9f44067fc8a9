"""Full-batch c4 parity study (BASELINE configs[3] per-GPU shard: 65,536 instances, N = 30, fp32,
thrust box [0, 65], hover reference, seed 1004): every instance's u0 / U / X from the device
(fp32, and fp64 on the same fp32-rounded inputs) against the plain-C fp64 oracle (oracle/c) on
those inputs.  Prints the error distribution and the active-set passes of the worst instances,
and saves the worst instances' inputs and outputs to ``--out`` for a CPU study.

Usage (GPU box): python tools/c4_full_parity.py [--B 65536] [--N 30] [--seed 1004] [--out F]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def relerr(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, dtype=np.float64).reshape(b.shape[0], -1)
    return np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, default=65536)
    ap.add_argument('--N', type=int, default=30)
    ap.add_argument('--seed', type=int, default=1004)
    ap.add_argument('--ref', default='hover')
    ap.add_argument('--worst', type=int, default=64)
    ap.add_argument('--out', default='gpurun_out/c4_worst.npz')
    ap.add_argument('--threads', type=int, default=16)
    ap.add_argument('--exact-xbar', action='store_true',
                    help='(study) solve in iterate mode at the fp64 rollout of u_ref rounded to fp32, '
                         'i.e. the fp32 solve without the fp32 rollout drift')
    a = ap.parse_args()
    import torch

    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle import c_oracle
    from oracle.ocp import OcpSpec
    B, N = a.B, a.N
    box = dict(lbu=np.zeros(4), ubu=np.full(4, 65.0))
    m = BatchedMPC(MPCConfig(N=N, dtype='f32', **box), max_batch=B)
    d = m.gen_inputs(B, seed=a.seed, ref=a.ref)
    if a.exact_xbar:
        from oracle.ocp import rollout
        x0h = d['x0'].double().cpu().numpy()
        xb = rollout(x0h, np.broadcast_to(d['uref'].double().cpu().numpy(), (B, N, 4)),
                     OcpSpec(N=N, **box)).astype(np.float32)
        u0 = m.solve_iterate(d['x0'], xb, d['uref'].expand(B, N, 4).contiguous(), d['xref'], d['uref']).clone()
    else:
        u0 = m.solve(d['x0'], d['xref'], d['uref'], want_traj=True).clone()
    X, U, st = m.get_state_trajectory().clone(), m.get_input_trajectory().clone(), m.get_status().clone()
    qs = m.qp_stats(B)
    torch.cuda.synchronize()
    # (study) the same solve without the refinement kernel: which instances it took, and their work
    os.environ['MPCB_AS_REFINE'] = '0'   # (read at every solve)
    try:
        m0 = BatchedMPC(MPCConfig(N=N, dtype='f32', **box), max_batch=B)
        if a.exact_xbar:
            m0.solve_iterate(d['x0'], xb, d['uref'].expand(B, N, 4).contiguous(), d['xref'], d['uref'])
        else:
            m0.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
        qs0 = m0.qp_stats(B).cpu().numpy()
    finally:
        os.environ.pop('MPCB_AS_REFINE')
    U0 = m0.get_input_trajectory().double().cpu().numpy()
    del m0
    import ctypes
    rl = (ctypes.c_int32 * 2)()
    if m.lib.mpcb_debug_ref_list(m._h, rl) == 0:
        print(f'refinement list: {rl[0]} instances listed (fp32 box, last chunk)')
    x0 = d['x0'].double().cpu().numpy()
    xr = d['xref'].double().cpu().numpy()
    ur = d['uref'].double().cpu().numpy()
    u0, X, U, st, qs = (t.double().cpu().numpy() if t.is_floating_point() else t.cpu().numpy()
                        for t in (u0, X, U, st, qs))
    # fp64 device solve of the same (fp32-rounded) inputs
    m64 = BatchedMPC(MPCConfig(N=N, dtype='f64', **box), max_batch=B)
    u64 = m64.solve(x0, xr, ur, want_traj=True).cpu().numpy()
    U64 = m64.get_input_trajectory().cpu().numpy()
    spec = OcpSpec(N=N, **box)
    t0 = time.time()
    o = c_oracle.solve(x0, xr, ur, spec, nthreads=a.threads)
    print(f'oracle/c: {B} instances in {time.time() - t0:.2f} s ({a.threads} threads)')
    print(f'statuses device {np.bincount(st, minlength=5).tolist()} oracle {np.bincount(o["status"], minlength=5).tolist()}')
    eu, eU, eX = relerr(u0, o['u0']), relerr(U, o['U']), relerr(X, o['X'])
    e64 = max(relerr(u64, o['u0']).max(), relerr(U64, o['U']).max())
    print(f'fp64 device vs oracle/c: {e64:.2e}')
    for name, e in (('u0', eu), ('U', eU), ('X', eX)):
        q = np.quantile(e, [0.5, 0.9, 0.99, 0.999, 1.0])
        print(f'fp32 {name}: quantiles 50/90/99/99.9/max ' + ' '.join(f'{v:.2e}' for v in q)
              + f'; > 5e-5: {(e > 5e-5).sum()}, > 1e-5: {(e > 1e-5).sum()}')
    dq = qs[:, 0] - qs0[:, 0]
    ref = np.nonzero(dq)[0]
    print(f'refined instances: {len(ref)}; extra forward-pass equivalents per refined instance: '
          f'{np.bincount(dq[ref]).nonzero()[0].tolist()} (counts {np.bincount(dq[ref])[np.bincount(dq[ref]) > 0].tolist()}); '
          f'extra backward stages max {int((qs[:, 1] - qs0[:, 1]).max())}')
    if len(ref):
        capped = ref[qs[ref, 0] > 200]
        okr = np.setdiff1d(ref, capped)
        if len(okr):
            print(f'refined and converged: {len(okr)}; U err max {eU[okr].max():.2e} median {np.median(eU[okr]):.2e}; '
                  f'u0 err max {eu[okr].max():.2e}; capped (> 200 forward-pass equivalents): {len(capped)} {capped[:8].tolist()}')
    wu = np.argsort(-eu)[:8]
    print('worst u0 instances: ' + '; '.join(
        f'{i}: err {eu[i]:.2e} |u0| max {np.abs(o["u0"][i]).max():.3f} U err {eU[i]:.2e} listed {dq[i] > 0}' for i in wu))
    eU0 = relerr(U0, o['U'])
    print(f'without refinement: U max {eU0.max():.2e}, > 5e-5: {(eU0 > 5e-5).sum()}')
    worst = np.argsort(-np.maximum(eU, eX))[:a.worst]
    npass = qs[:, 0]
    print(f'passes: mean {npass.mean():.2f} max {npass.max()}; worst-U instances passes {npass[worst[:16]].tolist()}')
    nfix = ((o['U'] <= 1e-9) | (o['U'] >= 65 - 1e-9)).sum(axis=(1, 2))
    print(f'active components (oracle): mean {nfix.mean():.2f}; worst instances {nfix[worst[:16]].tolist()}')
    for i in worst[:12]:
        print(f'  inst {i}: u0 {eu[i]:.2e} U {eU[i]:.2e} X {eX[i]:.2e} passes {npass[i]} active {nfix[i]}')
    os.makedirs(os.path.dirname(a.out) or '.', exist_ok=True)
    np.savez(a.out, idx=worst, x0=x0[worst], xref=xr[0], uref=ur[0], u0=u0[worst], U=U[worst], X=X[worst],
             oU=o['U'][worst], oX=o['X'][worst], passes=npass[worst], eu=eu, eU=eU, eX=eX, N=N)
    print(f'saved {a.out}')


if __name__ == '__main__':
    main()
