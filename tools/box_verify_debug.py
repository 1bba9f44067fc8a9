"""Diagnostic (GPU box): the fp32 input-box solve of selected c4 instances, with the objective's
exact gradient at the device's U evaluated on the host in fp64 over (a) the device's own fp32
linearisation (sim_step rollout + mpcb_linearize, what the kernel's fp64 verification sees) and
(b) the oracle's fp64 linearisation.  Prints, per instance, the fixed components whose gradient
(the box multiplier) has the wrong sign and the verification's tolerance there.

    python tools/box_verify_debug.py --ids 32481 62027 [--seed 1004 --N 30]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gradient(A, Bm, gap, x0, xbar, ubar, U, xref, uref, spec):
    """fp64 re-simulation of U through (A, B, gap) from x0, then the adjoint sweep: the exact
    gradient of the QP objective w.r.t. U and |terms| sums (as_body's verification)."""
    B, N = U.shape[0], spec.N
    s, Q, R, QN = spec.s, spec.Q, spec.R, spec.QN
    dx = x0 - xbar[:, 0]
    X = np.empty((B, N + 1, 12))
    for k in range(N):
        X[:, k] = xbar[:, k] + dx
        dx = np.einsum('bij,bj->bi', A[:, k], dx) + np.einsum('bij,bj->bi', Bm[:, k], U[:, k] - ubar[:, k]) + gap[:, k]
    X[:, N] = xbar[:, N] + dx
    lam = np.einsum('ij,bj->bi', QN, X[:, N] - xref[:, N])
    g = np.empty((B, N, 4))
    sc = np.empty((B, N, 4))
    for k in range(N - 1, -1, -1):
        eu = U[:, k] - uref[:, k]
        g[:, k] = s * eu @ R.T + np.einsum('bji,bj->bi', Bm[:, k], lam)
        sc[:, k] = (np.abs(s * R)[None] * np.abs(eu)[:, None, :]).sum(-1) + np.einsum('bji,bj->bi', np.abs(Bm[:, k]), np.abs(lam))
        lam = s * (X[:, k] - xref[:, k]) @ Q.T + np.einsum('bji,bj->bi', A[:, k], lam)
    return g, sc, X


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ids', type=int, nargs='+', required=True)
    ap.add_argument('--seed', type=int, default=1004)
    ap.add_argument('--N', type=int, default=30)
    ap.add_argument('--data-study', action='store_true')
    a = ap.parse_args()
    if a.data_study:
        return data_study(a.ids, a.seed, a.N)
    import torch

    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle.ocp import OcpSpec, mpc_solve
    N = a.N
    box = dict(lbu=np.zeros(4), ubu=np.full(4, 65.0))
    spec = OcpSpec(N=N, **box)
    mx = max(a.ids) + 1
    m = BatchedMPC(MPCConfig(N=N, dtype='f32', **box), max_batch=mx)
    d = m.gen_inputs(mx, seed=a.seed, ref='hover')
    ids = np.asarray(a.ids)
    x0 = d['x0'][ids].contiguous()
    m.solve(x0, d['xref'], d['uref'], want_traj=True)
    U = m.get_input_trajectory().double().cpu().numpy()
    qs = m.qp_stats(len(ids)).cpu().numpy()
    B = len(ids)
    # the device's fp32 linearisation: rollout by sim_step, then mpcb_linearize
    xb = torch.empty((B, N + 1, 12), dtype=torch.float32, device=x0.device)
    xb[:, 0] = x0
    ub = d['uref'].expand(B, N, 4).contiguous()
    for k in range(N):
        xb[:, k + 1] = m.sim_step(xb[:, k].contiguous(), ub[:, k].contiguous())
    A32, B32, xn = m.linearize(xb, ub)
    torch.cuda.synchronize()
    xbar = xb.double().cpu().numpy()
    ubar = ub.double().cpu().numpy()
    gap = xn.double().cpu().numpy() - xbar[:, 1:]
    xr = np.broadcast_to(d['xref'].double().cpu().numpy(), (B, N + 1, 12))
    ur = np.broadcast_to(d['uref'].double().cpu().numpy(), (B, N, 4))
    x0d = x0.double().cpu().numpy()
    g32, sc32, _ = gradient(A32.double().cpu().numpy(), B32.double().cpu().numpy(), gap, x0d, xbar, ubar, U, xr, ur, spec)
    o = mpc_solve(x0d, xr, ur, spec, return_lin=True)
    g64, sc64, _ = gradient(o['A'], o['B'], o['gap'], x0d, o['xbar'], o['ubar'], U, xr, ur, spec)
    tol_u = 16 * float(np.finfo(np.float32).eps) * 66.0
    for b in range(B):
        low, up = U[b] <= tol_u, U[b] >= 65 - tol_u
        e = np.abs(U[b] - o['U'][b])
        k, mm = np.unravel_index(e.argmax(), e.shape)
        print(f'inst {ids[b]}: qp_stats {qs[b].tolist()}; max |dU| {e.max():.3e} at ({k},{mm}) dev {U[b, k, mm]:.5f} oracle {o["U"][b, k, mm]:.5f}')
        for name, g, sc in (('device data', g32, sc32), ('oracle data', g64, sc64)):
            wrong = (low & (g[b] < 0)) | (up & (g[b] > 0))
            print(f'  {name}: gradient at ({k},{mm}) {g[b, k, mm]:.3e}, tol 2^-20 sum|terms| {sc[b, k, mm] * 2**-20:.3e}; '
                  f'wrong-sign fixed components {np.argwhere(wrong).tolist()} values {[f"{g[b, i, j]:.2e}" for i, j in np.argwhere(wrong)]}')




def data_study(ids, seed=1004, N=30):
    """(study) the oracle's exact QP solve on the device's fp32 [A|B] (mpcb_linearize at the
    oracle's rollout rounded to fp32) against the oracle's own: how far fp32 sensitivities alone
    move the minimiser."""
    import torch

    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle.ocp import OcpSpec, mpc_solve, pdas_solve
    box = dict(lbu=np.zeros(4), ubu=np.full(4, 65.0))
    spec = OcpSpec(N=N, **box)
    mx = max(ids) + 1
    m = BatchedMPC(MPCConfig(N=N, dtype='f32', **box), max_batch=mx)
    d = m.gen_inputs(mx, seed=seed, ref='hover')
    ids = np.asarray(ids)
    B = len(ids)
    x0 = d['x0'][ids].double().cpu().numpy()
    xr = np.broadcast_to(d['xref'].double().cpu().numpy(), (B, N + 1, 12))
    ur = np.broadcast_to(d['uref'].double().cpu().numpy(), (B, N, 4))
    o = mpc_solve(x0, xr, ur, spec, return_lin=True)
    A32, B32, _ = m.linearize(o['xbar'].astype(np.float32), o['ubar'].astype(np.float32))
    torch.cuda.synchronize()
    A32, B32 = A32.double().cpu().numpy(), B32.double().cpu().numpy()
    print('max |dA| %.2e (max |A| %.2e), max |dB| %.2e (max |B| %.2e)' % (
        np.abs(A32 - o['A']).max(), np.abs(o['A']).max(), np.abs(B32 - o['B']).max(), np.abs(o['B']).max()))
    for name, A, Bm in (('A32 B32', A32, B32), ('A32 B64', A32, o['B']), ('A64 B32', o['A'], B32),
                        ('A,B rounded', o['A'].astype(np.float32).astype(float), o['B'].astype(np.float32).astype(float))):
        dx, du, st, it, _ = pdas_solve(A, Bm, o['gap'], x0 - o['xbar'][:, 0], o['xbar'], o['ubar'], xr, ur, spec)
        U = o['ubar'] + du
        e = np.abs(U - o['U']).reshape(B, -1).max(1) / np.maximum(np.abs(o['U']).reshape(B, -1).max(1), 1)
        print(f'  exact QP on {name}: rel err U per instance {[f"{v:.2e}" for v in e]}')


if __name__ == '__main__':
    main()
