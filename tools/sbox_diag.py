"""Diagnostics for the state-box IPM in oracle.ocp (not a test): per-instance status and an LP
feasibility check of the condensed QP (scipy linprog)."""
import json
import sys

import numpy as np
from scipy.optimize import linprog

sys.path.insert(0, '.')
import oracle.ocp as ocp  # noqa: E402
from oracle.full import FullSpec, default_p25, mpc_solve17  # noqa: E402,F401

src = open('tests/test_gpu_full17.py').read()
exec(src[src.index('def _inputs'):src.index('def _mpc')])
LBU = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])
UBU = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
d = json.load(open('tests/golden/ocp_json_pin.json'))
lbx, ubx = np.array(d['lbx']), np.array(d['ubx'])


def condense(A, Bm, gap, dx0, N):
    NX, NU = A.shape[-1], Bm.shape[-1]
    Phi = np.zeros((N + 1, NX, N * NU))
    c = np.zeros((N + 1, NX))
    c[0] = dx0
    for k in range(N):
        Phi[k + 1] = A[k] @ Phi[k]
        Phi[k + 1][:, k * NU:(k + 1) * NU] += Bm[k]
        c[k + 1] = A[k] @ c[k] + gap[k]
    return Phi, c


def feasible(A, Bm, gap, dx0, xbar, ubar, N):   # see also oracle.ocp.lp_box_feasible
    Phi, c = condense(A, Bm, gap, dx0, N)
    NU = Bm.shape[-1]
    G = Phi[1:N].reshape(-1, N * NU)
    lo = (lbx - xbar[1:N] - c[1:N]).ravel()
    hi = (ubx - xbar[1:N] - c[1:N]).ravel()
    bnds = list(zip((LBU - ubar).ravel(), (UBU - ubar).ravel()))
    r = linprog(np.zeros(N * NU), A_ub=np.vstack([G, -G]), b_ub=np.concatenate([hi, -lo]), bounds=bnds,
                method='highs')
    return r.status


B, N = int(sys.argv[1]) if len(sys.argv) > 1 else 24, 20
x0, xref, uref, p = _inputs(B, N, 31)
x0[:, 3:17] *= 0.5
x0[:, 0:2] *= 0.5
o = mpc_solve17(x0, xref, uref, FullSpec(N=N), p)
sb = FullSpec(N=N, lbu=LBU, ubu=UBU)
A, Bm, gap, xbar, ubar = o['A'], o['B'], o['gap'], o['xbar'], o['ubar']
dx0 = x0 - xbar[:, 0]
with np.errstate(all='ignore'):
    dx, du, st, it = ocp.ipm_box_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, sb, lbx=lbx, ubx=ubx,
                                       max_iter=int(sys.argv[2]) if len(sys.argv) > 2 else 60)
for b in range(B):
    print(b, 'status', st[b], 'it', it[b], 'lp', feasible(A[b], Bm[b], gap[b], dx0[b], xbar[b], ubar[b], N),
          'finite', np.isfinite(du[b]).all())

