"""Diagnostics for the 17/6 state-box interior point (oracle.ocp.ipm_box_solve; not a test):
per-instance status and iterations next to an LP feasibility check of the same QP.

usage: python tools/sbox_diag.py [B] [max_iter]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from oracle.full import FullSpec, mpc_solve17  # noqa: E402
from oracle.ocp import ipm_box_solve, lp_box_feasible  # noqa: E402
from test_gpu_full17 import LBU17, UBU17, _inputs  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    max_iter = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    N = 20
    d = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'ocp_json_pin.json')))
    lbx, ubx = np.array(d['lbx']), np.array(d['ubx'])
    x0, xref, uref, p = _inputs(B, N, 31)
    x0[:, 3:17] *= 0.5
    x0[:, 0:2] *= 0.5
    o = mpc_solve17(x0, xref, uref, FullSpec(N=N), p)
    spec = FullSpec(N=N, lbu=LBU17, ubu=UBU17)
    dx0 = x0 - o['xbar'][:, 0]
    xr = np.broadcast_to(xref, (B, N + 1, 17))
    ur = np.broadcast_to(uref, (B, N, 6))
    with np.errstate(all='ignore'):
        _, du, st, it = ipm_box_solve(o['A'], o['B'], o['gap'], dx0, o['xbar'], o['ubar'], xr, ur, spec,
                                      max_iter=max_iter, lbx=lbx, ubx=ubx)
    feas = lp_box_feasible(o['A'], o['B'], o['gap'], dx0, o['xbar'], o['ubar'], spec, lbx, ubx)
    for b in range(B):
        print(b, 'status', st[b], 'it', it[b], 'lp_feasible', bool(feas[b]), 'finite', bool(np.isfinite(du[b]).all()))


if __name__ == '__main__':
    main()
