"""Explicit RK4 with exact forward sensitivities (oracle; test infrastructure only).

Restates acados ``sim_erk`` as configured by the reference: ``integrator_type='ERK'``
(``blastermodel.py:277``), 4 stages / 1 step per shooting interval
(``acados_ocp_blasterModel.json`` ``sim_method_num_stages`` / ``sim_method_num_steps``),
step h = Tf/N (JSON ``time_steps`` / ``Tsim``).  [acados sim_erk: classic Butcher tableau
(1/2, 1/2, 1; weights 1/6, 1/3, 1/3, 1/6) — third-party, unpinned beyond that.]

A, B are the exact derivatives of the discrete RK4 map, propagated in forward mode
through the four stages (what acados' forward VDE computes).
"""
from __future__ import annotations

import numpy as np

from .model import Params, f12, jac12


def rk4_step(x, u, h, P: Params, wind=None, f=f12):
    x = np.asarray(x, dtype=np.float64)
    k1 = f(x, u, P, wind)
    k2 = f(x + 0.5 * h * k1, u, P, wind)
    k3 = f(x + 0.5 * h * k2, u, P, wind)
    k4 = f(x + h * k3, u, P, wind)
    return x + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)


def rk4_sens(x, u, h, P: Params, wind=None):
    """Return (x_next, A, B) with A = d x_next / d x (nx x nx), B = d x_next / d u (nx x nu)."""
    x = np.asarray(x, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    nx, nu = x.shape[-1], u.shape[-1]
    bs = x.shape[:-1]
    S0 = np.zeros(bs + (nx, nx + nu))
    S0[..., :, :nx] = np.eye(nx)
    Eu = np.zeros(bs + (nu, nx + nu))
    Eu[..., :, nx:] = np.eye(nu)

    def dk(xs, dxs):
        Jf = jac12(xs, u, P, wind)
        return np.einsum('...ij,...jk->...ik', Jf[..., :, :nx], dxs) + \
            np.einsum('...ij,...jk->...ik', Jf[..., :, nx:], Eu)

    k1 = f12(x, u, P, wind)
    d1 = dk(x, S0)
    x2 = x + 0.5 * h * k1
    k2 = f12(x2, u, P, wind)
    d2 = dk(x2, S0 + 0.5 * h * d1)
    x3 = x + 0.5 * h * k2
    k3 = f12(x3, u, P, wind)
    d3 = dk(x3, S0 + 0.5 * h * d2)
    x4 = x + h * k3
    k4 = f12(x4, u, P, wind)
    d4 = dk(x4, S0 + h * d3)
    xn = x + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
    S = S0 + (h / 6.0) * (d1 + 2.0 * d2 + 2.0 * d3 + d4)
    return xn, S[..., :, :nx], S[..., :, nx:]
