"""The full 17-state / 6-input BLASTER OCP (oracle; test infrastructure only).

SURVEY §8 row f2.  The reference's actual controller (``blastermodel.py:70-292``, pinned numbers in
``acados_ocp_blasterModel.json``: N = 60, Tf = 2, ny = 23, W = diag(Q17, R6), W_e = 10 Q17, 25
parameters with T_blast = 21.582 at ``parameter_values[24]``):

* dynamics ``f17`` (``oracle.model``, pinned to the reference's own ``generateModel()`` by
  ``tests/golden/dynamics_ref17.npz``): the rigid body of ``f12`` plus the swivel angles
  alpha (alpha_dot = u[4:6]) that tilt the blaster thrust T_blast through R_gimbal, and the
  point-of-contact states (poc_dot = J_p v + J_euler eta_dot + J_angles alpha_dot);
* RK4 with exact sensitivities of the discrete map, here by the complex step
  (A e_j = Im Phi(x + i eps e_j) / eps, eps = 1e-30: exact to rounding, no subtraction), checked
  against the golden analytic Jacobians of f17 at the f level;
* the same Gauss-Newton LQ step and Riccati recursion as the 12/4 slice
  (``oracle.ocp.riccati_solve`` is dimension-generic); the input box (JSON idxbu) by the
  primal-dual interior point ``oracle.ocp.ipm_box_solve`` (acados uses HPIPM's interior point;
  the exact active set of the 12/4 path needs thousands of exchanges on this model).

The reference's state box (``idxbx``, stages 1..N-1, ``FullSpec.lbx/ubx``) goes through the same
interior point (explicit slacks with an infeasible start, ``oracle.ocp.ipm_box_solve``).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .model import Params, f17
from .ocp import STATUS_NAN, STATUS_OK, STATUS_QP_FAIL, ipm_box_solve, riccati_solve

NX17, NU17, NP17 = 17, 6, 25
EPS_CS = 1e-30


def default_Q17() -> np.ndarray:
    # simulation_blaster.py:24 (JSON cost.W diag[0:17])
    return np.diag([1e3] * 6 + [5.0] * 3 + [10.0] * 3 + [1e-2] * 2 + [1e3] * 3)


def default_R6() -> np.ndarray:
    # simulation_blaster.py:27 (JSON cost.W diag[17:23])
    return np.diag([0.05] * 4 + [1e-5] * 2)


def default_p25() -> np.ndarray:
    # JSON parameter_values: all Jacobian entries 0, T_blast = 2.2 * 9.81 (simulation_blaster.py:22,67)
    p = np.zeros(NP17)
    p[24] = 2.2 * 9.81
    return p


@dataclass
class FullSpec:
    N: int = 60
    dt: float = 2.0 / 60.0
    Q: np.ndarray = field(default_factory=default_Q17)
    R: np.ndarray = field(default_factory=default_R6)
    QN: np.ndarray | None = None          # default 10 Q (simulation_blaster.py:25)
    cost_scale: float | None = None       # default dt (acados time_steps)
    lbu: np.ndarray | None = None
    ubu: np.ndarray | None = None
    lbx: np.ndarray | None = None         # state box on stages 1..N-1 (JSON idxbx), needs lbu
    ubx: np.ndarray | None = None
    params: Params = field(default_factory=Params)
    max_as_iter: int = 200

    def __post_init__(self):
        if self.QN is None:
            self.QN = 10.0 * np.asarray(self.Q)

    @property
    def s(self) -> float:
        return self.dt if self.cost_scale is None else self.cost_scale

    @property
    def boxed(self) -> bool:
        return self.lbu is not None


def rk4_step17(x, u, p25, h, P: Params):
    k1 = f17(x, u, p25, P)
    k2 = f17(x + 0.5 * h * k1, u, p25, P)
    k3 = f17(x + 0.5 * h * k2, u, p25, P)
    k4 = f17(x + h * k3, u, p25, P)
    return x + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)


def _f17c(x, u, p25, P: Params):
    """f17 on complex arguments (the complex step); same algebra as oracle.model.f17."""
    from .model import _rb_core, unpack_params25
    Ja, Je, Jp, tb = unpack_params25(p25)
    a1, a2 = x[..., 12], x[..., 13]
    g3 = np.stack([np.sin(a1) * np.cos(a2), -np.sin(a2), np.cos(a1) * np.cos(a2)], axis=-1)
    extra = g3 * np.asarray(tb)[..., None]
    p_dot, eta_dot, v_dot, om_dot = _rb_core(x, u[..., 0:4], P, extra)
    adot = u[..., 4:6]
    poc = (np.einsum('...ij,...j->...i', Jp, x[..., 6:9]) + np.einsum('...ij,...j->...i', Je, eta_dot)
           + np.einsum('...ij,...j->...i', Ja, adot))
    return np.concatenate([p_dot, eta_dot, v_dot, om_dot, adot, poc], axis=-1)


def jac17(x, u, p25, P: Params):
    """[df/dx, df/du] of f17 by the complex step, shape (..., 17, 23)."""
    x = np.asarray(x, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    z = np.concatenate([x, u], axis=-1)
    out = np.empty(x.shape[:-1] + (NX17, NX17 + NU17))
    for j in range(NX17 + NU17):
        zc = z.astype(np.complex128)
        zc[..., j] += 1j * EPS_CS
        out[..., :, j] = _f17c(zc[..., :NX17], zc[..., NX17:], p25, P).imag / EPS_CS
    return out


def rk4_sens17(x, u, p25, h, P: Params):
    """(x_next, A, B) of the RK4 map by the complex step (exact derivatives of the discrete map)."""
    x = np.asarray(x, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    z = np.concatenate([x, u], axis=-1)
    xn = rk4_step17(x, u, p25, h, P)
    S = np.empty(x.shape[:-1] + (NX17, NX17 + NU17))

    def rk4c(xc, uc):
        k1 = _f17c(xc, uc, p25, P)
        k2 = _f17c(xc + 0.5 * h * k1, uc, p25, P)
        k3 = _f17c(xc + 0.5 * h * k2, uc, p25, P)
        k4 = _f17c(xc + h * k3, uc, p25, P)
        return xc + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)

    for j in range(NX17 + NU17):
        zc = z.astype(np.complex128)
        zc[..., j] += 1j * EPS_CS
        S[..., :, j] = rk4c(zc[..., :NX17], zc[..., NX17:]).imag / EPS_CS
    return xn, S[..., :, :NX17], S[..., :, NX17:]


def mpc_solve17(x0, xref, uref, spec: FullSpec, p25=None, mode='rollout', xbar=None, ubar=None):
    """One SQP_RTI step of the 17/6 OCP for a batch: x0 (B,17), xref (B|1,N+1,17), uref (B|1,N,6),
    p25 (B|1,25) the same vector on every stage, or (B|1,N,25) stage by stage (acados
    ``set(k, 'p', p)``, simulation_blaster.py:65-69: stage k's vector enters interval k)."""
    x0 = np.asarray(x0, dtype=np.float64)
    Bsz, N = x0.shape[0], spec.N
    xref = np.broadcast_to(np.asarray(xref, dtype=np.float64), (Bsz, N + 1, NX17))
    uref = np.broadcast_to(np.asarray(uref, dtype=np.float64), (Bsz, N, NU17))
    p25 = default_p25() if p25 is None else np.asarray(p25, dtype=np.float64)
    pk = np.broadcast_to(p25[..., :N, :] if p25.ndim == 3 else p25[..., None, :], (Bsz, N, NP17))
    P = spec.params
    if mode == 'rollout':
        ubar = uref.copy()
        xbar = np.empty((Bsz, N + 1, NX17))
        xbar[:, 0] = x0
        for k in range(N):
            xbar[:, k + 1] = rk4_step17(xbar[:, k], ubar[:, k], pk[:, k], spec.dt, P)
    else:
        xbar = np.asarray(xbar, dtype=np.float64)
        ubar = np.asarray(ubar, dtype=np.float64)
    A = np.empty((Bsz, N, NX17, NX17))
    Bm = np.empty((Bsz, N, NX17, NU17))
    gap = np.empty((Bsz, N, NX17))
    for k in range(N):
        xn, A[:, k], Bm[:, k] = rk4_sens17(xbar[:, k], ubar[:, k], pk[:, k], spec.dt, P)
        gap[:, k] = xn - xbar[:, k + 1]
    if mode == 'rollout':
        gap[:] = 0.0   # the rollout is gap-free by construction
    dx0 = x0 - xbar[:, 0]
    if spec.boxed:   # interior point (the active set needs thousands of exchanges here)
        dx, du, status, iters = ipm_box_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec,
                                              max_iter=spec.max_as_iter, lbx=spec.lbx, ubx=spec.ubx)
    else:
        dx, du, _, ok = riccati_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec)
        status = np.where(ok, STATUS_OK, STATUS_QP_FAIL).astype(np.int32)
        iters = np.zeros(Bsz, dtype=np.int32)
    X = xbar + dx
    U = ubar + du
    bad = ~(np.isfinite(X).all(axis=(1, 2)) & np.isfinite(U).all(axis=(1, 2)))
    status = np.where(bad, STATUS_NAN, status).astype(np.int32)
    return dict(u0=U[:, 0].copy(), X=X, U=U, status=status, iters=iters, xbar=xbar, ubar=ubar,
                A=A, B=Bm, gap=gap)


def sensitivity17(o, x0, xref, uref, spec: FullSpec, rel: float, trials: int = 1, seed: int = 0):
    """How far the exact boxed minimiser of the 17/6 OCP moves when its linearisation [A|B] (of
    ``o`` = mpc_solve17(...)) carries relative noise ``rel`` (2^-45: a few fp64 ulp; 2^-22: fp32):
    re-solved by the same interior point + polish, per instance the largest normwise move of U and
    of u0 (oracle.ocp.fp32_sensitivity's 17/6 counterpart; test infrastructure only).  An instance
    that moves by more than a parity bound under noise its arithmetic carries anyway is degenerate
    for that bound (a flat direction of a strongly constrained QP): tests/test_gpu_fuzz17.py counts
    such instances and holds them to the optimal objective."""
    x0 = np.asarray(x0, dtype=np.float64)
    Bsz, N = x0.shape[0], spec.N
    xr = np.broadcast_to(np.asarray(xref, dtype=np.float64), (Bsz, N + 1, NX17))
    ur = np.broadcast_to(np.asarray(uref, dtype=np.float64), (Bsz, N, NU17))
    rs = np.random.default_rng(seed)
    den = np.maximum(np.abs(o['U']).reshape(Bsz, -1).max(axis=1), 1.0)
    den0 = np.maximum(np.abs(o['u0']).max(axis=1), 1.0)
    worst = np.zeros(Bsz)
    for _ in range(trials):
        A = o['A'] * (1.0 + rel * rs.standard_normal(o['A'].shape))
        Bm = o['B'] * (1.0 + rel * rs.standard_normal(o['B'].shape))
        with np.errstate(all='ignore'):
            _, du, st, _ = ipm_box_solve(A, Bm, o['gap'], x0 - o['xbar'][:, 0], o['xbar'], o['ubar'], xr, ur, spec,
                                         max_iter=spec.max_as_iter, lbx=spec.lbx, ubx=spec.ubx)
        U = o['ubar'] + du
        mv = np.maximum(np.abs(U - o['U']).reshape(Bsz, -1).max(axis=1) / den,
                        np.abs(U[:, 0] - o['u0']).max(axis=1) / den0)
        worst = np.maximum(worst, np.where(st == STATUS_OK, mv, np.inf))
    return worst

