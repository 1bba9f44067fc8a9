"""BLASTER dynamics restated in NumPy fp64 (oracle; test infrastructure only).

Follows ``/root/reference/src/scripts/blastermodel.py``:

* moments (mixer)            ``:95-101``
* R = R_psi @ R_theta @ R_phi ``:103-122`` (ZYX intrinsic, body -> world, ENU, gravity -z ``:93``)
* Euler-rate map W            ``:128-141``; euler_dot = inv(W) @ omega ``:162``
* swivel rotation R_gimbal    ``:143-160`` (Ry(alpha1) @ Rx(alpha2))
* v_dot / omega_dot / poc_dot ``:163-165``; state/input/param layout ``:171-210``.

Two models:

* ``f17``: the full 17-state / 6-input / 25-parameter reference model.
* ``f12``: its exact rigid-body slice (x[0:12], u[0:4], alpha == 0 so R_gimbal = I), the model
  of the BASELINE configs.  Optional world-frame wind force (c5 extension, not in the
  reference) adds ``wind / mass`` to v_dot.

Everything is vectorised over a leading batch axis.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

GRAVITY = 9.81  # blastermodel.py:93


@dataclass
class Params:
    """Physical constants (``blasterModel.__init__`` args, blastermodel.py:16-45)."""

    mass: float = 9.0
    J: np.ndarray = field(default_factory=lambda: np.diag([0.50781, 0.47314, 0.72975]))
    lx: float = 0.3434
    ly: float = 0.3475
    c: float = 0.03
    g: float = GRAVITY
    t_blast: float = 0.0  # T_blast parameter p[24] (0 for the 12/4 quad configs)

    @property
    def Jinv(self) -> np.ndarray:
        return np.linalg.inv(np.asarray(self.J, dtype=np.float64))


def moments(T: np.ndarray, P: Params) -> np.ndarray:
    """Body moments from the 4 motor thrusts (blastermodel.py:95-101)."""
    T0, T1, T2, T3 = T[..., 0], T[..., 1], T[..., 2], T[..., 3]
    return np.stack([
        (T1 + T3 - T0 - T2) * P.ly,
        (-T0 - T3 + T1 + T2) * P.lx,
        (-T0 - T1 + T2 + T3) * P.c,
    ], axis=-1)


def rot_zyx(phi, theta, psi) -> np.ndarray:
    """R = Rz(psi) @ Ry(theta) @ Rx(phi) (blastermodel.py:103-122). Shape (..., 3, 3)."""
    cf, sf = np.cos(phi), np.sin(phi)
    ct, st = np.cos(theta), np.sin(theta)
    cp, sp = np.cos(psi), np.sin(psi)
    R = np.empty(np.shape(phi) + (3, 3), dtype=np.result_type(phi, theta, psi, 1.0))
    R[..., 0, 0] = cp * ct
    R[..., 0, 1] = cp * st * sf - sp * cf
    R[..., 0, 2] = cp * st * cf + sp * sf
    R[..., 1, 0] = sp * ct
    R[..., 1, 1] = sp * st * sf + cp * cf
    R[..., 1, 2] = sp * st * cf - cp * sf
    R[..., 2, 0] = -st
    R[..., 2, 1] = ct * sf
    R[..., 2, 2] = ct * cf
    return R


def euler_rate_inv(phi, theta) -> np.ndarray:
    """Closed-form inverse of R_to_omega (blastermodel.py:135-140); det = cos(theta)."""
    cf, sf = np.cos(phi), np.sin(phi)
    ct, st = np.cos(theta), np.sin(theta)
    tt = st / ct
    Wi = np.zeros(np.shape(phi) + (3, 3), dtype=np.result_type(phi, theta, 1.0))
    Wi[..., 0, 0] = 1.0
    Wi[..., 0, 1] = sf * tt
    Wi[..., 0, 2] = cf * tt
    Wi[..., 1, 1] = cf
    Wi[..., 1, 2] = -sf
    Wi[..., 2, 1] = sf / ct
    Wi[..., 2, 2] = cf / ct
    return Wi


def _rb_core(x, T, P: Params, thrust_extra_body=None, wind=None):
    """Shared rigid-body part: returns (p_dot, eta_dot, v_dot, omega_dot)."""
    phi, theta, psi = x[..., 3], x[..., 4], x[..., 5]
    v = x[..., 6:9]
    om = x[..., 9:12]
    R = rot_zyx(phi, theta, psi)
    Wi = euler_rate_inv(phi, theta)
    eta_dot = np.einsum('...ij,...j->...i', Wi, om)
    Tsum = T.sum(axis=-1)
    fb = np.zeros(np.shape(Tsum) + (3,), dtype=np.result_type(Tsum, x, 1.0))
    fb[..., 2] = Tsum
    if thrust_extra_body is not None:
        fb = fb + thrust_extra_body
    v_dot = np.einsum('...ij,...j->...i', R, fb) / P.mass
    v_dot[..., 2] -= P.g
    if wind is not None:
        v_dot = v_dot + np.asarray(wind) / P.mass
    J = np.asarray(P.J, dtype=np.float64)
    Jw = np.einsum('ij,...j->...i', J, om)
    om_dot = np.einsum('ij,...j->...i', P.Jinv, moments(T, P) - np.cross(om, Jw))
    return v, eta_dot, v_dot, om_dot


def f12(x: np.ndarray, u: np.ndarray, P: Params, wind=None) -> np.ndarray:
    """12-state/4-input slice of f_expl_expr (blastermodel.py:191-201 with alpha = 0)."""
    x = np.asarray(x, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    extra = None
    if P.t_blast != 0.0:
        extra = np.zeros(x.shape[:-1] + (3,))
        extra[..., 2] = P.t_blast  # R_gimbal = I at alpha = 0
    p_dot, eta_dot, v_dot, om_dot = _rb_core(x, u[..., 0:4], P, extra, wind)
    return np.concatenate([p_dot, eta_dot, v_dot, om_dot], axis=-1)


def unpack_params25(p25: np.ndarray):
    """Column-major vec of J_angles(3x2), J_euler(3x3), J_p(3x3), then T_blast (blastermodel.py:203-210)."""
    p25 = np.asarray(p25, dtype=np.float64)
    Ja = np.swapaxes(p25[..., 0:6].reshape(p25.shape[:-1] + (2, 3)), -1, -2)
    Je = np.swapaxes(p25[..., 6:15].reshape(p25.shape[:-1] + (3, 3)), -1, -2)
    Jp = np.swapaxes(p25[..., 15:24].reshape(p25.shape[:-1] + (3, 3)), -1, -2)
    return Ja, Je, Jp, p25[..., 24]


def f17(x: np.ndarray, u: np.ndarray, p25: np.ndarray, P: Params) -> np.ndarray:
    """Full 17-state/6-input reference model f_expl_expr (blastermodel.py:95-201)."""
    x = np.asarray(x, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    Ja, Je, Jp, tb = unpack_params25(p25)
    a1, a2 = x[..., 12], x[..., 13]
    # R_gimbal = Ry(alpha1) @ Rx(alpha2) (blastermodel.py:148-160); only its 3rd column matters.
    c1, s1 = np.cos(a1), np.sin(a1)
    c2, s2 = np.cos(a2), np.sin(a2)
    g3 = np.stack([s1 * c2, -s2, c1 * c2], axis=-1)  # Ry(a1) @ Rx(a2) @ e3
    extra = g3 * np.asarray(tb)[..., None]
    p_dot, eta_dot, v_dot, om_dot = _rb_core(x, u[..., 0:4], P, extra)
    adot = u[..., 4:6]
    poc_dot = (np.einsum('...ij,...j->...i', Jp, x[..., 6:9])
               + np.einsum('...ij,...j->...i', Je, eta_dot)
               + np.einsum('...ij,...j->...i', Ja, adot))
    return np.concatenate([p_dot, eta_dot, v_dot, om_dot, adot, poc_dot], axis=-1)


def jac12(x: np.ndarray, u: np.ndarray, P: Params, wind=None) -> np.ndarray:
    """Analytic Jacobian [df/dx, df/du] of ``f12`` — shape (..., 12, 16)."""
    x = np.asarray(x, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    bs = x.shape[:-1]
    Jf = np.zeros(bs + (12, 16))
    phi, theta, psi = x[..., 3], x[..., 4], x[..., 5]
    om = x[..., 9:12]
    wx, wy, wz = om[..., 0], om[..., 1], om[..., 2]
    cf, sf = np.cos(phi), np.sin(phi)
    ct, st = np.cos(theta), np.sin(theta)
    cp, sp = np.cos(psi), np.sin(psi)
    tt = st / ct
    sec = 1.0 / ct
    # p_dot = v
    for i in range(3):
        Jf[..., i, 6 + i] = 1.0
    # eta_dot = Wi(phi, theta) @ omega
    Jf[..., 3:6, 9:12] = euler_rate_inv(phi, theta)
    a = sf * wy + cf * wz           # appears in rows 3 and 5
    b = cf * wy - sf * wz           # d a / d phi
    Jf[..., 3, 3] = tt * b
    Jf[..., 4, 3] = -sf * wy - cf * wz
    Jf[..., 5, 3] = b * sec
    Jf[..., 3, 4] = a * sec * sec
    Jf[..., 5, 4] = a * st * sec * sec
    # v_dot = R e3 * Ttot / m + g
    Ttot = u[..., 0:4].sum(axis=-1) + P.t_blast
    s = Ttot / P.mass
    re3 = np.stack([cp * cf * st + sp * sf, sp * cf * st - cp * sf, cf * ct], axis=-1)
    d_phi = np.stack([-cp * sf * st + sp * cf, -sp * sf * st - cp * cf, -sf * ct], axis=-1)
    d_th = np.stack([cp * cf * ct, sp * cf * ct, -cf * st], axis=-1)
    d_psi = np.stack([-sp * cf * st + cp * sf, cp * cf * st + sp * sf, np.zeros_like(phi)], axis=-1)
    Jf[..., 6:9, 3] = d_phi * s[..., None]
    Jf[..., 6:9, 4] = d_th * s[..., None]
    Jf[..., 6:9, 5] = d_psi * s[..., None]
    for m in range(4):
        Jf[..., 6:9, 12 + m] = re3 / P.mass
    # omega_dot = Jinv (M(T) - omega x J omega)
    J = np.asarray(P.J, dtype=np.float64)
    Jinv = P.Jinv
    Jw = np.einsum('ij,...j->...i', J, om)

    def skew(w):
        S = np.zeros(w.shape[:-1] + (3, 3))
        S[..., 0, 1] = -w[..., 2]
        S[..., 0, 2] = w[..., 1]
        S[..., 1, 0] = w[..., 2]
        S[..., 1, 2] = -w[..., 0]
        S[..., 2, 0] = -w[..., 1]
        S[..., 2, 1] = w[..., 0]
        return S

    dcross = np.einsum('...ij,jk->...ik', skew(om), J) - skew(Jw)  # d(w x Jw)/dw
    Jf[..., 9:12, 9:12] = -np.einsum('ij,...jk->...ik', Jinv, dcross)
    dM = np.array([[-P.ly, P.ly, -P.ly, P.ly],
                   [-P.lx, P.lx, P.lx, -P.lx],
                   [-P.c, -P.c, P.c, P.c]])
    Jf[..., 9:12, 12:16] = Jinv @ dM
    return Jf
