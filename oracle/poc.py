"""Point-of-contact (POC) Jacobian solver restated in NumPy fp64 (oracle; test infrastructure only).

SURVEY §8 row f3.  Follows ``/root/reference/src/scripts/Jacobian_POC_Solver.py`` and
``htm.py``:

* stream model ``:62-83``: x = (p, v), p_dot = v, v_dot = -M_c v + g, g = (0, 0, -9.81),
  integrated by acados ERK with 4 stages and 10 steps over the horizon T (``:89-92``);
  [acados sim_erk: classic RK4, 10 equal steps — third-party, unpinned beyond that];
* initial condition ``setInitConditions`` ``:153-163``: T = T_w_b(phi, theta, psi, position)
  @ T_b_s2(alpha1, alpha2) (``htm.py:7-36``), p0 = T[:3, 3], v0 = T[:3, :3] @ (0, 0, -V);
  T_w_b uses SciPy's ``Rotation.from_euler('zyx', [psi, theta, phi])`` (extrinsic: Rx Ry Rz),
  called here exactly as the reference calls it;
* ground-hit time ``_solveRootFindingProblem`` ``:116-138``: Newton on z(T) with a forward-
  difference derivative (dT = 1e-5, ``:140-151``) from T = 0.1 until |z| <= 1e-3, negative
  iterates reflected;
* POC = p(T) and forward-difference Jacobians (eps = 1e-6, ``:222-296``) w.r.t. the Euler
  angles (3), the nozzle angles (2) and the position (3): one root solve per perturbation.

Reference quirk kept visible, not reproduced: with a NumPy ``position`` argument the in-place
``position += eps`` (``:286``) also moves ``self._positions``, so the position perturbations
accumulate; with the list the reference's ``__main__`` passes (``:305``) they do not.  This
restatement perturbs one coordinate at a time (the list behaviour).

Parity: the reference's own path needs acados (absent); there are no reference vectors for it.
Pinned pieces: the rotation (the reference's SciPy call itself), the RK4 integrator against the
closed-form solution of the linear stream ODE.  The rest is parity unpinned.
"""
from __future__ import annotations

import numpy as np
from scipy.spatial.transform import Rotation

G = np.array([0.0, 0.0, -9.81])   # Jacobian_POC_Solver.py:68
EPS_FD = 1e-6                      # :37
DT_NEWTON = 1e-5                   # :145
TOL_ROOT = 1e-3                    # :129
T0_ROOT = 0.1                      # :229
NSTEPS = 10                        # :92


def T_b_s2(a1, a2):
    """htm.py:7-28 (body -> nozzle), batched over a1, a2 (shape [B])."""
    a1 = np.asarray(a1, dtype=np.float64)
    a2 = np.asarray(a2, dtype=np.float64)
    B = a1.shape[0]
    h1 = np.broadcast_to(np.array([[1, 0, 0, 0.01672], [0, 1, 0, 0], [0, 0, 1, -0.22937], [0, 0, 0, 1.0]]),
                         (B, 4, 4))
    c1, s1, c2, s2 = np.cos(a1), np.sin(a1), np.cos(a2), np.sin(a2)
    z, o = np.zeros(B), np.ones(B)
    h2 = np.stack([np.stack([c1, z, s1, 0.0425 * o], -1), np.stack([z, o, z, z], -1),
                   np.stack([-s1, z, c1, z], -1), np.stack([z, z, z, o], -1)], -2)
    h3 = np.stack([np.stack([o, z, z, -0.05322 * o], -1), np.stack([z, c2, s2, z], -1),
                   np.stack([z, -s2, c2, -0.15946 * o], -1), np.stack([z, z, z, o], -1)], -2)
    return h1 @ h2 @ h3


def T_w_b(phi, theta, psi, position):
    """htm.py:30-36 (world <- body), the reference's SciPy call."""
    B = np.shape(phi)[0]
    T = np.broadcast_to(np.eye(4), (B, 4, 4)).copy()
    T[:, :3, :3] = Rotation.from_euler('zyx', np.stack([psi, theta, phi], -1)).as_matrix()
    T[:, :3, 3] = position
    return T


def init_conditions(euler, motor, position, stream_velocity):
    """setInitConditions (Jacobian_POC_Solver.py:153-163): (p0, v0) of the stream, [B, 6]."""
    euler = np.asarray(euler, dtype=np.float64)
    motor = np.asarray(motor, dtype=np.float64)
    position = np.asarray(position, dtype=np.float64)
    T = T_w_b(euler[:, 0], euler[:, 1], euler[:, 2], position) @ T_b_s2(motor[:, 0], motor[:, 1])
    v = np.array([0.0, 0.0, -float(stream_velocity)])
    return np.concatenate([T[:, :3, 3], T[:, :3, :3] @ v], axis=-1)


def integrate(x0, T, Mc):
    """ERK4, 10 steps over [0, T] (per-instance T), of p_dot = v, v_dot = -Mc v + g."""
    x = np.asarray(x0, dtype=np.float64).copy()
    Mc = np.asarray(Mc, dtype=np.float64)
    h = (np.asarray(T, dtype=np.float64) / NSTEPS)[:, None]

    def f(s):
        v = s[:, 3:]
        vd = -(v @ Mc.T if Mc.ndim == 2 else Mc * v) + G
        return np.concatenate([v, vd], axis=-1)

    for _ in range(NSTEPS):
        k1 = f(x)
        k2 = f(x + 0.5 * h * k1)
        k3 = f(x + 0.5 * h * k2)
        k4 = f(x + h * k3)
        x = x + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
    return x


def root_time(x0, Mc, max_iter=100):
    """_solveRootFindingProblem / _rootFindingStep (Jacobian_POC_Solver.py:116-151), batched.
    Returns (T [B], iterations [B], converged [B])."""
    B = x0.shape[0]
    TN = np.full(B, T0_ROOT)
    err = np.full(B, 100.0)
    it = np.zeros(B, dtype=np.int32)
    act = np.ones(B, dtype=bool)
    for _ in range(max_iter):
        act = np.abs(err) > TOL_ROOT
        if not act.any():
            break
        f = integrate(x0, TN, Mc)[:, 2]
        fp = (integrate(x0, TN + DT_NEWTON, Mc)[:, 2] - f) / DT_NEWTON
        TN1 = TN - f / fp
        TN1 = np.where(TN1 < 0, -TN1, TN1)
        e1 = integrate(x0, TN1, Mc)[:, 2]
        TN = np.where(act, TN1, TN)
        err = np.where(act, e1, err)
        it += act
    return TN, it, np.abs(err) <= TOL_ROOT


def solve_jacobians(euler, motor, position, stream_velocity, Mc, max_iter=100):
    """solveJacobians (Jacobian_POC_Solver.py:222-296) for a batch: POC [B,3], J_eul [B,3,3],
    J_mot [B,3,2], J_pos [B,3,3], converged [B]."""
    euler = np.asarray(euler, dtype=np.float64)
    motor = np.asarray(motor, dtype=np.float64)
    position = np.asarray(position, dtype=np.float64)
    B = euler.shape[0]

    def poc(e, m, p):
        x0 = init_conditions(e, m, p, stream_velocity)
        T, _, ok = root_time(x0, Mc, max_iter)
        return integrate(x0, T, Mc)[:, :3], ok

    P0, ok = poc(euler, motor, position)
    Je = np.empty((B, 3, 3))
    Jm = np.empty((B, 3, 2))
    Jp = np.empty((B, 3, 3))
    for i in range(3):
        e = euler.copy()
        e[:, i] = e[:, i] + EPS_FD
        Pp, o = poc(e, motor, position)
        Je[:, :, i] = (Pp - P0) / EPS_FD
        ok &= o
    for i in range(2):
        m = motor.copy()
        m[:, i] = m[:, i] + EPS_FD
        Pp, o = poc(euler, m, position)
        Jm[:, :, i] = (Pp - P0) / EPS_FD
        ok &= o
    for i in range(3):
        p = position.copy()
        p[:, i] = p[:, i] + EPS_FD
        Pp, o = poc(euler, motor, p)
        Jp[:, :, i] = (Pp - P0) / EPS_FD
        ok &= o
    return P0, Je, Jm, Jp, ok


def params25(J_mot, J_eul, J_pos, t_blast):
    """The model parameter vector (blastermodel.py:203-210): column-major vec of J_angles (3x2),
    J_euler (3x3), J_p (3x3), then T_blast."""
    B = J_mot.shape[0]
    return np.concatenate([np.swapaxes(J_mot, 1, 2).reshape(B, 6), np.swapaxes(J_eul, 1, 2).reshape(B, 9),
                           np.swapaxes(J_pos, 1, 2).reshape(B, 9), np.full((B, 1), float(t_blast))], axis=1)
