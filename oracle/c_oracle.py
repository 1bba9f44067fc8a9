"""ctypes wrapper of oracle/c/libmpc_oracle.so (test infrastructure / CPU baseline only)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from .ocp import OcpSpec

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get('MPCB_ORACLE_LIB') or os.path.join(_HERE, 'c', 'libmpc_oracle.so')


class _Params(ctypes.Structure):
    _fields_ = [('minv', ctypes.c_double), ('g', ctypes.c_double), ('t_blast', ctypes.c_double),
                ('lx', ctypes.c_double), ('ly', ctypes.c_double), ('c', ctypes.c_double),
                ('J', ctypes.c_double * 9), ('Jinv', ctypes.c_double * 9),
                ('Q', ctypes.c_double * 144), ('R', ctypes.c_double * 16), ('QN', ctypes.c_double * 144),
                ('dt', ctypes.c_double), ('s', ctypes.c_double)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(['make', '-s', '-C', os.path.dirname(LIB)])
        _lib = ctypes.CDLL(LIB)
        _lib.mpc_oracle_solve.restype = ctypes.c_int
    return _lib


def _params(spec: OcpSpec) -> _Params:
    P = spec.params
    p = _Params()
    p.minv, p.g, p.t_blast, p.lx, p.ly, p.c = 1.0 / P.mass, P.g, P.t_blast, P.lx, P.ly, P.c
    J = np.asarray(P.J, dtype=np.float64)
    for i, v in enumerate(J.reshape(-1)):
        p.J[i] = v
    for i, v in enumerate(np.linalg.inv(J).reshape(-1)):
        p.Jinv[i] = v
    for i, v in enumerate(np.asarray(spec.Q, dtype=np.float64).reshape(-1)):
        p.Q[i] = v
    for i, v in enumerate(np.asarray(spec.R, dtype=np.float64).reshape(-1)):
        p.R[i] = v
    for i, v in enumerate(np.asarray(spec.QN, dtype=np.float64).reshape(-1)):
        p.QN[i] = v
    p.dt, p.s = spec.dt, spec.s
    return p


def solve(x0, xref, uref, spec: OcpSpec, nthreads: int = 1, want_traj: bool = True, wind=None):
    """Rollout-mode SQP_RTI step (same algorithm as oracle.ocp.mpc_solve): unconstrained, or with
    the input box by the primal-dual active set of oracle.ocp.pdas_solve (then ``iters`` too)."""
    lib = load()
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    B, N = x0.shape[0], spec.N
    xr = np.ascontiguousarray(xref, dtype=np.float64)
    ur = np.ascontiguousarray(uref, dtype=np.float64)
    xr_sb = 0 if xr.shape[0] == 1 else (N + 1) * 12
    ur_sb = 0 if ur.shape[0] == 1 else N * 4
    u0 = np.empty((B, 4))
    X = np.empty((B, N + 1, 12)) if want_traj else None
    U = np.empty((B, N, 4)) if want_traj else None
    st = np.empty(B, dtype=np.int32)
    P = _params(spec)
    dp = ctypes.POINTER(ctypes.c_double)
    ptr = lambda a: a.ctypes.data_as(dp) if a is not None else None  # noqa: E731
    ip = ctypes.POINTER(ctypes.c_int)
    if spec.boxed:
        lb = np.ascontiguousarray(np.broadcast_to(np.asarray(spec.lbu, dtype=np.float64), (4,)))
        ub = np.ascontiguousarray(np.broadcast_to(np.asarray(spec.ubu, dtype=np.float64), (4,)))
        it = np.empty(B, dtype=np.int32)
        lib.mpc_oracle_solve_box(ctypes.c_int(B), ctypes.c_int(N), ctypes.byref(P), ptr(lb), ptr(ub),
                                 ctypes.c_int(spec.max_as_iter), ptr(x0), ptr(xr), ctypes.c_long(xr_sb), ptr(ur),
                                 ctypes.c_long(ur_sb), ptr(u0), ptr(X), ptr(U), st.ctypes.data_as(ip),
                                 it.ctypes.data_as(ip), ctypes.c_int(nthreads))
        return dict(u0=u0, X=X, U=U, status=st, iters=it)
    if wind is not None and spec.boxed:
        raise NotImplementedError('wind with the input box')
    wd = None if wind is None else np.ascontiguousarray(np.broadcast_to(wind, (B, 3)), dtype=np.float64)
    lib.mpc_oracle_solve(ctypes.c_int(B), ctypes.c_int(N), ctypes.byref(P), ptr(x0), ptr(xr),
                         ctypes.c_long(xr_sb), ptr(ur), ctypes.c_long(ur_sb), ptr(wd), ctypes.c_long(3),
                         ptr(u0), ptr(X), ptr(U),
                         st.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), ctypes.c_int(nthreads))
    return dict(u0=u0, X=X, U=U, status=st)


def latency_b1(x0, xref, uref, spec: OcpSpec, reps: int = 2000):
    """Per-instance solve latency of the plain-C port on the calling thread (c1 shape: one
    instance per call, as the reference's control loop simulation_blaster.py:56-107 solves it):
    ``reps`` single-instance solves cycling over the rows of ``x0`` (broadcast xref/uref), each
    timed inside C.  Returns the per-solve times in ms."""
    lib = load()
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    xr = np.ascontiguousarray(np.asarray(xref, dtype=np.float64)[:1])
    ur = np.ascontiguousarray(np.asarray(uref, dtype=np.float64)[:1])
    ns = np.empty(int(reps))
    P = _params(spec)
    dp = ctypes.POINTER(ctypes.c_double)
    bad = lib.mpc_oracle_latency_b1(ctypes.c_int(x0.shape[0]), ctypes.c_int(spec.N), ctypes.byref(P),
                                    x0.ctypes.data_as(dp), xr.ctypes.data_as(dp), ur.ctypes.data_as(dp),
                                    ctypes.c_int(int(reps)), ns.ctypes.data_as(dp))
    if bad:
        raise RuntimeError(f'{bad} failed solves in the latency sample')
    return ns * 1e-6
