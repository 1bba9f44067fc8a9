"""acados OCP JSON -> MPCConfig.

Reads the ``acados_ocp_<model>.json`` that the reference's ``AcadosOcpSolver(ocp, json_file=...)``
writes (src/scripts/acados_ocp_blasterModel.json, produced by blastermodel.py:289) and maps the
parts this build implements onto ``MPCConfig``:

* dims ``nx``/``nu``/``N``/``np`` (17/6/25 for the full model; ``slice_12_4=True`` cuts the
  rigid-body slice of the BASELINE configs out of a 17/6 description);
* LINEAR_LS cost with selector ``Vx``/``Vu`` (blastermodel.py:228-257): Q = W[:nx,:nx],
  R = W[nx:,nx:], Q_N = W_e; stage scaling = ``time_steps`` (acados' convention, uniform dt);
* input box ``idxbu``/``lbu``/``ubu`` (blastermodel.py:259-264), on both models (every input
  boxed, as the reference sets it; a partial idxbu raises);
* ``qp_solver_iter_max`` (500 in the reference JSON) as the QP iteration cap;
* ``parameter_values`` (the default p, T_blast at p[24]);
* ERK, 4 stages, 1 step, Gauss-Newton SQP_RTI with a full step (the only integrator / NLP
  configuration the device implements; anything else raises).

The physical constants (mass, J, l_x, l_y, c) are baked into the CasADi expressions, not the
JSON: they are keyword arguments with the reference's defaults (simulation_blaster.py:12-21).
The state box (``idxbx``/``lbx``/``ubx``, stages 1..N-1) is applied on the 17/6 model when it covers
every state (the reference's idxbx = range(nx)); otherwise, and on the 12/4 slice, it is returned
in ``info`` and reported as not applied.
"""
from __future__ import annotations

import json
import warnings

import numpy as np

from .config import NU, NU17, NX, NX17, MPCConfig


def _get(d, *path, default=None):
    for k in path:
        if not isinstance(d, dict) or k not in d:
            return default
        d = d[k]
    return d


def load_acados_ocp_json(src, slice_12_4: bool = False, dtype: str = 'f64', **physical):
    """Returns (MPCConfig, info) for a JSON path or an already-parsed dict.

    info: yref [ny] and yref_e [ny_e] (the JSON's stage / terminal references), p [np],
    idxbx / lbx / ubx (as in the JSON), and ``dropped`` (what was not mapped)."""
    d = json.load(open(src)) if isinstance(src, str) else src
    dims = d['dims']
    nx, nu, N = int(dims['nx']), int(dims['nu']), int(dims['N'])
    if (nx, nu) not in ((NX17, NU17), (NX, NU)):
        raise ValueError(f'nx/nu {nx}/{nu}: the BLASTER models are 17/6 and 12/4')
    so = d['solver_options']
    checks = {
        'integrator_type': ('ERK',),
        'nlp_solver_type': ('SQP_RTI',),
        'hessian_approx': ('GAUSS_NEWTON',),
        'globalization': ('FIXED_STEP',),
    }
    for key, ok in checks.items():
        if key in so and so[key] not in ok:
            raise ValueError(f'solver_options.{key} = {so[key]!r}: implemented {ok}')
    for key in ('sim_method_num_stages', 'sim_method_num_steps'):
        v = np.atleast_1d(so.get(key, 4 if 'stages' in key else 1))
        if not np.all(v == (4 if 'stages' in key else 1)):
            raise ValueError(f'solver_options.{key}: the device integrates classic RK4, 1 step')
    if float(so.get('nlp_solver_step_length', 1.0)) != 1.0:
        raise ValueError('nlp_solver_step_length must be 1.0 (full step)')
    ts = np.asarray(so.get('time_steps', [float(so['tf']) / N] * N), dtype=np.float64)
    if not np.allclose(ts, ts[0], rtol=1e-12, atol=0):
        raise ValueError('non-uniform time_steps are not implemented')
    dt = float(ts[0])

    cost = d.get('cost', d)
    if cost.get('cost_type', 'LINEAR_LS') != 'LINEAR_LS' or cost.get('cost_type_e', 'LINEAR_LS') != 'LINEAR_LS':
        raise ValueError('only LINEAR_LS costs are implemented')
    W = np.asarray(cost['W'], dtype=np.float64)
    We = np.asarray(cost['W_e'], dtype=np.float64)
    ny = nx + nu
    Vx = np.asarray(cost.get('Vx', np.eye(ny, nx)), dtype=np.float64)
    Vu = np.asarray(cost.get('Vu', np.eye(ny, nu, -nx)), dtype=np.float64)
    if W.shape != (ny, ny) or not (np.array_equal(Vx, np.eye(ny, nx)) and np.array_equal(Vu, np.eye(ny, nu, -nx))):
        raise ValueError('the cost must select y = [x; u] (Vx, Vu selectors, blastermodel.py:247-254)')
    Q, R = W[:nx, :nx], W[nx:, nx:]
    if np.abs(W[:nx, nx:]).max(initial=0.0) > 0:
        raise ValueError('cross weights between x and u are not implemented')

    con = d.get('constraints', d)
    lbu = ubu = None
    idxbu = list(np.atleast_1d(con.get('idxbu', [])).astype(int))
    if idxbu:
        # the device's input box covers every input (the reference's idxbu = range(nu),
        # blastermodel.py:261): a partial box would need +-1e20 rows that the interior point
        # would treat as real constraints (a 1e20 slack dominates its duality measure)
        if sorted(idxbu) != list(range(nu)):
            raise ValueError(f'idxbu {idxbu}: the device implements a box on every input (range({nu}))')
        lbu = np.empty(nu)
        ubu = np.empty(nu)
        lbu[idxbu] = np.asarray(con['lbu'], dtype=np.float64)
        ubu[idxbu] = np.asarray(con['ubu'], dtype=np.float64)
    p = np.asarray(d.get('parameter_values', np.zeros(int(dims.get('np', 0)))), dtype=np.float64)
    t_blast = float(p[24]) if p.size >= 25 else 0.0
    dropped = []
    idxbx = list(np.atleast_1d(con.get('idxbx', [])).astype(int))
    lbx = ubx = None
    if idxbx:
        # the device's state box covers every state (the reference sets idxbx = range(nx),
        # blastermodel.py:268) of the 17/6 model, together with the input box
        if (not slice_12_4 and nx == NX17 and sorted(idxbx) == list(range(nx)) and lbu is not None
                and np.isfinite(con['lbx']).all() and np.isfinite(con['ubx']).all()):
            lbx = np.empty(nx)
            ubx = np.empty(nx)
            lbx[idxbx] = np.asarray(con['lbx'], dtype=np.float64)
            ubx[idxbx] = np.asarray(con['ubx'], dtype=np.float64)
        else:
            dropped.append('state box idxbx (stages 1..N-1)')

    if slice_12_4 and nx == NX17:
        Q, R, We = Q[:NX, :NX], R[:NU, :NU], We[:NX, :NX]
        if lbu is not None:
            lbu, ubu = lbu[:NU], ubu[:NU]
        nx, nu = NX, NU
        dropped.append('alpha / POC states and swivel inputs (12/4 slice)')
    phys = dict(mass=9.0, J=np.diag([0.50781, 0.47314, 0.72975]), lx=0.3434, ly=0.3475, c=0.03)
    phys.update(physical)
    # HPIPM's iteration cap (JSON solver_options.qp_solver_iter_max, blastermodel.py:279) caps the
    # device's active-set / interior-point iterations
    max_it = int(so.get('qp_solver_iter_max', 200))
    cfg = MPCConfig(N=N, dt=dt, dtype=dtype, Q=Q, R=R, QN=We, cost_scale=dt, lbu=lbu, ubu=ubu,
                    lbx=lbx, ubx=ubx, t_blast=t_blast, nx=nx, nu=nu, max_as_iter=max_it, **phys)
    for what in dropped:
        warnings.warn(f'acados JSON: {what} not applied by the device path', stacklevel=2)
    info = dict(yref=np.asarray(cost.get('yref', np.zeros(ny)), dtype=np.float64),
                yref_e=np.asarray(cost.get('yref_e', np.zeros(nx)), dtype=np.float64),
                p=p, idxbx=idxbx, lbx=np.asarray(con.get('lbx', []), dtype=np.float64),
                ubx=np.asarray(con.get('ubx', []), dtype=np.float64), dropped=dropped)
    return cfg, info
