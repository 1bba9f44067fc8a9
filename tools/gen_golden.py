#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.  BUILD-CONTAINER TOOL ONLY.

Reads /root/reference (present only in the build container, never on the GPU box) and
writes small data files; the reference itself never enters the repo.

1. ``dynamics_ref17.npz`` — the reference's own ``blasterModel.generateModel()``
   (``src/scripts/blastermodel.py:47-212``) is executed with ``tools/refstub`` first on
   ``sys.path`` (a sympy-backed stand-in for the CasADi SX subset it touches, and a
   capture-only ``acados_template``).  Its symbolic ``f_expl_expr`` is evaluated (values and
   exact Jacobians) at seeded random points and at hover, for two of the reference's
   parameter sets (``simulation_blaster.py:12-22`` and ``blastermodel.py:296-306``).
2. ``ocp_capture.json`` — the OCP that ``generateController()`` (``blastermodel.py:214-292``)
   builds: W, W_e, Vx, Vu, Vx_e, bounds, solver options, parameter values.
3. ``ocp_json_pin.json`` — the same fields read (``json.load``) from the reference's
   serialized ``acados_ocp_blasterModel.json``.
4. ``mathutils_ref.npz`` — ``utils/MathUtils.py`` quaternion helpers evaluated at random
   quaternions.
5. ``mpc_c1.npz`` / ``mpc_small.npz`` — oracle-generated MPC outputs for the c1 shape and small
   c2-c4 slices (these pin the device against the oracle, not against acados).

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = '/root/reference'
OUT = os.path.join(REPO, 'tests', 'golden')


def _ref_imports():
    sys.path.insert(0, os.path.join(REPO, 'tools', 'refstub'))
    sys.path.insert(1, REF)
    sys.path.insert(2, os.path.join(REF, 'src', 'scripts'))
    import sympy as sp  # noqa: F401
    import blastermodel  # the reference module, unmodified
    import acados_template
    from utils import MathUtils
    return blastermodel, acados_template, MathUtils


def _sim_params():
    """simulation_blaster.py:12-30 (the set the JSON freezes)."""
    J = np.eye(3)
    J[0, 0], J[1, 1], J[2, 2] = 0.50781, 0.47314, 0.72975
    Q = np.zeros((17, 17))
    np.fill_diagonal(Q, [1e3] * 6 + [0.5e1] * 3 + [1e1] * 3 + [1e-2] * 2 + [1e3] * 3)
    R = np.zeros((6, 6))
    np.fill_diagonal(R, [5e-2] * 4 + [1e-5] * 2)
    sb = np.array([[-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0,
                    -0.0872665, -0.0872665, -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5],
                   [1.5, 1.5, 5.0, 0.174532925, 0.174532925, 0.349066, 1.0, 1.0, 1.0, 0.0872665,
                    0.0872665, 0.0872665, 1.22173, 0.523599, 1.5, 1.5, 2.5]])
    cb = np.array([[0, 0, 0, 0, -0.0872665, -0.0872665], [65, 65, 65, 65, 0.0872665, 0.0872665]])
    return dict(mass=9.0, J=J, l_x=0.3434, l_y=0.3475, N=60, Tf=2.0, c=0.03, Q=Q, R=R,
                Q_t=10 * Q, blastThruster=2.2 * 9.81, statesBound=sb, controlBound=cb)


def _main_params():
    """blastermodel.py:296-314 (__main__ set: mass 10)."""
    d = _sim_params()
    d.update(mass=10.0, N=30, Tf=1.0, blastThruster=2.2)
    return d


def _build(blastermodel, kw):
    b = blastermodel.blasterModel(kw['mass'], kw['J'], kw['l_x'], kw['l_y'], kw['N'], kw['Tf'],
                                  kw['c'], kw['Q'], kw['R'], kw['Q_t'], kw['blastThruster'],
                                  kw['statesBound'], kw['controlBound'])
    b.generateModel()
    return b


def gen_dynamics(blastermodel, rng):
    import sympy as sp
    out = {}
    for tag, kw in (('sim', _sim_params()), ('main', _main_params())):
        b = _build(blastermodel, kw)
        m = b._model
        xs = list(m.x.M)
        us = list(m.u.M)
        ps = list(m.p.M)
        f = m.f_expl_expr.M
        fx = f.jacobian(sp.Matrix(xs))
        fu = f.jacobian(sp.Matrix(us))
        lf = sp.lambdify([xs, us, ps], f, 'numpy')
        lfx = sp.lambdify([xs, us, ps], fx, 'numpy')
        lfu = sp.lambdify([xs, us, ps], fu, 'numpy')
        n = 64
        X = np.zeros((n + 1, 17))
        U = np.zeros((n + 1, 6))
        Pp = np.zeros((n + 1, 25))
        # row 0: hover (simulation_blaster.py:97 thrust 22.0725 N/motor), alpha = 0, T_blast = 0
        X[0, 2] = 3.5
        U[0, :4] = kw['mass'] * 9.81 / 4.0
        X[1:, 0:3] = rng.uniform(-1.5, 1.5, (n, 3))
        X[1:, 3:5] = rng.uniform(-0.6, 0.6, (n, 2))
        X[1:, 5] = rng.uniform(-np.pi, np.pi, n)
        X[1:, 6:12] = rng.uniform(-1.0, 1.0, (n, 6))
        X[1:, 12:14] = rng.uniform(-0.5, 0.5, (n, 2))
        X[1:, 14:17] = rng.uniform(-2.0, 2.0, (n, 3))
        U[1:, :4] = rng.uniform(0.0, 65.0, (n, 4))
        U[1:, 4:6] = rng.uniform(-0.0872665, 0.0872665, (n, 2))
        Pp[1:, :24] = rng.uniform(-1.0, 1.0, (n, 24))
        Pp[1:, 24] = rng.uniform(0.0, 25.0, n)
        Pp[1::4, 24] = 0.0
        F = np.array([np.asarray(lf(X[i], U[i], Pp[i]), dtype=float).reshape(-1) for i in range(n + 1)])
        FX = np.array([np.asarray(lfx(X[i], U[i], Pp[i]), dtype=float) for i in range(n + 1)])
        FU = np.array([np.asarray(lfu(X[i], U[i], Pp[i]), dtype=float) for i in range(n + 1)])
        out[tag] = dict(x=X, u=U, p=Pp, f=F, dfdx=FX, dfdu=FU, mass=kw['mass'], J=kw['J'],
                        lx=kw['l_x'], ly=kw['l_y'], c=kw['c'])
    np.savez_compressed(os.path.join(OUT, 'dynamics_ref17.npz'),
                        **{f'{t}_{k}': np.asarray(v) for t, d in out.items() for k, v in d.items()})
    return out


def gen_ocp_capture(blastermodel, acados_template):
    acados_template.CAPTURED.clear()
    b = _build(blastermodel, _sim_params())
    integ, ocp_solver = b.generateController()
    ocp = ocp_solver.ocp
    c, k, so = ocp.cost, ocp.constraints, ocp.solver_options
    cap = dict(
        N=int(ocp.dims.N), nx=int(ocp.model.x.size()[0]), nu=int(ocp.model.u.size()[0]),
        np=int(ocp.model.p.size()[0]),
        W=np.asarray(c.W, float).tolist(), W_e=np.asarray(c.W_e, float).tolist(),
        Vx=np.asarray(c.Vx, float).tolist(), Vu=np.asarray(c.Vu, float).tolist(),
        Vx_e=np.asarray(c.Vx_e, float).tolist(), yref=np.asarray(c.yref, float).tolist(),
        cost_type=c.cost_type, cost_type_e=c.cost_type_e,
        idxbu=np.asarray(k.idxbu).tolist(), lbu=np.asarray(k.lbu, float).tolist(),
        ubu=np.asarray(k.ubu, float).tolist(), idxbx=np.asarray(k.idxbx).tolist(),
        lbx=np.asarray(k.lbx, float).tolist(), ubx=np.asarray(k.ubx, float).tolist(),
        x0=np.asarray(k.x0, float).tolist(),
        qp_solver=so.qp_solver, hessian_approx=so.hessian_approx,
        integrator_type=so.integrator_type, nlp_solver_type=so.nlp_solver_type,
        qp_solver_iter_max=int(so.qp_solver_iter_max), qp_solver_cond_N=int(so.qp_solver_cond_N),
        levenberg_marquardt=float(so.levenberg_marquardt), tf=float(so.tf),
        parameter_values=np.asarray(ocp.parameter_values, float).tolist(),
        json_file=ocp_solver.json_file,
    )
    with open(os.path.join(OUT, 'ocp_capture.json'), 'w') as fh:
        json.dump(cap, fh, indent=1)
    return cap


def gen_json_pin():
    with open(os.path.join(REF, 'src', 'scripts', 'acados_ocp_blasterModel.json')) as fh:
        d = json.load(fh)
    c, k, so, dims = d['cost'], d['constraints'], d['solver_options'], d['dims']
    pin = dict(
        dims={kk: dims[kk] for kk in ('N', 'nx', 'nu', 'np', 'ny', 'ny_e', 'nbu', 'nbx', 'nbx_0', 'nbx_e')},
        W=c['W'], W_e=c['W_e'], Vx=c['Vx'], Vu=c['Vu'], Vx_e=c['Vx_e'], yref=c['yref'],
        cost_type=c['cost_type'], cost_type_e=c['cost_type_e'],
        idxbu=k['idxbu'], lbu=k['lbu'], ubu=k['ubu'], idxbx=k['idxbx'], lbx=k['lbx'], ubx=k['ubx'],
        idxbx_0=k['idxbx_0'], idxbxe_0=k['idxbxe_0'],
        parameter_values=d['parameter_values'],
        solver_options={kk: so[kk] for kk in (
            'Tsim', 'tf', 'time_steps', 'integrator_type', 'sim_method_num_stages',
            'sim_method_num_steps', 'nlp_solver_type', 'qp_solver', 'qp_solver_cond_N',
            'qp_solver_iter_max', 'hessian_approx', 'globalization', 'nlp_solver_step_length',
            'levenberg_marquardt')},
    )
    with open(os.path.join(OUT, 'ocp_json_pin.json'), 'w') as fh:
        json.dump(pin, fh, indent=1)
    return pin


def gen_mathutils(MathUtils, rng):
    import casadi  # the refstub
    n = 32
    q1 = rng.normal(size=(n, 4))
    q2 = rng.normal(size=(n, 4))
    q1 /= np.linalg.norm(q1, axis=1, keepdims=True)
    prod, inv, rot = [], [], []
    for i in range(n):
        a = casadi.SX(list(q1[i]))
        b = casadi.SX(list(q2[i]))
        prod.append(np.array(MathUtils.quatMultiplication(a, b).M, dtype=float).reshape(-1))
        inv.append(np.array(MathUtils.unitQuatInversion(a).M, dtype=float).reshape(-1))
        rot.append(np.array(MathUtils.quat2Rot(a).M, dtype=float))
    np.savez_compressed(os.path.join(OUT, 'mathutils_ref.npz'), q1=q1, q2=q2,
                        prod=np.array(prod), inv=np.array(inv), rot=np.array(rot))


def gen_mpc_fixtures():
    sys.path.insert(0, REPO)
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec, mpc_solve
    inp = make_inputs('c1')
    spec = OcpSpec(N=10)
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec)
    np.savez_compressed(os.path.join(OUT, 'mpc_c1.npz'), x0=inp['x0'], xref=inp['xref'],
                        uref=inp['uref'], u0=o['u0'], X=o['X'], U=o['U'], status=o['status'])
    blobs = {}
    for cfg, N, box in (('c2', 20, False), ('c3', 20, False), ('c4', 30, True)):
        inp = make_inputs(cfg, ids=np.arange(8, dtype=np.uint64))
        spec = OcpSpec(N=N, lbu=np.zeros(4) if box else None, ubu=np.full(4, 65.0) if box else None)
        o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec)
        for key in ('x0', 'xref', 'uref'):
            blobs[f'{cfg}_{key}'] = inp[key]
        for key in ('u0', 'X', 'U', 'status', 'iters'):
            blobs[f'{cfg}_{key}'] = o[key]
    np.savez_compressed(os.path.join(OUT, 'mpc_small.npz'), **blobs)


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20261015)
    blastermodel, acados_template, MathUtils = _ref_imports()
    gen_dynamics(blastermodel, rng)
    cap = gen_ocp_capture(blastermodel, acados_template)
    pin = gen_json_pin()
    # the captured OCP must equal the reference's serialized JSON (same parameter set)
    for key in ('W', 'W_e', 'Vx', 'Vu', 'Vx_e', 'lbu', 'ubu', 'lbx', 'ubx', 'parameter_values'):
        assert np.allclose(np.asarray(cap[key], float), np.asarray(pin[key], float)), key
    gen_mathutils(MathUtils, rng)
    gen_mpc_fixtures()
    print('golden fixtures written to', OUT)


if __name__ == '__main__':
    main()
