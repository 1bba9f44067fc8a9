"""Writes tests/golden/loop17_ref.npz: the receding-horizon loop of simulation_blaster.py:56-107 on
the reference's own OCP (acados_ocp_blasterModel.json: 17/6, N = 60, input box and state box on
stages 1..N-1, the JSON's parameter values) for B = 64 instances and NSIM = 20 steps, computed by
the oracle: per step one SQP_RTI step from the persistent iterate (oracle.full.mpc_solve17,
mode='iterate', initial iterate zeros as acados') and the plant step (oracle.full.rk4_step17 with
Tsim = Tf/N) applying u0.  Stores the inputs (x0, p, xref, uref) and the trajectories (Xs, Us),
the per-step statuses and the IPM iteration counts.  The initial states are the JSON test's
distribution (tests/test_gpu_rows.py::test_solve_from_reference_json_matches_oracle): hover at
z = 3 with small perturbations, inside the state box.

usage: python tools/make_loop17_fixture.py [--procs 8]"""
import os
import sys
import warnings
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
B, NSIM, SEED = 64, 20, 2027


def problem():
    from mpc_blaster_amd.acados_json import load_acados_ocp_json
    from oracle.full import FullSpec
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        cfg, info = load_acados_ocp_json(os.path.join(ROOT, 'tests', 'golden', 'ocp_json_pin.json'))
    N = cfg.N
    rng = np.random.default_rng(SEED)
    yref = info['yref']
    x0 = np.tile(yref[:17], (B, 1))
    x0[:, 2] = 3.0
    x0[:, 0:3] += rng.uniform(-0.3, 0.3, (B, 3))
    x0[:, 3:6] += rng.uniform(-0.05, 0.05, (B, 3))
    x0[:, 6:9] += rng.uniform(-0.2, 0.2, (B, 3))
    x0[:, 9:12] += rng.uniform(-0.02, 0.02, (B, 3))
    xref = np.where(np.arange(17) == 2, 3.5, yref[:17])
    xref = np.where(np.arange(17) == 14, 0.2, xref)          # POC_x reference, simulation_blaster.py:48
    uref = np.r_[np.full(4, 22.0725), yref[21:23]]
    spec = FullSpec(N=N, dt=cfg.dt, Q=cfg.Q, R=cfg.R, QN=cfg.QN, lbu=cfg.lbu, ubu=cfg.ubu, lbx=cfg.lbx,
                    ubx=cfg.ubx, max_as_iter=cfg.max_as_iter)
    return cfg, spec, x0, np.asarray(info['p'], dtype=np.float64), xref, uref


def run(ids, nsim=NSIM):
    """The oracle loop for instances ``ids`` (numpy; test infrastructure)."""
    from oracle.full import mpc_solve17, rk4_step17
    cfg, spec, x0, p, xref, uref = problem()
    N, b = spec.N, len(ids)
    x = x0[ids].copy()
    pb = np.tile(p, (b, 1))
    xr = np.broadcast_to(xref, (b, N + 1, 17))
    ur = np.broadcast_to(uref, (b, N, 6))
    xb, ub = np.zeros((b, N + 1, 17)), np.zeros((b, N, 6))
    Xs, Us = np.empty((b, nsim + 1, 17)), np.empty((b, nsim, 6))
    st, it = np.empty((b, nsim), np.int32), np.empty((b, nsim), np.int32)
    Xs[:, 0] = x
    for i in range(nsim):
        with np.errstate(all='ignore'):
            o = mpc_solve17(x, xr, ur, spec, pb, mode='iterate', xbar=xb, ubar=ub)
        xb, ub = o['X'], o['U']
        st[:, i], it[:, i] = o['status'], o['iters']
        Us[:, i] = o['u0']
        x = rk4_step17(x, o['u0'], pb, spec.dt, spec.params)
        Xs[:, i + 1] = x
    return Xs, Us, st, it


def main():
    procs = int(sys.argv[sys.argv.index('--procs') + 1]) if '--procs' in sys.argv else 8
    parts = np.array_split(np.arange(B), procs)
    with Pool(procs) as pool:
        res = pool.map(run, parts)
    Xs, Us, st, it = (np.concatenate([r[i] for r in res]) for i in range(4))
    cfg, spec, x0, p, xref, uref = problem()
    np.savez(os.path.join(ROOT, 'tests', 'golden', 'loop17_ref.npz'), x0=x0, p=p, xref=xref, uref=uref,
             Xs=Xs, Us=Us, status=st, iters=it, nsim=NSIM)
    print('status counts', np.bincount(st.ravel(), minlength=5), 'iterations max', it.max())


if __name__ == '__main__':
    main()
