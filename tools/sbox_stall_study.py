#!/usr/bin/env python3
"""The state-box interior point's stall rule (oracle.ocp IPM_SBOX_SHORT / _RUN, mpcb_full.h
IPM17_SBOX_SHORT / _RUN) chosen on the oracle's own traces of the 17/6 bench draws
(tools/bench_full17.py --bounds all: 4096 instances, N = 60, seed 1017).  CPU only, ~10 min with
4 processes: per instance the step lengths, duality measure and primal residual of every
iteration (oracle.ocp.ipm_box_solve trace) and the LP feasibility of its QP
(oracle.ocp.lp_box_feasible), then for each candidate (a, M) -- stop as infeasible after M steps in
a row shorter than a while not near the solution -- the longest such run among LP-feasible
instances and the iteration at which each LP-infeasible one would stop.

    python tools/sbox_stall_study.py [--parts 4] [--out /tmp/sbox_trace]
"""
import argparse
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def draws(N=60, BB=4096):
    """tools/bench_full17.py --bounds all: x0, xref, uref, p and the boxes."""
    rng = np.random.default_rng(1017)
    x0 = np.zeros((BB, 17))
    x0[:, 0:3] = rng.uniform(-1, 1, (BB, 3))
    x0[:, 2] += 3.5
    x0[:, 3:6] = rng.uniform(-0.17, 0.17, (BB, 3))
    x0[:, 6:9] = rng.uniform(-0.5, 0.5, (BB, 3))
    x0[:, 9:12] = rng.uniform(-0.087, 0.087, (BB, 3))
    xref = np.zeros((1, N + 1, 17))
    xref[..., 2], xref[..., 14] = 3.5, 0.2
    uref = np.zeros((1, N, 6))
    uref[..., :4] = 22.0725
    p = np.zeros((BB, 25))
    p[:, :24] = rng.uniform(-0.5, 0.5, (BB, 24))
    p[:, 24] = 2.2 * 9.81
    lbu = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])
    ubu = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
    lbx = np.array([-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0, -0.0872665,
                    -0.0872665, -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5])
    ubx = -lbx
    ubx[[2, 12]] = 5.0, 1.22173
    x0 = np.clip(x0, 0.5 * lbx, 0.5 * ubx)
    x0[:, 2] = 3.5 + rng.uniform(-0.5, 0.5, BB)
    return x0, xref, uref, p, lbu, ubu, lbx, ubx


def trace_part(part, nparts, out):
    from oracle.full import FullSpec, mpc_solve17
    from oracle.ocp import ipm_box_solve, lp_box_feasible
    N = 60
    x0, xref, uref, p, lbu, ubu, lbx, ubx = draws(N)
    sl = slice(part * len(x0) // nparts, (part + 1) * len(x0) // nparts)
    x0, p = x0[sl], p[sl]
    B = len(x0)
    spec = FullSpec(N=N, lbu=lbu, ubu=ubu, lbx=lbx, ubx=ubx)
    with np.errstate(all='ignore'):
        o = mpc_solve17(x0, xref, uref, FullSpec(N=N), p)
    A, Bm, gap, xbar, ubar = o['A'], o['B'], o['gap'], o['xbar'], o['ubar']
    dx0 = x0 - xbar[:, 0]
    feas = lp_box_feasible(A, Bm, gap, dx0, xbar, ubar, spec, lbx, ubx)
    tr = []
    with np.errstate(all='ignore'):
        _, _, st, it = ipm_box_solve(A, Bm, gap, dx0, xbar, ubar, np.broadcast_to(xref, (B, N + 1, 17)),
                                     np.broadcast_to(uref, (B, N, 6)), spec, max_iter=200, lbx=lbx, ubx=ubx,
                                     trace=tr)
    np.savez(f'{out}_{part}.npz', mu=np.array([t[0] for t in tr]), res=np.array([t[1] for t in tr]),
             alpha=np.array([t[2] for t in tr]), feas=feas, status=st, iters=it)


def study(out, nparts):
    parts = [np.load(f'{out}_{i}.npz') for i in range(nparts)]
    T = max(q['alpha'].shape[0] for q in parts)
    pad = lambda a: np.concatenate([a, np.full((T - a.shape[0], a.shape[1]), np.nan)], 0)
    al, res, mu = (np.concatenate([pad(q[k]) for q in parts], 1) for k in ('alpha', 'res', 'mu'))
    feas = np.concatenate([q['feas'] for q in parts])
    it = np.concatenate([q['iters'] for q in parts])
    print(f'{len(feas)} draws: {(~feas).sum()} LP-infeasible; iterations with the rule in effect: '
          f'feasible max {it[feas].max()}, infeasible max {it[~feas].max()}')
    for a in (1e-2, 2e-2, 3e-2, 5e-2, 7e-2, 1e-1):
        run = np.zeros(al.shape[1], int)
        longest = np.zeros(al.shape[1], int)
        for t in range(T):
            near = (mu[t] <= 1e-5) & (res[t] <= 1e-9)
            run = np.where(~np.isnan(al[t]) & (al[t] < a) & ~near, run + 1, 0)
            longest = np.maximum(longest, run)
        m0 = int(longest[feas].max())
        line = f'a = {a:.0e}: longest run among feasible {m0};'
        for M in (m0 + 1, m0 + 2, m0 + 3, m0 + 4):
            run = np.zeros(al.shape[1], int)
            stop = np.full(al.shape[1], -1)
            for t in range(T):
                near = (mu[t] <= 1e-5) & (res[t] <= 1e-9)
                run = np.where(~np.isnan(al[t]) & (al[t] < a) & ~near, run + 1, 0)
                hit = (run >= M) & (stop < 0)
                stop[hit] = t + 1
            line += f'  M={M}: infeasible stop max {stop[~feas].max()}'
        print(line)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--parts', type=int, default=4)
    ap.add_argument('--out', default='/tmp/sbox_trace')
    ap.add_argument('--part', type=int, default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.part is not None:
        trace_part(args.part, args.parts, args.out)
        return
    procs = [subprocess.Popen([sys.executable, __file__, '--parts', str(args.parts), '--out', args.out,
                               '--part', str(i)], env=dict(os.environ, OMP_NUM_THREADS='2'))
             for i in range(args.parts)]
    if any(p.wait() for p in procs):
        raise SystemExit('a trace part failed')
    study(args.out, args.parts)


if __name__ == '__main__':
    main()
