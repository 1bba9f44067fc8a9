#!/usr/bin/env python3
"""Why the 12/4 input box has an interior-point fallback (oracle.ocp.pdas_solve, mpcb_asipm.h).
CPU only (NumPy oracle).  On input-box draws with sine references and a +-5 N wind per instance
(tests/test_oracle_ocp.py hard_box_inputs) it counts the active-set passes of the oracle's
primal-dual active set under several backup rules, on the instances that need more than 60
passes with the shipped rule, against the interior point's iterations (adaptive centring, the
fallback's scheme, and Mehrotra's).

    python tools/pdas_hard_study.py [--B 3000] [--N 18] [--cap 1500]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from oracle.ocp import (OcpSpec, _ipm_box_mehrotra, ipm_box_solve, linearise, riccati_solve,  # noqa: E402
                        rollout)
from test_oracle_ocp import hard_box_inputs  # noqa: E402


def pdas(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec, pbar=3, backup='least', cap=1500):
    """oracle.ocp.pdas_solve without the fallback, with a choice of backup rule: 'least' (shipped:
    Murty's least index), 'largest', or 'stage' (every violation of the first violated stage)."""
    Bsz, N = xbar.shape[0], spec.N
    NU = Bm.shape[-1]
    lb = np.broadcast_to(np.asarray(spec.lbu, float), (NU,))
    ub = np.broadcast_to(np.asarray(spec.ubu, float), (NU,))
    low = np.zeros((Bsz, N, NU), bool)
    up = np.zeros((Bsz, N, NU), bool)
    done = np.zeros(Bsz, bool)
    iters = np.zeros(Bsz, np.int32)
    best = np.full(Bsz, 1 << 30)
    pcount = np.full(Bsz, pbar)
    flat = np.arange(N * NU).reshape(N, NU)
    for _ in range(cap):
        fixed = low | up
        delta = np.where(low, lb - ubar, np.where(up, ub - ubar, 0.0))
        _, du, mu, _ = riccati_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec, fixed, delta)
        iters[~done] += 1
        u = ubar + du
        v_lo, v_hi = ~fixed & (u < lb), ~fixed & (u > ub)
        v_fl, v_fu = low & (mu < 0), up & (mu > 0)
        V = v_lo | v_hi | v_fl | v_fu
        nV = V.sum(axis=(1, 2))
        done |= nV == 0
        if done.all():
            break
        full = (nV < best) | (pcount > 0)
        pcount = np.where(nV < best, pbar, np.where(full, pcount - 1, pcount))
        best = np.minimum(best, nV)
        if backup == 'least':
            single = flat[None] == np.where(V, flat[None], N * NU).reshape(Bsz, -1).min(axis=1)[:, None, None]
        elif backup == 'largest':
            single = flat[None] == np.where(V, flat[None], -1).reshape(Bsz, -1).max(axis=1)[:, None, None]
        else:
            ks = np.where(V.any(axis=2), np.arange(N)[None], N).min(axis=1)
            single = V & (np.arange(N)[None, :, None] == ks[:, None, None])
        sel = np.where(full[:, None, None], V, single) & ~done[:, None, None]
        low = np.where(sel & v_lo, True, np.where(sel & v_fl, False, low))
        up = np.where(sel & v_hi, True, np.where(sel & v_fu, False, up))
    return iters, done


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, default=3000)
    ap.add_argument('--N', type=int, default=18)
    ap.add_argument('--cap', type=int, default=1500)
    args = ap.parse_args()
    B, N = args.B, args.N
    inp = hard_box_inputs(B, N, 11)
    spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0))
    xref = np.broadcast_to(inp['xref'], (B, N + 1, 12))
    uref = np.broadcast_to(inp['uref'], (B, N, 4))
    ubar = uref.copy()
    xbar = rollout(inp['x0'], ubar, spec, inp['wind'])
    A, Bm, gap = linearise(xbar, ubar, spec, inp['wind'])
    qp = (A, Bm, gap, inp['x0'] - xbar[:, 0], xbar, ubar, xref, uref, spec)
    it, done = pdas(*qp, cap=60)
    hard = np.nonzero(~done)[0]
    print(f'{B} draws (N = {N}): {len(hard)} need more than 60 active-set passes', flush=True)
    sub = tuple(a[hard] if isinstance(a, np.ndarray) and a.shape[0] == B else a for a in qp)
    for pbar, backup in [(3, 'least'), (10, 'least'), (3, 'stage'), (3, 'largest')]:
        it, done = pdas(*sub, pbar=pbar, backup=backup, cap=args.cap)
        print(f'  active set, {pbar} full-exchange tries, backup {backup:7s}: passes median {np.median(it):5.0f} '
              f'p90 {np.percentile(it, 90):5.0f} max {it.max():5d}, unconverged after {args.cap}: {(~done).sum()}',
              flush=True)
    with np.errstate(all='ignore'):
        _, _, st, it = ipm_box_solve(*sub, max_iter=100, centring='adaptive')
        print(f'  interior point, adaptive centring: status {np.bincount(st, minlength=5).tolist()}, '
              f'iterations mean {it.mean():.1f} max {it.max()}')
        _, _, st, it = _ipm_box_mehrotra(*sub, max_iter=100)
        print(f'  interior point, Mehrotra: status {np.bincount(st, minlength=5).tolist()}, '
              f'iterations mean {it.mean():.1f} max {it.max()}')


if __name__ == '__main__':
    main()
