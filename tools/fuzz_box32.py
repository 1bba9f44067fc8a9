"""Diagnostic (GPU box): the fp32 input-box cases of the randomised parity sweep
(tests/test_gpu_fuzz.py draw) over a case range, each against the fp64 NumPy oracle on the same
fp32-rounded inputs: per case the normwise worst u0 / U / X errors, how many instances exceed
5e-5 and how many of those the oracle's interior point handled (``fallback``).

    python tools/fuzz_box32.py [--first 0] [--cases 248] [--nmax 40]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--first', type=int, default=0)
    ap.add_argument('--cases', type=int, default=248)
    ap.add_argument('--nmax', type=int, default=40)
    a = ap.parse_args()
    import torch

    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec, fp32_sensitivity, mpc_solve
    from test_gpu_fuzz import draw, relerr
    worst = []
    for case in range(a.first, a.first + a.cases):
        c = draw(case)
        if not (c['box'] and c['dtype'] == 'f32') or c['N'] > a.nmax:
            continue
        N, B = c['N'], c['B']
        rng = np.random.default_rng(c['seed'])
        inp = make_inputs(c['ref'], ids=np.arange(B, dtype=np.uint64) + np.uint64(c['seed'] % 100000), N=N)
        wind = 5.0 * (2.0 * rng.random((B, 3)) - 1.0) if c['wind'] else None
        cast = lambda v: None if v is None else v.astype(np.float32).astype(np.float64)  # noqa: E731
        x0, xref, uref, wind = cast(inp['x0']), cast(inp['xref']), cast(inp['uref']), cast(wind)
        spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0))
        m = BatchedMPC(MPCConfig(N=N, dtype='f32', lbu=spec.lbu, ubu=spec.ubu), max_batch=B + int(c['extra'] * B))
        if c['iterate']:
            xbar = cast(xref + rng.normal(scale=0.05, size=(B, N + 1, 12)))
            ubar = cast(uref + rng.normal(scale=1.0, size=(B, N, 4)))
            m.solve_iterate(x0, xbar, ubar, xref, uref, wind=wind)
            o = mpc_solve(x0, xref, uref, spec, wind=wind, mode='iterate', xbar=xbar, ubar=ubar, return_lin=True)
        else:
            m.solve(x0, xref, uref, wind=wind)
            o = mpc_solve(x0, xref, uref, spec, wind=wind, return_lin=True)
        ill = fp32_sensitivity(o, x0, xref, uref, spec) > 1e-5
        torch.cuda.synchronize()
        U1 = m.get_input_trajectory().cpu().numpy().copy()
        qs = m.qp_stats(B).cpu().numpy()
        os.environ['MPCB_AS_REFINE'] = '0'   # (read at every solve): which instances were refined
        try:
            if c['iterate']:
                m.solve_iterate(x0, xbar, ubar, xref, uref, wind=wind)
            else:
                m.solve(x0, xref, uref, wind=wind)
            U0 = m.get_input_trajectory().cpu().numpy()
        finally:
            os.environ.pop('MPCB_AS_REFINE')
        refined = (U0 != U1).reshape(B, -1).any(axis=1)
        if c['iterate']:
            m.solve_iterate(x0, xbar, ubar, xref, uref, wind=wind)
        else:
            m.solve(x0, xref, uref, wind=wind)
        torch.cuda.synchronize()
        eu = relerr(m.get_control().cpu().numpy(), o['u0'])
        eU = relerr(m.get_input_trajectory().cpu().numpy(), o['U'])
        eX = relerr(m.get_state_trajectory().cpu().numpy(), o['X'])
        st = m.get_status().cpu().numpy()
        bad = (np.maximum(np.maximum(eu, eU), eX) > 5e-5) & ~ill
        fb = o['fallback']
        print(f'case {case} N={N} B={B} iterate={c["iterate"]} wind={c["wind"]} ref={c["ref"]}: '
              f'u0 {eu.max():.2e} U {eU.max():.2e} X {eX.max():.2e}; fp32-ill {int(ill.sum())}; '
              f'well-conditioned > 5e-5: {bad.sum()} (max {np.maximum(np.maximum(eu, eU), eX)[~ill].max(initial=0):.2e}) '
              f'(of them oracle-fallback {int((bad & fb).sum())}); fallbacks {int(fb.sum())}; '
              f'status match {bool((st == o["status"]).all())}; refined {int(refined.sum())}, '
              f'bad and refined {int((bad & refined).sum())}', flush=True)
        for i in np.nonzero(bad & ~fb)[0][:3]:
            print(f'    bad non-fallback instance {i}: u0 {eu[i]:.2e} U {eU[i]:.2e} X {eX[i]:.2e} '
                  f'refined {bool(refined[i])} passes {qs[i].tolist()} oracle iters {o["iters"][i]}', flush=True)
        worst.append(np.maximum(np.maximum(eu, eU), eX)[~ill].max(initial=0))
        del m
    print(f'cases {len(worst)}: worst {max(worst):.2e}; over 5e-5: {sum(w > 5e-5 for w in worst)}')


if __name__ == '__main__':
    main()
