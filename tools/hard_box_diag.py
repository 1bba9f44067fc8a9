"""Diagnostic (GPU box): the fp32 input box on tests/test_oracle_ocp.py hard_box_inputs (sine
references, +-5 N wind), per instance against the fp64 oracle: the instances beyond 5e-5 that
oracle.ocp.fp32_sensitivity does not flag, with their pass counts and whether the refinement
kernel changed them (MPCB_AS_REFINE=0 A/B).

    python tools/hard_box_diag.py [--N 18 --B 192 --seed 11]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--N', type=int, default=18)
    ap.add_argument('--B', type=int, default=192)
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--case', type=int, default=None, help='a fp32 box case of tests/test_gpu_fuzz.py draw instead')
    a = ap.parse_args()
    import torch

    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle.ocp import OcpSpec, fp32_sensitivity, mpc_solve
    from test_gpu_fuzz import relerr
    from test_oracle_ocp import hard_box_inputs
    cast = lambda v: None if v is None else v.astype(np.float32).astype(np.float64)  # noqa: E731
    kw = {}
    if a.case is None:
        N, B = a.N, a.B
        inp = hard_box_inputs(B, N, a.seed)
        x0, xref, uref, wind = (cast(inp[k]) for k in ('x0', 'xref', 'uref', 'wind'))
    else:
        from oracle.inputs import make_inputs
        from test_gpu_fuzz import draw
        c = draw(a.case)
        N, B = c['N'], c['B']
        rng = np.random.default_rng(c['seed'])
        inp = make_inputs(c['ref'], ids=np.arange(B, dtype=np.uint64) + np.uint64(c['seed'] % 100000), N=N)
        wind = 5.0 * (2.0 * rng.random((B, 3)) - 1.0) if c['wind'] else None
        x0, xref, uref, wind = cast(inp['x0']), cast(inp['xref']), cast(inp['uref']), cast(wind)
        if c['iterate']:
            kw = dict(mode='iterate', xbar=cast(xref + rng.normal(scale=0.05, size=(B, N + 1, 12))),
                      ubar=cast(uref + rng.normal(scale=1.0, size=(B, N, 4))))
    spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0))
    m = BatchedMPC(MPCConfig(N=N, dtype='f32', lbu=spec.lbu, ubu=spec.ubu), max_batch=B)
    res = {}
    for ref in ('1', '0'):
        os.environ['MPCB_AS_REFINE'] = ref
        if kw:
            m.solve_iterate(x0, kw['xbar'], kw['ubar'], xref, uref, wind=wind)
        else:
            m.solve(x0, xref, uref, wind=wind)
        torch.cuda.synchronize()
        res[ref] = (m.get_input_trajectory().double().cpu().numpy(), m.qp_stats(B).cpu().numpy())
    os.environ.pop('MPCB_AS_REFINE')
    o = mpc_solve(x0, xref, uref, spec, wind=wind, return_lin=True, **kw)
    sens = fp32_sensitivity(o, x0, xref, uref, spec)
    U, qs = res['1']
    e = relerr(U, o['U'])
    e0 = relerr(res['0'][0], o['U'])
    refined = (res['1'][0] != res['0'][0]).reshape(B, -1).any(axis=1)
    bad = np.nonzero((e > 5e-5) & (sens <= 1e-5))[0]
    print(f'{len(bad)} well-conditioned instances beyond 5e-5 (of {B}); refined {int(refined.sum())}')
    for i in bad[:12]:
        print(f'  {i}: err {e[i]:.2e} (without refinement {e0[i]:.2e}) sens {sens[i]:.1e} qp_stats {qs[i].tolist()} '
              f'(without {res["0"][1][i].tolist()}) oracle iters {o["iters"][i]} fallback {bool(o["fallback"][i])} '
              f'refined {bool(refined[i])}')
        # the active sets: device (within 1e-6 of a bound) against the oracle's (1e-9)
        du, ou = U[i], o['U'][i]
        dl, dh = du <= 1e-6 * 65, du >= 65 - 1e-6 * 65
        ol, oh = ou <= 1e-9, ou >= 65 - 1e-9
        diff = np.argwhere((dl != ol) | (dh != oh))
        k, m_ = np.unravel_index(np.argmax(np.abs(du - ou)), du.shape)
        print(f'      active: device {int(dl.sum())}+{int(dh.sum())} oracle {int(ol.sum())}+{int(oh.sum())}; '
              f'differ at {[(int(a), int(b), round(float(du[a, b]), 5), round(float(ou[a, b]), 5)) for a, b in diff[:6]]}; '
              f'worst (k={k}, m={m_}) device {du[k, m_]:.6f} oracle {ou[k, m_]:.6f}')


if __name__ == '__main__':
    main()
