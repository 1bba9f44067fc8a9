"""Randomised GPU parity sweep of the full 17/6 path (the reference's own OCP family): seeded
random horizon, batch, handle size, boxes (none / input / input + state), rollout or iterate mode,
per-instance or stage-varying parameters, fp64 or fp32, through the C ABI against the oracle
(oracle/full.py) on identical inputs.  Unboxed: fp64 1e-9 normwise; fp32 u0 5e-3 against the fp64
oracle (measured up to 1.1e-3: the 6x6 input block with its alpha-rate weight 1e-5 is
ill-conditioned in single precision).  Boxed QPs are held to optimality, since along nearly flat
directions the minimiser is ill-determined (sweeps of cases 0-127: an fp64 state-box instance
6.4e-7 off the oracle's minimiser at an objective 2.4e-14 from it; fp32 input-box u0 up to 6e-2 off
at objectives within 1.6e-6; a tighter fp32 interior-point stop changed nothing): the QP
objective of the device's U (states by the oracle's linearised dynamics) within 1e-9 (fp64) /
1e-5 (fp32) of the oracle's, fp64 state rows within 1e-9 of the box and the fp64 minimiser within
1e-5.  Statuses equal, except OK against MINSTEP on at most 1 in 20 fp64 state-box instances (the
polish certifies a near-degenerate instance on one side only: 1 of 57 in case 66).  No state box
in fp32 (refused by the library).
"""
import os

import numpy as np
import pytest

from oracle.full import FullSpec, default_p25, mpc_solve17, sensitivity17

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

MINSTEP = 3   # mpcb.h MPCB_STATUS_MINSTEP
CASES = int(os.environ.get('MPCB_FUZZ_CASES', 16))   # (a deeper sweep on demand, from case
FIRST = int(os.environ.get('MPCB_FUZZ_FIRST', 0))          # MPCB_FUZZ_FIRST on)
LBU17 = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])
UBU17 = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
SB_LO = np.array([-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0, -0.0872665, -0.0872665,
                  -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5])
SB_HI = np.array([1.5, 1.5, 5.0, 0.174532925, 0.174532925, 0.349066, 1.0, 1.0, 1.0, 0.0872665, 0.0872665,
                  0.0872665, 1.22173, 0.523599, 1.5, 1.5, 2.5])


def relerr(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, dtype=np.float64).reshape(b.shape[0], -1)
    return np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1.0)


def draw(case):
    rng = np.random.default_rng(9100 + case)
    bounds = ('none', 'input', 'all')[int(rng.integers(3))]
    dtype = 'f32' if (bounds != 'all' and rng.random() < 0.3) else 'f64'
    return dict(bounds=bounds, dtype=dtype, N=int(rng.integers(5, 61)), B=int(rng.integers(1, 97)),
                iterate=bool(rng.random() < 0.35), stage_p=bool(rng.random() < 0.3),
                extra=int(rng.integers(0, 64)), seed=int(rng.integers(1 << 30)))


def inputs(B, N, rng, stage_p):
    x0 = np.zeros((B, 17))
    x0[:, 0:3] = rng.uniform(-1, 1, (B, 3))
    x0[:, 2] += 3.5
    x0[:, 3:6] = rng.uniform(-0.17, 0.17, (B, 3))
    x0[:, 6:9] = rng.uniform(-0.5, 0.5, (B, 3))
    x0[:, 9:12] = rng.uniform(-0.087, 0.087, (B, 3))
    x0[:, 12:14] = rng.uniform(-0.2, 0.2, (B, 2))
    x0[:, 14:17] = rng.uniform(-0.3, 0.3, (B, 3))
    x0 = np.clip(x0, 0.5 * SB_LO, 0.5 * SB_HI)   # (inside the state box's stage-1 reach)
    x0[:, 2] = 3.5 + rng.uniform(-0.5, 0.5, B)
    xref = np.zeros((B, N + 1, 17))
    xref[..., 2] = 3.5
    xref[..., 14] = 0.2
    uref = np.zeros((B, N, 6))
    uref[..., :4] = 22.0725
    if stage_p:
        p = np.tile(default_p25(), (B, N, 1))
        p[..., :24] = rng.uniform(-0.5, 0.5, (B, N, 24))
    else:
        p = np.tile(default_p25(), (B, 1))
        p[:, :24] = rng.uniform(-0.5, 0.5, (B, 24))
    return x0, xref, uref, p


def qp_objective(o, U, x0, xref, uref, spec):
    """The step's QP objective at input trajectory U (clipped into the input box), states by the
    oracle's linearised dynamics (o: mpc_solve17's A, B, gap, xbar, ubar); also the largest
    state-box violation of those states (0 without a state box)."""
    A, Bm, gap, xbar, ubar = o['A'], o['B'], o['gap'], o['xbar'], o['ubar']
    B, N = U.shape[0], spec.N
    U = np.asarray(U, dtype=np.float64)
    if spec.lbu is not None:
        U = np.clip(U, spec.lbu, spec.ubu)
    du = U - ubar
    dx = np.empty((B, N + 1, 17))
    dx[:, 0] = x0 - xbar[:, 0]
    for k in range(N):
        dx[:, k + 1] = np.einsum('bij,bj->bi', A[:, k], dx[:, k]) + np.einsum('bij,bj->bi', Bm[:, k], du[:, k]) + gap[:, k]
    X = xbar + dx
    ex = X - np.broadcast_to(xref, (B, N + 1, 17))
    eu = U - np.broadcast_to(uref, (B, N, 6))
    J = spec.s * (np.einsum('bki,ij,bkj->b', ex[:, :N], spec.Q, ex[:, :N]) + np.einsum('bki,ij,bkj->b', eu, spec.R, eu))
    J = J + np.einsum('bi,ij,bj->b', ex[:, N], spec.QN, ex[:, N])
    viol = np.zeros(B)
    if spec.lbx is not None:
        Xs = X[:, 1:N]
        viol = np.maximum(np.maximum(spec.lbx - Xs, Xs - spec.ubx), 0).max(axis=(1, 2))
    return J, viol


@pytest.mark.parametrize('case', range(FIRST, FIRST + CASES))
def test_random_full17_config_matches_oracle(case):
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    c = draw(case)
    N, B, dtype = c['N'], c['B'], c['dtype']
    rng = np.random.default_rng(c['seed'])
    x0, xref, uref, p = inputs(B, N, rng, c['stage_p'])
    kw = {}
    if c['bounds'] in ('input', 'all'):
        kw.update(lbu=LBU17, ubu=UBU17)
    if c['bounds'] == 'all':
        kw.update(lbx=SB_LO, ubx=SB_HI)
    m = BatchedMPC(MPCConfig.full(N=N, dtype=dtype, **kw), max_batch=B + c['extra'])
    cast = (lambda a: a.astype(np.float32).astype(np.float64)) if dtype == 'f32' else (lambda a: a)
    x0, xref, uref, p = cast(x0), cast(xref), cast(uref), cast(p)
    m.set_params(p)
    spec = FullSpec(N=N, **kw)
    if c['iterate']:
        xb = cast(x0[:, None, :] + rng.normal(0, 0.03, (B, N + 1, 17)))
        ub = cast(uref + rng.normal(0, 0.5, (B, N, 6)))
        m.solve_iterate(x0, xb, ub, xref, uref)
        o = mpc_solve17(x0, xref, uref, spec, p, mode='iterate', xbar=xb, ubar=ub)
    else:
        m.solve(x0, xref, uref)
        o = mpc_solve17(x0, xref, uref, spec, p)
    torch.cuda.synchronize()
    u0 = m.get_control().cpu().numpy()
    X = m.get_state_trajectory().cpu().numpy()
    U = m.get_input_trajectory().cpu().numpy()
    st = m.get_status().cpu().numpy()
    e = [relerr(u0, o['u0']).max(), relerr(X, o['X']).max(), relerr(U, o['U']).max()]
    print(f'case {case} {c}: rel err u0 {e[0]:.2e} X {e[1]:.2e} U {e[2]:.2e}, status '
          f'{np.bincount(st, minlength=5).tolist()} oracle {np.bincount(o["status"], minlength=5).tolist()}')
    ok = (st == 0) & (o['status'] == 0)
    if c['bounds'] != 'none':
        Jd, vd = qp_objective(o, U, x0, xref, uref, spec)
        Jo, vo = qp_objective(o, o['U'], x0, xref, uref, spec)
        jgap = Jd / np.abs(Jo) - 1.0
        print(f'  objective gap max {jgap[ok].max(initial=0):.2e}, state-box violation device '
              f'{vd[ok].max(initial=0):.1e} oracle {vo[ok].max(initial=0):.1e}')
    emax = max(relerr(u0, o['u0'])[ok].max(initial=0), relerr(X, o['X'])[ok].max(initial=0),
               relerr(U, o['U'])[ok].max(initial=0))
    if dtype == 'f64':
        # same statuses, except that the state box's polish may certify ONE instance on one side and
        # leave it at the interior point's conditioning limit (MINSTEP) on the other (1 of 57 in
        # case 66 of the 128-case sweep)
        diff = st != o['status']
        minstep = {0, MINSTEP}
        assert all({int(a), int(b)} <= minstep for a, b in zip(st[diff], o['status'][diff]))
        assert diff.sum() <= 1
        if c['bounds'] == 'none':
            assert emax <= 1e-9
        else:
            # optimal and feasible as the oracle's; the minimiser within 1e-8 on every instance
            # that is not degenerate at fp64 precision (its exact minimiser moves by more than
            # 1e-9 under a few ulp of noise on [A|B], oracle.full.sensitivity17: a flat direction)
            flat = sensitivity17(o, x0, xref, uref, spec, rel=2.0 ** -45) > 1e-9
            w = ok & ~flat
            ew = max(relerr(u0, o['u0'])[w].max(initial=0), relerr(X, o['X'])[w].max(initial=0),
                     relerr(U, o['U'])[w].max(initial=0))
            print(f'  fp64 boxed: {int((ok & flat).sum())} of {int(ok.sum())} degenerate; the others within {ew:.1e}')
            assert jgap[ok].max(initial=0) <= 1e-9 and vd[ok].max(initial=0) <= 1e-9 and ew <= 1e-8
    else:
        assert (st == 0).all()
        if c['bounds'] == 'none':
            assert e[0] <= 5e-3
        else:
            # the input box in fp32: held to the optimal objective; u0 against the fp64 minimiser
            # is reported with the instances' fp32 sensitivity (the measured reason it can be far)
            sens = sensitivity17(o, x0, xref, uref, spec, rel=2.0 ** -22)
            eu = relerr(u0, o['u0'])
            pin = sens <= 1e-5
            print(f'  fp32 boxed: u0 max {eu.max():.1e}; fp32 sensitivity max {sens.max():.1e}; '
                  f'u0 on the {int(pin.sum())} fp32-pinnable instances {eu[pin].max(initial=0):.1e}')
            assert jgap.max() <= 1e-5
