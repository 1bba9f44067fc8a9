"""The 17/6 oracle: dynamics Jacobians pinned to the reference's own
generateModel() (exact sympy Jacobians in tests/golden/dynamics_ref17.npz), RK4 sensitivities
against central differences, and the LQ step against an independent dense solve."""
import os

import numpy as np
import pytest

from oracle.full import FullSpec, default_p25, jac17, mpc_solve17, rk4_sens17, rk4_step17
from oracle.model import Params

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def _params(d, t):
    return Params(mass=float(d[t + '_mass']), J=d[t + '_J'], lx=float(d[t + '_lx']),
                  ly=float(d[t + '_ly']), c=float(d[t + '_c']))


@pytest.mark.parametrize('tag', ['sim', 'main'])
def test_jac17_matches_reference_symbolic_jacobians(tag):
    d = np.load(os.path.join(GOLD, 'dynamics_ref17.npz'))
    P = _params(d, tag)
    J = jac17(d[tag + '_x'], d[tag + '_u'], d[tag + '_p'], P)
    for got, ref in ((J[..., :17], d[tag + '_dfdx']), (J[..., 17:], d[tag + '_dfdu'])):
        assert np.abs(got - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max())


def _random_point(B, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-0.3, 0.3, (B, 17))
    x[:, 2] += 3.5
    u = np.concatenate([rng.uniform(10, 30, (B, 4)), rng.uniform(-0.08, 0.08, (B, 2))], axis=1)
    p = np.tile(default_p25(), (B, 1))
    p[:, :24] = rng.uniform(-0.5, 0.5, (B, 24))
    return x, u, p


def test_rk4_sens17_matches_central_differences():
    P = Params()
    x, u, p = _random_point(4, 1)
    h = 1.0 / 30.0
    _, A, Bm = rk4_sens17(x, u, p, h, P)
    eps = 1e-6
    for j in range(17):
        e = np.zeros(17)
        e[j] = eps
        fd = (rk4_step17(x + e, u, p, h, P) - rk4_step17(x - e, u, p, h, P)) / (2 * eps)
        assert np.abs(fd - A[:, :, j]).max() < 1e-7
    for j in range(6):
        e = np.zeros(6)
        e[j] = eps
        fd = (rk4_step17(x, u + e, p, h, P) - rk4_step17(x, u - e, p, h, P)) / (2 * eps)
        assert np.abs(fd - Bm[:, :, j]).max() < 1e-7


def _dense_unconstrained(o, xref, uref, spec):
    """Condensed QP in du (dx_0 given), solved densely: an independent check of the Riccati."""
    A, Bm, gap, xbar, ubar = o['A'], o['B'], o['gap'], o['xbar'], o['ubar']
    Bsz, N = xbar.shape[0], spec.N
    nx, nu = 17, 6
    out = np.empty((Bsz, N, nu))
    for b in range(Bsz):
        c = np.zeros((N + 1, nx))
        G = np.zeros((N + 1, nx, N * nu))
        c[0] = o['X'][b, 0] - xbar[b, 0]
        for k in range(N):
            c[k + 1] = A[b, k] @ c[k] + gap[b, k]
            G[k + 1] = A[b, k] @ G[k]
            G[k + 1][:, k * nu:(k + 1) * nu] += Bm[b, k]
        H = np.zeros((N * nu, N * nu))
        g = np.zeros(N * nu)
        for k in range(N + 1):
            W = spec.QN if k == N else spec.s * spec.Q
            e = c[k] + xbar[b, k] - xref[b, k]
            H += G[k].T @ W @ G[k]
            g += G[k].T @ W @ e
        for k in range(N):
            sl = slice(k * nu, (k + 1) * nu)
            H[sl, sl] += spec.s * spec.R
            g[sl] += spec.s * spec.R @ (ubar[b, k] - uref[b, k])
        out[b] = np.linalg.solve(H, -g).reshape(N, nu)
    return out


@pytest.mark.parametrize('mode', ['rollout', 'iterate'])
def test_mpc_solve17_matches_dense_qp(mode):
    N, B = 6, 3
    spec = FullSpec(N=N)
    x0, _, p = _random_point(B, 2)
    xref = np.zeros((B, N + 1, 17))
    xref[..., 2] = 3.5
    uref = np.zeros((B, N, 6))
    uref[..., :4] = 22.0725
    kw = {}
    if mode == 'iterate':
        rng = np.random.default_rng(3)
        kw = dict(xbar=x0[:, None, :] + rng.normal(0, 0.05, (B, N + 1, 17)),
                  ubar=uref + rng.normal(0, 0.5, (B, N, 6)))
    o = mpc_solve17(x0, xref, uref, spec, p, mode=mode, **kw)
    assert (o['status'] == 0).all()
    du = _dense_unconstrained(o, xref, uref, spec)
    assert np.abs((o['U'] - o['ubar']) - du).max() <= 1e-8 * max(1.0, np.abs(du).max())


def test_ipm_box_matches_dense_bvls_and_kkt():
    """The interior point of the 17/6 input box (oracle.ocp.ipm_box_solve) against an
    independent condensed box-QP solve (SciPy BVLS) and the KKT conditions."""
    from oracle.ocp import dense_box_qp
    N, B = 10, 4
    lbu = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])
    ubu = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
    spec = FullSpec(N=N, lbu=lbu, ubu=ubu)
    x0, _, p = _random_point(B, 5)
    x0[:, 3:6] *= 0.5
    xref = np.zeros((B, N + 1, 17))
    xref[..., 2] = 3.5
    uref = np.zeros((B, N, 6))
    uref[..., :4] = 22.0725
    o = mpc_solve17(x0, xref, uref, spec, p)
    assert (o['status'] == 0).all() and o['iters'].max() < 60
    du = o['U'] - o['ubar']
    assert (o['U'] >= lbu - 1e-12).all() and (o['U'] <= ubu + 1e-12).all()
    dd = dense_box_qp(o['A'], o['B'], o['gap'], np.zeros((B, 17)), o['xbar'], o['ubar'], xref, uref, spec)
    assert np.abs(du - dd).max() <= 1e-6 * max(1.0, np.abs(dd).max())


def test_ipm_state_box_kkt():
    """The reference's state box (acados_ocp_blasterModel.json idxbx/lbx/ubx, stages 1..N-1) on
    top of the input box: the interior point's solution satisfies the KKT conditions of the
    condensed QP (multipliers >= 0 by NNLS on the near-active rows; stationarity, feasibility and
    the duality gap that bounds the suboptimality), and the state box is active on a good share
    of the rows."""
    import json

    from oracle.ocp import dense_kkt_certificate
    d = json.load(open(os.path.join(GOLD, 'ocp_json_pin.json')))
    lbx, ubx = np.array(d['lbx']), np.array(d['ubx'])
    N, B = 20, 6
    spec = FullSpec(N=N, lbu=np.array(d['lbu']), ubu=np.array(d['ubu']), lbx=lbx, ubx=ubx)
    rng = np.random.default_rng(31)
    x0 = rng.uniform(0.25 * lbx, 0.25 * ubx, (B, 17))
    x0[:, 2] = 3.5 + rng.uniform(-0.5, 0.5, B)
    xref = np.zeros((B, N + 1, 17))
    xref[..., 2] = 3.5
    xref[..., 14] = 0.2
    uref = np.zeros((B, N, 6))
    uref[..., :4] = 22.0725
    p = np.tile(default_p25(), (B, 1))
    p[:, :24] = rng.uniform(-0.5, 0.5, (B, 24))
    o = mpc_solve17(x0, xref, uref, spec, p)
    assert (o['status'] == 0).all() and o['iters'].max() < 60
    X = o['X'][:, 1:N]
    assert (X >= lbx - 1e-9).all() and (X <= ubx + 1e-9).all()
    n_act = ((X - lbx < 1e-6) | (ubx - X < 1e-6)).sum()
    assert n_act >= B * 10
    du = o['U'] - o['ubar']
    stat, viol, gap = dense_kkt_certificate(o['A'], o['B'], o['gap'], np.zeros((B, 17)), o['xbar'], o['ubar'],
                                            xref, uref, spec, du, lbx=lbx, ubx=ubx)
    assert stat.max() <= 1e-12 and viol.max() <= 1e-10 and gap.max() <= 1e-8, (stat, viol, gap)


def test_ipm_state_box_thin_interior_instances_converge(monkeypatch):
    """The two LP-feasible bench instances whose Newton system breaks before mu = 1e-8
    (tests/golden/sbox_thin_interior.npz).  Without the polish the interior point's iterate at the
    breakdown is all there is: a reduced-accuracy point, reported as acados' MINSTEP.  With it
    (oracle.ocp.al_polish) the active set is identified and U is the exact solution on it: a KKT
    certificate of the condensed QP to rounding; an LP says both QPs are feasible."""
    import oracle.ocp as ocp
    from oracle.ocp import IPM_BREAK_TOL, STATUS_MINSTEP, dense_kkt_certificate, lp_box_feasible
    d = np.load(os.path.join(GOLD, 'sbox_thin_interior.npz'))
    lbx, ubx, x0, p = d['lbx'], d['ubx'], d['x0'], d['p']
    N, B = int(d['N']), x0.shape[0]
    xref = np.zeros((B, N + 1, 17))
    xref[..., 2], xref[..., 14] = 3.5, 0.2
    uref = np.zeros((B, N, 6))
    uref[..., :4] = 22.0725
    lbu = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])
    ubu = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
    spec = FullSpec(N=N, lbu=lbu, ubu=ubu, lbx=lbx, ubx=ubx)
    diag = {}
    orig = ocp.al_polish
    monkeypatch.setattr(ocp, 'al_polish', lambda *a, **k: orig(*a, diag=diag, **k))
    with np.errstate(all='ignore'):
        o = mpc_solve17(x0, xref, uref, spec, p)
    assert IPM_BREAK_TOL >= 1e-5
    assert (o['status'] == 0).all(), o['status']
    assert diag['done'].all() and (diag['passes'] >= 1).all()
    dx0 = x0 - o['xbar'][:, 0]
    assert lp_box_feasible(o['A'], o['B'], o['gap'], dx0, o['xbar'], o['ubar'], spec, lbx, ubx).all()
    stat, viol, gap = dense_kkt_certificate(o['A'], o['B'], o['gap'], dx0, o['xbar'], o['ubar'], xref, uref, spec,
                                            o['U'] - o['ubar'], lbx=lbx, ubx=ubx)
    assert stat.max() <= 1e-12 and viol.max() <= 1e-10 and gap.max() <= 1e-5, (stat, viol, gap)
    monkeypatch.setattr(ocp, 'POLISH_ITERS', 0)
    with np.errstate(all='ignore'):
        o0 = mpc_solve17(x0, xref, uref, spec, p)
    assert (o0['status'] == STATUS_MINSTEP).all(), o0['status']   # both stopped at the breakdown
    stat0, _, _ = dense_kkt_certificate(o0['A'], o0['B'], o0['gap'], dx0, o0['xbar'], o0['ubar'], xref, uref, spec,
                                        o0['U'] - o0['ubar'], lbx=lbx, ubx=ubx)
    assert stat0.max() > 1e3 * stat.max()


def test_polish_active_set_changes(monkeypatch):
    """The polish's one-change-per-pass active-set correction: with the midpoint ratio test
    (lambda > s) the second thin-interior instance starts from a set holding rows that are not
    active at the solution (their equalities are inconsistent with the rest); the passes release
    them and still end at the exact solution (same U as from the default classification)."""
    import oracle.ocp as ocp
    d = np.load(os.path.join(GOLD, 'sbox_thin_interior.npz'))
    lbx, ubx, x0, p = d['lbx'], d['ubx'], d['x0'][1:], d['p'][1:]
    N = int(d['N'])
    xref = np.zeros((1, N + 1, 17))
    xref[..., 2], xref[..., 14] = 3.5, 0.2
    uref = np.zeros((1, N, 6))
    uref[..., :4] = 22.0725
    spec = FullSpec(N=N, lbu=np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665]),
                    ubu=np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665]), lbx=lbx, ubx=ubx)
    with np.errstate(all='ignore'):
        ref = mpc_solve17(x0, xref, uref, spec, p)
    diag = {}
    orig = ocp.al_polish
    monkeypatch.setattr(ocp, 'al_polish', lambda *a, **k: orig(*a, diag=diag, **k))
    monkeypatch.setattr(ocp, 'POLISH_ACT', 1.0)
    with np.errstate(all='ignore'):
        o = mpc_solve17(x0, xref, uref, spec, p)
    assert (o['status'] == 0).all() and diag['done'].all() and diag['passes'][0] >= 4
    wmin = [t[1][0] for t in diag['trace']]
    assert min(wmin) < 0                                   # a release happened
    assert np.abs(o['U'] - ref['U']).max() <= 1e-7 * np.abs(ref['U']).max()


def test_loop17_fixture_is_the_oracle_loop():
    """tests/golden/loop17_ref.npz (the GPU closed-loop test's reference) is what the oracle's loop
    gives: two instances, the first three steps, recomputed here."""
    import importlib.util
    spec_ = importlib.util.spec_from_file_location('mkloop', os.path.join(os.path.dirname(GOLD), '..', 'tools',
                                                                        'make_loop17_fixture.py'))
    mk = importlib.util.module_from_spec(spec_)
    spec_.loader.exec_module(mk)
    d = np.load(os.path.join(GOLD, 'loop17_ref.npz'))
    Xs, Us, st, it = mk.run(np.array([0, 1]), nsim=3)
    assert np.abs(Us - d['Us'][:2, :3]).max() <= 1e-12 * np.abs(d['Us']).max()
    assert np.abs(Xs - d['Xs'][:2, :4]).max() <= 1e-12 * np.abs(d['Xs']).max()
    assert np.array_equal(st, d['status'][:2, :3])
