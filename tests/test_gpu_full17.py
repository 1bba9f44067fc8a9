"""GPU parity of the full 17/6 model path through the C ABI vs the oracle
(oracle/full.py, whose dynamics Jacobians are pinned to the reference's generateModel()).

Tolerance: fp64 per-instance ||y_dev - y_oracle||_inf / max(||y_oracle||_inf, 1) <= 1e-9 on u0,
X and U (north_star asks 1e-5); [A|B] and the plant step <= 1e-11 absolute.  fp32 is checked on
u0 against the fp64 oracle with a 5e-4 normwise bound (achieved 2.7e-5; the alpha-rate weight 1e-5 of the
reference makes the 6x6 input block ill-conditioned in single precision)."""
import os

import numpy as np
import pytest

from oracle.full import FullSpec, default_p25, mpc_solve17, rk4_sens17, rk4_step17
from oracle.model import Params

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

LBU17 = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])   # JSON idxbu/lbu/ubu
UBU17 = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
SB_LO = np.array([-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0, -0.0872665, -0.0872665,
                  -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5])     # statesBound (JSON lbx/ubx)
SB_HI = np.array([1.5, 1.5, 5.0, 0.174532925, 0.174532925, 0.349066, 1.0, 1.0, 1.0, 0.0872665, 0.0872665,
                  0.0872665, 1.22173, 0.523599, 1.5, 1.5, 2.5])


def relerr(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, dtype=np.float64).reshape(b.shape[0], -1)
    return np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1.0)


def _inputs(B, N, seed):
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 17))
    x0[:, 0:3] = rng.uniform(-1, 1, (B, 3))
    x0[:, 2] += 3.5
    x0[:, 3:6] = rng.uniform(-0.17, 0.17, (B, 3))
    x0[:, 6:9] = rng.uniform(-0.5, 0.5, (B, 3))
    x0[:, 9:12] = rng.uniform(-0.087, 0.087, (B, 3))
    x0[:, 12:14] = rng.uniform(-0.2, 0.2, (B, 2))
    x0[:, 14:17] = rng.uniform(-0.3, 0.3, (B, 3))
    xref = np.zeros((B, N + 1, 17))
    xref[..., 2] = 3.5
    xref[..., 14] = 0.2            # POC_x reference (simulation_blaster.py:48)
    uref = np.zeros((B, N, 6))
    uref[..., :4] = 22.0725
    p = np.tile(default_p25(), (B, 1))
    p[:, :24] = rng.uniform(-0.5, 0.5, (B, 24))
    return x0, xref, uref, p


def _mpc(N, dtype='f64', max_batch=64):
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    return BatchedMPC(MPCConfig.full(N=N, dtype=dtype), max_batch=max_batch)


def test_linearize17_matches_oracle():
    N, B = 4, 5
    m = _mpc(N, max_batch=B)
    rng = np.random.default_rng(11)
    x0, _, uref, p = _inputs(B, N, 11)
    xb = x0[:, None, :] + rng.normal(0, 0.05, (B, N + 1, 17))
    ub = uref + rng.normal(0, 0.5, (B, N, 6))
    m.set_params(p)
    A, Bm, xn = (t.cpu().numpy() for t in m.linearize(xb, ub))
    P = Params()
    for k in range(N):
        xr, Ar, Br = rk4_sens17(xb[:, k], ub[:, k], p, 2.0 / 60.0, P)
        assert np.abs(A[:, k] - Ar).max() < 1e-11
        assert np.abs(Bm[:, k] - Br).max() < 1e-11
        assert np.abs(xn[:, k] - xr).max() < 1e-11


def test_sim_step17_matches_oracle():
    B = 70
    m = _mpc(10, max_batch=B)
    x0, _, uref, p = _inputs(B, 10, 12)
    m.set_params(p)
    xo = m.sim_step(x0, uref[:, 0]).cpu().numpy()
    ref = rk4_step17(x0, uref[:, 0], p, 2.0 / 60.0, Params())
    assert np.abs(xo - ref).max() < 1e-11


@pytest.mark.parametrize('B,N', [(1, 10), (7, 12), (33, 60)])
def test_solve17_rollout_matches_oracle_fp64(B, N):
    m = _mpc(N, max_batch=B)
    x0, xref, uref, p = _inputs(B, N, 100 + B)
    m.set_params(p)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    o = mpc_solve17(x0, xref, uref, FullSpec(N=N), p)
    assert (m.get_status().cpu().numpy() == o['status']).all()
    e = [relerr(m.get_control().cpu().numpy(), o['u0']).max(),
         relerr(m.get_state_trajectory().cpu().numpy(), o['X']).max(),
         relerr(m.get_input_trajectory().cpu().numpy(), o['U']).max()]
    print(f'17/6 fp64 B={B} N={N}: u0 {e[0]:.2e} X {e[1]:.2e} U {e[2]:.2e}')
    assert max(e) <= 1e-9


def test_solve17_iterate_and_default_params_match_oracle():
    N, B = 15, 9
    m = _mpc(N, max_batch=B)
    x0, xref, uref, _ = _inputs(B, N, 7)
    rng = np.random.default_rng(8)
    xb = x0[:, None, :] + rng.normal(0, 0.05, (B, N + 1, 17))
    ub = uref + rng.normal(0, 0.5, (B, N, 6))
    m.set_params(None)   # defaults: zero Jacobian blocks, T_blast = 2.2 * 9.81
    m.solve_iterate(x0, xb, ub, xref, uref)
    torch.cuda.synchronize()
    o = mpc_solve17(x0, xref, uref, FullSpec(N=N), None, mode='iterate', xbar=xb, ubar=ub)
    assert relerr(m.get_state_trajectory().cpu().numpy(), o['X']).max() <= 1e-9
    assert relerr(m.get_input_trajectory().cpu().numpy(), o['U']).max() <= 1e-9
    assert (m.get_status().cpu().numpy() == 0).all()


@pytest.mark.parametrize('box', [False, True])
def test_solve17_chunked_ragged_batches_match_oracle(box, monkeypatch):
    """Several workspace chunks whose last wavefront is ragged (MPCB_CHUNK=64, B=150: chunks of
    64, 64, 22 instances): the 16-lane kernel's extra groups run on private padding slots of the
    workspace and must neither disturb the valid instances nor write outputs."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    monkeypatch.setenv('MPCB_CHUNK', '64')
    N, B = 12, 150
    kw = dict(lbu=LBU17, ubu=UBU17) if box else {}
    m = BatchedMPC(MPCConfig.full(N=N, **kw), max_batch=B)
    x0, xref, uref, p = _inputs(B, N, 404)
    m.set_params(p)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    o = mpc_solve17(x0, xref, uref, FullSpec(N=N, **kw), p)
    tol = 1e-9 if not box else 1e-7
    assert (m.get_status().cpu().numpy() == o['status']).all()
    assert relerr(m.get_control().cpu().numpy(), o['u0']).max() <= tol
    assert relerr(m.get_state_trajectory().cpu().numpy(), o['X']).max() <= tol
    assert relerr(m.get_input_trajectory().cpu().numpy(), o['U']).max() <= tol


def test_solve17_fp32_close_to_fp64_oracle():
    N, B = 20, 16
    m = _mpc(N, 'f32', max_batch=B)
    x0, xref, uref, p = _inputs(B, N, 21)
    m.set_params(p)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    o = mpc_solve17(x0, xref, uref, FullSpec(N=N), p)
    e = relerr(m.get_control().cpu().numpy(), o['u0']).max()
    print(f'17/6 fp32 u0 err {e:.2e}')
    assert e <= 5e-4


@pytest.mark.parametrize('states_bound', [False, True])
def test_acados_facade_full_model_runs_reference_loop(states_bound):
    """simulation_blaster.py:56-107 through the compat facade on the FULL 17/6 model
    (blasterModel(..., full_model=True), the reference's controlBound enforced): set(0,'lbx'/'ubx'),
    set(k,'p'), cost_set(k,'yref'), solve(), get(0,'u'), then the plant integrator — against the
    oracle's SQP_RTI iterate."""
    import warnings
    from mpc_blaster_amd.compat.blastermodel import blasterModel
    J = np.diag([0.50781, 0.47314, 0.72975])
    Q = np.diag([1e3] * 6 + [5.0] * 3 + [10.0] * 3 + [1e-2] * 2 + [1e3] * 3)
    R = np.diag([5e-2] * 4 + [1e-5] * 2)
    N = 12
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        b = blasterModel(9.0, J, 0.3434, 0.3475, N, N / 30.0, 0.03, Q, R, 10 * Q, 2.2,
                         np.stack([SB_LO, SB_HI]) if states_bound else np.full((2, 17), np.nan),
                         np.stack([LBU17, UBU17]), full_model=True)
        b.generateModel()
        integrator, ocp_solver = b.generateController()
    rng = np.random.default_rng(4)
    p = default_p25()
    p[:24] = rng.uniform(-0.3, 0.3, 24)
    x = np.zeros(17)
    x[2] = 3.0
    yref = np.zeros(23)
    yref[2], yref[14] = 3.5, 0.2                      # simulation_blaster.py:48
    spec = FullSpec(N=N, lbu=LBU17, ubu=UBU17)          # controlBound (simulation_blaster.py:30)
    if states_bound:                                    # statesBound (simulation_blaster.py:28-29)
        spec = FullSpec(N=N, lbu=LBU17, ubu=UBU17, lbx=SB_LO, ubx=SB_HI)
    tol = 1e-7 if states_bound else 1e-9
    xbar, ubar = np.zeros((1, N + 1, 17)), np.zeros((1, N, 6))
    xr = np.broadcast_to(yref[:17], (1, N + 1, 17))
    ur = np.zeros((1, N, 6))
    for j in range(N + 1):
        ocp_solver.set(j, 'p', p)                     # simulation_blaster.py:69
    integrator.set('p', p)
    for i in range(4):
        ocp_solver.set(0, 'lbx', x)
        ocp_solver.set(0, 'ubx', x)
        for k in range(N + 1):
            ocp_solver.cost_set(k, 'yref', yref if k < N else yref[:17])
        assert ocp_solver.solve() == 0
        u = ocp_solver.get(0, 'u')
        o = mpc_solve17(x[None], xr, ur, spec, p[None], mode='iterate', xbar=xbar, ubar=ubar)
        xbar, ubar = o['X'], o['U']
        assert o['status'][0] == 0
        assert relerr(u[None], o['u0']).max() < tol
        assert relerr(ocp_solver.get(N, 'x')[None], o['X'][:, N]).max() < tol
        integrator.set('x', x)
        integrator.set('u', u)
        assert integrator.solve() == 0
        xn = integrator.get('x')
        ref = rk4_step17(x[None], u[None], p[None], 1.0 / 30.0, Params())[0]
        assert np.abs(xn - ref).max() < 1e-11
        x = xn



@pytest.mark.parametrize('mode', ['rollout', 'iterate'])
def test_solve17_input_box_matches_oracle_interior_point(mode):
    """The reference's input box on the full model by the interior point: the device iterate
    equals the oracle's (same iteration, <= 1e-9; achieved ~1e-13) and both match an independent dense box-QP solve (SciPy BVLS on the condensed
    problem, <= 1e-5: its own accuracy on this ill-conditioned Hessian)."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle.ocp import dense_box_qp
    N, B = 20, 24
    m = BatchedMPC(MPCConfig.full(N=N, lbu=LBU17, ubu=UBU17), max_batch=B)
    x0, xref, uref, p = _inputs(B, N, 31)
    m.set_params(p)
    spec = FullSpec(N=N, lbu=LBU17, ubu=UBU17)
    kw = {}
    if mode == 'iterate':
        rng = np.random.default_rng(32)
        kw = dict(xbar=x0[:, None, :] + rng.normal(0, 0.05, (B, N + 1, 17)),
                  ubar=uref + rng.normal(0, 0.5, (B, N, 6)))
        m.solve_iterate(x0, kw['xbar'], kw['ubar'], xref, uref)
    else:
        m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    o = mpc_solve17(x0, xref, uref, spec, p, mode=mode, **kw)
    assert (o['status'] == 0).all()
    assert (m.get_status().cpu().numpy() == 0).all()
    U = m.get_input_trajectory().cpu().numpy()
    assert (U >= LBU17 - 1e-9).all() and (U <= UBU17 + 1e-9).all()
    act = np.isclose(o['U'], LBU17, atol=1e-6) | np.isclose(o['U'], UBU17, atol=1e-6)
    assert act.any()                                   # the box is active somewhere
    e = [relerr(m.get_control().cpu().numpy(), o['u0']).max(),
         relerr(m.get_state_trajectory().cpu().numpy(), o['X']).max(), relerr(U, o['U']).max()]
    dd = dense_box_qp(o['A'], o['B'], o['gap'], x0 - o['xbar'][:, 0], o['xbar'], o['ubar'],
                      np.broadcast_to(xref, (B, N + 1, 17)), np.broadcast_to(uref, (B, N, 6)), spec)
    eb = relerr(U - o['ubar'], dd).max()
    print(f'17/6 box fp64 {mode}: u0 {e[0]:.2e} X {e[1]:.2e} U {e[2]:.2e} vs oracle, {eb:.2e} vs BVLS; '
          f'{act.mean():.1%} of (k, m) at a bound, oracle iterations max {o["iters"].max()}')
    assert max(e) <= 1e-9
    assert eb <= 1e-5


def _sbox_inputs(B, N, seed):
    """x0 inside a quarter of the reference's state box (tests/golden/ocp_json_pin.json)."""
    import json
    d = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'ocp_json_pin.json')))
    lbx, ubx = np.array(d['lbx']), np.array(d['ubx'])
    x0, xref, uref, p = _inputs(B, N, seed)
    rng = np.random.default_rng(seed + 1)
    x0 = rng.uniform(0.25 * lbx, 0.25 * ubx, (B, 17))
    x0[:, 2] = 3.5 + rng.uniform(-0.5, 0.5, B)
    return x0, xref, uref, p, lbx, ubx


@pytest.mark.parametrize('mode', ['rollout', 'iterate'])
def test_solve17_state_box_matches_oracle_interior_point(mode):
    """The reference's state box (JSON idxbx, stages 1..N-1) with its input box: the device
    interior point and its active-set polish (oracle.ocp.al_polish) equal the oracle's (<= 1e-9:
    the polished point is the exact solution of the equality-constrained QP on the active set, so
    the two no longer differ by where each interior point stopped) and carry a KKT certificate of
    the condensed QP (oracle.ocp.dense_kkt_certificate: NNLS multipliers >= 0, stationarity,
    feasibility, and a duality gap that bounds the suboptimality)."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle.ocp import dense_kkt_certificate
    N, B = 20, 24
    x0, xref, uref, p, lbx, ubx = _sbox_inputs(B, N, 41)
    m = BatchedMPC(MPCConfig.full(N=N, lbu=LBU17, ubu=UBU17, lbx=lbx, ubx=ubx), max_batch=B)
    m.set_params(p)
    spec = FullSpec(N=N, lbu=LBU17, ubu=UBU17, lbx=lbx, ubx=ubx)
    kw = {}
    if mode == 'iterate':
        rng = np.random.default_rng(42)
        kw = dict(xbar=x0[:, None, :] + rng.normal(0, 0.01, (B, N + 1, 17)),
                  ubar=uref + rng.normal(0, 0.5, (B, N, 6)))
        m.solve_iterate(x0, kw['xbar'], kw['ubar'], xref, uref)
    else:
        m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    o = mpc_solve17(x0, xref, uref, spec, p, mode=mode, **kw)
    assert (o['status'] == 0).all()
    assert (m.get_status().cpu().numpy() == 0).all()
    X = m.get_state_trajectory().cpu().numpy()
    U = m.get_input_trajectory().cpu().numpy()
    assert (X[:, 1:N] >= lbx - 1e-9).all() and (X[:, 1:N] <= ubx + 1e-9).all()
    n_act = ((o['X'][:, 1:N] - lbx < 1e-6) | (ubx - o['X'][:, 1:N] < 1e-6)).sum()
    assert n_act >= B * 5                              # the state box is active
    e = [relerr(m.get_control().cpu().numpy(), o['u0']).max(), relerr(X, o['X']).max(), relerr(U, o['U']).max()]
    stat, viol, gap = dense_kkt_certificate(o['A'], o['B'], o['gap'], x0 - o['xbar'][:, 0], o['xbar'], o['ubar'],
                                            np.broadcast_to(xref, (B, N + 1, 17)),
                                            np.broadcast_to(uref, (B, N, 6)), spec, U - o['ubar'], lbx=lbx, ubx=ubx)
    print(f'17/6 state box fp64 {mode}: u0 {e[0]:.2e} X {e[1]:.2e} U {e[2]:.2e} vs oracle; KKT certificate: '
          f'stationarity {stat.max():.1e} violation {viol.max():.1e} duality gap {gap.max():.1e}; '
          f'{n_act} active state rows, oracle iterations max {o["iters"].max()}')
    assert max(e) <= 1e-9
    assert stat.max() <= 1e-10 and viol.max() <= 1e-10 and gap.max() <= 1e-5
    # the kernel's own count of interior-point iterations and polish passes (mpcb_qp_stats)
    qs = m.qp_stats(B).cpu().numpy()
    print(f'   device iterations {qs[:, 0].tolist()} oracle {o["iters"].tolist()}; polish passes {qs[:, 1].tolist()}')
    assert (np.abs(qs[:, 0] - o['iters']) <= 1).all() and (qs[:, 1] >= 1).all()


def test_solve17_state_box_infeasible_instances_flagged():
    """x0 over the whole rate range: some state-box QPs have no feasible point (an LP says so).
    The device flags exactly those with MPCB_STATUS_QP_FAIL, as the oracle does, and solves the
    rest as the oracle does."""
    import json
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle.ocp import lp_box_feasible
    d = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'ocp_json_pin.json')))
    lbx, ubx = np.array(d['lbx']), np.array(d['ubx'])
    N, B = 20, 64
    x0, xref, uref, p = _inputs(B, N, 77)
    m = BatchedMPC(MPCConfig.full(N=N, lbu=LBU17, ubu=UBU17, lbx=lbx, ubx=ubx), max_batch=B)
    m.set_params(p)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    spec = FullSpec(N=N, lbu=LBU17, ubu=UBU17, lbx=lbx, ubx=ubx)
    with np.errstate(all='ignore'):
        o = mpc_solve17(x0, xref, uref, spec, p)
    st = m.get_status().cpu().numpy()
    feas = lp_box_feasible(o['A'], o['B'], o['gap'], x0 - o['xbar'][:, 0], o['xbar'], o['ubar'], spec, lbx, ubx)
    print(f'17/6 state box: {int((~feas).sum())} of {B} infeasible; device status {np.bincount(st)}')
    assert (~feas).any() and feas.sum() >= B // 2
    assert np.array_equal(st == 0, feas) and np.array_equal(o['status'] == 0, feas)
    assert (st[~feas] == 4).all()
    # the feasible ones: the polish takes both interior points (which stop up to an iteration apart
    # at the conditioning limit on near-degenerate instances: 2.3e-5 apart in u0 before it) to the
    # same exact active-set solution
    from oracle.ocp import dense_kkt_certificate
    ok = feas
    U = m.get_input_trajectory().cpu().numpy()
    e_u0 = relerr(m.get_control().cpu().numpy()[ok], o["u0"][ok]).max()
    e_U = relerr(U[ok], o['U'][ok]).max()
    print(f"feasible instances: u0 vs oracle {e_u0:.2e}, U {e_U:.2e}")
    assert e_u0 <= 1e-8 and e_U <= 1e-8
    stat, viol, gap = dense_kkt_certificate(o['A'][ok], o['B'][ok], o['gap'][ok], (x0 - o['xbar'][:, 0])[ok],
                                            o['xbar'][ok], o['ubar'][ok], np.broadcast_to(xref, (B, N + 1, 17))[ok],
                                            np.broadcast_to(uref, (B, N, 6))[ok], spec, (U - o['ubar'])[ok],
                                            lbx=lbx, ubx=ubx)
    # (gap bounds f(z) - f*; the objectives are ~1e3 here, so 1e-4 is 1e-7 relative)
    assert stat.max() <= 1e-10 and viol.max() <= 1e-10 and gap.max() <= 1e-4, (stat.max(), viol.max(), gap.max())


def test_full17_phase_timing_events():
    """mpcb_set_timing / mpcb_last_timing on the 17/6 path: nominal17, riccati17, lin17ws device
    ms from HIP events, and timing changes no result."""
    N, B = 12, 16
    m = _mpc(N, max_batch=B)
    x0, xref, uref, p = _inputs(B, N, 5)
    m.set_params(p)
    a = m.solve(x0, xref, uref).clone()
    m.set_timing(True)
    b = m.solve(x0, xref, uref)
    t = m.last_timing()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert t['nominal'] > 0 and t['riccati'] > 0 and t['linearise'] > 0


def test_solve17_fp32_input_box_close_to_fp64_oracle():
    """fp32 interior point on the input box (tolerances scaled to fp32: mu <= 1e-6, residual
    <= 1e-5): every instance converges and u0 stays within 1e-3 (relative to max(1, |u|)) of
    the fp64 oracle.  The state box needs fp64 (mpcb_create refuses it in fp32)."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig, _lib
    N, B = 20, 24
    x0, xref, uref, p = _inputs(B, N, 31)
    m = BatchedMPC(MPCConfig.full(N=N, dtype='f32', lbu=LBU17, ubu=UBU17), max_batch=B)
    m.set_params(p)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    o = mpc_solve17(x0, xref, uref, FullSpec(N=N, lbu=LBU17, ubu=UBU17), p)
    assert (o['status'] == 0).all()
    st = m.get_status().cpu().numpy()
    e = relerr(m.get_control().cpu().numpy().astype(np.float64), o['u0']).max()
    print(f'17/6 fp32 input box: u0 err {e:.2e}, status {np.bincount(st)}')
    assert (st == 0).all()
    assert e <= 1e-3
    with pytest.raises(_lib.MpcbError, match='f64'):
        BatchedMPC(MPCConfig.full(N=N, dtype='f32', lbu=LBU17, ubu=UBU17, lbx=-np.ones(17), ubx=np.ones(17)),
                   max_batch=B)


def _reference_blaster_model(**kw):
    """blasterModel(...) with simulation_blaster.py:12-30's exact arguments (N = 60, Tf = 2,
    blastThruster = 2.2 * 9.81, statesBound, controlBound) on the full model."""
    from mpc_blaster_amd.compat.blastermodel import blasterModel
    J = np.eye(3)
    J[0, 0], J[1, 1], J[2, 2] = 0.50781, 0.47314, 0.72975
    Q = np.zeros((17, 17))
    np.fill_diagonal(Q, [1e3, 1e3, 1e3, 1e3, 1e3, 1e3, 0.5e1, 0.5e1, 0.5e1, 1e1, 1e1, 1e1, 1e-2, 1e-2,
                         1e3, 1e3, 1e3])
    R = np.zeros((6, 6))
    np.fill_diagonal(R, [5e-2, 5e-2, 5e-2, 5e-2, 1e-5, 1e-5])
    return blasterModel(9.0, J, 0.3434, 0.3475, 60, 2.0, 0.03, Q, R, 10 * Q, 2.2 * 9.81,
                        np.stack([SB_LO, SB_HI]), np.stack([LBU17, UBU17]), full_model=True, **kw)


def test_facade_reference_arguments_default_then_stage_varying_p():
    """The reference's own constructor arguments: the first solve runs before any set('p') on
    acados' default parameter vector (T_blast = 2.2*9.81 whatever blastThruster is,
    blastermodel.py:280-282), the second with a different p on every stage (set(k, 'p') per
    stage, simulation_blaster.py:65-69) — both against the oracle's SQP_RTI iterate."""
    b = _reference_blaster_model()
    b.generateModel()
    assert b._cfg.t_blast == pytest.approx(21.582, rel=1e-15)
    integrator, ocp = b.generateController()
    N = 60
    spec = FullSpec(N=N, lbu=LBU17, ubu=UBU17, lbx=SB_LO, ubx=SB_HI)
    x = np.zeros(17)                                      # simulation_blaster.py:46
    yref = np.zeros(23)
    yref[2], yref[14] = 3.5, 0.2                          # simulation_blaster.py:48
    xr = np.broadcast_to(yref[:17], (1, N + 1, 17))
    ur = np.zeros((1, N, 6))
    rng = np.random.default_rng(11)
    pk = np.tile(default_p25(), (N, 1))
    pk[:, :24] = rng.uniform(-0.3, 0.3, (N, 24))
    xbar, ubar = np.zeros((1, N + 1, 17)), np.zeros((1, N, 6))
    for it in range(2):
        if it == 1:
            for k in range(N):
                ocp.set(k, 'p', pk[k])
        ocp.set(0, 'lbx', x)
        ocp.set(0, 'ubx', x)
        for k in range(N + 1):
            ocp.cost_set(k, 'yref', yref if k < N else yref[:17])
        assert ocp.solve() == 0
        o = mpc_solve17(x[None], xr, ur, spec, None if it == 0 else pk[None], mode='iterate',
                        xbar=xbar, ubar=ubar)
        xbar, ubar = o['X'], o['U']
        assert o['status'][0] == 0
        eu = relerr(ocp.get(0, 'u')[None], o['u0']).max()
        ex = relerr(np.stack([ocp.get(k, 'x') for k in range(N + 1)])[None], o['X']).max()
        print(f'solve {it}: u0 err {eu:.2e}, X err {ex:.2e}')
        assert eu < 1e-7 and ex < 1e-7


def test_set_params_rows_checked_against_batch():
    """A solve / linearize / sim_step over more instances than the parameter rows is refused
    (no out-of-bounds device read); broadcast rows (one vector) serve any batch."""
    from mpc_blaster_amd._lib import MpcbError
    N, B = 6, 5
    x0, xref, uref, p = _inputs(B, N, 3)
    m = _mpc(N, max_batch=B)
    m.set_params(p[:2])
    with pytest.raises(MpcbError, match='parameter rows'):
        m.solve(x0, xref, uref)
    with pytest.raises(MpcbError, match='parameter rows'):
        m.sim_step(x0, uref[:, 0])
    m.set_params(p[:1])
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    o = mpc_solve17(x0, xref, uref, FullSpec(N=N), p[:1])
    assert relerr(m.get_control().cpu().numpy(), o['u0']).max() < 1e-9


def test_set_t_blast_updates_default_parameter_in_place():
    N, B = 8, 4
    x0, xref, uref, _ = _inputs(B, N, 5)
    m = _mpc(N, max_batch=B)
    h = m._h.value
    m.set_t_blast(15.0)
    assert m._h.value == h
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    p = default_p25()
    p[24] = 15.0
    o = mpc_solve17(x0, xref, uref, FullSpec(N=N), p[None])
    assert relerr(m.get_control().cpu().numpy(), o['u0']).max() < 1e-9


def test_full_size_17_input_box_properties():
    """The reference OCP at its own horizon (N = 60) with the input box, 4096 instances (the
    tools/bench_full17.py size): every status OK, every input inside the box, the interior point's
    u0 equal to the oracle's on a sample of instances."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    N, B = 60, 4096
    x0, xref, uref, p = _inputs(B, N, 2026)
    m = BatchedMPC(MPCConfig.full(N=N, lbu=LBU17, ubu=UBU17), max_batch=B)
    m.set_params(p)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    st = m.get_status().cpu().numpy()
    U = m.get_input_trajectory().cpu().numpy()
    assert (st == 0).all(), np.bincount(st)
    assert (U >= LBU17 - 1e-9).all() and (U <= UBU17 + 1e-9).all()
    idx = np.arange(0, B, 257)
    o = mpc_solve17(x0[idx], xref[idx], uref[idx], FullSpec(N=N, lbu=LBU17, ubu=UBU17), p[idx])
    assert (o['status'] == 0).all()
    e = relerr(m.get_control().cpu().numpy()[idx], o['u0']).max()
    print(f'17/6 input box N=60 B=4096: sampled u0 vs oracle {e:.2e}, oracle iterations max {o["iters"].max()}')
    assert e <= 1e-7


def test_solve17_state_box_thin_interior_instance_converges():
    """LP-feasible state-box QPs whose Riccati recursion loses positive definiteness before
    mu = 1e-8 (tests/golden/sbox_thin_interior.npz, tools/make_sbox_fixture.py; lambda / s ~ 1e16
    on strongly active rows).  Both interior points stop at that limit (the device on the second
    instance one iteration before the oracle: mu 1.3e-6 against 6.6e-8, u0 2.4e-5 apart); the
    polish then identifies the active set and both end at its exact solution, with a KKT
    certificate."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle.ocp import dense_kkt_certificate
    d = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'sbox_thin_interior.npz'))
    lbx, ubx = d['lbx'], d['ubx']
    x0, p = d['x0'], d['p']
    N, B = int(d['N']), x0.shape[0]
    xref = np.zeros((1, N + 1, 17))
    xref[..., 2], xref[..., 14] = 3.5, 0.2
    uref = np.zeros((1, N, 6))
    uref[..., :4] = 22.0725
    m = BatchedMPC(MPCConfig.full(N=N, lbu=LBU17, ubu=UBU17, lbx=lbx, ubx=ubx), max_batch=B)
    m.set_params(p)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    spec = FullSpec(N=N, lbu=LBU17, ubu=UBU17, lbx=lbx, ubx=ubx)
    with np.errstate(all='ignore'):
        o = mpc_solve17(x0, xref, uref, spec, p)
    st = m.get_status().cpu().numpy()
    U = m.get_input_trajectory().cpu().numpy()
    e = relerr(m.get_control().cpu().numpy(), o['u0']).max()
    stat, viol, gap = dense_kkt_certificate(o['A'], o['B'], o['gap'], x0 - o['xbar'][:, 0], o['xbar'], o['ubar'],
                                            np.broadcast_to(xref, (B, N + 1, 17)), np.broadcast_to(uref, (B, N, 6)),
                                            spec, U - o['ubar'], lbx=lbx, ubx=ubx)
    print(f'17/6 thin-interior state box: device status {st}, oracle {o["status"]} after {o["iters"]} iterations; '
          f'u0 {e:.2e} vs oracle; KKT stationarity {stat.max():.1e} violation {viol.max():.1e} gap {gap.max():.1e}')
    assert (o['status'] == 0).all() and (st == 0).all()
    assert e <= 1e-7   # north_star 1e-5; measured 4.6e-9
    assert stat.max() <= 1e-10 and viol.max() <= 1e-10 and gap.max() <= 1e-5   # (gap: objective ~1e3)


def test_closed_loop17_reference_ocp_matches_oracle():
    """The receding-horizon loop of simulation_blaster.py:56-107 on the reference's own OCP
    (acados_ocp_blasterModel.json: 17/6, N = 60, input box and state box, the JSON's parameters),
    batched: B = 64 instances, 20 steps of SQP_RTI from the persistent iterate plus the plant step,
    all on the device (mpc_blaster_amd.closed_loop) against the oracle's loop
    (tests/golden/loop17_ref.npz, tools/make_loop17_fixture.py) at <= 1e-5 per step (north_star)."""
    import warnings
    from mpc_blaster_amd import BatchedMPC, load_acados_ocp_json
    from mpc_blaster_amd.closed_loop import closed_loop
    d = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'loop17_ref.npz'))
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        cfg, info = load_acados_ocp_json(os.path.join(os.path.dirname(__file__), 'golden', 'ocp_json_pin.json'))
    x0, nsim = d['x0'], int(d['nsim'])
    B, N = x0.shape[0], cfg.N
    m = BatchedMPC(cfg, max_batch=B)
    m.set_params(np.tile(d['p'], (B, 1)))
    xr = np.broadcast_to(d['xref'], (1, N + 1, 17))
    ur = np.broadcast_to(d['uref'], (1, N, 6))
    Xs, Us, st = closed_loop(m, x0, xr, ur, nsim)
    torch.cuda.synchronize()
    Xs, Us, st = Xs.cpu().numpy(), Us.cpu().numpy(), st.cpu().numpy()
    eu = max(relerr(Us[:, i], d['Us'][:, i]).max() for i in range(nsim))
    ex = max(relerr(Xs[:, i], d['Xs'][:, i]).max() for i in range(nsim + 1))
    print(f'17/6 closed loop B={B} x {nsim} steps: u0 {eu:.2e} x {ex:.2e} vs oracle; statuses '
          f'{np.bincount(d["status"].ravel(), minlength=5)} (oracle, all steps)')
    assert np.array_equal(st, d['status'].max(axis=1))
    assert eu <= 1e-5 and ex <= 1e-5
