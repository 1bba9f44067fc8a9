"""GPU checks of the smaller SURVEY §8 rows through the C ABI:

* f4  — a solve from the reference's own OCP description (``load_acados_ocp_json`` on
  tests/golden/ocp_json_pin.json = acados_ocp_blasterModel.json) vs ``oracle.full.mpc_solve17``;
* c   — the committed oracle fixture ``mpc_small.npz`` (8 instances each of c2, c3, c4 at fp64)
  reproduced by the device;
* a10 — the device quaternion helpers (``mpcb_quat_ops``) vs ``mathutils_ref.npz``, the
  values the reference's own ``utils/MathUtils.py`` produced (tools/gen_golden.py).

Tolerances: fp64 per-instance ||y_dev - y_ref||_inf / max(||y_ref||_inf, 1) <= 1e-9 (north_star
asks 1e-5); the quaternion helpers <= 1e-14 absolute (a handful of fp64 products)."""
import os
import warnings

import numpy as np
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def relerr(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, dtype=np.float64).reshape(b.shape[0], -1)
    return np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1.0)


def test_solve_from_reference_json_matches_oracle():
    """f4 end to end: MPCConfig from the reference JSON (17/6, N = 60, input box idxbu and state box
    idxbx on stages 1..N-1, default parameters with T_blast = 2.2*9.81, qp_solver_iter_max 500),
    stage references = the JSON's yref, near-hover initial states inside the state box."""
    from mpc_blaster_amd import BatchedMPC, load_acados_ocp_json
    from oracle.full import FullSpec, mpc_solve17
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        cfg, info = load_acados_ocp_json(os.path.join(GOLD, 'ocp_json_pin.json'))
    assert cfg.lbx is not None and cfg.lbu is not None and cfg.max_as_iter == 500
    B, N = 8, cfg.N
    rng = np.random.default_rng(2026)
    yref = info['yref']
    x0 = np.tile(yref[:17], (B, 1))
    x0[:, 2] = 3.0
    x0[:, 0:3] += rng.uniform(-0.3, 0.3, (B, 3))
    x0[:, 3:6] += rng.uniform(-0.05, 0.05, (B, 3))
    x0[:, 6:9] += rng.uniform(-0.2, 0.2, (B, 3))
    x0[:, 9:12] += rng.uniform(-0.02, 0.02, (B, 3))
    xref = np.broadcast_to(np.where(np.arange(17) == 2, 3.5, yref[:17]), (B, N + 1, 17)).copy()
    uref = np.broadcast_to(np.r_[np.full(4, 22.0725), yref[21:23]], (B, N, 6)).copy()
    m = BatchedMPC(cfg, max_batch=B)
    m.set_params(None)                      # the JSON parameter_values (p[24] = T_blast)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    spec = FullSpec(N=N, dt=cfg.dt, Q=cfg.Q, R=cfg.R, QN=cfg.QN, lbu=cfg.lbu, ubu=cfg.ubu,
                    lbx=cfg.lbx, ubx=cfg.ubx, max_as_iter=cfg.max_as_iter)
    o = mpc_solve17(x0, xref, uref, spec, np.tile(info['p'], (B, 1)))
    st = m.get_status().cpu().numpy()
    assert (o['status'] == 0).all() and (st == 0).all()
    e = [relerr(m.get_control().cpu().numpy(), o['u0']).max(),
         relerr(m.get_state_trajectory().cpu().numpy(), o['X']).max(),
         relerr(m.get_input_trajectory().cpu().numpy(), o['U']).max()]
    print(f'JSON-loaded 17/6 boxed solve: u0 {e[0]:.2e} X {e[1]:.2e} U {e[2]:.2e}')
    assert max(e) <= 1e-6          # interior point stopped at mu <= 1e-12 (the state-box bound)


@pytest.mark.parametrize('cfg', ['c2', 'c3', 'c4'])
def test_mpc_small_fixture(cfg):
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    d = np.load(os.path.join(GOLD, 'mpc_small.npz'))
    x0, xref, uref = d[f'{cfg}_x0'], d[f'{cfg}_xref'], d[f'{cfg}_uref']
    B, N = x0.shape[0], uref.shape[1]
    box = cfg == 'c4'
    m = BatchedMPC(MPCConfig(N=N, dtype='f64', lbu=np.zeros(4) if box else None,
                             ubu=np.full(4, 65.0) if box else None), max_batch=B)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    assert np.array_equal(m.get_status().cpu().numpy(), d[f'{cfg}_status'])
    assert relerr(m.get_control().cpu().numpy(), d[f'{cfg}_u0']).max() <= 1e-9
    assert relerr(m.get_state_trajectory().cpu().numpy(), d[f'{cfg}_X']).max() <= 1e-9
    assert relerr(m.get_input_trajectory().cpu().numpy(), d[f'{cfg}_U']).max() <= 1e-9


def test_quat_ops_match_reference_mathutils():
    from mpc_blaster_amd import mathutils
    d = np.load(os.path.join(GOLD, 'mathutils_ref.npz'))
    prod = mathutils.quat_multiply(d['q1'], d['q2']).cpu().numpy()
    inv = mathutils.unit_quat_inverse(d['q1']).cpu().numpy()
    rot = mathutils.quat_to_rot(d['q1']).cpu().numpy()
    assert np.abs(prod - d['prod']).max() <= 1e-14
    assert np.abs(inv - d['inv']).max() == 0.0
    assert np.abs(rot - d['rot']).max() <= 1e-14
    # a single quaternion and a [2, 3, 4] batch keep their leading shape
    assert mathutils.quat_to_rot(d['q1'][0]).shape == (3, 3)
    assert mathutils.quat_multiply(d['q1'][:6].reshape(2, 3, 4), d['q2'][:6].reshape(2, 3, 4)).shape == (2, 3, 4)
