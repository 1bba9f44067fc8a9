"""Oracle OCP/QP checks: JSON pin, Riccati vs dense QP, PDAS vs independent BVLS, KKT."""
import json
import os

import numpy as np
import pytest

from oracle.inputs import make_inputs, CONFIGS
from oracle.ocp import OcpSpec, dense_box_qp, default_Q, default_R, mpc_solve, stage_cost

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def test_ocp_definition_pinned_to_reference_json():
    pin = json.load(open(os.path.join(GOLD, 'ocp_json_pin.json')))
    cap = json.load(open(os.path.join(GOLD, 'ocp_capture.json')))
    W = np.asarray(pin['W'])
    # 12/4 slice of the JSON-pinned weights is what OcpSpec defaults to
    assert np.allclose(np.diag(W)[:12], np.diag(default_Q()))
    assert np.allclose(np.diag(W)[17:21], np.diag(default_R()))
    assert np.allclose(np.asarray(pin['W_e']), 10 * np.asarray(pin['W'])[:17, :17])
    so = pin['solver_options']
    assert so['integrator_type'] == 'ERK' and set(so['sim_method_num_stages']) == {4}
    assert set(so['sim_method_num_steps']) == {1}
    assert so['nlp_solver_type'] == 'SQP_RTI' and so['hessian_approx'] == 'GAUSS_NEWTON'
    assert so['globalization'] == 'FIXED_STEP' and so['nlp_solver_step_length'] == 1.0
    assert np.allclose(so['time_steps'], 1.0 / 30.0) and so['tf'] == 2.0
    assert pin['lbu'][:4] == [0.0] * 4 and pin['ubu'][:4] == [65.0] * 4
    assert abs(pin['parameter_values'][24] - 2.2 * 9.81) < 1e-12
    # the OCP the reference code builds equals its serialized JSON
    for key in ('W', 'W_e', 'lbu', 'ubu', 'lbx', 'ubx'):
        assert np.allclose(np.asarray(cap[key]), np.asarray(pin[key]))
    assert cap['qp_solver'] == 'PARTIAL_CONDENSING_HPIPM' and cap['qp_solver_cond_N'] == 60


@pytest.mark.parametrize('cfg,N', [('c1', 10), ('c2', 20), ('c3', 20)])
def test_riccati_equals_dense_qp(cfg, N):
    inp = make_inputs(cfg, ids=np.arange(3, dtype=np.uint64))
    spec = OcpSpec(N=N)
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, return_lin=True)
    big = OcpSpec(N=N, lbu=np.full(4, -1e9), ubu=np.full(4, 1e9))
    du = dense_box_qp(o['A'], o['B'], o['gap'], np.zeros((3, 12)), o['xbar'], o['ubar'],
                      inp['xref'], inp['uref'], big)
    U = o['ubar'] + du
    assert np.abs(U - o['U']).max() <= 1e-7 * np.abs(o['U']).max()


def test_pdas_equals_bvls_box_qp():
    inp = make_inputs('c4', ids=np.arange(6, dtype=np.uint64))
    spec = OcpSpec(N=30, lbu=np.zeros(4), ubu=np.full(4, 65.0))
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, return_lin=True)
    assert (o['status'] == 0).all()
    du = dense_box_qp(o['A'], o['B'], o['gap'], np.zeros((6, 12)), o['xbar'], o['ubar'],
                      inp['xref'], inp['uref'], spec)
    assert np.abs(o['ubar'] + du - o['U']).max() < 1e-6
    assert (o['U'] >= -1e-12).all() and (o['U'] <= 65 + 1e-12).all()
    # bounds are genuinely active in this config
    assert ((o['U'] == 0.0) | (o['U'] == 65.0)).any()


def test_optimality_gn_step_is_descent_on_lq_model():
    # perturbing the returned controls can only raise the LQ objective (strict convexity)
    inp = make_inputs('c2', ids=np.arange(2, dtype=np.uint64))
    spec = OcpSpec(N=20)
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, return_lin=True)
    base = stage_cost(o['X'], o['U'], inp['xref'], inp['uref'], spec)
    rng = np.random.default_rng(3)
    for _ in range(5):
        dU = rng.normal(scale=0.5, size=o['U'].shape)
        dX = np.zeros_like(o['X'])
        for k in range(20):
            dX[:, k + 1] = np.einsum('bij,bj->bi', o['A'][:, k], dX[:, k]) + np.einsum('bij,bj->bi', o['B'][:, k], dU[:, k])
        c = stage_cost(o['X'] + dX, o['U'] + dU, inp['xref'], inp['uref'], spec)
        assert (c > base).all()


def test_golden_c1_reproduces():
    d = np.load(os.path.join(GOLD, 'mpc_c1.npz'))
    o = mpc_solve(d['x0'], d['xref'], d['uref'], OcpSpec(N=10))
    assert np.allclose(o['X'], d['X'], rtol=1e-12, atol=1e-12)
    assert np.allclose(o['u0'], d['u0'], rtol=1e-12, atol=1e-12)


def test_inputs_reproducible_per_instance():
    a = make_inputs('c3', ids=np.arange(10, dtype=np.uint64))
    b = make_inputs('c3', ids=np.arange(5, 10, dtype=np.uint64))
    assert np.array_equal(a['x0'][5:], b['x0'])
    assert np.array_equal(a['xref'][5:], b['xref'])
    assert CONFIGS['c5']['batch'] == 1048576


def hard_box_inputs(B, N, seed):
    """Input-box draws on which the active set's backup rule is slow: sine references plus a
    +-5 N wind per instance (tests/test_gpu_edges.py uses the same draws on the device)."""
    inp = make_inputs('c3', ids=np.arange(B, dtype=np.uint64) + np.uint64(seed), N=N)
    inp['wind'] = 5.0 * (2.0 * np.random.default_rng(seed).random((B, 3)) - 1.0)
    return inp


def test_pdas_hands_slow_instances_to_the_interior_point():
    """oracle.ocp.pdas_solve's fallback: instances still unconverged after AS_IPM_AFTER passes are
    solved by the interior point; they end OK and agree with the independent BVLS solve."""
    from oracle.ocp import AS_IPM_AFTER
    N, B = 18, 192
    inp = hard_box_inputs(B, N, 11)
    spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0))
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, wind=inp['wind'], return_lin=True)
    assert (o['status'] == 0).all()
    fb = np.nonzero(o['iters'] > AS_IPM_AFTER)[0]
    assert len(fb) >= 5   # the draw has slow instances
    sel = fb[:6]
    du = dense_box_qp(o['A'][sel], o['B'][sel], o['gap'][sel], np.zeros((len(sel), 12)), o['xbar'][sel],
                      o['ubar'][sel], inp['xref'][sel], inp['uref'][sel], spec)
    assert np.abs(o['ubar'][sel] + du - o['U'][sel]).max() < 1e-5
    assert (o['U'] >= -1e-9).all() and (o['U'] <= 65 + 1e-9).all()
