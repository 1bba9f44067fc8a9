"""Oracle dynamics vs golden vectors produced by the reference's own generateModel()."""
import json
import os

import numpy as np
import pytest

from oracle.model import Params, f12, f17, jac12, euler_rate_inv
from oracle.rk4 import rk4_sens, rk4_step

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def dyn():
    return np.load(os.path.join(GOLD, 'dynamics_ref17.npz'))


def _params(d, t):
    return Params(mass=float(d[t + '_mass']), J=d[t + '_J'], lx=float(d[t + '_lx']),
                  ly=float(d[t + '_ly']), c=float(d[t + '_c']))


@pytest.mark.parametrize('tag', ['sim', 'main'])
def test_f17_matches_reference_generateModel(dyn, tag):
    P = _params(dyn, tag)
    F = f17(dyn[tag + '_x'], dyn[tag + '_u'], dyn[tag + '_p'], P)
    ref = dyn[tag + '_f']
    assert np.abs(F - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize('tag', ['sim', 'main'])
def test_f12_is_exact_slice_of_reference(dyn, tag):
    P = _params(dyn, tag)
    x, u, p = dyn[tag + '_x'], dyn[tag + '_u'], dyn[tag + '_p']
    for i in range(x.shape[0]):
        P.t_blast = float(p[i, 24])
        x17 = x[i].copy()
        x17[12:14] = 0.0  # alpha = 0 slice
        ref = f17(x17[None], u[i][None], p[i][None], P)[0]
        got = f12(x[i, :12][None], u[i, :4][None], P)[0]
        assert np.allclose(got, ref[:12], rtol=1e-14, atol=1e-12)
    # rows with T_blast = 0: the reference's own f rows 0..11 and their Jacobian blocks
    m = p[:, 24] == 0.0
    P.t_blast = 0.0
    got = f12(x[m, :12], u[m, :4], P)
    assert np.allclose(got, dyn[tag + '_f'][m, :12], rtol=1e-13, atol=1e-12)
    J = jac12(x[m, :12], u[m, :4], P)
    assert np.allclose(J[:, :, :12], dyn[tag + '_dfdx'][m, :12, :12], rtol=1e-12, atol=1e-11)
    assert np.allclose(J[:, :, 12:], dyn[tag + '_dfdu'][m, :12, :4], rtol=1e-12, atol=1e-11)


def test_hover_known_answer():
    # simulation_blaster.py:97: 22.0725 N per motor holds hover for m = 9 (9*9.81/4)
    x = np.zeros((1, 12))
    x[0, 2] = 3.5
    u = np.full((1, 4), 22.0725)
    assert np.abs(f12(x, u, Params())).max() < 1e-14


def test_euler_rate_inverse_closed_form():
    rng = np.random.default_rng(1)
    phi, th = rng.uniform(-1.2, 1.2, (2, 100))
    W = np.zeros((100, 3, 3))
    W[:, 0, 0] = 1
    W[:, 0, 2] = -np.sin(th)
    W[:, 1, 1] = np.cos(phi)
    W[:, 1, 2] = np.sin(phi) * np.cos(th)
    W[:, 2, 1] = -np.sin(phi)
    W[:, 2, 2] = np.cos(phi) * np.cos(th)
    assert np.allclose(euler_rate_inv(phi, th) @ W, np.eye(3), atol=1e-12)


def test_rk4_sensitivities_match_central_differences():
    rng = np.random.default_rng(2)
    P = Params()
    x = rng.uniform(-0.5, 0.5, (16, 12))
    u = rng.uniform(5, 40, (16, 4))
    h = 1.0 / 30.0
    _, A, B = rk4_sens(x, u, h, P)
    S = np.concatenate([A, B], axis=2)
    z = np.concatenate([x, u], axis=1)
    eps = 1e-6
    for j in range(16):
        zp, zm = z.copy(), z.copy()
        zp[:, j] += eps
        zm[:, j] -= eps
        fd = (rk4_step(zp[:, :12], zp[:, 12:], h, P) - rk4_step(zm[:, :12], zm[:, 12:], h, P)) / (2 * eps)
        assert np.abs(S[:, :, j] - fd).max() < 1e-8


def test_mathutils_known_answers():
    """utils/MathUtils.py helpers (unused by the path) vs the oracle restatement."""
    from oracle.mathutils import quat_multiply, unit_quat_inverse, quat_to_rot
    d = np.load(os.path.join(GOLD, 'mathutils_ref.npz'))
    assert np.allclose(quat_multiply(d['q1'], d['q2']), d['prod'], atol=1e-14)
    assert np.allclose(unit_quat_inverse(d['q1']), d['inv'], atol=1e-15)
    assert np.allclose(quat_to_rot(d['q1']), d['rot'], atol=1e-14)
