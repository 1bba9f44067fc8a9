"""POC Jacobian oracle: integrator against the closed-form stream solution,
rotation against the reference's own SciPy call, root finder and Jacobian structure on the
reference's __main__ case (Jacobian_POC_Solver.py:303-306).  The reference path itself needs
acados (absent), so the end-to-end numbers are parity unpinned."""
import numpy as np
from scipy.spatial.transform import Rotation

from oracle.poc import (G, T_w_b, init_conditions, integrate, params25, root_time,
                        solve_jacobians)
from oracle.model import unpack_params25


def test_rk4_matches_closed_form_stream():
    rng = np.random.default_rng(0)
    x0 = rng.normal(size=(16, 6)) * np.array([1, 1, 1, 50, 50, 150])
    T = rng.uniform(0.001, 0.1, 16)
    for Mc in (1.0, 0.3):
        x = integrate(x0, T, Mc)
        v0 = x0[:, 3:]
        vinf = G / Mc
        e = np.exp(-Mc * T)[:, None]
        p = x0[:, :3] + vinf * T[:, None] + (v0 - vinf) * (1 - e) / Mc
        v = vinf + (v0 - vinf) * e
        assert np.abs(x[:, :3] - p).max() < 1e-9
        assert np.abs(x[:, 3:] - v).max() < 1e-7


def test_rotation_is_the_reference_scipy_call():
    rng = np.random.default_rng(1)
    e = rng.uniform(-0.5, 0.5, (8, 3))
    T = T_w_b(e[:, 0], e[:, 1], e[:, 2], np.zeros((8, 3)))
    for i in range(8):   # htm.py:33: R.from_euler('zyx', [psi, theta, phi])
        ref = Rotation.from_euler('zyx', [e[i, 2], e[i, 1], e[i, 0]]).as_matrix()
        assert np.abs(T[i, :3, :3] - ref).max() < 1e-15


def test_reference_main_case():
    e, m, p = np.array([[0, -0.05, 0.0]]), np.array([[0.2117, 0.0]]), np.array([[0.6, 0, 3.5]])
    P0, Je, Jm, Jp, ok = solve_jacobians(e, m, p, 150.0, 1.0)
    assert ok.all()
    x0 = init_conditions(e, m, p, 150.0)
    T, it, conv = root_time(x0, 1.0)
    assert conv.all() and 0 < T[0] < 0.1
    assert abs(integrate(x0, T, 1.0)[0, 2]) <= 1e-3   # lands on the ground (z = 0)
    assert abs(P0[0, 2]) <= 1e-3
    # a translation moves the POC with it in x and y
    assert np.allclose(Jp[0, :2, :2], np.eye(2), atol=1e-6)
    p25 = params25(Jm, Je, Jp, 21.582)
    Ja, Je2, Jp2, tb = unpack_params25(p25)
    assert np.array_equal(Ja, Jm) and np.array_equal(Je2, Je) and np.array_equal(Jp2, Jp)
