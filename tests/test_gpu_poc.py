"""GPU parity of the batched POC Jacobian solver vs oracle/poc.py.

Tolerance: POC <= 1e-11 absolute; Jacobians <= 1e-5 absolute (achieved ~1e-6) — the
reference's forward differences (eps = 1e-6, Jacobian_POC_Solver.py:37) of Newton iterates whose
slope is itself a forward difference (dT = 1e-5, :145) amplify the ~1e-16 relative rounding
differences of two fp64 implementations by up to ~1e10 in the perturbed ground-hit times."""
import numpy as np
import pytest

from oracle.poc import params25, solve_jacobians

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu


def _poses(B, seed):
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.uniform(-0.15, 0.15, (B, 3)), rng.uniform(-0.3, 0.3, (B, 2)),
                           rng.uniform(-1, 1, (B, 2)), rng.uniform(2.0, 4.0, (B, 1))], axis=1)


@pytest.mark.parametrize('Mc', [1.0, 'matrix'])
def test_poc_jacobians_match_oracle(Mc):
    from mpc_blaster_amd.poc import poc_jacobians
    B = 203
    pose = _poses(B, 3)
    M = np.diag([1.0, 0.8, 1.2]) if Mc == 'matrix' else Mc
    o = {k: v.cpu().numpy() for k, v in poc_jacobians(pose, 150.0, M, t_blast=21.582).items()}
    P0, Je, Jm, Jp, ok = solve_jacobians(pose[:, 0:3], pose[:, 3:5], pose[:, 5:8], 150.0, M)
    assert (o['status'] == 0).all() and ok.all()
    assert np.abs(o['poc'] - P0).max() < 1e-11
    for got, ref in ((o['J_eul'], Je), (o['J_mot'], Jm), (o['J_pos'], Jp)):
        assert np.abs(got - ref).max() < 1e-5
    assert np.abs(o['p25'] - params25(Jm, Je, Jp, 21.582)).max() < 1e-5


def test_reference_class_surface():
    from mpc_blaster_amd.poc import JacobianPOCSolver
    s = JacobianPOCSolver(150, 1.0, 0.00015)   # Jacobian_POC_Solver.py:303
    s.initialise()
    assert s.solveJacobians([0, -0.05, 0], [0.2117, 0], [0.6, 0, 3.5]) == 0
    J_mot, J_eul, J_pos = s.getJacobians()
    P0, Je, Jm, Jp, _ = solve_jacobians([[0, -0.05, 0]], [[0.2117, 0]], [[0.6, 0, 3.5]], 150.0, 1.0)
    assert np.abs(s._POC - P0[0]).max() < 1e-11
    assert np.abs(J_mot - Jm[0]).max() < 1e-5 and np.abs(J_eul - Je[0]).max() < 1e-5
    assert np.abs(J_pos - Jp[0]).max() < 1e-5
