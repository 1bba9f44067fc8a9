"""The plain-C oracle restatement (CPU baseline) agrees with the NumPy oracle."""
import numpy as np
import pytest

from oracle import c_oracle
from oracle.inputs import make_inputs
from oracle.ocp import OcpSpec, mpc_solve


@pytest.mark.parametrize('cfg,N', [('c1', 10), ('c2', 20), ('c3', 20), ('c5', 40)])
def test_c_oracle_matches_numpy(cfg, N):
    inp = make_inputs(cfg, ids=np.arange(16, dtype=np.uint64), N=N)
    spec = OcpSpec(N=N)
    a = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, wind=inp['wind'])
    b = c_oracle.solve(inp['x0'], inp['xref'], inp['uref'][:1], spec, nthreads=2, wind=inp['wind'])
    assert (b['status'] == 0).all()
    for k in ('u0', 'X', 'U'):
        err = np.abs(a[k] - b[k]).max() / max(np.abs(a[k]).max(), 1.0)
        assert err < 1e-11, (k, err)


def test_c_oracle_box_matches_numpy_pdas():
    """The C restatement of the input-box active set (BASELINE c4) takes the NumPy oracle's
    iterations: same statuses, iteration counts and solution (c4 draws, N = 30)."""
    N = 30
    inp = make_inputs('c4', ids=np.arange(64, dtype=np.uint64), N=N)
    spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0))
    a = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec)
    b = c_oracle.solve(inp['x0'], inp['xref'], inp['uref'][:1], spec, nthreads=2)
    assert np.array_equal(a['status'], b['status']) and (b['status'] == 0).all()
    assert np.array_equal(a['iters'], b['iters'])
    for k in ('u0', 'X', 'U'):
        err = np.abs(a[k] - b[k]).max() / max(np.abs(a[k]).max(), 1.0)
        assert err < 1e-11, (k, err)


def test_c_oracle_latency_b1_runs_single_instances():
    """The c1-shape latency sampler (bench.py cpu_baseline.c1_latency_ms): one instance per C call,
    every solve OK, positive per-solve times."""
    from oracle import c_oracle
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec
    inp = make_inputs('c1', ids=np.arange(4, dtype=np.uint64), N=10)
    ms = c_oracle.latency_b1(inp['x0'], inp['xref'], inp['uref'], OcpSpec(N=10), reps=16)
    assert ms.shape == (16,) and (ms > 0).all() and (ms < 1000).all()
