"""The plain-C oracle restatement (CPU baseline) agrees with the NumPy oracle."""
import numpy as np
import pytest

from oracle import c_oracle
from oracle.inputs import make_inputs
from oracle.ocp import OcpSpec, mpc_solve


@pytest.mark.parametrize('cfg,N', [('c1', 10), ('c2', 20), ('c3', 20)])
def test_c_oracle_matches_numpy(cfg, N):
    inp = make_inputs(cfg, ids=np.arange(16, dtype=np.uint64), N=N)
    spec = OcpSpec(N=N)
    a = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec)
    b = c_oracle.solve(inp['x0'], inp['xref'], inp['uref'][:1], spec, nthreads=2)
    assert (b['status'] == 0).all()
    for k in ('u0', 'X', 'U'):
        err = np.abs(a[k] - b[k]).max() / max(np.abs(a[k]).max(), 1.0)
        assert err < 1e-11, (k, err)
