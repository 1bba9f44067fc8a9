"""The oracle's degeneracy flags that the GPU parity sweeps use to decide which instances a
precision can pin (oracle.ocp.fp32_sensitivity for the 12/4 input box, tests/test_gpu_fuzz.py;
oracle.full.sensitivity17 for the 17/6 boxes, tests/test_gpu_fuzz17.py), checked on the CPU:
without noise the re-solve reproduces the minimiser exactly, and the moves grow with the noise."""
import numpy as np

from oracle.full import FullSpec, mpc_solve17, sensitivity17
from oracle.inputs import make_inputs
from oracle.ocp import OcpSpec, fp32_sensitivity, mpc_solve


def test_fp32_sensitivity_zero_noise_and_c4_scale():
    N, B = 30, 24
    inp = make_inputs('c4', ids=np.arange(B, dtype=np.uint64), N=N)
    spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0))
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, return_lin=True)
    assert (o['status'] == 0).all()
    s0 = fp32_sensitivity(o, inp['x0'], inp['xref'], inp['uref'], spec, rel=0.0)
    assert s0.max() <= 1e-12
    s = fp32_sensitivity(o, inp['x0'], inp['xref'], inp['uref'], spec)
    big = fp32_sensitivity(o, inp['x0'], inp['xref'], inp['uref'], spec, rel=2.0 ** -12)
    print(f'c4 draws: fp32 sensitivity max {s.max():.1e}, at 2^-12 noise {big.max():.1e}')
    # (c4's hover draws are well conditioned: ~1e-6, below the sweeps' 1e-5 flag)
    assert np.isfinite(s).all() and s.max() < 1e-5
    assert big.max() > s.max()


def test_sensitivity17_zero_noise_and_growth():
    N, B = 10, 4
    lbu = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])
    ubu = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
    spec = FullSpec(N=N, lbu=lbu, ubu=ubu)
    from test_oracle_full import _random_point
    x0, _, p = _random_point(B, 5)
    x0[:, 3:6] *= 0.5
    xref = np.zeros((B, N + 1, 17))
    xref[..., 2] = 3.5
    uref = np.zeros((B, N, 6))
    uref[..., :4] = 22.0725
    o = mpc_solve17(x0, xref, uref, spec, p)
    assert (o['status'] == 0).all()
    s0 = sensitivity17(o, x0, xref, uref, spec, rel=0.0)
    s45 = sensitivity17(o, x0, xref, uref, spec, rel=2.0 ** -45)
    s22 = sensitivity17(o, x0, xref, uref, spec, rel=2.0 ** -22)
    print(f'17/6 input box: sensitivity 0 -> {s0.max():.1e}, 2^-45 -> {s45.max():.1e}, 2^-22 -> {s22.max():.1e}')
    assert s0.max() <= 1e-12
    assert np.isfinite(s22).all() and s22.max() >= s45.max()
