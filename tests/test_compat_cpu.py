"""Host logic of the acados-subset facade (no GPU): the reference constructor's default
parameter vector and how set(k, 'p') reaches the device handle."""
import numpy as np
import pytest

from mpc_blaster_amd.compat.acados import AcadosOcpSolver
from mpc_blaster_amd.compat.blastermodel import DEFAULT_T_BLAST, blasterModel
from mpc_blaster_amd.config import MPCConfig


def _reference_args():
    """simulation_blaster.py:12-30, verbatim values."""
    J = np.eye(3)
    J[0, 0], J[1, 1], J[2, 2] = 0.50781, 0.47314, 0.72975
    Q = np.zeros((17, 17))
    np.fill_diagonal(Q, [1e3] * 6 + [5.0] * 3 + [10.0] * 3 + [1e-2] * 2 + [1e3] * 3)
    R = np.zeros((6, 6))
    np.fill_diagonal(R, [5e-2] * 4 + [1e-5] * 2)
    sb = np.array([[-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0, -0.0872665,
                    -0.0872665, -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5],
                   [1.5, 1.5, 5.0, 0.174532925, 0.174532925, 0.349066, 1.0, 1.0, 1.0, 0.0872665, 0.0872665,
                    0.0872665, 1.22173, 0.523599, 1.5, 1.5, 2.5]])
    cb = np.array([[0, 0, 0, 0, -0.0872665, -0.0872665], [65, 65, 65, 65, 0.0872665, 0.0872665]])
    return (9.0, J, 0.3434, 0.3475, 60, 2.0, 0.03, Q, R, 10 * Q, 2.2 * 9.81, sb, cb)


@pytest.mark.parametrize('full', [True, False])
def test_default_t_blast_is_the_reference_constant(full):
    """blastermodel.py:280-282 hard-codes params[-1] = 2.2*9.81 whatever blastThruster is;
    simulation_blaster.py:22 passes blastThruster = 2.2*9.81 (it must not become 211.7 N)."""
    b = blasterModel(*_reference_args(), full_model=full)
    b.generateModel()
    assert DEFAULT_T_BLAST == pytest.approx(21.582, rel=1e-15)
    assert b._cfg.t_blast == pytest.approx(21.582, rel=1e-15)
    b2 = blasterModel(*_reference_args()[:10], 2.2, *_reference_args()[11:], full_model=full)
    b2.generateModel()
    assert b2._cfg.t_blast == pytest.approx(21.582, rel=1e-15)


class _Handle:
    """Records what the facade hands to the device handle."""

    def __init__(self):
        self.calls = []

    def set_params(self, p):
        self.calls.append(('p', None if p is None else np.array(p)))

    def set_t_blast(self, t):
        self.calls.append(('t', t))


def _facade(cfg, B=1):
    o = AcadosOcpSolver.__new__(AcadosOcpSolver)
    o.cfg, o.B, o.nx, o.nu = cfg, B, cfg.nx, cfg.nu
    o._p = np.zeros((B, cfg.N + 1, 25))
    o._p[..., 24] = cfg.t_blast
    o._p_dirty = False
    o.mpc = _Handle()
    return o


def test_set_p_per_stage_full_model():
    cfg = MPCConfig.full(N=5)
    o = _facade(cfg)
    rng = np.random.default_rng(0)
    p = rng.normal(size=25)
    for k in range(cfg.N + 1):
        o.set(k, 'p', p)
    o._upload_params()
    kind, v = o.mpc.calls[-1]
    assert kind == 'p' and v.shape == (1, 25) and np.array_equal(v[0], p)   # one vector, all stages
    o.set(3, 'p', 2 * p)                                # stage 3 differs -> [B, N, 25]
    o._upload_params()
    kind, v = o.mpc.calls[-1]
    assert v.shape == (1, cfg.N, 25)
    assert np.array_equal(v[0, 3], 2 * p) and np.array_equal(v[0, 2], p)
    o.set(cfg.N, 'p', 3 * p)                            # the terminal stage has no dynamics
    o._upload_params()
    assert o.mpc.calls[-1][1].shape == (1, cfg.N, 25)
    with pytest.raises(IndexError):
        o.set(cfg.N + 1, 'p', p)


def test_set_p_on_the_slice_maps_t_blast_and_rejects_stage_varying():
    cfg = MPCConfig(N=4, t_blast=DEFAULT_T_BLAST)
    o = _facade(cfg)
    for k in range(cfg.N):
        o.set(k, 'p', np.zeros(25))
    o._upload_params()
    assert o.mpc.calls == [('t', 0.0)]
    o.cfg.t_blast = 0.0
    p = np.zeros(25)
    p[24] = 5.0
    o.set(1, 'p', p)
    with pytest.raises(NotImplementedError):
        o._upload_params()
    assert o._p_dirty    # the rejected parameters stay pending: the next solve() raises again
    with pytest.raises(NotImplementedError):
        o._upload_params()


def test_library_abi_version_is_checked_at_load(tmp_path):
    """A library of another C ABI version is refused before any call (a stale v3
    library would read mpcb_set_params' row count as its device pointer)."""
    import subprocess

    from mpc_blaster_amd import _lib
    src = tmp_path / 'stale.c'
    src.write_text('int mpcb_abi_version(void) { return 3; }\n' + ''.join(
        f'int {n}(void) {{ return 0; }}\n' for n in _lib.EXPORTS if n != 'mpcb_abi_version'))
    so = tmp_path / 'libstale.so'
    subprocess.check_call(['gcc', '-shared', '-fPIC', str(src), '-o', str(so)])
    with pytest.raises(_lib.LibraryMissing, match='ABI version 3'):
        _lib.load(str(so))


def test_slice_refuses_a_finite_state_box():
    """The 12/4 slice has no state box: the reference's finite statesBound raises there (instead of
    being silently dropped); the default model is the reference's 17/6 OCP, which enforces it."""
    b = blasterModel(*_reference_args(), full_model=False)
    b.generateModel()
    with pytest.raises(NotImplementedError, match='statesBound'):
        b.generateController()
    b2 = blasterModel(*_reference_args())
    b2.generateModel()
    assert b2._cfg.nx == 17 and b2._cfg.lbx is not None


def test_fp32_refuses_a_finite_state_box():
    """One constraint policy: the 17/6 state box is fp64-only on the device, so
    an fp32 model with the reference's finite statesBound raises like the 12/4 slice does instead
    of warning and solving without it; a non-finite statesBound is accepted in fp32."""
    b = blasterModel(*_reference_args(), dtype='f32')
    with pytest.raises(NotImplementedError, match='statesBound'):
        b.generateModel()
        b.generateController()
    args = list(_reference_args())
    args[11] = np.full_like(np.asarray(args[11], dtype=np.float64), np.inf)
    b2 = blasterModel(*args, dtype='f32')
    b2.generateModel()
    assert b2._cfg.lbx is None
