"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle on identical inputs.

Tolerances (north_star: 1e-5 relative in fp64):
* fp64: per-instance ||y_dev - y_oracle||_inf / max(||y_oracle||_inf, 1) <= 1e-9 (achieved
  ~1e-12; RK4/trig rounding only).
* fp32: the same normwise metric <= 5e-5 on u0, U and X (achieved ~2e-6; fp32 Riccati with a
  symmetric-by-construction P, SURVEY §7 ii);
  the achieved numbers are printed by tests and recorded in DESIGN.md.
"""
import os

import numpy as np
import pytest

from oracle.inputs import make_inputs
from oracle.model import Params
from oracle.ocp import OcpSpec, mpc_solve, stage_cost
from oracle.rk4 import rk4_sens

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


_PATH_ENV = {   # path -> library overrides (the defaults pick by batch size)
    'split': {'MPCB_SPLIT_MIN_BATCH': '1'},                          # nominal / Riccati / forward
    'small': {'MPCB_SPLIT_MIN_BATCH': '1', 'MPCB_SMALL_MAX': '1000000'},  # cached-[A|B] passes
    'fused': {'MPCB_SPLIT_MIN_BATCH': str(1 << 40)},               # single-kernel solver
}


def _mpc(N, dtype='f64', box=False, max_batch=4096, path=None, **kw):
    """path: None (library default by batch size) or a key of _PATH_ENV (forced via env)."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    cfg = MPCConfig(N=N, dtype=dtype, lbu=np.zeros(4) if box else None,
                    ubu=np.full(4, 65.0) if box else None, **kw)
    env = _PATH_ENV.get(path, {})
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return BatchedMPC(cfg, max_batch=max_batch)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _spec(N, box=False):
    return OcpSpec(N=N, lbu=np.zeros(4) if box else None, ubu=np.full(4, 65.0) if box else None)


def relerr(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, dtype=np.float64).reshape(b.shape[0], -1)
    return np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1.0)


def test_library_is_the_native_hip_build():
    from mpc_blaster_amd import _lib
    lib = _lib.load()
    assert os.path.basename(lib._name) == 'libmpcblaster.so'
    assert lib.mpcb_abi_version() == 5


def test_linearize_matches_oracle_fp64():
    N, B = 5, 37
    m = _mpc(N, 'f64', max_batch=B)
    rng = np.random.default_rng(5)
    xb = rng.uniform(-0.6, 0.6, (B, N + 1, 12))
    ub = rng.uniform(5.0, 40.0, (B, N, 4))
    A, Bm, xn = (t.cpu().numpy() for t in m.linearize(xb, ub))
    P = Params()
    for k in range(N):
        xr, Ar, Br = rk4_sens(xb[:, k], ub[:, k], 1.0 / 30.0, P)
        assert np.abs(A[:, k] - Ar).max() < 1e-12
        assert np.abs(Bm[:, k] - Br).max() < 1e-12
        assert np.abs(xn[:, k] - xr).max() < 1e-12


def test_gen_inputs_bit_exact_fp64():
    m = _mpc(20, 'f64', max_batch=1000)
    d = m.gen_inputs(1000, seed=1003, id_offset=123, ref='sine', wind=True)
    o = make_inputs('c3', ids=np.arange(123, 1123, dtype=np.uint64))
    assert np.array_equal(d['x0'].cpu().numpy(), o['x0'])
    from oracle.inputs import make_wind, draws
    assert np.array_equal(d['wind'].cpu().numpy(), make_wind(draws(1003, np.arange(123, 1123))))
    assert np.abs(d['xref'].cpu().numpy() - o['xref']).max() < 1e-14
    assert np.all(d['uref'].cpu().numpy() == 22.0725)


def test_c1_golden_fp64():
    d = np.load(os.path.join(GOLD, 'mpc_c1.npz'))
    m = _mpc(10, 'f64', max_batch=1)
    m.solve(d['x0'], d['xref'], d['uref'])
    torch.cuda.synchronize()
    assert relerr(m.get_control().cpu().numpy(), d['u0']).max() < 1e-9
    assert relerr(m.get_state_trajectory().cpu().numpy(), d['X']).max() < 1e-9
    assert relerr(m.get_input_trajectory().cpu().numpy(), d['U']).max() < 1e-9
    assert m.get_status().cpu().numpy().tolist() == [0]


@pytest.mark.parametrize('cfg,N,dtype,box,path', [
    ('c2', 20, 'f64', False, 'fused'), ('c3', 20, 'f64', False, 'fused'),
    ('c3', 20, 'f32', False, 'fused'), ('c2', 10, 'f32', False, 'fused'),
    ('c2', 20, 'f64', False, 'split'), ('c3', 20, 'f64', False, 'split'),
    ('c3', 20, 'f32', False, 'split'), ('c2', 10, 'f32', False, 'split'),
    ('c2', 20, 'f64', False, 'small'), ('c3', 20, 'f32', False, 'small'),
    ('c4', 30, 'f64', True, None), ('c4', 30, 'f32', True, None),
])
def test_solve_matches_oracle(cfg, N, dtype, box, path):
    B = 203   # ragged: not a multiple of the 4-instance wave
    inp = make_inputs(cfg, ids=np.arange(B, dtype=np.uint64), N=N)
    m = _mpc(N, dtype, box, max_batch=B, path=path)
    m.solve(inp['x0'], inp['xref'], inp['uref'])
    torch.cuda.synchronize()
    u0 = m.get_control().cpu().numpy()
    X = m.get_state_trajectory().cpu().numpy()
    U = m.get_input_trajectory().cpu().numpy()
    st = m.get_status().cpu().numpy()
    # the oracle sees exactly the inputs the device saw (fp32 inputs rounded first)
    cast = (lambda a: a.astype(np.float32).astype(np.float64)) if dtype == 'f32' else (lambda a: a)
    o = mpc_solve(cast(inp['x0']), cast(inp['xref']), cast(inp['uref']), _spec(N, box))
    e_u, e_x, e_U = relerr(u0, o['u0']), relerr(X, o['X']), relerr(U, o['U'])
    print(f'{cfg} N={N} {dtype} box={box} path={path}: max rel err u0 {e_u.max():.2e} X {e_x.max():.2e} U {e_U.max():.2e}')
    assert (st == o['status']).all() and (st == 0).all()
    tol_u, tol_x = (1e-9, 1e-9) if dtype == 'f64' else (5e-5, 5e-5)
    assert e_u.max() < tol_u and e_U.max() < tol_u and e_x.max() < tol_x
    if box:
        assert (U >= -1e-6).all() and (U <= 65 + 1e-4).all()


@pytest.mark.parametrize('path', ['fused', 'split', 'small'])
def test_iterate_mode_matches_oracle_fp64(path):
    """acados SQP_RTI semantics: linearise at a given iterate with gaps and dx0 != 0."""
    N, B = 12, 41
    rng = np.random.default_rng(9)
    inp = make_inputs('c2', ids=np.arange(B, dtype=np.uint64), N=N)
    xbar = inp['xref'] + rng.normal(scale=0.05, size=(B, N + 1, 12))
    ubar = inp['uref'] + rng.normal(scale=1.0, size=(B, N, 4))
    m = _mpc(N, 'f64', max_batch=B, path=path)
    m.solve_iterate(inp['x0'], xbar, ubar, inp['xref'], inp['uref'])
    torch.cuda.synchronize()
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], _spec(N), mode='iterate', xbar=xbar, ubar=ubar)
    assert relerr(m.get_control().cpu().numpy(), o['u0']).max() < 1e-9
    assert relerr(m.get_state_trajectory().cpu().numpy(), o['X']).max() < 1e-9


@pytest.mark.parametrize('path', ['fused', 'split', 'small'])
def test_wind_extension_fp64(path):
    N, B = 8, 16
    inp = make_inputs('c5', ids=np.arange(B, dtype=np.uint64), N=N)
    m = _mpc(N, 'f64', max_batch=B, path=path)
    m.solve(inp['x0'], inp['xref'], inp['uref'], wind=inp['wind'])
    torch.cuda.synchronize()
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], _spec(N), wind=inp['wind'])
    assert relerr(m.get_control().cpu().numpy(), o['u0']).max() < 1e-9


def test_sim_step_and_histogram():
    B = 1000
    m = _mpc(20, 'f64', max_batch=B)
    rng = np.random.default_rng(4)
    x = rng.uniform(-0.5, 0.5, (B, 12))
    u = rng.uniform(0, 65, (B, 4))
    xo = m.sim_step(x, u).cpu().numpy()
    from oracle.rk4 import rk4_step
    assert np.abs(xo - rk4_step(x, u, 1.0 / 30.0, Params())).max() < 1e-12
    counts = m.histogram(u, 0.0, 65.0, 64).cpu().numpy()
    ref = np.stack([np.histogram(np.clip(u[:, i], 0, 65 - 1e-9), bins=64, range=(0, 65))[0] for i in range(4)])
    assert np.array_equal(counts, ref)


@pytest.mark.parametrize('mode', ['rollout', 'iterate'])
def test_wrapped_euler_angles_quad_rollout_fp64(mode):
    """The quad-lane rollout (split path, chunks <= 16384) carries each lane's Euler angle through
    the RK4 stages itself (mpcb_split.hip rk4_nom_own).  Angles offset by 2*pi*k, up to past 2^19
    rad where sin/cos leave the Cody-Waite range for the ocml fallback on that lane only, with the
    reference offset alike, must still match the oracle.  Tolerance: the stage angle x + h/2*k is
    rounded at |x| ~ 6e5 to ~1.2e-10 absolute (the device contracts it into one fma, NumPy rounds
    twice), which moves sin/cos by that much; 1e-9 elsewhere."""
    N, B = 12, 24
    inp = make_inputs('c2', ids=np.arange(B, dtype=np.uint64), N=N)
    k = np.array([0, 1, -3, 1e3, -1e4, 1e5, 9e4, 83500.0] * 3)[:B]   # 2*pi*83500 > 2^19
    off = np.zeros((B, 12))
    off[:, 3] = 2 * np.pi * np.roll(k, 1)
    off[:, 4] = 2 * np.pi * np.roll(k, 2)
    off[:, 5] = 2 * np.pi * k
    x0 = inp['x0'] + off
    xref = inp['xref'] + off[:, None, :]
    m = _mpc(N, 'f64', max_batch=B, path='split')
    spec = _spec(N)
    if mode == 'rollout':
        m.solve(x0, xref, inp['uref'])
        o = mpc_solve(x0, xref, inp['uref'], spec)
    else:
        rng = np.random.default_rng(3)
        xbar = xref + rng.normal(scale=0.05, size=xref.shape)
        ubar = inp['uref'] + rng.normal(scale=1.0, size=inp['uref'].shape)
        m.solve_iterate(x0, xbar, ubar, xref, inp['uref'])
        o = mpc_solve(x0, xref, inp['uref'], spec, mode='iterate', xbar=xbar, ubar=ubar)
    torch.cuda.synchronize()
    e_u = relerr(m.get_control().cpu().numpy(), o['u0'])
    e_x = relerr(m.get_state_trajectory().cpu().numpy() - off[:, None, :], o['X'] - off[:, None, :])
    big = np.abs(off).max(axis=1) > 1e3
    print(f'{mode}: small offsets u0 {e_u[~big].max():.2e} X {e_x[~big].max():.2e}; '
          f'large u0 {e_u[big].max():.2e} X {e_x[big].max():.2e}')
    assert (m.get_status().cpu().numpy() == 0).all()
    assert e_u[~big].max() < 1e-9 and e_x[~big].max() < 1e-9
    assert e_u[big].max() < 1e-6 and e_x[big].max() < 1e-6


@pytest.mark.parametrize('path', ['fused', 'split', 'small'])
def test_u0_only_path_equals_full_path(path):
    N, B = 20, 64
    inp = make_inputs('c3', ids=np.arange(B, dtype=np.uint64), N=N)
    m = _mpc(N, 'f32', max_batch=B, path=path)
    a = m.solve(inp['x0'], inp['xref'], inp['uref'], want_traj=False).clone()
    b = m.solve(inp['x0'], inp['xref'], inp['uref'], want_traj=True)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize('path,box', [('fused', False), ('split', False), ('small', False), (None, True)])
def test_phase_timing_events(path, box):
    """mpcb_set_timing / mpcb_last_timing: per-phase device ms, and timing changes no result."""
    N, B = 20, 256
    inp = make_inputs('c3', ids=np.arange(B, dtype=np.uint64), N=N)
    m = _mpc(N, 'f32', box=box, max_batch=B, path=path)
    a = m.solve(inp['x0'], inp['xref'], inp['uref'], want_traj=False).clone()
    m.set_timing(True)
    b = m.solve(inp['x0'], inp['xref'], inp['uref'], want_traj=False)
    t = m.last_timing()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert t['riccati'] > 0
    if m.path == 'split' and not box:
        assert t['nominal'] > 0 and t['forward'] < t['riccati']   # u0 only: no forward kernel
    elif box:
        assert t['nominal'] > 0 and t['forward'] > 0              # active-set kernel
    else:
        assert t['nominal'] == 0 and t['forward'] == 0


def test_full_size_c3_properties():
    """BASELINE c3 at full size: statuses, finiteness, shard invariance, sampled oracle parity."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    B, N = 65536, 20
    m = BatchedMPC(MPCConfig(N=N, dtype='f32'), max_batch=B)
    d = m.gen_inputs(B, seed=1003, ref='sine')
    u0 = m.solve(d['x0'], d['xref'], d['uref'], want_traj=True).clone()
    X = m.get_state_trajectory().clone()
    st = m.get_status().clone()
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert torch.isfinite(u0).all() and torch.isfinite(X).all()
    # shard invariance: instances 40000.. solved alone give identical bits
    sl = slice(40000, 40000 + 777)
    u_sub = m.solve(d['x0'][sl], d['xref'][sl], d['uref'], want_traj=False)
    torch.cuda.synchronize()
    assert torch.equal(u_sub, u0[sl])
    # sampled oracle parity
    idx = np.arange(0, B, 4099)
    x0 = d['x0'][idx].double().cpu().numpy()
    xr = d['xref'][idx].double().cpu().numpy()
    o = mpc_solve(x0, xr, np.full((len(idx), N, 4), np.float32(22.0725), dtype=np.float64), _spec(N))
    assert relerr(u0[idx].cpu().numpy(), o['u0']).max() < 5e-5
    assert relerr(X[idx].cpu().numpy(), o['X']).max() < 5e-5


@pytest.mark.parametrize('B', [4096, 20000])
def test_full_size_c2_properties(B):
    """BASELINE c2 at the bench's size (4096 per GPU, fp64, N = 20, hover) on the default path the
    bench times (the fused rollout + Riccati launch and the 16-lane forward pass), and the same
    workload above the 16384-instance small-chunk threshold (the thread-per-instance rollout and
    forward pass, captured-scalar P2): every status 0, shard invariance (a slice solved alone gives
    identical bits), and sampled parity against the fp64 oracle at 1e-9."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    N = 20
    m = BatchedMPC(MPCConfig(N=N, dtype='f64'), max_batch=B)
    d = m.gen_inputs(B, seed=1002, ref='hover')
    u0 = m.solve(d['x0'], d['xref'], d['uref'], want_traj=True).clone()
    X = m.get_state_trajectory().clone()
    U = m.get_input_trajectory().clone()
    st = m.get_status().clone()
    torch.cuda.synchronize()
    k = m.last_kernels()
    assert k == m.plan_kernels(B)
    if B <= 16384:
        assert k == {'riccati': 'mpcb::row_riccati_kernel<false, true>', 'forward': 'mpcb::fwd_rm_kernel<double, false>'}
    else:
        assert k['nominal'] == 'mpcb::nominal_kernel<double, false>'
        assert k['forward'] == 'mpcb::forward_kernel<double, false, false>'
    assert int((st != 0).sum()) == 0
    assert torch.isfinite(u0).all() and torch.isfinite(X).all() and torch.isfinite(U).all()
    sl = slice(B // 3, B // 3 + 203)   # a ragged slice, off the quad boundary
    u_sub = m.solve(d['x0'][sl], d['xref'], d['uref'], want_traj=True).clone()
    X_sub = m.get_state_trajectory().clone()
    torch.cuda.synchronize()
    assert torch.equal(u_sub, u0[sl]) and torch.equal(X_sub, X[sl])
    idx = np.unique(np.r_[np.arange(0, B, 61), B - 1])
    o = mpc_solve(d['x0'][idx].cpu().numpy(), d['xref'].cpu().numpy(), d['uref'].cpu().numpy(), _spec(N))
    assert relerr(u0[idx].cpu().numpy(), o['u0']).max() < 1e-9
    assert relerr(X[idx].cpu().numpy(), o['X']).max() < 1e-9
    assert relerr(U[idx].cpu().numpy(), o['U']).max() < 1e-9


@pytest.mark.parametrize('want_traj', [False, True])
@pytest.mark.parametrize('path', [None, 'fused'])
def test_c5_matches_oracle_fp32(want_traj, path):
    """BASELINE c5 (configs[4]): N = 40, fp32, hover reference, per-instance wind force; the
    u0-only P2 (want_traj=False: the Riccati kernel writes u0, no forward pass) and the full
    trajectory, against the fp64 oracle on the fp32-rounded inputs."""
    B, N = 203, 40
    inp = make_inputs('c5', ids=np.arange(B, dtype=np.uint64), N=N)
    m = _mpc(N, 'f32', max_batch=B, path=path)
    m.solve(inp['x0'], inp['xref'], inp['uref'], wind=inp['wind'], want_traj=want_traj)
    torch.cuda.synchronize()
    cast = lambda a: a.astype(np.float32).astype(np.float64)
    o = mpc_solve(cast(inp['x0']), cast(inp['xref']), cast(inp['uref']), _spec(N), wind=cast(inp['wind']))
    e_u = relerr(m.get_control().cpu().numpy(), o['u0'])
    msg = f'c5 N=40 f32 path={path} traj={want_traj}: u0 {e_u.max():.2e}'
    assert (m.get_status().cpu().numpy() == 0).all()
    assert e_u.max() < 5e-5
    if want_traj:
        e_x = relerr(m.get_state_trajectory().cpu().numpy(), o['X'])
        e_U = relerr(m.get_input_trajectory().cpu().numpy(), o['U'])
        msg += f' X {e_x.max():.2e} U {e_U.max():.2e}'
        assert e_x.max() < 5e-5 and e_U.max() < 5e-5
    print(msg)


def _host_histogram(u0, lo=0.0, hi=65.0, nbins=64):
    """The kernel's binning restated: bin = floor((double(u) - lo) * nbins / (hi - lo)), clipped."""
    v = np.asarray(u0, dtype=np.float64)
    b = np.floor((v - lo) * (nbins / (hi - lo)))
    b = np.where(np.isnan(v), nbins - 1, np.clip(b, 0, nbins - 1)).astype(np.int64)
    return np.stack([np.bincount(b[:, m], minlength=nbins) for m in range(v.shape[1])])


def test_full_size_c5_histogram_properties():
    """BASELINE c5 per-GPU shard (131072 of 1048576 on 8 GPUs, N = 40, fp32, wind): every status
    0, u0 finite; the 64-bin per-motor histogram sums to B per motor and equals the host binning
    of the device u0 bit for bit; the u0-only solve equals the trajectory solve; sampled parity."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    B, N = 131072, 40
    m = BatchedMPC(MPCConfig(N=N, dtype='f32'), max_batch=B)
    d = m.gen_inputs(B, seed=1005, id_offset=3 * B, ref='hover', wind=True)   # rank 3's ids
    u0 = m.solve(d['x0'], d['xref'], d['uref'], wind=d['wind'], want_traj=False).clone()
    st = m.get_status().clone()
    counts = m.histogram(u0, 0.0, 65.0, 64)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert torch.isfinite(u0).all()
    c = counts.cpu().numpy()
    assert (c.sum(axis=1) == B).all()
    assert np.array_equal(c, _host_histogram(u0.cpu().numpy()))
    # the u0-only Riccati kernel and the full path agree
    u_full = m.solve(d['x0'], d['xref'], d['uref'], wind=d['wind'], want_traj=True)
    torch.cuda.synchronize()
    assert torch.equal(u_full, u0)
    # the device's synthetic inputs are the oracle's (fp32-rounded) and sampled instances match it
    idx = np.arange(0, B, 5003)
    o_in = make_inputs('c5', ids=np.uint64(3 * B) + idx.astype(np.uint64), N=N)
    cast = lambda a: a.astype(np.float32).astype(np.float64)
    assert np.array_equal(d['x0'][idx].double().cpu().numpy(), cast(o_in['x0']))
    assert np.array_equal(d['wind'][idx].double().cpu().numpy(), cast(o_in['wind']))
    o = mpc_solve(cast(o_in['x0']), cast(o_in['xref']), cast(o_in['uref']), _spec(N), wind=cast(o_in['wind']))
    e = relerr(u0[idx].cpu().numpy(), o['u0'])
    print(f'c5 full size: sampled u0 err {e.max():.2e}; hist bins occupied {int((c > 0).sum())}')
    assert e.max() < 5e-5


def test_full_size_c4_box_properties():
    """BASELINE c4 per-GPU shard (65536, N=30, fp32, thrust box [0, 65]): every instance reaches
    its KKT point (no MAXITER), bounds hold, sampled oracle parity, and the single-kernel
    active-set solver (MPCB_BOX_IMPL=v1) agrees on a slice."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    B, N = 65536, 30
    cfg = MPCConfig(N=N, dtype='f32', lbu=np.zeros(4), ubu=np.full(4, 65.0))
    m = BatchedMPC(cfg, max_batch=B)
    d = m.gen_inputs(B, seed=1004, ref='hover')
    u0 = m.solve(d['x0'], d['xref'], d['uref'], want_traj=True).clone()
    U = m.get_input_trajectory().clone()
    st = m.get_status().clone()
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    # a free component is accepted up to the fp32 rounding band of the violation test beyond its
    # bound: tol_u = 16 eps32 (|lb| + |ub| + 1) = 1.26e-4 (mpcb_as.hip / mpcb_box.hip)
    tol_u = 16 * float(np.finfo(np.float32).eps) * 66.0
    assert (U >= -tol_u).all() and (U <= 65 + tol_u).all()
    idx = np.arange(0, B, 2731)
    x0 = d['x0'][idx].double().cpu().numpy()
    xr = np.broadcast_to(d['xref'][0].double().cpu().numpy(), (len(idx), N + 1, 12)).copy()
    o = mpc_solve(x0, xr, np.full((len(idx), N, 4), np.float32(22.0725), dtype=np.float64), _spec(N, box=True))
    assert (o['status'] == 0).all()
    assert relerr(u0[idx].cpu().numpy(), o['u0']).max() < 5e-5
    assert relerr(U[idx].cpu().numpy(), o['U']).max() < 5e-5
    os.environ['MPCB_BOX_IMPL'] = 'v1'
    try:
        m1 = BatchedMPC(cfg, max_batch=512)
    finally:
        os.environ.pop('MPCB_BOX_IMPL')
    assert m1.path == 'fused'
    u1 = m1.solve(d['x0'][:512], d['xref'], d['uref'], want_traj=False)
    torch.cuda.synchronize()
    assert relerr(u1.cpu().numpy(), u0[:512].cpu().numpy()).max() < 5e-5


def test_full_batch_c4_every_instance_matches_c_oracle():
    """BASELINE c4 per-GPU shard, ALL 65,536 instances (seed 1004, N = 30, fp32, thrust box
    [0, 65]) against the plain-C fp64 oracle (oracle/c: the same active set in exact-order C,
    pinned to the NumPy oracle by tests/test_c_oracle.py) on the same fp32-rounded inputs: u0, U
    and X of every instance within 5e-5 normwise.  Before the fp64-residual refinement kernel
    (mpcb_as.h refine_verify) 24 instances were off by up to 5.7e-4 in U (a component fixed at
    a bound that the exact solution leaves free) and 7 by up to 9.2e-5 in u0."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from oracle import c_oracle
    B, N = 65536, 30
    box = dict(lbu=np.zeros(4), ubu=np.full(4, 65.0))
    m = BatchedMPC(MPCConfig(N=N, dtype='f32', **box), max_batch=B)
    d = m.gen_inputs(B, seed=1004, ref='hover')
    m.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
    u0, X, U = (t.double().cpu().numpy() for t in (m.get_control(), m.get_state_trajectory(),
                                                   m.get_input_trajectory()))
    st = m.get_status().cpu().numpy()
    x0 = d['x0'].double().cpu().numpy()
    o = c_oracle.solve(x0, d['xref'].double().cpu().numpy(), d['uref'].double().cpu().numpy(),
                       _spec(N, box=True), nthreads=min(16, os.cpu_count() or 1))
    e_u, e_U, e_x = relerr(u0, o['u0']), relerr(U, o['U']), relerr(X, o['X'])
    print(f'c4 full batch (65536): max rel err u0 {e_u.max():.2e} U {e_U.max():.2e} X {e_x.max():.2e}; '
          f'> 1e-5: u0 {(e_u > 1e-5).sum()} U {(e_U > 1e-5).sum()} X {(e_x > 1e-5).sum()}')
    assert (st == 0).all() and (o['status'] == 0).all()
    assert e_u.max() <= 5e-5 and e_U.max() <= 5e-5 and e_x.max() <= 5e-5


@pytest.mark.parametrize('dtype', ['f32', 'f64'])
def test_box_work_counter_grid_is_bit_identical(dtype):
    """The active-set kernel's resident grid (a group whose instance converged takes the next one
    from a per-chunk work counter, mpcb_as.hip) computes each instance with the same arithmetic as
    one wave per quad (MPCB_AS_PERSIST=0): U, X and status are bit-identical, over several chunks
    (MPCB_CHUNK=1024: the counter is reset per chunk) with a ragged last chunk and quad, and a
    sampled slice (plus every instance with a non-zero status) matches the oracle."""
    B, N = 3001, 20
    old = os.environ.get('MPCB_CHUNK')
    os.environ['MPCB_CHUNK'] = '1024'
    try:
        m = _mpc(N, dtype, box=True, max_batch=B)
    finally:
        if old is None:
            os.environ.pop('MPCB_CHUNK')
        else:
            os.environ['MPCB_CHUNK'] = old
    assert m.path == 'split'
    d = m.gen_inputs(B, seed=2024, ref='hover')
    res = []
    for persist in ('1', '0'):
        os.environ['MPCB_AS_PERSIST'] = persist
        try:
            u0 = m.solve(d['x0'], d['xref'], d['uref'], want_traj=True).clone()
        finally:
            os.environ.pop('MPCB_AS_PERSIST')
        res.append((u0, m.get_input_trajectory().clone(), m.get_state_trajectory().clone(),
                    m.get_status().clone()))
    torch.cuda.synchronize()
    for a, b in zip(*res):
        assert torch.equal(a, b)
    st = res[0][3].cpu().numpy()
    bad = np.nonzero(st)[0]
    assert len(bad) <= 2 and (st[bad] == 2).all()   # MPCB_STATUS_MAXITER
    idx = np.unique(np.concatenate([[0, 1, 1023, 1024, 2047, 2048, 3000], bad]))
    x0 = d['x0'][idx].double().cpu().numpy()
    xr = np.broadcast_to(d['xref'][0].double().cpu().numpy(), (len(idx), N + 1, 12)).copy()
    ur = np.broadcast_to(d['uref'][0].double().cpu().numpy(), (len(idx), N, 4)).copy()
    o = mpc_solve(x0, xr, ur, _spec(N, box=True))
    tol = 5e-5 if dtype == 'f32' else 1e-9
    # (the oracle's active-set loop also stops at max_iter on the instances the device flags; their
    # last iterates are not a KKT point and are compared only by status)
    assert (o['status'] == st[idx]).all()
    ok = o['status'] == 0
    assert ok.sum() >= 7 and relerr(res[0][1][idx].cpu().numpy(), o['U'])[ok].max() < tol


def test_closed_loop_matches_oracle_fp64():
    """Receding-horizon loop (simulation_blaster.py:56-107) with the persistent SQP_RTI iterate."""
    from mpc_blaster_amd.closed_loop import closed_loop
    from oracle.rk4 import rk4_step
    N, B, nsim = 10, 6, 12
    inp = make_inputs('c2', ids=np.arange(B, dtype=np.uint64), N=N)
    m = _mpc(N, 'f64', max_batch=B)
    Xs, Us, st = closed_loop(m, inp['x0'], inp['xref'], inp['uref'], nsim)
    torch.cuda.synchronize()
    xbar = np.zeros((B, N + 1, 12))
    ubar = np.zeros((B, N, 4))
    x = inp['x0'].copy()
    for i in range(nsim):
        o = mpc_solve(x, inp['xref'], inp['uref'], _spec(N), mode='iterate', xbar=xbar, ubar=ubar)
        xbar, ubar = o['X'], o['U']
        assert relerr(Us[:, i].cpu().numpy(), o['u0']).max() < 1e-8
        x = rk4_step(x, o['u0'], 1.0 / 30.0, Params())
        assert relerr(Xs[:, i + 1].cpu().numpy(), x).max() < 1e-8
    assert (st.cpu().numpy() == 0).all()


@pytest.mark.parametrize('t_blast', ['default', 'zero'])
def test_acados_facade_runs_reference_loop(t_blast):
    """simulation_blaster.py-style loop through the compat facade (12/4 slice of the reference
    parameter set, reference-length 17/23 vectors sliced).  ``default``: no set('p'), so the
    slice flies with acados' default T_blast = 2.2*9.81 (blastermodel.py:280-282); ``zero``:
    set(k, 'p') / integrator.set('p') with p[24] = 0 on every stage (a quad without the blaster),
    applied on the same device handle."""
    from mpc_blaster_amd.compat.blastermodel import blasterModel
    J = np.diag([0.50781, 0.47314, 0.72975])
    Q = np.zeros((17, 17))
    np.fill_diagonal(Q, [1e3] * 6 + [5.0] * 3 + [10.0] * 3 + [1e-2] * 2 + [1e3] * 3)
    R = np.zeros((6, 6))
    np.fill_diagonal(R, [5e-2] * 4 + [1e-5] * 2)
    cb = np.array([[0, 0, 0, 0, -0.0872665, -0.0872665], [65, 65, 65, 65, 0.0872665, 0.0872665]])
    N = 15
    b = blasterModel(9.0, J, 0.3434, 0.3475, N, N / 30.0, 0.03, Q, R, 10 * Q, 0.0,
                     np.full((2, 17), np.nan), cb, full_model=False)
    b.generateModel()
    integrator, ocp_solver = b.generateController()
    x = np.zeros(17)
    yref = np.zeros(23)
    yref[2] = 3.5
    lbu, ubu = np.zeros(4), np.full(4, 65.0)
    tb = 2.2 * 9.81 if t_blast == 'default' else 0.0
    P = Params(t_blast=tb)
    spec = OcpSpec(N=N, lbu=lbu, ubu=ubu, params=P)
    xbar, ubar = np.zeros((1, N + 1, 12)), np.zeros((1, N, 4))
    xs = x[:12].copy()
    handle = ocp_solver.mpc._h.value
    if t_blast == 'zero':
        for k in range(N):
            ocp_solver.set(k, 'p', np.zeros(25))
        integrator.set('p', np.zeros(25))
    for i in range(5):
        ocp_solver.set(0, 'lbx', x)
        ocp_solver.set(0, 'ubx', x)
        for k in range(N + 1):
            ocp_solver.cost_set(k, 'yref', yref if k < N else yref[:17])
        status = ocp_solver.solve()
        u = ocp_solver.get(0, 'u')
        o = mpc_solve(xs[None], np.broadcast_to(np.r_[0, 0, 3.5, [0] * 9], (1, N + 1, 12)),
                      np.zeros((1, N, 4)), spec, mode='iterate', xbar=xbar, ubar=ubar)
        xbar, ubar = o['X'], o['U']
        assert status == 0
        assert relerr(u[None], o['u0']).max() < 1e-8
        assert abs(ocp_solver.get_cost() - float(stage_cost(o['X'], o['U'], np.broadcast_to(np.r_[0, 0, 3.5, [0] * 9], (1, N + 1, 12)), np.zeros((1, N, 4)), spec)[0])) < 1e-6 * max(1.0, ocp_solver.get_cost())
        integrator.set('x', x)
        integrator.set('u', np.r_[u, 0.0, 0.0])
        assert integrator.solve() == 0
        x = np.r_[integrator.get('x'), np.zeros(5)]
        from oracle.rk4 import rk4_step
        xs = rk4_step(xs[None], o['u0'], 1.0 / 30.0, P)[0]
        assert np.abs(x[:12] - xs).max() < 1e-9
    assert ocp_solver.mpc._h.value == handle     # T_blast changed in place, not by re-creation


@pytest.mark.parametrize('dtype', ['f32', 'f64'])
@pytest.mark.parametrize('mode', ['rollout', 'iterate'])
def test_box_long_horizon_w64_matches_oracle(dtype, mode):
    """The 64-bit stage-mask active-set kernels (as_kernel_*<false, *>, 32 < N <= 64):
    the reference horizon N=60 with the input box, ragged B, both modes, against the oracle; and
    the work-counter grid bit-identical to one wave per quad (MPCB_AS_PERSIST=0) on the same
    instantiation."""
    N, B = 60, 157
    inp = make_inputs('c4', ids=np.arange(B, dtype=np.uint64), N=N)
    cast = (lambda a: a.astype(np.float32).astype(np.float64)) if dtype == 'f32' else (lambda a: a)
    m = _mpc(N, dtype, box=True, max_batch=B, path='split')
    kw = {}
    if mode == 'iterate':
        rng = np.random.default_rng(60)
        kw = dict(xbar=cast(inp['xref'] + rng.normal(scale=0.05, size=(B, N + 1, 12))),
                  ubar=cast(inp['uref'] + rng.normal(scale=2.0, size=(B, N, 4))))
    res = []
    for persist in ('1', '0'):
        os.environ['MPCB_AS_PERSIST'] = persist
        try:
            if mode == 'iterate':
                m.solve_iterate(inp['x0'], kw['xbar'], kw['ubar'], inp['xref'], inp['uref'])
            else:
                m.solve(inp['x0'], inp['xref'], inp['uref'])
            torch.cuda.synchronize()
        finally:
            os.environ.pop('MPCB_AS_PERSIST')
        res.append((m.get_control().clone(), m.get_input_trajectory().clone(),
                    m.get_state_trajectory().clone(), m.get_status().clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    u0, U, X, st = (t.double().cpu().numpy() if t.is_floating_point() else t.cpu().numpy() for t in res[0])
    o = mpc_solve(cast(inp['x0']), cast(inp['xref']), cast(inp['uref']), _spec(N, box=True),
                  mode=mode, **kw)
    tol = 5e-5 if dtype == 'f32' else 1e-9
    assert (st == o['status']).all()
    ok = o['status'] == 0
    assert ok.sum() >= B - 2
    e_u, e_U, e_x = relerr(u0, o['u0'])[ok], relerr(U, o['U'])[ok], relerr(X, o['X'])[ok]
    print(f'box N={N} {dtype} {mode}: max rel err u0 {e_u.max():.2e} U {e_U.max():.2e} X {e_x.max():.2e}')
    assert e_u.max() < tol and e_U.max() < tol and e_x.max() < tol
    assert (U >= -1e-5).all() and (U <= 65 + 1e-4).all()


_J_GENERAL = np.array([[0.50781, 0.012, -0.008], [0.012, 0.47314, 0.015], [-0.008, 0.015, 0.72975]])


@pytest.mark.parametrize('dtype,mode', [('f64', 'rollout'), ('f64', 'iterate'), ('f32', 'rollout')])
def test_row_rollout_general_inertia_matches_oracle(dtype, mode):
    """The 16-lane row rollout (chunks <= 16384, mpcb_rollout.hip) with a NON-diagonal inertia:
    the general quadratic form of w x Jw and, in fp64, the general tangent of the exported
    [A|B] (template DJ = false; the reference's diagonal J takes DJ = true everywhere else), at
    an odd horizon and a ragged batch, against the oracle with the same J."""
    from oracle.model import Params
    N, B = 13, 37
    inp = make_inputs('c2', ids=np.arange(B, dtype=np.uint64), N=N)
    spec = OcpSpec(N=N, params=Params(J=_J_GENERAL))
    m = _mpc(N, dtype, max_batch=B, path='split', J=_J_GENERAL)
    cast = (lambda a: a.astype(np.float32).astype(np.float64)) if dtype == 'f32' else (lambda a: a)
    if mode == 'iterate':
        rng = np.random.default_rng(13)
        xbar = inp['xref'] + rng.normal(scale=0.05, size=(B, N + 1, 12))
        ubar = inp['uref'] + rng.normal(scale=1.0, size=(B, N, 4))
        m.solve_iterate(inp['x0'], xbar, ubar, inp['xref'], inp['uref'])
        o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, mode='iterate', xbar=xbar, ubar=ubar)
    else:
        m.solve(inp['x0'], inp['xref'], inp['uref'])
        o = mpc_solve(cast(inp['x0']), cast(inp['xref']), cast(inp['uref']), spec)
    torch.cuda.synchronize()
    tol = 1e-9 if dtype == 'f64' else 5e-5
    e_u = relerr(m.get_control().cpu().numpy(), o['u0'])
    e_x = relerr(m.get_state_trajectory().cpu().numpy(), o['X'])
    e_U = relerr(m.get_input_trajectory().cpu().numpy(), o['U'])
    print(f'general J {dtype} {mode}: max rel err u0 {e_u.max():.2e} X {e_x.max():.2e} U {e_U.max():.2e}')
    assert (m.get_status().cpu().numpy() == 0).all()
    assert e_u.max() < tol and e_x.max() < tol and e_U.max() < tol


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_row_rollout_sincos_redo_matches_oracle(dtype):
    """The row rollout's speculative interval (mpcb_rollout.hip `interval`): sin/cos without
    range fallbacks, stages 1..3 (fp64) by angle addition over the stage offset, and a redo of the
    interval with the full reduction when an angle lane leaves those ranges.  Waves mixing normal
    instances with fast body rates (stage offsets above 1/8 rad) and huge roll angles (the
    sin/cos large-argument fallback) against the oracle."""
    N, B = 20, 40
    inp = make_inputs('c2', ids=np.arange(B, dtype=np.uint64), N=N)
    x0 = inp['x0'].copy()
    if dtype == 'f64':   # fast rates: offsets h/2 * rate > 1/8 (fp32 has no angle addition)
        x0[0:12:2, 9:12] = [[14.0, -11.0, 9.0]]
    big = np.zeros(B, bool)
    big[1:12:4] = True
    x0[big, 3] += 1.0e6 if dtype == 'f64' else 1.0e4   # beyond the reduction's range
    m = _mpc(N, dtype, max_batch=B, path='split')
    m.solve(x0, inp['xref'], inp['uref'])
    torch.cuda.synchronize()
    u0, X, U = (t.cpu().numpy().copy() for t in (m.get_control(), m.get_state_trajectory(),
                                                  m.get_input_trajectory()))
    assert (m.get_status().cpu().numpy() == 0).all() and np.isfinite(X).all()
    if dtype == 'f64':
        o = mpc_solve(x0, inp['xref'], inp['uref'], OcpSpec(N=N))
        e_u, e_x, e_U = relerr(u0, o['u0']), relerr(X, o['X']), relerr(U, o['U'])
        print(f'sincos redo f64: max rel err u0 {e_u.max():.2e} X {e_x.max():.2e} U {e_U.max():.2e}')
        assert e_u.max() < 1e-9 and e_x.max() < 1e-9 and e_U.max() < 1e-9
    else:
        # a roll of 1e4 rad carries ~1e-3 rad of fp32 rounding, so those instances have no fp32
        # oracle; the others are checked against it, and must come out bit for bit as in a batch
        # without the large angles (the redo runs sc() = sc_core() on their lanes)
        cast = lambda a: a.astype(np.float32).astype(np.float64)
        o = mpc_solve(cast(x0[~big]), cast(inp['xref'][~big]), cast(inp['uref'][~big]), OcpSpec(N=N))
        e_u = relerr(u0[~big], o['u0'])
        e_U = relerr(U[~big], o['U'])
        print(f'sincos redo f32: max rel err u0 {e_u.max():.2e} U {e_U.max():.2e}')
        assert e_u.max() < 5e-5 and e_U.max() < 5e-5
        x1 = x0.copy()
        x1[big, 3] -= 1.0e4
        m.solve(x1, inp['xref'], inp['uref'])
        torch.cuda.synchronize()
        assert np.array_equal(m.get_control().cpu().numpy()[~big], u0[~big])
        assert np.array_equal(m.get_state_trajectory().cpu().numpy()[~big], X[~big])


@pytest.mark.parametrize('mode', ['rollout', 'iterate'])
def test_fused_rollout_riccati_equals_two_kernels(mode):
    """c2's row_riccati_kernel (P1 and P2 of a quad in one launch) against the same two bodies as
    two launches (MPCB_FUSE_P12=0): the same operations, so the same bits."""
    N, B = 20, 45
    inp = make_inputs('c2', ids=np.arange(B, dtype=np.uint64), N=N)
    rng = np.random.default_rng(21)
    xbar = inp['xref'] + rng.normal(scale=0.05, size=(B, N + 1, 12))
    ubar = inp['uref'] + rng.normal(scale=1.0, size=(B, N, 4))
    res = []
    for fuse in ('1', '0'):
        os.environ['MPCB_FUSE_P12'] = fuse
        try:
            m = _mpc(N, 'f64', max_batch=B, path='split')
            if mode == 'iterate':
                m.solve_iterate(inp['x0'], xbar, ubar, inp['xref'], inp['uref'])
            else:
                m.solve(inp['x0'], inp['xref'], inp['uref'])
            torch.cuda.synchronize()
        finally:
            os.environ.pop('MPCB_FUSE_P12')
        res.append([t.cpu().numpy().copy() for t in (m.get_control(), m.get_state_trajectory(),
                                                      m.get_input_trajectory(), m.get_status())])
    for a, b in zip(*res):
        assert np.array_equal(a, b)


@pytest.mark.parametrize('N', [20, 7])
def test_rollout_tangent_export_equals_captured_scalar_path(N):
    """fp64 small chunks: the rollout that integrates the sensitivities and exports [A|B]
    (SplitArgs::tin, the default) against the round-3 split whose P2 integrates them from the
    captured scalars (MPCB_P1_TAN=0): the same solve to rounding, both modes."""
    B = 61
    inp = make_inputs('c2', ids=np.arange(B, dtype=np.uint64), N=N)
    res = []
    for tan in ('1', '0'):
        os.environ['MPCB_P1_TAN'] = tan
        try:
            m = _mpc(N, 'f64', max_batch=B, path='split')
        finally:
            os.environ.pop('MPCB_P1_TAN')
        m.solve(inp['x0'], inp['xref'], inp['uref'])
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in (m.get_control(), m.get_state_trajectory(), m.get_input_trajectory())])
    for a, b in zip(*res):
        assert relerr(a, b).max() < 1e-12
