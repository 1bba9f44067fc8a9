"""GPU edge cases of the solve path through the C ABI: empty batches, a non-finite instance inside
a batch, the shortest horizon and long horizons.

* Empty batch: every path returns without launching anything and without an error.
* A NaN in one instance's x0: that instance reports a non-OK status, and every other instance's
  outputs are bit-identical to the same batch with a finite x0 in its place (instances are
  independent on every path: the fused row kernel, the thread-per-instance forward, the
  active-set work counter, the 17/6 interior point).  This found the row rollout's wave-wide
  slow-path redo (mpcb_row.h), which changed the last bits of the NaN instance's wave-mates.
* N = 1 and long horizons against the oracle at the fp64 bound of tests/test_gpu_parity.py
  (1e-9 normwise); the long unconstrained horizon takes the two-launch fallback of the fused
  kernel (its LDS staging exceeds the one-wave-per-SIMD share: mpcb_capi.hip select_path).
"""
import numpy as np
import pytest

from oracle.inputs import make_inputs
from oracle.ocp import OcpSpec, mpc_solve

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

STATUS_OK = 0


def relerr(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, dtype=np.float64).reshape(b.shape[0], -1)
    return np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1.0)


def _mpc(N, dtype, box, max_batch, env=None, monkeypatch=None):
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    cfg = MPCConfig(N=N, dtype=dtype, lbu=np.zeros(4) if box else None,
                    ubu=np.full(4, 65.0) if box else None)
    return BatchedMPC(cfg, max_batch=max_batch)


def _outputs(m):
    torch.cuda.synchronize()
    return [t.cpu().numpy().copy() for t in (m.get_control(), m.get_state_trajectory(),
                                             m.get_input_trajectory(), m.get_status())]


@pytest.mark.parametrize('N,dtype,box', [(20, 'f64', False), (20, 'f32', False), (30, 'f32', True)])
def test_empty_batch_is_a_noop(N, dtype, box):
    m = _mpc(N, dtype, box, 64)
    x0 = np.zeros((0, 12))
    xref = np.zeros((1, N + 1, 12))
    uref = np.full((1, N, 4), 22.0725)
    u0 = m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    assert tuple(u0.shape) == (0, 4)
    assert tuple(m.get_status().shape) == (0,)
    if box:
        assert tuple(m.qp_stats(0).shape) == (0, 2)
    # and the handle still solves afterwards
    inp = make_inputs('c4' if box else 'c2', ids=np.arange(5, dtype=np.uint64), N=N)
    m.solve(inp['x0'], inp['xref'], inp['uref'])
    assert (_outputs(m)[3] == STATUS_OK).all()


@pytest.mark.parametrize('cfg,N,dtype,box,B', [
    ('c2', 20, 'f64', False, 4096),    # fused row kernel + 16-lane forward
    ('c2', 20, 'f64', False, 203),     # small-batch path
    ('c3', 20, 'f32', False, 20000),   # thread-per-instance rollout / forward, captured-scalar P2
    ('c4', 30, 'f32', True, 1000),     # P2 exports + active-set work counter
    ('c4', 30, 'f64', True, 300),
])
def test_nonfinite_instance_is_flagged_and_isolated(cfg, N, dtype, box, B):
    inp = make_inputs(cfg, ids=np.arange(B, dtype=np.uint64), N=N)
    bad = [17, B - 2]
    m = _mpc(N, dtype, box, B)
    x_ok = inp['x0'].copy()
    x_ok[bad] = x_ok[[b - 1 for b in bad]]
    m.solve(x_ok, inp['xref'], inp['uref'])
    ref = _outputs(m)
    x_nan = inp['x0'].copy()
    x_nan[bad[0], 3] = np.nan
    x_nan[bad[1], 0] = np.inf
    m.solve(x_nan, inp['xref'], inp['uref'])
    got = _outputs(m)
    st = got[3]
    print(f'{cfg} {dtype} box={box} B={B}: status of the non-finite instances {st[bad].tolist()}')
    assert (st[bad] != STATUS_OK).all()
    keep = np.setdiff1d(np.arange(B), bad)
    assert (st[keep] == STATUS_OK).all() and (ref[3] == STATUS_OK).all()
    for name, a, b in zip(('u0', 'X', 'U'), got[:3], ref[:3]):
        diff = np.nonzero((a[keep] != b[keep]).reshape(len(keep), -1).any(axis=1))[0]
        if len(diff):
            print(f'  {name}: {len(diff)} instances differ, e.g. {keep[diff[:12]].tolist()}, max abs '
                  f'{np.abs(a[keep] - b[keep]).max():.3e}')
    for a, b in zip(got[:3], ref[:3]):
        assert np.array_equal(a[keep], b[keep])


@pytest.mark.parametrize('N,box,path', [(1, False, None), (1, True, None), (1, False, 'split'),
                                        (200, False, None), (200, False, 'split'), (64, True, None)])
def test_horizon_extremes_match_oracle_fp64(N, box, path, monkeypatch):
    B = 37 if path is None else 2048
    cfg = 'c4' if box else 'c3'
    inp = make_inputs(cfg, ids=np.arange(B, dtype=np.uint64), N=N)
    env = {'MPCB_SPLIT_MIN_BATCH': '1'} if path == 'split' else {}
    m = _mpc(N, 'f64', box, B, env, monkeypatch)
    m.solve(inp['x0'], inp['xref'], inp['uref'])
    u0, X, U, st = _outputs(m)
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'],
                  OcpSpec(N=N, lbu=np.zeros(4) if box else None, ubu=np.full(4, 65.0) if box else None))
    e = max(relerr(u0, o['u0']).max(), relerr(X, o['X']).max(), relerr(U, o['U']).max())
    print(f'N={N} box={box} path={path} B={B}: max rel err {e:.2e}')
    assert (st == o['status']).all() and (st == STATUS_OK).all()
    assert e < 1e-9


@pytest.mark.parametrize('states', [False, True])
def test_full17_nonfinite_instance_is_flagged_and_isolated(states):
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from test_gpu_full17 import LBU17, SB_HI, SB_LO, UBU17, _inputs
    N, B = 20, 64
    kw = dict(lbx=SB_LO, ubx=SB_HI) if states else {}
    m = BatchedMPC(MPCConfig.full(N=N, lbu=LBU17, ubu=UBU17, **kw), max_batch=B)
    x0, xref, uref, p = _inputs(B, N, 41)
    m.set_params(p)
    x_ok = x0.copy()
    x_ok[9] = x_ok[8]
    m.solve(x_ok, xref, uref)
    ref = _outputs(m)
    x_nan = x0.copy()
    x_nan[9, 5] = np.nan
    m.solve(x_nan, xref, uref)
    got = _outputs(m)
    print(f'17/6 boxes (states {states}): status of the non-finite instance {int(got[3][9])}')
    assert got[3][9] != STATUS_OK
    keep = np.setdiff1d(np.arange(B), [9])
    assert (got[3][keep] == ref[3][keep]).all()
    for a, b in zip(got[:3], ref[:3]):
        assert np.array_equal(a[keep], b[keep])


@pytest.mark.parametrize('cfg,N,dtype,box,B', [
    ('c2', 20, 'f64', False, 4096),    # fused row kernel + 16-lane forward
    ('c3', 20, 'f32', False, 20000),   # thread-per-instance path
    ('c4', 30, 'f32', True, 3000),     # active-set work counter
    ('c5', 40, 'f32', False, 70000),   # two chunks (65,536 + 4,464), wind
])
def test_batch_order_invariance(cfg, N, dtype, box, B):
    """Reversing the batch reverses the outputs bit for bit: an instance's result depends neither
    on its wave-mates nor on its position in the chunk or on which chunk holds it."""
    inp = make_inputs(cfg, ids=np.arange(B, dtype=np.uint64), N=N)
    m = _mpc(N, dtype, box, B)
    wind = inp['wind']
    m.solve(inp['x0'], inp['xref'], inp['uref'], wind=wind)
    fwd = _outputs(m)
    rev = {k: (None if v is None else np.ascontiguousarray(v[::-1] if v.shape[0] == B else v))
           for k, v in inp.items()}
    m.solve(rev['x0'], rev['xref'], rev['uref'], wind=rev['wind'])
    bwd = _outputs(m)
    for name, a, b in zip(('u0', 'X', 'U', 'status'), fwd, bwd):
        same = np.array_equal(a, b[::-1])
        if not same:
            d = np.nonzero((a != b[::-1]).reshape(B, -1).any(axis=1))[0]
            print(f'{cfg}: {name} differs on {len(d)} instances, e.g. {d[:12].tolist()}')
        assert same
    assert (fwd[3] == STATUS_OK).all()


@pytest.mark.parametrize('dtype,mode', [('f64', 'rollout'), ('f64', 'iterate'), ('f32', 'rollout')])
def test_box_slow_instances_take_the_interior_point(dtype, mode):
    """The 12/4 input box's fallback (mpcb_asipm.h): on draws where the active set's backup rule is
    slow (sine references, +-5 N wind) the instances unconverged after AS_IPM_AFTER passes are
    solved by the interior point, as in oracle.ocp.pdas_solve.  fp64: the device against the oracle
    at 1e-9 normwise, same statuses (all OK).  fp32: the interior point stops at mu <= 1e-8
    (IpmTol<float>) about 1e-4 off the minimiser, and its active set then goes through the
    refinement kernel (crossover, mpcb_asipm.h), so every instance that fp32 data can pin
    (oracle.ocp.fp32_sensitivity <= 1e-5) is held to 5e-5 normwise, the others (counted) to the
    QP's optimal objective; all inside the box."""
    from test_oracle_ocp import hard_box_inputs
    from oracle.ocp import AS_IPM_AFTER
    N, B = 18, 192
    inp = hard_box_inputs(B, N, 11)
    m = _mpc(N, dtype, True, B)
    cast = (lambda a: a.astype(np.float32).astype(np.float64)) if dtype == 'f32' else (lambda a: a)
    x0, xref, uref, wind = (cast(inp[k]) for k in ('x0', 'xref', 'uref', 'wind'))
    spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0))
    if mode == 'iterate':
        rng = np.random.default_rng(3)
        xbar = cast(xref + rng.normal(scale=0.05, size=(B, N + 1, 12)))
        ubar = cast(uref + rng.normal(scale=1.0, size=(B, N, 4)))
        m.solve_iterate(x0, xbar, ubar, xref, uref, wind=wind)
        o = mpc_solve(x0, xref, uref, spec, wind=wind, mode='iterate', xbar=xbar, ubar=ubar)
    else:
        m.solve(x0, xref, uref, wind=wind)
        o = mpc_solve(x0, xref, uref, spec, wind=wind)
    u0, X, U, st = _outputs(m)
    fb = o['fallback']
    e = max(relerr(u0, o['u0']).max(), relerr(X, o['X']).max(), relerr(U, o['U']).max())
    print(f'{dtype} {mode}: {fb.sum()} instances took the interior point in the oracle ({(o["iters"] > AS_IPM_AFTER).sum()} '
          f'after {AS_IPM_AFTER} passes), max rel err {e:.2e}, status {np.bincount(st, minlength=5).tolist()}')
    assert fb.sum() >= 5
    assert (st == 0).all() and (o['status'] == 0).all()
    if dtype == 'f64':
        assert e < 1e-9
    else:
        from oracle.ocp import fp32_sensitivity
        from test_gpu_fuzz import qp_objective
        o = mpc_solve(x0, xref, uref, spec, wind=wind, return_lin=True,
                      **(dict(mode='iterate', xbar=xbar, ubar=ubar) if mode == 'iterate' else {}))
        ill = fp32_sensitivity(o, x0, xref, uref, spec) > 1e-5
        ew = max(relerr(u0, o['u0'])[~ill].max(), relerr(X, o['X'])[~ill].max(), relerr(U, o['U'])[~ill].max())
        gap = qp_objective(o, U, x0, xref, uref, spec) / np.abs(qp_objective(o, o['U'], x0, xref, uref, spec)) - 1.0
        print(f'  fp32: {int(ill.sum())} of {B} fp32-ill-conditioned; the others max rel err {ew:.2e}; '
              f'objective gap max {gap.max():.2e}')
        assert ew < 5e-5 and (gap < 1e-5).all()
    tb = 1e-7 if dtype == 'f64' else 2e-4   # (interior iterates; fp32: the violation tolerance tol_u)
    assert (U >= -tb).all() and (U <= 65 + tb).all()


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_box_fallback_and_refinement_are_order_and_run_invariant(dtype):
    """The hand-over paths (interior point fallback, fp32 refinement list, mpcb_asipm.h /
    as_ref_kernel_f32) take instances through device-side queues filled by atomics, so their ORDER
    varies from run to run; an instance's result must not.  On the hard-box draw (many hand-overs):
    reversing the batch reverses every output bit for bit, and a soak of 12 repeated solves of a
    4x-tiled batch (several waves racing on the same queues) returns the first solve's bits each
    time."""
    from test_oracle_ocp import hard_box_inputs
    N, B = 18, 192
    inp = hard_box_inputs(B, N, 11)
    cast = (lambda a: a.astype(np.float32).astype(np.float64)) if dtype == 'f32' else (lambda a: a)
    x0, xref, uref, wind = (cast(inp[k]) for k in ('x0', 'xref', 'uref', 'wind'))
    m = _mpc(N, dtype, True, 4 * B)
    m.solve(x0, xref, uref, wind=wind)
    fwd = _outputs(m)
    r = lambda a: np.ascontiguousarray(a[::-1]) if a.shape[0] == B else a  # noqa: E731
    m.solve(r(x0), r(xref), r(uref), wind=r(wind))
    bwd = _outputs(m)
    for name, a, b in zip(('u0', 'X', 'U', 'status'), fwd, bwd):
        assert np.array_equal(a, b[::-1]), f'{dtype}: {name} depends on batch order'
    t = lambda a: np.ascontiguousarray(np.concatenate([a] * 4)) if a.shape[0] == B else a  # noqa: E731
    x4, xr4, ur4, w4 = t(x0), t(xref), t(uref), t(wind)
    m.solve(x4, xr4, ur4, wind=w4)
    first = _outputs(m)
    for a, b in zip(first, fwd):
        assert np.array_equal(a[:B], b) and np.array_equal(a[3 * B:], b)
    for k in range(12):
        m.solve(x4, xr4, ur4, wind=w4)
        got = _outputs(m)
        for name, a, b in zip(('u0', 'X', 'U', 'status'), got, first):
            assert np.array_equal(a, b), f'{dtype}: soak solve {k}: {name} differs'
    print(f'{dtype}: order and 12-solve soak bit-identical; status {np.bincount(fwd[3], minlength=5).tolist()}')


def test_box_interior_point_from_start_matches_oracle():
    """max_as_iter = 1: every instance whose unconstrained solution leaves the box goes straight to
    the interior point (mpcb.h max_as_iter), on the device as in oracle.ocp.pdas_solve."""
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    from test_oracle_ocp import hard_box_inputs
    N, B = 18, 192
    inp = hard_box_inputs(B, N, 12)
    m = BatchedMPC(MPCConfig(N=N, dtype='f64', lbu=np.zeros(4), ubu=np.full(4, 65.0), max_as_iter=1), max_batch=B)
    m.solve(inp['x0'], inp['xref'], inp['uref'], wind=inp['wind'])
    u0, X, U, st = _outputs(m)
    spec = OcpSpec(N=N, lbu=np.zeros(4), ubu=np.full(4, 65.0), max_as_iter=1)
    o = mpc_solve(inp['x0'], inp['xref'], inp['uref'], spec, wind=inp['wind'])
    e = max(relerr(u0, o['u0']).max(), relerr(X, o['X']).max(), relerr(U, o['U']).max())
    print(f'interior point from the start: {o["fallback"].sum()} of {B} handed over, max rel err {e:.2e}')
    assert o['fallback'].sum() > B // 2
    assert (st == 0).all() and (o['status'] == 0).all()
    assert e < 1e-9
