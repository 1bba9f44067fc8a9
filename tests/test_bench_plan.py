"""CPU checks that tie bench.py's roofline to the committed profiles: the kernels a bench workload
launches come from the library's own device-free plan (mpcb_plan_kernels, the selection code of
mpcb_create / mpcb_solve), and every one of them has an entry in that workload's committed PMC
summary (profiles/pmc_<w>.json), so ``roofline.traffic`` / ``executed_frac`` are never null for
want of a name (round-4 verdict item 1)."""
import json
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def bench():
    from mpc_blaster_amd.build import build
    build()
    import bench as b
    return b


@pytest.mark.parametrize('w', ['c2', 'c3', 'c4', 'c5'])
def test_every_bench_kernel_is_in_the_committed_pmc_summary(bench, w):
    wl = dict(bench.WORKLOADS[w], name=w)
    names = bench.phase_kernels(wl)
    assert 'riccati' in names
    per = json.load(open(os.path.join(REPO, 'profiles', f'pmc_{w}.json')))['per_kernel']
    for phase, k in names.items():
        assert k in per, (phase, k, sorted(per))
        # and pmc_kernel finds it (it exits on a committed summary without the kernel)
        assert bench.pmc_kernel(w, k) == per[k]


def test_pmc_kernel_refuses_a_summary_without_the_kernel(bench):
    with pytest.raises(SystemExit, match='no entry for the dominant kernel'):
        bench.pmc_kernel('c3', 'mpcb::riccati_kernel_f32<false, false>')


def test_flop_count_for_every_planned_kernel(bench):
    """kernel_flops knows every kernel any workload's plan names (rollout and iterate modes)."""
    from mpc_blaster_amd import MPCConfig, _lib
    for w, wl in bench.WORKLOADS.items():
        wl = dict(wl, name=w)
        box = wl['box']
        cfg = MPCConfig(N=wl['N'], dtype=wl['dtype'], lbu=np.zeros(4) if box else None,
                        ubu=np.full(4, 65.0) if box else None)
        for it in (False, True):
            r = {'qp': {'bwd_stages': 1.0, 'fwd_passes': 1.0}}
            for phase, k in _lib.plan_kernels(cfg.to_c(), wl['batch'], wl['batch'], iterate=it).items():
                assert bench.kernel_flops(wl, r, phase, k) > 0


def test_plan_follows_the_selection_switches():
    """The plan is the launch code run dry: the switches tests exercise change it the same way."""
    from mpc_blaster_amd import MPCConfig, _lib
    cfg = MPCConfig(N=20, dtype='f64').to_c()
    assert _lib.plan_kernels(cfg, 4096, 4096) == {
        'riccati': 'mpcb::row_riccati_kernel<false, true>', 'forward': 'mpcb::fwd_rm_kernel<double, false>'}
    os.environ['MPCB_FUSE_P12'] = '0'
    try:
        two = _lib.plan_kernels(cfg, 4096, 4096)
    finally:
        del os.environ['MPCB_FUSE_P12']
    assert two['nominal'] == 'mpcb::nominal_row_kernel<double, false, true, true>'
    assert two['riccati'] == 'mpcb::riccati_kernel_f64<true, false, true>'
    os.environ['MPCB_P1_TAN'] = '0'
    try:
        cap = _lib.plan_kernels(cfg, 4096, 4096, iterate=True)
    finally:
        del os.environ['MPCB_P1_TAN']
    assert cap['nominal'] == 'mpcb::nominal_row_kernel<double, true, true, false>'
    assert cap['riccati'] == 'mpcb::riccati_kernel_f64<true, true, false>'
    # chunks above 16384: thread-per-instance rollout and forward, no tangent export
    big = _lib.plan_kernels(cfg, 65536, 65536)
    assert big['nominal'] == 'mpcb::nominal_kernel<double, false>'
    assert big['forward'] == 'mpcb::forward_kernel<double, false, false>'
    # a non-diagonal inertia selects the general-J row kernels
    J = np.diag([0.50781, 0.47314, 0.72975])
    J[0, 1] = J[1, 0] = 0.01
    g = _lib.plan_kernels(MPCConfig(N=20, dtype='f64', J=J).to_c(), 4096, 4096)
    assert g['riccati'] == 'mpcb::row_riccati_kernel<false, false>'
    # the 17/6 model: nominal17q, the stage-parallel linearisation and the interior point
    full = _lib.plan_kernels(MPCConfig.full().to_c(), 4096, 4096)
    assert full == {'nominal': 'mpcb::nominal17q_kernel<double>', 'linearise': 'mpcb::lin17ws_kernel<double>',
                    'riccati': 'mpcb::q17::riccati17q_kernel<double, false, false>'}


def test_plan_refuses_bad_arguments():
    from mpc_blaster_amd import MPCConfig, _lib
    cfg = MPCConfig(N=20, dtype='f64').to_c()
    with pytest.raises(_lib.MpcbError):
        _lib.plan_kernels(cfg, 4096, 8192)
    cfg.nx = 9
    with pytest.raises(_lib.MpcbError):
        _lib.plan_kernels(cfg, 4096, 16)
