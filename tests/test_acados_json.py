"""acados OCP JSON loader on the reference's pinned description
(tests/golden/ocp_json_pin.json = the numbers of src/scripts/acados_ocp_blasterModel.json)."""
import json
import os
import warnings

import numpy as np
import pytest

from mpc_blaster_amd import MPCConfig, load_acados_ocp_json

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def _nested():
    """The pin re-nested into acados' JSON layout (dims / cost / constraints / solver_options)."""
    f = json.load(open(os.path.join(GOLD, 'ocp_json_pin.json')))
    cost = {k: f[k] for k in ('W', 'W_e', 'Vx', 'Vu', 'Vx_e', 'yref', 'cost_type', 'cost_type_e')}
    con = {k: f[k] for k in ('idxbu', 'lbu', 'ubu', 'idxbx', 'lbx', 'ubx', 'idxbx_0', 'idxbxe_0')}
    return dict(dims=f['dims'], cost=cost, constraints=con, parameter_values=f['parameter_values'],
                solver_options=f['solver_options'])


def test_full_model_matches_reference_defaults():
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        cfg, info = load_acados_ocp_json(_nested())
    ref = MPCConfig.full()
    assert (cfg.nx, cfg.nu, cfg.N) == (17, 6, 60)
    assert cfg.dt == pytest.approx(1.0 / 30.0, rel=1e-15)
    for a in ('Q', 'R', 'QN'):
        assert np.array_equal(getattr(cfg, a), getattr(ref, a)), a
    assert cfg.t_blast == pytest.approx(21.582, rel=1e-12)
    assert info['idxbx'] == list(range(17)) and len(info['lbx']) == 17
    assert not any('state box' in str(x.message) for x in w)        # applied on the 17/6 model
    assert np.array_equal(cfg.lbx, info['lbx']) and np.array_equal(cfg.ubx, info['ubx'])
    assert cfg.lbx[2] == 0.0 and cfg.ubx[12] == pytest.approx(1.22173)
    assert np.array_equal(cfg.lbu, [0, 0, 0, 0, -0.0872665, -0.0872665])
    assert np.array_equal(cfg.ubu, [65, 65, 65, 65, 0.0872665, 0.0872665])


def test_slice_12_4_matches_baseline_config():
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        cfg, _ = load_acados_ocp_json(_nested(), slice_12_4=True)
    base = MPCConfig(N=60)
    assert (cfg.nx, cfg.nu) == (12, 4) and cfg.lbx is None
    for a in ('Q', 'R', 'QN'):
        assert np.array_equal(getattr(cfg, a), getattr(base, a)), a
    assert np.array_equal(cfg.lbu, np.zeros(4)) and np.array_equal(cfg.ubu, np.full(4, 65.0))
    assert cfg.t_blast == pytest.approx(21.582, rel=1e-12)


def test_rejects_unimplemented_solver_options():
    d = _nested()
    d['solver_options'] = dict(d['solver_options'], integrator_type='IRK')
    with pytest.raises(ValueError, match='integrator_type'):
        load_acados_ocp_json(d)
    d = _nested()
    d['solver_options'] = dict(d['solver_options'], sim_method_num_stages=[2] * 60)
    with pytest.raises(ValueError, match='num_stages'):
        load_acados_ocp_json(d)


def test_qp_iteration_cap_and_partial_box():
    """qp_solver_iter_max (500 in the reference JSON) becomes the device's QP iteration
    cap; a partial idxbu is refused rather than filled with +-1e20 rows."""
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        cfg, _ = load_acados_ocp_json(_nested())
        assert cfg.max_as_iter == 500
        d = _nested()
        d['constraints'] = dict(d['constraints'], idxbu=[0, 1, 2, 3], lbu=[0.0] * 4, ubu=[65.0] * 4)
        with pytest.raises(ValueError, match='idxbu'):
            load_acados_ocp_json(d)
