"""Single-instance per-step latency (the reference's own use: one MPC solve per 10 Hz control
step, mavros_blaster_sim.py:35, timed per step at simulation_blaster.py:107).

``measure_b1`` times, with the device synchronised after every step:

* ``c1_device_ms``  — BASELINE configs[0] (12/4, N = 10, fp64, hover) at B = 1, inputs and
  outputs resident on the device (the kernels alone plus launch);
* ``c1_host_ms``    — the same with NumPy inputs and u0* copied back to the host (H2D + solve +
  D2H), i.e. what ``solve(x0, x_ref, u_ref)`` / ``get_control()`` cost a caller holding host arrays;
* ``ref_loop_ms``   — one step of the reference script's loop through the acados-subset facade on
  the reference's own OCP (17/6, N = 60, input and state box, simulation_blaster.py:12-30 and
  :56-107: set(0,'lbx'/'ubx'), cost_set(k,'yref'), solve(), get(0,'u'), plant step).
"""
from __future__ import annotations

import time

import numpy as np


def _timed(fn, n, warm=3):
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    t = np.array(t) * 1e3
    return float(np.median(t)), float(np.percentile(t, 99))


def measure_b1(n: int = 200, device: int = 0) -> dict:
    import torch

    from .api import BatchedMPC
    from .config import MPCConfig
    out = {}
    m = BatchedMPC(MPCConfig(N=10, dtype='f64'), max_batch=1, device=device)
    x0 = np.array([[0.3, -0.2, 0.1, 0.05, -0.04, 0.1, 0.2, 0.1, -0.1, 0.02, -0.01, 0.03]])
    xref = np.zeros((1, 11, 12))
    uref = np.full((1, 10, 4), 22.0725)            # hover thrust per motor
    dev = lambda a: torch.as_tensor(a, dtype=torch.float64, device=device)  # noqa: E731
    dx0, dxr, dur = dev(x0), dev(xref), dev(uref)
    out['c1_device_ms'], out['c1_device_p99_ms'] = _timed(lambda: m.solve(dx0, dxr, dur), n)

    def host_step():
        m.solve(x0, xref, uref)
        return m.get_control().cpu().numpy()
    out['c1_host_ms'], out['c1_host_p99_ms'] = _timed(host_step, n)
    m.close()

    from .compat.blastermodel import blasterModel
    J = np.diag([0.50781, 0.47314, 0.72975])
    Q = np.diag([1e3] * 6 + [5.0] * 3 + [10.0] * 3 + [1e-2] * 2 + [1e3] * 3)
    R = np.diag([5e-2] * 4 + [1e-5] * 2)
    lbu = [0, 0, 0, 0, -0.0872665, -0.0872665]
    ubu = [65, 65, 65, 65, 0.0872665, 0.0872665]
    sb_lo = [-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0, -0.0872665,
             -0.0872665, -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5]
    sb_hi = [1.5, 1.5, 5.0, 0.174532925, 0.174532925, 0.349066, 1.0, 1.0, 1.0, 0.0872665, 0.0872665,
             0.0872665, 1.22173, 0.523599, 1.5, 1.5, 2.5]
    b = blasterModel(9.0, J, 0.3434, 0.3475, 60, 2.0, 0.03, Q, R, 10 * Q, 2.2 * 9.81,
                     np.array([sb_lo, sb_hi]), np.array([lbu, ubu]), full_model=True, device=device)
    b.generateModel()
    integrator, ocp = b.generateController()
    yref = np.zeros(23)
    yref[2], yref[14] = 3.5, 0.2            # simulation_blaster.py:48
    state = {'x': np.zeros(17)}

    def ref_step():
        x = state['x']
        ocp.set(0, 'lbx', x)
        ocp.set(0, 'ubx', x)
        for k in range(61):
            ocp.cost_set(k, 'yref', yref if k < 60 else yref[:17])
        ocp.solve()
        u = ocp.get(0, 'u')
        integrator.set('x', x)
        integrator.set('u', u)
        integrator.solve()
        state['x'] = integrator.get('x')
    out['ref_loop_ms'], out['ref_loop_p99_ms'] = _timed(ref_step, max(20, n // 10))
    out['note'] = ('median / p99 over sequential steps, device synchronised each step; the reference '
                   'control period is 100 ms (10 Hz, mavros_blaster_sim.py:35)')
    return out
