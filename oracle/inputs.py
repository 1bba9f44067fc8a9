"""Synthetic MPC inputs for the BASELINE configs (oracle copy; test infrastructure only).

SURVEY.md §8(d): one Philox4x32-10 stream keyed by (seed, global instance id) so any shard or
subset of the batch reproduces exactly.  Bit-identical (fp64) to the device generator
``mpc_blaster_amd/csrc/mpcb_inputs.hip``.  Per instance 18 uniforms in [0, 1):

* cols 0-11  x0 = x_hover + a * (2u - 1),  a = [1,1,1 | .17,.17,.35 | .5,.5,.5 | .087 x3]
* cols 12-14 wind force (c5) = 5 * (2u - 1) N per world axis
* cols 15-17 sinusoid (c3): amplitude 0.2 + 0.8u, omega 0.5 + 1.5u, phase 2*pi*u

Hover: z = 3.5 m (``simulation_blaster.py:48`` yref), thrust 22.0725 N/motor
(``simulation_blaster.py:97`` commented-out hover input; = 9 * 9.81 / 4).
"""
from __future__ import annotations

import numpy as np

from .philox import uniform

NX, NU = 12, 4
HOVER_Z = 3.5
HOVER_T = 22.0725
X0_HALF_RANGE = np.array([1.0, 1.0, 1.0, 0.17, 0.17, 0.35, 0.5, 0.5, 0.5, 0.087, 0.087, 0.087])
N_UNIFORM = 18

CONFIGS = {
    # name: (seed, batch, N, dtype, ref kind, box, wind)
    'c1': dict(seed=1001, batch=1, N=10, dtype='f64', ref='hover', box=False, wind=False),
    'c2': dict(seed=1002, batch=4096, N=20, dtype='f64', ref='hover', box=False, wind=False),
    'c3': dict(seed=1003, batch=65536, N=20, dtype='f32', ref='sine', box=False, wind=False),
    'c4': dict(seed=1004, batch=262144, N=30, dtype='f32', ref='hover', box=True, wind=False),
    'c5': dict(seed=1005, batch=1048576, N=40, dtype='f32', ref='hover', box=False, wind=True),
}


def hover_state() -> np.ndarray:
    x = np.zeros(NX)
    x[2] = HOVER_Z
    return x


def draws(seed: int, ids) -> np.ndarray:
    return uniform(seed, np.asarray(ids, dtype=np.uint64), N_UNIFORM)


def make_x0(U: np.ndarray) -> np.ndarray:
    t = 2.0 * U[:, 0:12] - 1.0
    return hover_state()[None, :] + X0_HALF_RANGE[None, :] * t


def make_wind(U: np.ndarray) -> np.ndarray:
    return 5.0 * (2.0 * U[:, 12:15] - 1.0)


def make_sine_ref(U: np.ndarray, N: int, dt: float):
    """Per-instance circular reference with its analytic velocity; u_ref = hover."""
    amp = 0.2 + 0.8 * U[:, 15]
    om = 0.5 + 1.5 * U[:, 16]
    ph = 2.0 * np.pi * U[:, 17]
    Bsz = U.shape[0]
    xr = np.zeros((Bsz, N + 1, NX))
    t = np.arange(N + 1) * dt
    ang = om[:, None] * t[None, :] + ph[:, None]
    wt = om[:, None] * t[None, :]
    xr[:, :, 0] = amp[:, None] * np.sin(ang)
    xr[:, :, 1] = amp[:, None] * np.cos(ang)
    xr[:, :, 2] = HOVER_Z + 0.2 * np.sin(wt)
    xr[:, :, 6] = amp[:, None] * om[:, None] * np.cos(ang)
    xr[:, :, 7] = -amp[:, None] * om[:, None] * np.sin(ang)
    xr[:, :, 8] = 0.2 * om[:, None] * np.cos(wt)
    return xr


def make_inputs(cfg: str, ids=None, dt: float = 1.0 / 30.0, N: int | None = None):
    """Return dict(x0, xref, uref, wind) for the instance ids of config ``cfg`` (fp64)."""
    c = CONFIGS[cfg]
    N = c['N'] if N is None else N
    if ids is None:
        ids = np.arange(c['batch'], dtype=np.uint64)
    U = draws(c['seed'], ids)
    Bsz = U.shape[0]
    x0 = make_x0(U)
    if c['ref'] == 'sine':
        xref = make_sine_ref(U, N, dt)
    else:
        xref = np.broadcast_to(hover_state(), (Bsz, N + 1, NX)).copy()
    uref = np.full((Bsz, N, NU), HOVER_T)
    wind = make_wind(U) if c['wind'] else None
    return dict(x0=x0, xref=xref, uref=uref, wind=wind)
