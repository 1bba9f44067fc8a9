"""MPCConfig: the problem definition handed to the HIP library (``mpcb_config``).

Defaults are the 12-state/4-input slice of the reference's JSON-pinned parameter set
(``src/scripts/simulation_blaster.py:12-30`` = ``acados_ocp_blasterModel.json``):
m = 9.0, J = diag(0.50781, 0.47314, 0.72975), l_x = 0.3434, l_y = 0.3475, c = 0.03,
Q = diag(1e3 x6, 5 x3, 10 x3), R = 0.05 I4, Q_N = 10 Q (``Q_t = 10*Q``, :25),
thrust box [0, 65] N (:30), dt = Tf/N = 1/30 s (JSON ``time_steps``), stage cost scaled by dt
(acados LINEAR_LS ``scaling = time_steps[k]``).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib

NX, NU = 12, 4          # the rigid-body slice (BASELINE configs)
NX17, NU17 = 17, 6      # the full reference model


def _default_Q(nx=NX):
    # simulation_blaster.py:24 (JSON cost.W diag[0:17]); the 12/4 slice keeps the first 12
    q = [1e3] * 6 + [5.0] * 3 + [10.0] * 3 + [1e-2] * 2 + [1e3] * 3
    return np.diag(q[:nx])


def _default_R(nu=NU):
    # simulation_blaster.py:27 (JSON cost.W diag[17:23])
    r = [0.05] * 4 + [1e-5] * 2
    return np.diag(r[:nu])


@dataclass
class MPCConfig:
    """nx/nu select the model: 12/4 (the rigid-body slice, BASELINE configs, MI355X-tuned
    kernels) or 17/6 (the full reference model; ``MPCConfig.full()`` gives the JSON-pinned OCP)."""
    N: int = 20
    dt: float = 1.0 / 30.0
    dtype: str = 'f64'                 # 'f64' | 'f32'
    mass: float = 9.0
    J: np.ndarray = field(default_factory=lambda: np.diag([0.50781, 0.47314, 0.72975]))
    lx: float = 0.3434
    ly: float = 0.3475
    c: float = 0.03
    g: float = 9.81
    t_blast: float = 0.0
    Q: np.ndarray | None = None        # default diag of simulation_blaster.py:24
    R: np.ndarray | None = None        # default diag of simulation_blaster.py:27
    QN: np.ndarray | None = None       # default 10 * Q
    cost_scale: float | None = None    # default dt
    lbu: np.ndarray | None = None      # None -> no input box
    ubu: np.ndarray | None = None
    lbx: np.ndarray | None = None      # 17/6 state box on stages 1..N-1 (needs lbu/ubu)
    ubx: np.ndarray | None = None
    max_as_iter: int = 200
    nx: int = NX
    nu: int = NU

    def __post_init__(self):
        if (self.nx, self.nu) not in ((NX, NU), (NX17, NU17)):
            raise ValueError(f'nx/nu {self.nx}/{self.nu}: the models are 12/4 and 17/6')
        self.Q = _default_Q(self.nx) if self.Q is None else np.asarray(self.Q, dtype=np.float64)
        self.R = _default_R(self.nu) if self.R is None else np.asarray(self.R, dtype=np.float64)
        self.QN = 10.0 * self.Q if self.QN is None else np.asarray(self.QN, dtype=np.float64)
        self.J = np.asarray(self.J, dtype=np.float64)
        nx, nu = self.nx, self.nu
        if self.Q.shape != (nx, nx) or self.QN.shape != (nx, nx) or self.R.shape != (nu, nu):
            raise ValueError(f'Q/QN must be {nx}x{nx} and R {nu}x{nu} for the {nx}/{nu} model')
        if self.dtype not in ('f64', 'f32'):
            raise ValueError(f'dtype {self.dtype!r}')
        if (self.lbu is None) != (self.ubu is None):
            raise ValueError('lbu and ubu must be given together')
        if (self.lbx is None) != (self.ubx is None):
            raise ValueError('lbx and ubx must be given together')
        if self.lbx is not None and (nx != NX17 or self.lbu is None):
            raise ValueError('the state box is implemented for the 17/6 model together with the input box')

    @classmethod
    def full(cls, **kw) -> 'MPCConfig':
        """The reference's own OCP (acados_ocp_blasterModel.json, simulation_blaster.py:12-30):
        17/6 model, N = 60, Tf = 2 (dt = 1/30), T_blast = 2.2 * 9.81, W = diag(Q17, R6),
        W_e = 10 Q17.  Pass ``lbu``/``ubu`` for the reference's input box (JSON idxbu: thrusts
        [0, 65] N, swivel rates +-0.0873 rad/s) and ``lbx``/``ubx`` for its state box (JSON idxbx,
        stages 1..N-1)."""
        d = dict(N=60, dt=2.0 / 60.0, t_blast=2.2 * 9.81, nx=NX17, nu=NU17)
        d.update(kw)
        return cls(**d)

    @property
    def boxed(self) -> bool:
        return self.lbu is not None

    @property
    def scale(self) -> float:
        return self.dt if self.cost_scale is None else float(self.cost_scale)

    def to_c(self) -> _lib.MpcbConfig:
        c = _lib.MpcbConfig()
        c.nx, c.nu, c.N = int(self.nx), int(self.nu), int(self.N)
        c.dtype = _lib.MPCB_F64 if self.dtype == 'f64' else _lib.MPCB_F32
        c.box_u = 1 if self.boxed else 0
        c.max_as_iter = int(self.max_as_iter)
        c.dt = float(self.dt)
        c.cost_scale = self.scale
        c.mass, c.lx, c.ly, c.c, c.g, c.t_blast = (float(v) for v in (
            self.mass, self.lx, self.ly, self.c, self.g, self.t_blast))
        for i, v in enumerate(self.J.reshape(-1)):
            c.J[i] = float(v)
        for i, v in enumerate(self.Q.reshape(-1)):
            c.Q[i] = float(v)
        for i, v in enumerate(self.QN.reshape(-1)):
            c.QN[i] = float(v)
        for i, v in enumerate(self.R.reshape(-1)):
            c.R[i] = float(v)
        if self.boxed:
            lb = np.broadcast_to(np.asarray(self.lbu, dtype=np.float64), (self.nu,))
            ub = np.broadcast_to(np.asarray(self.ubu, dtype=np.float64), (self.nu,))
            for i in range(self.nu):
                c.lbu[i], c.ubu[i] = float(lb[i]), float(ub[i])
        if self.lbx is not None:
            c.box_x = 1
            lb = np.broadcast_to(np.asarray(self.lbx, dtype=np.float64), (self.nx,))
            ub = np.broadcast_to(np.asarray(self.ubx, dtype=np.float64), (self.nx,))
            for i in range(self.nx):
                c.lbx[i], c.ubx[i] = float(lb[i]), float(ub[i])
        return c

    @property
    def torch_dtype(self):
        import torch
        return torch.float64 if self.dtype == 'f64' else torch.float32
