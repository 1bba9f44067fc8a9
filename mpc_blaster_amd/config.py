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

NX, NU = 12, 4


def _default_Q():
    return np.diag([1e3] * 6 + [5.0] * 3 + [10.0] * 3)


def _default_R():
    return np.diag([0.05] * 4)


@dataclass
class MPCConfig:
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
    Q: np.ndarray = field(default_factory=_default_Q)
    R: np.ndarray = field(default_factory=_default_R)
    QN: np.ndarray | None = None       # default 10 * Q
    cost_scale: float | None = None    # default dt
    lbu: np.ndarray | None = None      # None -> no input box
    ubu: np.ndarray | None = None
    max_as_iter: int = 200

    def __post_init__(self):
        self.Q = np.asarray(self.Q, dtype=np.float64)
        self.R = np.asarray(self.R, dtype=np.float64)
        self.QN = 10.0 * self.Q if self.QN is None else np.asarray(self.QN, dtype=np.float64)
        self.J = np.asarray(self.J, dtype=np.float64)
        if self.Q.shape != (NX, NX) or self.QN.shape != (NX, NX) or self.R.shape != (NU, NU):
            raise ValueError('Q/QN must be 12x12 and R 4x4 for the 12-state/4-input model')
        if self.dtype not in ('f64', 'f32'):
            raise ValueError(f'dtype {self.dtype!r}')
        if (self.lbu is None) != (self.ubu is None):
            raise ValueError('lbu and ubu must be given together')

    @property
    def boxed(self) -> bool:
        return self.lbu is not None

    @property
    def scale(self) -> float:
        return self.dt if self.cost_scale is None else float(self.cost_scale)

    def to_c(self) -> _lib.MpcbConfig:
        c = _lib.MpcbConfig()
        c.nx, c.nu, c.N = NX, NU, int(self.N)
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
            lb = np.broadcast_to(np.asarray(self.lbu, dtype=np.float64), (NU,))
            ub = np.broadcast_to(np.asarray(self.ubu, dtype=np.float64), (NU,))
            for i in range(NU):
                c.lbu[i], c.ubu[i] = float(lb[i]), float(ub[i])
        return c

    @property
    def torch_dtype(self):
        import torch
        return torch.float64 if self.dtype == 'f64' else torch.float32
