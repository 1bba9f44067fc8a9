"""acados-subset facades over the HIP solver (the calls src/scripts actually make).

Reference call sites (SURVEY §8 b): ``ocp_solver.set(0,'lbx'|'ubx',x)`` / ``set(k,'p',p)``
(simulation_blaster.py:60-69), ``cost_set(k,'yref',y)`` (:63-78), ``solve()`` (:80),
``get(0,'u')`` / ``get(k,'x')`` (:87-89), ``get_cost()`` (:86); plant
``integrator.set('x'|'u'|'p', v)`` / ``solve()`` / ``get('x')`` (:82-104).

Semantics kept from acados SQP_RTI (JSON ``nlp_solver_type``): one Gauss-Newton step per
``solve()`` from the PERSISTENT iterate (initially all zeros; no shift between calls), x0 via
``lbx_0 = ubx_0``; ``get(k,'x')`` returns the new iterate (= linear prediction).  Each call
is synchronous like acados'.  ``batch`` > 1 keeps B independent solvers in one object: every
``set``/``cost_set`` value may then carry a leading batch axis.

Models: with a 17/6 config (``MPCConfig.full()``, ``blasterModel(..., full_model=True)``) the
facade is the reference's own OCP — vectors pass through unchanged and ``set(k, 'p', p)``
reaches the device parameters.  With the 12/4 rigid-body slice (the BASELINE configs) reference-
length vectors are accepted and sliced (x[0:12]; y = [x(17); u(6)] -> x[0:12], u[0:4]).
"""
from __future__ import annotations

import warnings

import numpy as np

from ..config import NU, NX, MPCConfig

NX_REF, NU_REF = 17, 6


def _torch():
    import torch
    return torch


def _as_batch(v, n, B, name):
    v = np.asarray(v, dtype=np.float64)
    if v.ndim == 1 or (v.ndim == 2 and v.shape[1] == 1 and v.shape[0] != B):
        v = v.reshape(1, -1)
    if v.shape[-1] != n:
        raise ValueError(f'{name}: length {v.shape[-1]} != {n}')
    return np.broadcast_to(v, (B, n))


def _slice_x(v, B, name, nx=NX):
    v = np.asarray(v, dtype=np.float64)
    n = v.shape[-1] if v.ndim else 0
    if n == NX_REF and nx == NX:
        v = v[..., :NX]
    return _as_batch(v, nx, B, name)


def _slice_u(v, B, name, nu=NU):
    v = np.asarray(v, dtype=np.float64)
    if v.shape[-1] == NU_REF and nu == NU:
        v = v[..., :NU]
    return _as_batch(v, nu, B, name)


def _slice_y(v, B, name, nx=NX, nu=NU):
    v = np.asarray(v, dtype=np.float64)
    n = v.shape[-1]
    if n == NX_REF + NU_REF and nx == NX:
        v = np.concatenate([v[..., :NX], v[..., NX_REF:NX_REF + NU]], axis=-1)
    return _as_batch(v, nx + nu, B, name)


class AcadosOcpSolver:
    """``AcadosOcpSolver`` subset: set / cost_set / solve / get / get_cost (B instances)."""

    def __init__(self, config: MPCConfig, batch: int = 1, device: int = 0, json_file=None):
        from ..api import BatchedMPC
        torch = _torch()
        self.cfg = config
        self.B = int(batch)
        self.json_file = json_file
        self.mpc = BatchedMPC(config, max_batch=self.B, device=device)
        dev = f'cuda:{self.mpc.device}'
        N = config.N
        dt = config.torch_dtype
        self._dev = dev
        self.nx, self.nu = config.nx, config.nu
        NX, NU = self.nx, self.nu
        self.xbar = torch.zeros((self.B, N + 1, NX), dtype=dt, device=dev)   # acados init: zeros
        self.ubar = torch.zeros((self.B, N, NU), dtype=dt, device=dev)
        self.x0 = np.zeros((self.B, NX))
        self._lbx0 = None
        self.yref = np.zeros((self.B, N + 1, NX + NU))
        self.status = np.zeros(self.B, dtype=np.int32)
        # acados parameter_values per stage (blastermodel.py:280-282: zeros, T_blast = p[24]);
        # uploaded at the next solve() when a set(k, 'p') changed them
        self._p = np.zeros((self.B, N + 1, 25))
        self._p[..., 24] = config.t_blast
        self._p_dirty = False

    @property
    def N(self):
        return self.cfg.N

    # -------------------------------------------------------------- setters
    def set(self, stage: int, field: str, value):
        torch = _torch()
        if field in ('lbx', 'ubx'):
            if stage != 0:
                raise NotImplementedError('state boxes beyond stage 0 are not part of this build')
            v = _slice_x(value, self.B, field, self.nx)
            if field == 'lbx':
                self._lbx0 = v.copy()
            else:
                if self._lbx0 is not None and not np.array_equal(self._lbx0, v):
                    raise NotImplementedError('stage-0 state box must be an equality (lbx_0 == ubx_0)')
                self.x0 = v.copy()
        elif field == 'x':
            self.xbar[:, stage] = torch.as_tensor(np.array(_slice_x(value, self.B, 'x', self.nx)),
                                                  dtype=self.xbar.dtype, device=self._dev)
        elif field == 'u':
            self.ubar[:, stage] = torch.as_tensor(np.array(_slice_u(value, self.B, 'u', self.nu)),
                                                  dtype=self.ubar.dtype, device=self._dev)
        elif field == 'p':
            if not 0 <= stage <= self.N:
                raise IndexError(f'stage {stage} outside 0..{self.N}')
            self._p[:, stage] = _as_batch(value, 25, self.B, 'p')
            self._p_dirty = True
        else:
            raise KeyError(f'field {field!r} not supported')

    def _upload_params(self):
        """Hand the per-stage parameters to the device (acados keeps p per stage; the terminal
        stage has no dynamics, so stages 0..N-1 are what the solve reads).  The dirty flag is
        cleared only once the device has accepted them: a rejected set keeps failing."""
        p = self._p[:, :self.N]
        if self.nx == NX_REF:
            same_stages = bool(np.all(p == p[:, :1]))
            same_rows = bool(np.all(p == p[:1]))
            self.mpc.set_params(p[:1, 0] if (same_stages and same_rows) else
                                (p[:, 0] if same_stages else p))
            self._p_dirty = False
            return
        # 12/4 slice: T_blast (p[24]) is the model's only parameter there, a handle scalar
        t = p[..., 24]
        if not np.all(t == t.flat[0]):
            raise NotImplementedError('the 12/4 slice takes one T_blast for every instance and stage '
                                      '(stage- or instance-varying p[24] needs the 17/6 model)')
        if np.any(p[..., :24] != 0):
            warnings.warn('POC Jacobian parameters only affect the POC states, which the 12/4 '
                          'model does not carry; ignored', stacklevel=3)
        if float(t.flat[0]) != self.cfg.t_blast:
            self.mpc.set_t_blast(float(t.flat[0]))
        self._p_dirty = False

    def cost_set(self, stage: int, field: str, value):
        if field != 'yref':
            raise KeyError(f'cost field {field!r} not supported (weights are fixed at creation)')
        if stage == self.N:
            self.yref[:, stage, :self.nx] = _slice_x(value, self.B, 'yref_e', self.nx)
        else:
            self.yref[:, stage] = _slice_y(value, self.B, 'yref', self.nx, self.nu)

    # -------------------------------------------------------------- solve
    def solve(self) -> int:
        torch = _torch()
        if self._p_dirty:
            self._upload_params()
        xr = self.yref[:, :, :self.nx]
        ur = self.yref[:, :self.N, self.nx:]
        self.mpc.solve_iterate(self.x0, self.xbar, self.ubar, xr, ur,
                               out=(torch.empty((self.B, self.nu), dtype=self.xbar.dtype, device=self._dev),
                                    self.xbar, self.ubar,
                                    torch.empty((self.B,), dtype=torch.int32, device=self._dev)))
        torch.cuda.synchronize(self.mpc.device)
        self.status = self.mpc.get_status().cpu().numpy()
        return int(self.status.max())

    # -------------------------------------------------------------- getters
    def get(self, stage: int, field: str):
        if field == 'x':
            v = self.xbar[:, stage].cpu().numpy()
        elif field == 'u':
            v = self.ubar[:, stage].cpu().numpy()
        else:
            raise KeyError(f'field {field!r} not supported')
        return v[0] if self.B == 1 else v

    def get_cost(self):
        """Objective at the current iterate (what acados' get_cost() evaluates)."""
        torch = _torch()
        dt = self.xbar.dtype
        Q = torch.as_tensor(self.cfg.Q, dtype=dt, device=self._dev)
        R = torch.as_tensor(self.cfg.R, dtype=dt, device=self._dev)
        QN = torch.as_tensor(self.cfg.QN, dtype=dt, device=self._dev)
        yr = torch.as_tensor(self.yref, dtype=dt, device=self._dev)
        ex = self.xbar[:, :-1] - yr[:, :-1, :self.nx]
        eu = self.ubar - yr[:, :-1, self.nx:]
        eN = self.xbar[:, -1] - yr[:, -1, :self.nx]
        c = 0.5 * self.cfg.scale * (torch.einsum('bki,ij,bkj->b', ex, Q, ex) + torch.einsum('bki,ij,bkj->b', eu, R, eu))
        c = c + 0.5 * torch.einsum('bi,ij,bj->b', eN, QN, eN)
        c = c.cpu().numpy()
        return float(c[0]) if self.B == 1 else c


class AcadosSimSolver:
    """``AcadosSimSolver`` subset: set('x'|'u'|'p'|'T') / solve() / get('x') — one RK4 step."""

    def __init__(self, config: MPCConfig, batch: int = 1, device: int = 0, json_file=None):
        from ..api import BatchedMPC
        self.cfg = config
        self.B = int(batch)
        self.mpc = BatchedMPC(config, max_batch=self.B, device=device)
        self.nx, self.nu = config.nx, config.nu
        self.x = np.zeros((self.B, self.nx))
        self.u = np.zeros((self.B, self.nu))
        self.T = config.dt          # JSON Tsim = Tf/N
        self.xn = self.x.copy()

    def set(self, field: str, value):
        if field == 'x':
            self.x = _slice_x(value, self.B, 'x', self.nx).copy()
        elif field == 'u':
            self.u = _slice_u(value, self.B, 'u', self.nu).copy()
        elif field == 'p':
            p = _as_batch(value, 25, self.B, 'p')
            if self.nx == NX_REF:
                self.mpc.set_params(p[:1] if np.all(p == p[:1]) else p)
            else:
                if not np.all(p[:, 24] == p[0, 24]):
                    raise NotImplementedError('the 12/4 slice takes one T_blast for every instance')
                if float(p[0, 24]) != self.cfg.t_blast:
                    self.mpc.set_t_blast(float(p[0, 24]))
        elif field == 'T':
            self.T = float(value)
        else:
            raise KeyError(f'field {field!r} not supported')

    def solve(self) -> int:
        torch = _torch()
        xo = self.mpc.sim_step(self.x, self.u, T=self.T)
        torch.cuda.synchronize(self.mpc.device)
        self.xn = xo.cpu().numpy()
        return 0 if np.isfinite(self.xn).all() else 1

    def get(self, field: str):
        if field != 'x':
            raise KeyError(f'field {field!r} not supported')
        return self.xn[0] if self.B == 1 else self.xn
