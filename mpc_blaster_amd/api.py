"""Batch API over the HIP library: ``solve(x0, x_ref, u_ref)`` / ``get_control()``.

This is the north_star call surface for the per-control-step solve that the reference runs
one instance at a time through ``ocp_solver.solve()`` (src/scripts/simulation_blaster.py:80).
Device buffers are torch ROCm tensors (plumbing only); every computation runs in
libmpcblaster.so.  Calls are asynchronous on torch's current stream; results are valid once
that stream is synchronised (``torch.cuda.synchronize()`` or reading them on the host).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

from . import _lib
from .config import MPCConfig


def _torch():
    import torch
    return torch


class BatchedMPC:
    """A handle bound to one GPU holding the workspace for up to ``max_batch`` instances."""

    def __init__(self, config: MPCConfig, max_batch: int, device: int | None = None):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError('BatchedMPC needs a ROCm GPU (torch.cuda.is_available() is False)')
        self.lib = _lib.load()
        self.cfg = config
        self.device = torch.cuda.current_device() if device is None else int(device)
        self._tdev = torch.device('cuda', self.device)
        self.max_batch = int(max_batch)
        self._c = config.to_c()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.mpcb_create(ctypes.byref(self._c), self.device, self.max_batch,
                                            ctypes.byref(h)))
        self._h = h
        self.dtype = config.torch_dtype
        self.nx, self.nu = config.nx, config.nu
        self._u0 = self._X = self._U = self._status = None
        self._params = None

    # ------------------------------------------------------------------ helpers
    def close(self):
        if getattr(self, '_h', None) is not None and self._h.value:
            self.lib.mpcb_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def workspace_bytes(self) -> int:
        return int(self.lib.mpcb_workspace_bytes(self._h))

    @property
    def path(self) -> str:
        """'split' (nominal / Riccati / forward kernels) or 'fused' (one kernel)."""
        return 'split' if self.lib.mpcb_path(self._h) == 1 else 'fused'

    def set_timing(self, enable: bool = True):
        """Record HIP events around each kernel phase of later solves (see ``last_timing``)."""
        _lib.check(self.lib.mpcb_set_timing(self._h, 1 if enable else 0))

    def last_timing(self) -> dict:
        """Device ms of the last timed solve's phases: nominal, riccati (dominant), forward
        (17/6 model: nominal, riccati = Riccati + forward or the interior point, linearise)."""
        ms = (ctypes.c_float * 3)()
        _lib.check(self.lib.mpcb_last_timing(self._h, ms))
        if self.nx == 17:
            return dict(nominal=ms[0], riccati=ms[1], linearise=ms[2])
        return dict(nominal=ms[0], riccati=ms[1], forward=ms[2])

    def last_kernels(self) -> dict:
        """{phase: rocprof kernel name} of what the last solve launched (phases as ``last_timing``)."""
        return _lib.kernel_names(lambda b, n: self.lib.mpcb_last_kernels(self._h, b, n), self.nx == 17)

    def plan_kernels(self, B: int, iterate: bool = False, want_traj: bool = True) -> dict:
        """{phase: rocprof kernel name} a solve of B instances launches on this handle's config."""
        return _lib.plan_kernels(self._c, self.max_batch, B, iterate, want_traj)

    def _dev(self, t, shape_tail, name, batch=None, allow_broadcast=False):
        """Coerce to a contiguous device tensor of the handle dtype; return (tensor, stride)."""
        torch = _torch()
        if isinstance(t, np.ndarray) and not t.flags.writeable:
            t = t.copy()   # torch.as_tensor warns on read-only arrays
        t = torch.as_tensor(t, dtype=self.dtype, device=self._tdev)
        if t.dim() == len(shape_tail):
            t = t.unsqueeze(0)
        if tuple(t.shape[1:]) != tuple(shape_tail):
            raise ValueError(f'{name}: expected shape [B, {", ".join(map(str, shape_tail))}], '
                             f'got {tuple(t.shape)}')
        t = t.contiguous()
        n = math.prod(shape_tail)
        if batch is not None and t.shape[0] != batch:
            if allow_broadcast and t.shape[0] == 1:
                return t, 0
            raise ValueError(f'{name}: batch {t.shape[0]} != {batch}')
        return t, n

    def _stream(self):
        return ctypes.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    def _outputs(self, B, want_traj):
        torch = _torch()
        dev = self._tdev
        N = self.cfg.N
        self._u0 = torch.empty((B, self.nu), dtype=self.dtype, device=dev)
        self._status = torch.empty((B,), dtype=torch.int32, device=dev)
        if want_traj:
            self._X = torch.empty((B, N + 1, self.nx), dtype=self.dtype, device=dev)
            self._U = torch.empty((B, N, self.nu), dtype=self.dtype, device=dev)
        else:
            self._X = self._U = None

    @staticmethod
    def _ptr(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)

    # ------------------------------------------------------------------ API
    def solve(self, x0, x_ref, u_ref, wind=None, want_traj: bool = True, out=None):
        """One SQP_RTI step per instance, linearised at the RK4 rollout of u_ref from x0.

        x0 [B,12]; x_ref [B|1,N+1,12]; u_ref [B|1,N,4]; wind [B|1,3] (optional).
        Returns the first-step controls u0* [B,4] (device tensor, async).
        """
        N = self.cfg.N
        x0, _ = self._dev(x0, (self.nx,), 'x0')
        B = x0.shape[0]
        if B > self.max_batch:
            raise ValueError(f'batch {B} > max_batch {self.max_batch}')
        xr, xr_sb = self._dev(x_ref, (N + 1, self.nx), 'x_ref', B, allow_broadcast=True)
        ur, ur_sb = self._dev(u_ref, (N, self.nu), 'u_ref', B, allow_broadcast=True)
        wd, wd_sb = (None, 0) if wind is None else self._dev(wind, (3,), 'wind', B, allow_broadcast=True)
        if out is None:
            self._outputs(B, want_traj)
        else:
            self._u0, self._X, self._U, self._status = out
        self._keep = (x0, xr, ur, wd)
        _lib.check(self.lib.mpcb_solve(
            self._h, B, self._ptr(x0), self.nx, self._ptr(xr), xr_sb, self._ptr(ur), ur_sb,
            self._ptr(wd), wd_sb, self._ptr(self._u0), self._ptr(self._X), self._ptr(self._U),
            self._ptr(self._status), self._stream()))
        return self._u0

    def solve_iterate(self, x0, xbar, ubar, x_ref, u_ref, wind=None, out=None):
        """acados SQP_RTI step from the persistent iterate (xbar [B,N+1,12], ubar [B,N,4])."""
        N = self.cfg.N
        x0, _ = self._dev(x0, (self.nx,), 'x0')
        B = x0.shape[0]
        xb, _ = self._dev(xbar, (N + 1, self.nx), 'xbar', B)
        ub, _ = self._dev(ubar, (N, self.nu), 'ubar', B)
        xr, xr_sb = self._dev(x_ref, (N + 1, self.nx), 'x_ref', B, allow_broadcast=True)
        ur, ur_sb = self._dev(u_ref, (N, self.nu), 'u_ref', B, allow_broadcast=True)
        wd, wd_sb = (None, 0) if wind is None else self._dev(wind, (3,), 'wind', B, allow_broadcast=True)
        if out is None:
            self._outputs(B, True)
        else:
            self._u0, self._X, self._U, self._status = out
        self._keep = (x0, xb, ub, xr, ur, wd)
        _lib.check(self.lib.mpcb_solve_iterate(
            self._h, B, self._ptr(x0), self.nx, self._ptr(xb), self._ptr(ub), self._ptr(xr), xr_sb,
            self._ptr(ur), ur_sb, self._ptr(wd), wd_sb, self._ptr(self._u0), self._ptr(self._X),
            self._ptr(self._U), self._ptr(self._status), self._stream()))
        return self._u0

    def set_params(self, p):
        """Parameters of the full 17/6 model (acados ``set(k, 'p', p)``,
        simulation_blaster.py:65-69): column-major J_angles 3x2, J_euler 3x3, J_p 3x3, T_blast.

        Shapes: [25] or [B|1, 25] (every stage alike), or [B|1, N|N+1, 25] stage by stage (the
        terminal stage N has no dynamics; its row is ignored).  ``None`` restores the defaults
        (zeros, T_blast = ``config.t_blast`` / ``set_t_blast``)."""
        if self.nx != 17:
            raise ValueError('set_params is for the 17/6 model; the 12/4 slice takes set_t_blast')
        if p is None:
            self._params = None
            _lib.check(self.lib.mpcb_set_params(self._h, 0, ctypes.c_void_p(0), 0, 0))
            return
        torch = _torch()
        N = self.cfg.N
        if isinstance(p, np.ndarray) and not p.flags.writeable:
            p = p.copy()   # torch.as_tensor warns on read-only arrays
        t = torch.as_tensor(p, dtype=self.dtype, device=self._tdev)
        if t.dim() == 1:
            t = t.reshape(1, 1, -1)
        elif t.dim() == 2:
            t = t.unsqueeze(1)
        if t.dim() != 3 or t.shape[-1] != 25 or t.shape[1] not in (1, N, N + 1):
            raise ValueError(f'p: expected [25], [B|1, 25] or [B|1, N|N+1, 25], got {tuple(p.shape)}')
        # acados ``set`` copies: a private device copy, so later writes to the caller's tensor
        # do not reach the solver (the library reads the pointer at every solve, mpcb.h)
        t = t.contiguous().clone()
        self._params = t   # the library keeps the device pointer: hold the tensor
        rows, stages = t.shape[0], t.shape[1]
        sb = 0 if rows == 1 else stages * 25
        kb = 0 if stages == 1 else 25
        _lib.check(self.lib.mpcb_set_params(self._h, rows, self._ptr(t), sb, kb))

    def set_t_blast(self, t_blast: float):
        """Blaster thrust p[24] (blastermodel.py:210) as a scalar for every instance and stage:
        the 12/4 slice's body-z force; on the 17/6 model the default parameter vector's T_blast.
        Updates the handle in place (no re-creation)."""
        _lib.check(self.lib.mpcb_set_t_blast(self._h, float(t_blast)))
        self.cfg.t_blast = float(t_blast)

    def qp_stats(self, B=None):
        """Input-box work statistics of the last solve: int32 [B, 2] device tensor per instance
        (mpcb_qp_stats): 12/4 (forward passes, masked backward stages); 17/6 (interior-point
        iterations, polish passes)."""
        torch = _torch()
        B = self._u0.shape[0] if B is None else int(B)
        out = torch.empty((B, 2), dtype=torch.int32, device=self._tdev)
        _lib.check(self.lib.mpcb_qp_stats(self._h, B, self._ptr(out), self._stream()))
        return out

    def get_control(self):
        """First-step control u0* of the last solve, [B,4] device tensor."""
        if self._u0 is None:
            raise RuntimeError('solve() has not been called')
        return self._u0

    def get_state_trajectory(self):
        """Predicted state trajectory X = xbar + dx of the last solve, [B,N+1,12]."""
        if self._X is None:
            raise RuntimeError('no trajectory: call solve(..., want_traj=True)')
        return self._X

    def get_input_trajectory(self):
        if self._U is None:
            raise RuntimeError('no trajectory: call solve(..., want_traj=True)')
        return self._U

    def get_status(self):
        return self._status

    def linearize(self, xbar, ubar, wind=None):
        """A [B,N,12,12], B [B,N,12,4], Phi(xbar_k, ubar_k) [B,N,12] (debug / parity)."""
        torch = _torch()
        N = self.cfg.N
        xb, _ = self._dev(xbar, (N + 1, self.nx), 'xbar')
        B = xb.shape[0]
        ub, _ = self._dev(ubar, (N, self.nu), 'ubar', B)
        wd, wd_sb = (None, 0) if wind is None else self._dev(wind, (3,), 'wind', B, allow_broadcast=True)
        dev = self._tdev
        A = torch.empty((B, N, self.nx, self.nx), dtype=self.dtype, device=dev)
        Bm = torch.empty((B, N, self.nx, self.nu), dtype=self.dtype, device=dev)
        xn = torch.empty((B, N, self.nx), dtype=self.dtype, device=dev)
        _lib.check(self.lib.mpcb_linearize(self._h, B, self._ptr(xb), self._ptr(ub), self._ptr(wd),
                                           wd_sb, self._ptr(A), self._ptr(Bm), self._ptr(xn),
                                           self._stream()))
        self._keep = (xb, ub, wd)
        return A, Bm, xn

    def sim_step(self, x, u, T=None, wind=None):
        """Plant integrator: one RK4 step of length T (default dt) — AcadosSimSolver.solve()."""
        torch = _torch()
        xs, _ = self._dev(x, (self.nx,), 'x')
        B = xs.shape[0]
        us, _ = self._dev(u, (self.nu,), 'u', B)
        wd, wd_sb = (None, 0) if wind is None else self._dev(wind, (3,), 'wind', B, allow_broadcast=True)
        xo = torch.empty_like(xs)
        _lib.check(self.lib.mpcb_sim_step(self._h, B, self._ptr(xs), self._ptr(us), self._ptr(wd),
                                          wd_sb, float(self.cfg.dt if T is None else T),
                                          self._ptr(xo), self._stream()))
        self._keep = (xs, us, wd)
        return xo

    def gen_inputs(self, B, seed, id_offset=0, ref='hover', wind=False):
        """Synthetic inputs on device (SURVEY §8 d): x0 [B,12], x_ref, u_ref (broadcast for hover)."""
        torch = _torch()
        N = self.cfg.N
        dev = self._tdev
        x0 = torch.empty((B, self.nx), dtype=self.dtype, device=dev)
        if ref == 'sine':
            xr = torch.empty((B, N + 1, self.nx), dtype=self.dtype, device=dev)
            xr_sb, kind = (N + 1) * self.nx, 1
        else:
            xr = torch.empty((1, N + 1, self.nx), dtype=self.dtype, device=dev)
            xr_sb, kind = 0, 0
        ur = torch.empty((1, N, self.nu), dtype=self.dtype, device=dev)
        wd = torch.empty((B, 3), dtype=self.dtype, device=dev) if wind else None
        _lib.check(self.lib.mpcb_gen_inputs(self._h, B, int(seed), int(id_offset), kind,
                                            self._ptr(x0), self._ptr(xr), xr_sb, self._ptr(ur), 0,
                                            self._ptr(wd), self._stream()))
        return dict(x0=x0, xref=xr, uref=ur, wind=wd)

    def histogram(self, u0, lo=0.0, hi=65.0, nbins=64, counts=None):
        """Accumulate a per-motor histogram of u0 into int64 counts [4, nbins] (device)."""
        torch = _torch()
        u, _ = self._dev(u0, (self.nu,), 'u0')
        if counts is None:
            counts = torch.zeros((self.nu, nbins), dtype=torch.int64, device=self._tdev)
        _lib.check(self.lib.mpcb_histogram(self._h, u.shape[0], self._ptr(u), float(lo), float(hi),
                                           int(nbins), self._ptr(counts), self._stream()))
        return counts
