"""Batched point-of-contact Jacobians over ``mpcb_poc_jacobians``.

``JacobianPOCSolver`` keeps the reference class's call surface
(src/scripts/Jacobian_POC_Solver.py: ``Jacobian_POC_Solver(streamVelocity, M_c, Ts)``,
``initialise()``, ``solveJacobians(euler_angles, motor_angles, position)``,
``getJacobians() -> (J_mot, J_eul, J_pos)``, ``_POC``) for one pose, and ``solve_batch`` runs
B poses in one launch; ``params25`` gives the model parameter vectors that
``BatchedMPC.set_params`` takes (the J_angles / J_euler / J_p blocks of blastermodel.py:203-210).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def poc_jacobians(pose, stream_velocity, M_c=1.0, t_blast=2.2 * 9.81, max_iter=100, device=None):
    """pose [B, 8] (phi, theta, psi, alpha1, alpha2, x, y, z).  Returns a dict of device tensors:
    poc [B,3], J_eul [B,3,3], J_mot [B,3,2], J_pos [B,3,3], p25 [B,25], status [B]."""
    import torch
    lib = _lib.load()
    dev = f'cuda:{torch.cuda.current_device() if device is None else device}'
    pose = torch.as_tensor(pose, dtype=torch.float64, device=dev).reshape(-1, 8).contiguous()
    B = pose.shape[0]
    Mc = np.asarray(M_c, dtype=np.float64)
    Mc = (Mc * np.eye(3) if Mc.ndim == 0 else Mc.reshape(3, 3)).reshape(-1)
    out = dict(poc=torch.empty((B, 3), dtype=torch.float64, device=dev),
               J_eul=torch.empty((B, 3, 3), dtype=torch.float64, device=dev),
               J_mot=torch.empty((B, 3, 2), dtype=torch.float64, device=dev),
               J_pos=torch.empty((B, 3, 3), dtype=torch.float64, device=dev),
               p25=torch.empty((B, 25), dtype=torch.float64, device=dev),
               status=torch.empty((B,), dtype=torch.int32, device=dev))
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    rc = lib.mpcb_poc_jacobians(B, ptr(pose), float(stream_velocity), (ctypes.c_double * 9)(*Mc),
                                int(max_iter), float(t_blast), ptr(out['poc']), ptr(out['J_eul']),
                                ptr(out['J_mot']), ptr(out['J_pos']), ptr(out['p25']),
                                ptr(out['status']), stream)
    if rc != 0:
        raise _lib.MpcbError(f'mpcb_poc_jacobians failed ({rc})')
    return out


class JacobianPOCSolver:
    """Reference-compatible single-pose surface (Jacobian_POC_Solver.py:20-300)."""

    def __init__(self, streamVelocity, M_c, Ts):
        self._streamVelocity = float(streamVelocity)
        self._M_c = M_c
        self._Ts = float(Ts)
        self._POC = np.zeros(3)
        self._J_pos = np.zeros((3, 3))
        self._J_eul = np.zeros((3, 3))
        self._J_mot = np.zeros((3, 2))

    def initialise(self):
        # the reference builds its acados integrator and solves a warm-up pose (:55-59)
        self.solveJacobians([0, 0, 0], [0, 0], [0, 0, 4])

    def solveJacobians(self, euler_angles, motor_angles, position):
        pose = np.concatenate([np.asarray(euler_angles, dtype=np.float64).reshape(3),
                               np.asarray(motor_angles, dtype=np.float64).reshape(2),
                               np.asarray(position, dtype=np.float64).reshape(3)])[None]
        o = poc_jacobians(pose, self._streamVelocity, self._M_c)
        self._POC = o['poc'][0].cpu().numpy()
        self._J_eul = o['J_eul'][0].cpu().numpy()
        self._J_mot = o['J_mot'][0].cpu().numpy()
        self._J_pos = o['J_pos'][0].cpu().numpy()
        return int(o['status'][0].item())

    def getJacobians(self):
        return self._J_mot, self._J_eul, self._J_pos
