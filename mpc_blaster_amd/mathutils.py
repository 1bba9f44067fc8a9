"""Quaternion helpers of ``utils/MathUtils.py`` on the device.

``mpcb_quat_ops`` (include/mpcb.h) evaluates, for a batch of fp64 quaternions q = [w, x, y, z]
(``MathUtils.py:9``): the Hamilton product (``quatMultiplication``, :5-23), the unit-quaternion
inverse (``unitQuatInversion``, :25-39) and the rotation matrix (``quat2Rot``, :41-54).  The
reference builds them on CasADi SX and never calls them on the MPC path (imported at
``blastermodel.py:4``).  Inputs may be NumPy arrays or tensors, [4] or [..., 4]; results are
float64 tensors on the device.
"""
from __future__ import annotations

import ctypes

from . import _lib


def _quat(q, device):
    import torch
    t = torch.as_tensor(q, dtype=torch.float64, device=device)
    if t.shape[-1] != 4:
        raise ValueError(f'quaternions have 4 components, got shape {tuple(t.shape)}')
    return t.reshape(-1, 4).contiguous(), t.shape[:-1]


def _run(q1, q2=None, prod=False, inv=False, rot=False, device=None):
    import torch
    dev = torch.device('cuda', torch.cuda.current_device()) if device is None else torch.device(device)
    a, lead = _quat(q1, dev)
    b = None
    if q2 is not None:
        b, lead2 = _quat(q2, dev)
        if lead2 != lead:
            raise ValueError('q1 and q2 must have the same shape')
    B = a.shape[0]
    out_p = torch.empty((B, 4), dtype=torch.float64, device=dev) if prod else None
    out_i = torch.empty((B, 4), dtype=torch.float64, device=dev) if inv else None
    out_r = torch.empty((B, 3, 3), dtype=torch.float64, device=dev) if rot else None
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)  # noqa: E731
    lib = _lib.load()
    with torch.cuda.device(dev):
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(lib.mpcb_quat_ops(B, ptr(a), ptr(b), ptr(out_p), ptr(out_i), ptr(out_r), stream))
    return out_p, out_i, out_r, lead


def quat_multiply(q1, q2, device=None):
    """q1 (x) q2 (MathUtils.quatMultiplication)."""
    p, _, _, lead = _run(q1, q2, prod=True, device=device)
    return p.reshape(*lead, 4)


def unit_quat_inverse(q, device=None):
    """Conjugate of a unit quaternion (MathUtils.unitQuatInversion)."""
    _, i, _, lead = _run(q, inv=True, device=device)
    return i.reshape(*lead, 4)


def quat_to_rot(q, device=None):
    """3x3 rotation matrix of a unit quaternion (MathUtils.quat2Rot)."""
    _, _, r, lead = _run(q, rot=True, device=device)
    return r.reshape(*lead, 3, 3)
