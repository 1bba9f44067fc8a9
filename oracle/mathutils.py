"""Quaternion helpers of ``utils/MathUtils.py``, restated for NumPy arrays —
ORACLE, test infrastructure only (the product runs them on the device: mpc_blaster_amd.mathutils).

The reference defines them on CasADi SX and never calls them on the MPC path (imported at
``blastermodel.py:4``, unused).  Convention: q = [w, x, y, z] (``MathUtils.py:9``).
"""
from __future__ import annotations

import numpy as np


def quat_multiply(q1, q2):
    """Hamilton product (MathUtils.quatMultiplication, MathUtils.py:5-23)."""
    a = np.asarray(q1, dtype=np.float64)
    b = np.asarray(q2, dtype=np.float64)
    w1, x1, y1, z1 = (a[..., i] for i in range(4))
    w2, x2, y2, z2 = (b[..., i] for i in range(4))
    return np.stack([
        w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
    ], axis=-1)


def unit_quat_inverse(q):
    """Conjugate of a unit quaternion (MathUtils.unitQuatInversion, MathUtils.py:25-39)."""
    q = np.asarray(q, dtype=np.float64)
    return q * np.array([1.0, -1.0, -1.0, -1.0])


def quat_to_rot(q):
    """Rotation matrix of a unit quaternion (MathUtils.quat2Rot, MathUtils.py:41-54)."""
    e = np.asarray(q, dtype=np.float64)
    e0, e1, e2, e3 = (e[..., i] for i in range(4))
    R = np.empty(e.shape[:-1] + (3, 3))
    R[..., 0, 0] = 2 * (e0 ** 2 + e1 ** 2) - 1
    R[..., 0, 1] = 2 * (e1 * e2 - e0 * e3)
    R[..., 0, 2] = 2 * (e1 * e3 + e0 * e2)
    R[..., 1, 0] = 2 * (e1 * e2 + e0 * e3)
    R[..., 1, 1] = 2 * (e0 ** 2 + e2 ** 2) - 1
    R[..., 1, 2] = 2 * (e2 * e3 - e0 * e1)
    R[..., 2, 0] = 2 * (e1 * e3 - e0 * e2)
    R[..., 2, 1] = 2 * (e2 * e3 + e0 * e1)
    R[..., 2, 2] = 2 * (e0 ** 2 + e3 ** 2) - 1
    return R
