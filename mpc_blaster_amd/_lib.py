"""ctypes binding of libmpcblaster.so (the C ABI declared in include/mpcb.h).

The HIP library is the product: there is no CPU fallback.  If the shared object is missing
the import of any compute entry point raises, loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = 'libmpcblaster.so'
LIB_PATH = os.path.join(_HERE, LIB_NAME)

ABI_VERSION = 5
MPCB_F64, MPCB_F32 = 0, 1
MPCB_MAX_NX, MPCB_MAX_NU = 17, 6
STATUS_OK, STATUS_NAN, STATUS_MAXITER, STATUS_MINSTEP, STATUS_QP_FAIL = 0, 1, 2, 3, 4

EXPORTS = ('mpcb_create', 'mpcb_destroy', 'mpcb_last_error', 'mpcb_abi_version',
           'mpcb_workspace_bytes', 'mpcb_path', 'mpcb_solve', 'mpcb_solve_iterate', 'mpcb_linearize',
           'mpcb_sim_step', 'mpcb_gen_inputs', 'mpcb_histogram', 'mpcb_set_timing',
           'mpcb_last_timing', 'mpcb_set_params', 'mpcb_set_t_blast', 'mpcb_qp_stats', 'mpcb_poc_jacobians',
           'mpcb_quat_ops', 'mpcb_plan_kernels', 'mpcb_last_kernels')
# the timing / launch-log slots of the split path (mpcb_last_timing, mpcb_plan_kernels) and of the
# 17/6 model
PHASES_12 = ('nominal', 'riccati', 'forward', 'linearise')
PHASES_17 = ('nominal', 'riccati', 'linearise', '')


class MpcbConfig(ctypes.Structure):
    """Mirror of ``mpcb_config`` (include/mpcb.h)."""

    _fields_ = [
        ('nx', ctypes.c_int32), ('nu', ctypes.c_int32), ('N', ctypes.c_int32),
        ('dtype', ctypes.c_int32), ('box_u', ctypes.c_int32), ('max_as_iter', ctypes.c_int32),
        ('box_x', ctypes.c_int32), ('reserved', ctypes.c_int32),
        ('dt', ctypes.c_double), ('cost_scale', ctypes.c_double),
        ('mass', ctypes.c_double), ('lx', ctypes.c_double), ('ly', ctypes.c_double),
        ('c', ctypes.c_double), ('g', ctypes.c_double), ('t_blast', ctypes.c_double),
        ('J', ctypes.c_double * 9),
        ('Q', ctypes.c_double * (MPCB_MAX_NX * MPCB_MAX_NX)),
        ('R', ctypes.c_double * (MPCB_MAX_NU * MPCB_MAX_NU)),
        ('QN', ctypes.c_double * (MPCB_MAX_NX * MPCB_MAX_NX)),
        ('lbu', ctypes.c_double * MPCB_MAX_NU), ('ubu', ctypes.c_double * MPCB_MAX_NU),
        ('lbx', ctypes.c_double * MPCB_MAX_NX), ('ubx', ctypes.c_double * MPCB_MAX_NX),
    ]


_lib = None


class LibraryMissing(ImportError):
    pass


def load(path: str | None = None):
    """Load (once) and type the shared library; raises LibraryMissing if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get('MPCB_LIB') or LIB_PATH
    if not os.path.exists(p):
        raise LibraryMissing(
            f'{p} not found: build it with `python -c "import __graft_entry__ as g; g.build()"` '
            '(hipcc --offload-arch=gfx950).  There is no CPU fallback.')
    lib = ctypes.CDLL(p)
    vp, i64, i32, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
    u64 = ctypes.c_uint64
    lib.mpcb_create.argtypes = [ctypes.POINTER(MpcbConfig), i32, i64, ctypes.POINTER(vp)]
    lib.mpcb_destroy.argtypes = [vp]
    lib.mpcb_last_error.restype = ctypes.c_char_p
    lib.mpcb_last_error.argtypes = []
    lib.mpcb_abi_version.argtypes = []
    lib.mpcb_workspace_bytes.argtypes = [vp]
    lib.mpcb_workspace_bytes.restype = i64
    lib.mpcb_path.argtypes = [vp]
    lib.mpcb_solve.argtypes = [vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp]
    lib.mpcb_solve_iterate.argtypes = [vp, i64, vp, i64, vp, vp, vp, i64, vp, i64, vp, i64,
                                       vp, vp, vp, vp, vp]
    lib.mpcb_linearize.argtypes = [vp, i64, vp, vp, vp, i64, vp, vp, vp, vp]
    lib.mpcb_sim_step.argtypes = [vp, i64, vp, vp, vp, i64, dbl, vp, vp]
    lib.mpcb_gen_inputs.argtypes = [vp, i64, u64, u64, i32, vp, vp, i64, vp, i64, vp, vp]
    lib.mpcb_histogram.argtypes = [vp, i64, vp, dbl, dbl, i32, vp, vp]
    lib.mpcb_set_timing.argtypes = [vp, i32]
    lib.mpcb_last_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    lib.mpcb_set_params.argtypes = [vp, i64, vp, i64, i64]
    lib.mpcb_set_t_blast.argtypes = [vp, dbl]
    lib.mpcb_qp_stats.argtypes = [vp, i64, vp, vp]
    lib.mpcb_poc_jacobians.argtypes = [i64, vp, dbl, ctypes.POINTER(dbl), i32, dbl, vp, vp, vp, vp, vp,
                                       vp, vp]
    lib.mpcb_quat_ops.argtypes = [i64, vp, vp, vp, vp, vp, vp]
    lib.mpcb_plan_kernels.argtypes = [ctypes.POINTER(MpcbConfig), i64, i64, i32, i32, ctypes.c_char_p, i64]
    lib.mpcb_last_kernels.argtypes = [vp, ctypes.c_char_p, i64]
    for name in EXPORTS:
        if name not in ('mpcb_last_error', 'mpcb_workspace_bytes'):
            getattr(lib, name).restype = i32
    got = int(lib.mpcb_abi_version())
    if got != ABI_VERSION:
        # a stale library would read arguments of a changed signature as the wrong types
        # (mpcb_set_params gained two arguments in v4), so refuse it before any call
        raise LibraryMissing(f'{p} has C ABI version {got}, this binding expects {ABI_VERSION}: '
                             'rebuild it (__graft_entry__.build())')
    if path is None:
        _lib = lib
    return lib


class MpcbError(RuntimeError):
    pass


def kernel_names(fill, full: bool) -> dict:
    """{phase: rocprof kernel name} from mpcb_plan_kernels / mpcb_last_kernels (``fill(buf, len)``
    calls one of them), phases without a launch omitted."""
    buf = ctypes.create_string_buffer(4096)
    check(fill(buf, len(buf)))
    names = buf.value.decode().split('\n')
    keys = PHASES_17 if full else PHASES_12
    return {k: n for k, n in zip(keys, names) if k and n}


def plan_kernels(cfg: MpcbConfig, max_batch: int, B: int, iterate: bool = False, want_traj: bool = True) -> dict:
    """The kernels a handle of (cfg, max_batch) launches for a solve of B instances, without a
    device (include/mpcb.h mpcb_plan_kernels)."""
    lib = load()
    return kernel_names(lambda b, n: lib.mpcb_plan_kernels(ctypes.byref(cfg), int(max_batch), int(B),
                                                           1 if iterate else 0, 1 if want_traj else 0, b, n),
                        cfg.nx == 17)


def check(rc: int):
    if rc != 0:
        msg = load().mpcb_last_error()
        raise MpcbError(f'mpcb error {rc}: {msg.decode() if msg else ""}')
