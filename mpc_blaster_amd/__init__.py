"""mpc_blaster_amd — MI355X-native batched MPC for the BLASTER quadrotor (sml93/mpc_blaster).

The hot path (RK4 rollout + linearisation, Gauss-Newton SQP_RTI QP by Riccati, input-box
active set) runs in hand-written HIP kernels for gfx950 inside ``libmpcblaster.so``; this
package is the thin host side:

* ``BatchedMPC``  — north_star batch surface ``solve(x0, x_ref, u_ref)`` / ``get_control()``.
* ``compat``      — acados-subset facade (``AcadosOcpSolver`` / ``AcadosSimSolver``) and a
  ``blasterModel``-compatible constructor so reference driver loops run with an import swap.
* ``dist``        — one process per GPU, instance sharding, RCCL gather of u0* / histograms.
* ``load_acados_ocp_json`` — an acados OCP JSON (the reference's generated description) as an
  ``MPCConfig`` (12/4 slice or the full 17/6 model).
"""
from .acados_json import load_acados_ocp_json  # noqa: F401
from .config import MPCConfig, NX, NU, NX17, NU17  # noqa: F401
from ._lib import LibraryMissing, MpcbError, load as load_library  # noqa: F401


def __getattr__(name):
    if name == 'BatchedMPC':
        from .api import BatchedMPC
        return BatchedMPC
    raise AttributeError(name)
