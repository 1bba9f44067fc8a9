"""Drop-in surface for the reference's driver scripts.

``from mpc_blaster_amd.compat.blastermodel import blasterModel`` replaces
``from blastermodel import blasterModel`` (src/scripts/simulation_blaster.py:1): its
``generateController()`` returns ``(AcadosSimSolver, AcadosOcpSolver)``-compatible objects
backed by libmpcblaster, so the closed-loop script body runs unchanged.
"""
from .acados import AcadosOcpSolver, AcadosSimSolver  # noqa: F401
from .blastermodel import blasterModel  # noqa: F401
