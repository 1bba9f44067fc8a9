"""Capture-only stand-in for the acados_template classes the reference instantiates.

TEST TOOL ONLY (tools/gen_golden.py, build container).  Records the OCP the reference's
``blasterModel.generateController()`` builds (cost, constraints, solver options) so it can be
compared with ``acados_ocp_blasterModel.json``.  Solves nothing.
"""
CAPTURED = []


class _Bag:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class AcadosModel(_Bag):
    pass


class AcadosOcp:
    def __init__(self):
        self.model = None
        self.dims = _Bag()
        self.cost = _Bag()
        self.constraints = _Bag()
        self.solver_options = _Bag()
        self.parameter_values = None


class AcadosSim(AcadosOcp):
    pass


class AcadosOcpSolver:
    def __init__(self, ocp, json_file=None):
        self.ocp = ocp
        self.json_file = json_file
        CAPTURED.append(('ocp', ocp, json_file))


class AcadosSimSolver:
    def __init__(self, ocp, json_file=None):
        self.ocp = ocp
        CAPTURED.append(('sim', ocp, json_file))
