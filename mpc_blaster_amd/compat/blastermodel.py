"""``blasterModel``-compatible constructor (src/scripts/blastermodel.py:14-292).

Same signature and call sequence as the reference:
``blasterModel(mass, J, l_x, l_y, N, Tf, c, Q, R, Q_t, blastThruster, statesBound,
controlBound)``, ``.generateModel()``, ``.generateController() -> (integrator, ocp_solver)``.
By default (``full_model=True``) it keeps the reference's 17/6 model, its weights, its input box
(controlBound: thrusts and swivel rates) and its state box (statesBound, stages 1..N-1,
blastermodel.py:268-270) unchanged — the device's 17/6 path, so swapping the import is all a
reference script needs; a statesBound with non-finite entries leaves the state box off.
``full_model=False`` selects the 12/4 rigid-body slice of the BASELINE configs: Q[:12,:12],
R[:4,:4], thrust bounds controlBound[:, :4].  The slice has no state box: a finite statesBound
there raises NotImplementedError at generateController (a silently unenforced constraint would
change the reference's OCP).
"""
from __future__ import annotations

import numpy as np

from ..config import NU, NU17, NX, NX17, MPCConfig
from .acados import AcadosOcpSolver, AcadosSimSolver

# acados parameter_values[24] of generateController (blastermodel.py:280-282; JSON :3423)
DEFAULT_T_BLAST = 2.2 * 9.81


class blasterModel:  # noqa: N801  (reference class name)
    def __init__(self, mass, J, l_x, l_y, N, Tf, c, Q, R, Q_t, blastThruster, statesBound,
                 controlBound, dtype: str = 'f64', batch: int = 1, device: int = 0,
                 full_model: bool = True):
        self._M = float(mass)
        self._J = np.asarray(J, dtype=np.float64)
        self._arm_length_x = float(l_x)
        self._arm_length_y = float(l_y)
        self._c = float(c)
        self._N = int(N)
        self._Tf = float(Tf)
        self._Q_weight = np.asarray(Q, dtype=np.float64)
        self._Q_weight_t = np.asarray(Q_t, dtype=np.float64)
        self._R_weight = np.asarray(R, dtype=np.float64)
        self._blastThruster = float(blastThruster)
        self._statesBound = np.asarray(statesBound, dtype=np.float64)
        self._controlBound = np.asarray(controlBound, dtype=np.float64)
        self._dtype, self._batch, self._device = dtype, int(batch), int(device)
        self._full = bool(full_model)
        self._cfg = None

    def _state_box(self):
        """statesBound as the 17/6 state box (needs the input box too, as the device does)."""
        sb = self._statesBound
        if sb.shape == (2, NX17) and np.isfinite(sb).all() and self._controlBound.size > 0:
            if self._dtype != 'f64':
                # one policy with the 12/4 slice: a silently unenforced constraint would change
                # the reference's OCP (blastermodel.py:268-270)
                raise NotImplementedError('statesBound (blastermodel.py:268-270): the state box needs '
                                 "dtype='f64' on the device; pass a non-finite statesBound to "
                                 'solve without it in fp32')
            return dict(lbx=sb[0].copy(), ubx=sb[1].copy())
        return {}

    def generateModel(self):
        """Builds the problem definition (the dynamics themselves live in the HIP kernels)."""
        cb = self._controlBound
        if self._full:
            # generateController's default parameter vector: zeros and T_blast = 2.2 * 9.81,
            # hard-coded whatever blastThruster is (blastermodel.py:280-282); the scripts then
            # set p stage by stage (simulation_blaster.py:65-69)
            self._cfg = MPCConfig(
                N=self._N, dt=self._Tf / self._N, dtype=self._dtype, mass=self._M, J=self._J,
                lx=self._arm_length_x, ly=self._arm_length_y, c=self._c,
                Q=self._Q_weight[:NX17, :NX17], R=self._R_weight[:NU17, :NU17],
                QN=self._Q_weight_t[:NX17, :NX17], t_blast=DEFAULT_T_BLAST,
                nx=NX17, nu=NU17,
                lbu=cb[0][:NU17] if cb.size else None, ubu=cb[1][:NU17] if cb.size else None,
                **self._state_box())
            return 0
        self._cfg = MPCConfig(
            N=self._N, dt=self._Tf / self._N, dtype=self._dtype, mass=self._M, J=self._J,
            lx=self._arm_length_x, ly=self._arm_length_y, c=self._c,
            Q=self._Q_weight[:NX, :NX], R=self._R_weight[:NU, :NU], QN=self._Q_weight_t[:NX, :NX],
            lbu=cb[0][:NU], ubu=cb[1][:NU],
            # the same default parameter vector (blastermodel.py:280-282): T_blast = 2.2 * 9.81
            # until set(k, 'p', p) changes it (a quad without the blaster sets p[24] = 0)
            t_blast=DEFAULT_T_BLAST)
        return 0

    def generateController(self):
        if self._cfg is None:
            self.generateModel()
        if not self._full and self._statesBound.size and np.isfinite(self._statesBound).any():
            raise NotImplementedError(
                'statesBound (blastermodel.py:268-270) on the 12/4 slice: the slice has no state box; '
                'use full_model=True (the default: the reference 17/6 OCP with its state box) or pass '
                'a non-finite statesBound')
        ocp = AcadosOcpSolver(self._cfg, batch=self._batch, device=self._device,
                              json_file='acados_ocp_blasterModel.json')
        sim = AcadosSimSolver(MPCConfig(**{**self._cfg.__dict__}), batch=self._batch,
                              device=self._device)
        return sim, ocp
