"""CPU oracle for the batched BLASTER MPC hot path — TEST INFRASTRUCTURE ONLY.

This package is the parity checker, never the product. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``mpc_blaster_amd``) never imports, links or executes anything here.

What it restates (fp64 NumPy, vectorised over the batch):

* ``oracle.model``  – the BLASTER dynamics ``f_expl_expr`` of
  ``/root/reference/src/scripts/blastermodel.py:95-201`` (17-state/6-input) and its exact
  12-state/4-input rigid-body slice, plus the analytic Jacobians.
* ``oracle.rk4``    – acados ``sim_erk`` semantics (4 stages, 1 step, h = Tf/N; options at
  ``blastermodel.py:277`` / JSON ``acados_ocp_blasterModel.json`` ``sim_method_num_stages``,
  ``sim_method_num_steps``) with exact forward sensitivities of the discrete map.
* ``oracle.ocp``    – one Gauss-Newton SQP_RTI step of the LINEAR_LS OCP of
  ``blastermodel.py:226-287``: Riccati recursion for the LQ QP, and an exact primal-dual
  active-set loop (plus a dense primal active-set cross-check) for input boxes.
* ``oracle.philox`` / ``oracle.inputs`` – the counter-based synthetic input generator
  (Philox4x32-10) of SURVEY.md §8(d), bit-identical to the device generator.
* ``oracle/c``      – a plain-C restatement of the same RK4 + Riccati path used as the timed
  CPU baseline (``bench.py`` ``cpu_baseline``).

Parity pinning:

* Dynamics f and ∂f: PINNED — ``tests/golden/dynamics_*.npz`` were produced by running the
  reference's own ``blasterModel.generateModel()`` (``tools/gen_golden.py``).
* OCP definition (dims, W, W_e, bounds, time steps, parameter values): PINNED against
  ``acados_ocp_blasterModel.json`` (fixture ``tests/golden/ocp_json_pin.json``).
* RK4 sensitivities: pinned by central finite differences of the pinned f.
* QP / SQP_RTI arithmetic: acados + HPIPM are absent from the reference and the image —
  **parity unpinned** beyond the KKT conditions of the QP (unique minimiser of a strictly
  convex QP), which the tests check independently of the Riccati code.
"""
