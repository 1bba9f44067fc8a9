/*
 * mpcb.h — C ABI of libmpcblaster.so, the MI355X-native batched MPC hot path.
 *
 * Drop-in boundary for the per-control-step solve of sml93/mpc_blaster.  The reference crosses
 * this boundary once per control step at ``ocp_solver.solve()``
 * (src/scripts/simulation_blaster.py:80, mavros_blaster_sim.py:85), i.e. acados'
 * AcadosOcpSolver over its ctypes-loaded generated library; the plant step is
 * ``integrator.solve()`` (simulation_blaster.py:94-104, AcadosSimSolver).  Each entry point
 * below names the reference interface it replaces.
 *
 * Conventions
 *  - Plain C: pointers + sizes, no C++ or torch types.  Every call returns 0 or a negative
 *    MPCB_E_* code; ``mpcb_last_error()`` gives a thread-local message.
 *  - Array arguments are DEVICE pointers (HBM, caller-owned, e.g. torch ROCm tensors) of the
 *    handle's dtype (double when cfg.dtype == MPCB_F64, float when MPCB_F32).  Per-instance
 *    strides are in ELEMENTS; a stride of 0 broadcasts one array to the whole batch.
 *  - Calls are asynchronous on ``hip_stream`` (NULL = default stream).  The Python facade
 *    synchronises to keep acados' synchronous semantics.
 *  - A handle is bound to one device, owns its workspace, and is not re-entrant.
 *  - Per-instance ``status`` (acados codes: 0 success, 1 NaN detected, 2 max iterations,
 *    3 MINSTEP, 4 QP failure) is separate from the call-level return code.
 *  - Arrays handed to a setter (mpcb_set_params) are read by later solves, not copied: the
 *    caller keeps them alive and unchanged until the next set call (the Python facade passes a
 *    private copy, so it keeps acados' copy semantics of ``set``).
 */
#ifndef MPCB_H
#define MPCB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCB_ABI_VERSION 5

enum { MPCB_F64 = 0, MPCB_F32 = 1 };
enum { MPCB_MODE_ROLLOUT = 0, MPCB_MODE_ITERATE = 1 };
enum {
  MPCB_OK = 0,
  MPCB_E_INVALID = -1,   /* bad argument / shape */
  MPCB_E_HIP = -2,       /* HIP runtime error */
  MPCB_E_NOMEM = -3,     /* workspace allocation failed */
  MPCB_E_UNSUPPORTED = -4
};
/* per-instance solver status, acados' codes (ACADOS_SUCCESS, _NAN_DETECTED, _MAXITER, _MINSTEP,
 * _QP_FAILURE).  MINSTEP: the fp64 17/6 interior point stopped at its conditioning limit (a
 * breakdown or collapsed step once mu <= 1e-5 on a feasible iterate) and no active-set polish
 * certified the point: the outputs are that reduced-accuracy iterate.  With the state box the
 * polish runs first (MINSTEP = it did not certify); the input box alone (Mehrotra) has no polish,
 * so every such stop there reports MINSTEP (oracle: ocp._ipm_box_mehrotra, the same rule). */
enum { MPCB_STATUS_OK = 0, MPCB_STATUS_NAN = 1, MPCB_STATUS_MAXITER = 2, MPCB_STATUS_MINSTEP = 3,
       MPCB_STATUS_QP_FAIL = 4 };

#define MPCB_MAX_NX 17
#define MPCB_MAX_NU 6

/*
 * Problem definition: replaces the ``blasterModel(mass, J, l_x, l_y, N, Tf, c, Q, R, Q_t,
 * blastThruster, statesBound, controlBound)`` constructor + ``generateController()``
 * (src/scripts/blastermodel.py:16, :214-292) that build the acados OCP.
 * Matrices are row-major, leading dimension nx (Q, QN) or nu (R).
 */
typedef struct mpcb_config {
  int32_t nx;            /* 12 (rigid-body slice, the BASELINE configs) or 17 (full model) */
  int32_t nu;            /* 4 or 6 */
  int32_t N;             /* horizon (ocp.dims.N, blastermodel.py:226) */
  int32_t dtype;         /* MPCB_F64 | MPCB_F32 */
  int32_t box_u;         /* 1: lbu <= u <= ubu on stages 0..N-1 (idxbu, blastermodel.py:261) */
  int32_t max_as_iter;   /* box_u iteration cap.  17/6: interior-point iterations.  12/4: active-set
                            passes, at most 48 (AS_IPM_AFTER); an instance not converged by then is
                            solved by the interior point (<= 100 iterations, mpcb_asipm.h) */
  int32_t box_x;         /* 17/6 only, needs box_u: lbx <= x_k <= ubx on stages 1..N-1 (idxbx,
                            blastermodel.py:268-270 statesBound; JSON constraints.lbx/ubx) */
  int32_t reserved;
  double dt;             /* Tf / N (solver_options.tf, blastermodel.py:287) */
  double cost_scale;     /* stage-cost scaling; acados uses time_steps[k] = dt */
  double mass, lx, ly, c, g, t_blast;   /* 17/6: t_blast is the default parameter p[24] */
  double J[9];           /* inertia (row-major 3x3) */
  double Q[MPCB_MAX_NX * MPCB_MAX_NX];   /* stage state weight  (W[:nx,:nx]) */
  double R[MPCB_MAX_NU * MPCB_MAX_NU];   /* stage input weight  (W[nx:,nx:]) */
  double QN[MPCB_MAX_NX * MPCB_MAX_NX];  /* terminal weight (W_e = Q_t) */
  double lbu[MPCB_MAX_NU], ubu[MPCB_MAX_NU];
  double lbx[MPCB_MAX_NX], ubx[MPCB_MAX_NX];   /* state box (box_x) */
} mpcb_config;

typedef struct mpcb_handle mpcb_handle;

/* Library / device lifetime.  Replaces AcadosOcpSolver(ocp, json_file) construction
 * (blastermodel.py:289): validates the config, uploads weights, sizes the workspace. */
int mpcb_create(const mpcb_config* cfg, int device, int64_t max_batch, mpcb_handle** out);
int mpcb_destroy(mpcb_handle* h);
const char* mpcb_last_error(void);
int mpcb_abi_version(void);
/* Workspace bytes owned by the handle (informational). */
int64_t mpcb_workspace_bytes(const mpcb_handle* h);
/* Kernel path chosen at creation: 1 = split nominal / Riccati / forward kernels (unconstrained),
 * 0 = single-kernel solver (input boxes; small batches when MPCB_SPLIT_MIN_BATCH asks for it). */
int mpcb_path(const mpcb_handle* h);
/* Optional device timing of later solves: HIP events recorded on the launch stream around each
 * kernel phase.  ``mpcb_last_timing`` waits for the last timed solve and writes the device
 * milliseconds of its phases: ms[0] nominal rollout, ms[1] Riccati (the dominant kernel; the
 * single launch on the fused / box paths), ms[2] forward pass; on the 17/6 model ms[0] nominal17,
 * ms[1] riccati17 (Riccati + forward, the interior point with boxes), ms[2] lin17ws (the
 * stage-parallel linearisation).  Summed over chunks (up to 64).
 * No reference counterpart (acados' ``get_stats('time_tot')`` is host wall time). */
int mpcb_set_timing(mpcb_handle* h, int enable);
int mpcb_last_timing(mpcb_handle* h, float ms[3]);
/* Kernels of a solve, one line per timing phase (the slots of mpcb_last_timing: nominal, Riccati,
 * forward pass / 17/6 linearisation; a fourth line for the small-chunk path's linearisation),
 * as rocprofv3 names the dispatches ("mpcb::riccati_kernel_f32<false, false, false>"), an empty
 * line for a phase without a launch; NUL-terminated in buf[len].
 * mpcb_plan_kernels: what mpcb_solve (mode MPCB_MODE_ROLLOUT, want_traj: X and U requested) or
 * mpcb_solve_iterate (MPCB_MODE_ITERATE) of B instances would launch on a handle created with
 * (cfg, max_batch) -- the same selection code, run without a device (no HIP call).
 * mpcb_last_kernels: what the handle's last solve launched.
 * No reference counterpart (profiling aid: ties a roofline to the rocprof dispatch it cites). */
int mpcb_plan_kernels(const mpcb_config* cfg, int64_t max_batch, int64_t B, int mode, int want_traj,
                      char* buf, int64_t len);
int mpcb_last_kernels(const mpcb_handle* h, char* buf, int64_t len);

/*
 * One SQP_RTI step for B independent instances, linearised at the RK4 rollout of u_ref from
 * x0 (north_star surface ``solve(x0, x_ref, u_ref)``).  Replaces, per instance, the call
 * sequence ocp_solver.set(0,'lbx'/'ubx',x0) / cost_set(k,'yref',...) / solve() /
 * get(0,'u') / get(k,'x') (simulation_blaster.py:60-89).
 *   x0    [B, nx]            stride x0_sb
 *   xref  [B|1, N+1, nx]     stride xref_sb (0 = broadcast)
 *   uref  [B|1, N, nu]       stride uref_sb
 *   wind  [B|1, 3] or NULL   world-frame disturbance force (build extension, c5)
 *   u0    [B, nu]            first-step control u0* (required)
 *   X     [B, N+1, nx]|NULL  predicted state trajectory xbar + dx (linear prediction)
 *   U     [B, N, nu]|NULL    predicted controls (X and U 16-byte aligned)
 *   status[B] int32          per-instance status
 */
int mpcb_solve(mpcb_handle* h, int64_t B,
               const void* x0, int64_t x0_sb,
               const void* xref, int64_t xref_sb,
               const void* uref, int64_t uref_sb,
               const void* wind, int64_t wind_sb,
               void* u0, void* X, void* U, int32_t* status, void* hip_stream);

/*
 * acados SQP_RTI semantics: linearise at the persistent iterate (xbar [B,N+1,nx],
 * ubar [B,N,nu]) with gaps, x0 enforced through dx_0 = x0 - xbar_0; outputs the full-step
 * iterate X = xbar + dx, U = ubar + du (X/U may alias xbar/ubar).  This is what one
 * ``ocp_solver.solve()`` does on the persistent solver object (simulation_blaster.py:80).
 */
int mpcb_solve_iterate(mpcb_handle* h, int64_t B,
                       const void* x0, int64_t x0_sb,
                       const void* xbar, const void* ubar,
                       const void* xref, int64_t xref_sb,
                       const void* uref, int64_t uref_sb,
                       const void* wind, int64_t wind_sb,
                       void* u0, void* X, void* U, int32_t* status, void* hip_stream);

/*
 * Linearisation only (debug / parity): RK4 + exact forward sensitivities of every shooting
 * interval.  A [B,N,nx,nx], Bm [B,N,nx,nu], xnext [B,N,nx] = Phi(xbar_k, ubar_k).
 * Replaces acados sim_erk with sens_forward (what SQP_RTI evaluates inside solve()).
 */
int mpcb_linearize(mpcb_handle* h, int64_t B, const void* xbar, const void* ubar,
                   const void* wind, int64_t wind_sb,
                   void* A, void* Bm, void* xnext, void* hip_stream);

/*
 * Plant integrator: x_out[b] = Phi(x[b], u[b]) with step T (one RK4 step).  Replaces
 * AcadosSimSolver set('x')/set('u')/solve()/get('x') (simulation_blaster.py:94-104).
 */
int mpcb_sim_step(mpcb_handle* h, int64_t B, const void* x, const void* u, const void* wind,
                  int64_t wind_sb, double T, void* x_out, void* hip_stream);

/*
 * Synthetic inputs (SURVEY §8 d): Philox4x32-10 keyed by (seed, id_offset + i).
 *   ref_kind 0 = hover reference, 1 = per-instance sinusoid (c3);  wind may be NULL.
 * Writes x0 [B,nx], xref [B,N+1,nx] (or [1,...] if ref_kind==0 and xref_sb==0), uref likewise.
 */
int mpcb_gen_inputs(mpcb_handle* h, int64_t B, uint64_t seed, uint64_t id_offset, int ref_kind,
                    void* x0, void* xref, int64_t xref_sb, void* uref, int64_t uref_sb,
                    void* wind, void* hip_stream);

/*
 * Model parameters of the full 17/6 model (nx == 17): acados ``ocp_solver.set(k, 'p', p)``,
 * stage by stage (simulation_blaster.py:65-69; the vector layout of blastermodel.py:203-210:
 * column-major vec of J_angles 3x2, J_euler 3x3, J_p 3x3, then T_blast).
 *   params     DEVICE array; the 25-vector of instance b at stage k starts at
 *              params[b * params_sb + k * params_kb] (elements).  params_sb == 0: one row for
 *              every instance; params_kb == 0: the same vector on every stage 0..N-1 (the
 *              terminal stage has no dynamics).  mpcb_sim_step reads stage 0.
 *   count      instance rows the array holds: a later solve / linearize / sim_step of B > count
 *              instances fails with MPCB_E_INVALID unless params_sb == 0.
 * The caller keeps the array alive for those later calls.  NULL restores the defaults (zeros,
 * T_blast = mpcb_set_t_blast / cfg.t_blast, acados ``parameter_values``, blastermodel.py:280-282).
 * MPCB_E_UNSUPPORTED on a 12/4 handle (its only parameter is T_blast: mpcb_set_t_blast).
 */
int mpcb_set_params(mpcb_handle* h, int64_t count, const void* params, int64_t params_sb,
                    int64_t params_kb);

/*
 * T_blast, the blaster thrust p[24] (blastermodel.py:210), as a host scalar.  12/4 model: the
 * body-z force of the rigid-body slice for every instance and stage of later calls (replaces
 * ``set(k, 'p', p)`` with the Jacobian blocks zero; no re-creation of the handle).  17/6 model:
 * the default parameter vector's p[24] (used while no device parameters are set).  Waits for the
 * device (a configuration call, not a per-step one).
 */
int mpcb_set_t_blast(mpcb_handle* h, double t_blast);

/*
 * Point-of-contact Jacobians of the blaster stream for B vehicle poses (fp64, runs on the
 * current device / ``hip_stream``, no handle).  Replaces Jacobian_POC_Solver.solveJacobians
 * (src/scripts/Jacobian_POC_Solver.py:222-296, htm.py:7-36): stream ODE p' = v,
 * v' = -Mc v + g by RK4 with 10 steps, Newton ground-hit time (dT 1e-5, from 0.1, |z| <= 1e-3),
 * forward differences with eps 1e-6.
 *   pose   [B, 8]  phi, theta, psi, alpha1, alpha2, x, y, z (device)
 *   Mc     host double[9], the stream drag matrix (row-major; scalar M_c -> M_c I)
 *   poc [B,3], J_eul [B,3,3], J_mot [B,3,2], J_pos [B,3,3]; p25 [B,25] or NULL: the model
 *   parameter vector of blastermodel.py:203-210 (vec J_mot | vec J_eul | vec J_pos | t_blast)
 *   status [B]: 0, or MPCB_STATUS_MAXITER if a root solve hit max_iter
 */
int mpcb_poc_jacobians(int64_t B, const double* pose, double stream_velocity, const double* Mc,
                       int max_iter, double t_blast, double* poc, double* J_eul, double* J_mot,
                       double* J_pos, double* p25, int32_t* status, void* hip_stream);

/*
 * Work statistics of the last solve on an input-box handle.  12/4 (the active-set QP, c4): per
 * instance ``out[2b]`` = forward passes until its active set was the KKT point (including the
 * first, after the unconstrained Riccati pass) and ``out[2b+1]`` = backward stages its masked
 * Riccati passes recomputed (restarts skip the stages above the highest changed one); an instance
 * the active set handed to the interior point (mpcb_config.max_as_iter) adds its iterations to
 * ``out[2b]`` and N per iteration to ``out[2b+1]``.  17/6 (the
 * interior point): ``out[2b]`` = interior-point iterations (Newton directions computed),
 * ``out[2b+1]`` = polish passes (fp64 state box).  ``out`` is a DEVICE int32 array [B, 2], B <= that
 * solve's batch.  Reference counterpart: HPIPM's ``get_stats('qp_iter')``.  MPCB_E_UNSUPPORTED on
 * handles without an input box.
 */
int mpcb_qp_stats(mpcb_handle* h, int64_t B, int32_t* out, void* hip_stream);

/*
 * Quaternion helpers of utils/MathUtils.py (q = [w, x, y, z], MathUtils.py:9) for B pairs, fp64,
 * device arrays: prod[b] = q1[b] (x) q2[b] (quatMultiplication, :5-23), inv[b] = conj(q1[b])
 * (unitQuatInversion, :25-39), rot[b] = R(q1[b]) row-major 3x3 (quat2Rot, :41-54).  Any output
 * may be NULL; q2 may be NULL when prod is.  The reference evaluates them on CasADi SX and never
 * on the MPC path (imported at blastermodel.py:4).
 */
int mpcb_quat_ops(int64_t B, const double* q1, const double* q2, double* prod, double* inv,
                  double* rot, void* hip_stream);

/* Histogram of u0 per input channel over [lo, hi) into counts[nu][nbins] (int64, accumulated). */
int mpcb_histogram(mpcb_handle* h, int64_t B, const void* u0, double lo, double hi, int nbins,
                   int64_t* counts, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* MPCB_H */
