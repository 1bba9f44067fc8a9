// mpcb_kernels.h — host-visible launch interface of the HIP kernels (internal to the library).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mpcb_model.h"

namespace mpcb {

constexpr int NX = 12;
constexpr int NU = 4;
constexpr int NZ = NX + NU;      // directions per instance = lanes per instance group
constexpr int GROUPS = 64 / NZ;  // instances per wavefront (4)
constexpr int NBOX_XTRA = 18;    // per-lane box-mode scratch values per stage (see solve kernel)

// Device-resident weights (row-major), uploaded once per handle.
template <class T>
struct Weights {
  T Q[NX * NX];
  T R[NU * NU];
  T QN[NX * NX];
  T lbu[NU], ubu[NU];
  // the 6 constant columns of [A|B] (position e_p, velocity e_v + hv e_p, hv = the RK4 tangent's
  // (h/6)*6) laid out like an ABT2 record -- entry i of slot s at i * 10 + s -- so a lane of a
  // constant direction reads its column with the variable lanes' strided loads (mpcb_as.hip)
  T ctab[NX * 10];
};

template <class T>
struct SolveArgs {
  int64_t B;
  int N;
  int mode;          // MPCB_MODE_ROLLOUT / MPCB_MODE_ITERATE
  int box;           // input boxes on
  int max_as_iter;
  int small;         // 1: small unconstrained chunk: parallel linearisation + cached-[A|B] passes
  int fwd16;         // 1: P2 exports [A|B]^T and the forward pass runs in the 16-lane layout
  int quad_p1;       // P1 variant: 2 = a 16-lane row per instance (f split over the lanes,
                     // mpcb_rollout.hip), 1 = a lane quad per instance (sin/cos split), 0 = a
                     // thread per instance
  T h;               // RK4 step
  T s;               // stage cost scaling
  Model<T> M;
  const Weights<T>* W;
  const T* x0; int64_t x0_sb;
  const T* xref; int64_t xref_sb;
  const T* uref; int64_t uref_sb;
  const T* wind; int64_t wind_sb;
  const T* xbar; const T* ubar;
  T* u0; T* X; T* U; int32_t* status;
  T* scratch;            // per-slot workspace
  int64_t slot_elems;    // elements per slot (one slot = one wavefront = GROUPS instances)
};

template <class T> hipError_t launch_solve(const SolveArgs<T>& a, int grid, hipStream_t st);

// Launch log of the solve paths (mpcb_plan_kernels / mpcb_last_kernels, include/mpcb.h): every
// solve-path launcher notes the kernel it launches in the slot of its timing phase
// (mpcb_last_timing: 0 nominal, 1 Riccati / the single launch, 2 forward pass or the 17/6
// stage-parallel linearisation; 3 the small-chunk path's linearisation).  In a dry run (the plan
// of a config, no device) the launchers note their kernels and make no HIP call, so the plan and
// the launches come from the same selection code.
constexpr int LOG_SLOTS = 4;
struct LaunchLog {
  const void* fn[LOG_SLOTS];
  bool dry;
};
LaunchLog& launch_log();   // thread-local (mpcb_capi.hip)
inline bool dry_run() { return launch_log().dry; }
#define MPCB_LAUNCH(PH, K, G, BLK, LDS, ST, ...)                                \
  do {                                                                          \
    ::mpcb::launch_log().fn[PH] = reinterpret_cast<const void*>(&K);            \
    if (!::mpcb::launch_log().dry) hipLaunchKernelGGL(K, G, BLK, LDS, ST, __VA_ARGS__); \
  } while (0)
enum { PH_NOMINAL = 0, PH_RICCATI = 1, PH_FORWARD = 2, PH_LIN17 = 2, PH_LIN = 3 };
// Static LDS of the fp64 Riccati body (riccati_body: GroupLds x 4, SW, Cst), the same in
// row_riccati_kernel and riccati_kernel_f64 (tools/kernel_meta.py: 24064 B); mpcb_create sizes
// the fused launch with it and launch_split checks it against the code object before the first
// fused launch (the solve fails loudly if it grew).
constexpr size_t RICCATI_F64_STATIC_LDS = 24064;

// Split (unconstrained) path: three launches per chunk of instances.
//   P1 nominal  (thread / instance): rollout or iterate, captures linearisation scalars
//   P2 riccati  (16 lanes / instance): tangent columns of [A|B] + Riccati, writes gains
//   P3 forward  (thread / instance): dx/du propagation (RK4 JVP), writes u0, X, U, status
// Chunk workspace layouts, structure-of-arrays blocked by instance quads (mpcb_split.hip soa();
// c = chunk-local instance, nb = chunk size rounded up to a multiple of 4):
//   XU [(N+1)][16][nb]  xbar_k | ubar_k
//   CC [N][80][nb]      4 RK stages x 20 linearisation scalars
//   GP [N][12][nb]      gap Phi(xbar_k, ubar_k) - xbar_{k+1}      (iterate mode only)
//   KR [N][52][nb]      K_k (48, K[m][i] at row 4*i+m) | kff_k (4)
constexpr int XU_REC = 16, CCS_REC = 80, GP_REC = 12, KR_REC = 52;
// Exported linearisation (16-lane forward pass, active-set kernel).  Only the NVAR columns of
// [A|B] that depend on the linearisation point are stored: the attitude (3..5), body-rate
// (9..11) and input (12..15) directions.  The others are constant for this model -- f does not
// depend on p and v enters only p_dot -- so A e_p = e_p and A e_v = e_v + h e_p exactly.
// Element orders put the 16 lanes of an instance on CONSECUTIVE elements for every access:
//   AB  [A|B]_{i, var_col(t)} at i*NVAR + t (backward: lane j reads its column)
//   ABT [A|B]_{i, var_col(t)} at t*12 + i   (forward: state lane i reads row i)
//   GH  input row m of the stage Hessian, entry i (16 = h_u) at i*4 + m
//   PS  P_k column j entry i (12 = p_k[j]) at i*12 + j
constexpr int NVAR = 10;
__host__ __device__ constexpr int var_col(int t) { return t < 3 ? 3 + t : 6 + t; }
__host__ __device__ constexpr int var_index(int j) { return (j >= 3 && j < 6) ? j - 3 : (j >= 9 ? j - 6 : -1); }
constexpr int AB_REC = 12 * NVAR, GH_REC = 4 * 17, PS_REC = 12 * 13;
// Row-major exports (SplitArgs::rm = 1: the input-box kernel mpcb_as.hip and the 16-lane forward
// pass of small unconstrained chunks).  Per stage the 4 instances of a quad follow each other and
// each instance's record is contiguous, so a lane's row (or column) is a run of aligned vectors
// (mpcb_split.h rec2()); rows carry no padding beyond what the vector width needs:
//   AB2  [10][12]  column var_col(t) of [A|B], 12 entries       (backward: lane var_col(t))
//   ABT2 [12][10]  row i of [A|B] at the variable columns t < 10 (forward: state lane i; the
//                  iterate-mode gap comes from GP)
//   KR2  [4][14]   row m of K (12 entries), slot 12 = k_m
//   GH2  [4][20]   row m of the stage Hessian's input rows (16 entries), slot 16 = h_u[m]; written
//                  by the active-set kernel's masked backward, only where component m is fixed
//   PS2  [12][8]   P_k packed by symmetry: lane j keeps P[j][(j + d) % 12], d = 0..6, and p_k[j]
//                  in slot 7 (84 slots for its 78 distinct entries); written by P2's unconstrained
//                  pass and by every stage the active-set kernel recomputes (its restart points)
constexpr int ABT2_W = NVAR, KR2_W = 14, PS2_W = 8;
static_assert(sizeof(Weights<float>::ctab) == NX * ABT2_W * sizeof(float), "ctab is one ABT2 record");
// The active-set kernel's backward reads its [A|B] column out of the ABT2 rows (12 strided loads:
// the masked backward recomputes ~2/3 of the stage-instances once, the forward passes read the
// rows ~4 times), so P2 writes [A|B] once (round 3: a separate AB2 column export cost more).
constexpr int AB2_REC = 12 * NVAR, ABT2_REC = 12 * ABT2_W, KR2_REC = 4 * KR2_W, GH2_REC = 4 * 20,
              PS2_REC = 12 * PS2_W;

// the 12/4 input box: active-set passes before an unconverged instance goes to the interior-point
// fallback (oracle.ocp.AS_IPM_AFTER; mpcb_asipm.h)
constexpr int AS_IPM_AFTER = 48;
// ... or after the first pass when it violates more than 7/20 of the horizon's input components
// (oracle.ocp.AS_IPM_NV_NUM / _DEN)
constexpr int AS_IPM_NV_NUM = 7, AS_IPM_NV_DEN = 20;
// the fp32 input box's refinement list (SplitArgs::as_ref, mpcb_as.h as_ref_put): a header of
// AS_REF_HDR words, then AS_REF_W per listed instance
constexpr int AS_REF_HDR = 4, AS_REF_W = 24, AS_REF_KC = 20;   // (KC: the restart stage, -1 or N - 1)
// ... which also lists converged instances whose first-stage controls are all below this (N)
constexpr double AS_REF_U0 = 2.0;
// ... and converged instances that needed this many active-set passes or more
constexpr int AS_REF_PASSES = 10;
// ... and converged instances whose set fixes at least this fraction of the input components
constexpr int AS_REF_FIX_NUM = 3, AS_REF_FIX_DEN = 10;

template <class T>
struct SplitArgs {
  int64_t b0;        // first global instance of the chunk
  int64_t nb;        // instances in the chunk
  int N;
  int mode;
  T h, s;
  Model<T> M;
  const Weights<T>* W;
  const T* x0; int64_t x0_sb;
  const T* xref; int64_t xref_sb;
  const T* uref; int64_t uref_sb;
  const T* wind; int64_t wind_sb;
  const T* xbar; const T* ubar;
  T* u0; T* X; T* U; int32_t* status;
  T* XU; T* CC; T* GP; T* KR;
  T* AB; T* ABT; T* GH;   // box path: P2 exports the linearisation and the Hessian's input rows
  T* PS;             // box path: value-function snapshots for restarts
  int32_t* qp_stats; // box path (nullable): per global instance [forward passes, masked backward
                     // stages] until its active set converged
  int* as_queue;     // box path (nullable): the active-set kernel's work counter
  const int32_t* as_order;   // (MPCB_AS_ORDER_DBG builds, nullable) ticket -> chunk instance
  int* as_fb;        // box path (nullable): the interior-point fallback's list ([0] count, [2 + t]
                     // chunk instance), filled by the active-set kernel (mpcb_asipm.h)
  int* as_ref;       // fp32 box path (nullable): the refinement list (mpcb_as.h AS_REF_*), filled by
                     // the active-set kernel, walked by the refinement kernel
  int as_ref_cap;    // entries the refinement list holds
  int max_as_iter;
  int small;         // 1: small unconstrained chunk: parallel linearisation + cached-[A|B] passes
  int fwd16;         // 1: P2 exports [A|B]^T and the forward pass runs in the 16-lane layout
  int quad_p1;       // P1 variant: 2 = a 16-lane row per instance (f split over the lanes,
                     // mpcb_rollout.hip), 1 = a lane quad per instance (sin/cos split), 0 = a
                     // thread per instance
  int tin;           // 1: the row rollout integrated the tangents and exported [A|B] as the ABT2
                     // rows (mpcb_row.h TAN); P2 reads its columns from them (no CC record), in
                     // the same launch (row_riccati_kernel); 2: the same as two launches
                     // (MPCB_FUSE_P12=0)
  int fwd;           // 1: run P3 (trajectories or iterate mode); 0: P2 writes u0/status
  int rm;            // 1: P2 writes the row-major exports (ABT2, KR2, PS2 in a.ABT/a.KR/a.PS)
  int imajor;        // row-major exports instance-major (an instance's N records contiguous: the
                     // unconstrained fp64 forward, measured -2 % per c2 step) or stage-major (the box
                     // path: P2's scattered export stores measured 10 % slower instance-major at c4)
};
// ev (nullable): 4 events recorded on st before P1, after P1, after P2 and after P3.
template <class T> hipError_t launch_split(const SplitArgs<T>& a, hipStream_t st,
                                           hipEvent_t* ev = nullptr);
template <class T> hipError_t launch_as(const SplitArgs<T>& a, hipStream_t st);
template <class T> hipError_t launch_fwd_rm(const SplitArgs<T>& a, hipStream_t st);
template <class T> hipError_t launch_small(const SplitArgs<T>& a, hipStream_t st);
template <class T> hipError_t launch_nominal_row(const SplitArgs<T>& a, hipStream_t st);   // mpcb_rollout.hip
template <class T> int64_t split_elems_per_instance(int N, int iterate, int box = 0);  // per instance
template <class T> int64_t solve_slot_elems(int N, int box);

template <class T>
hipError_t launch_linearize(int64_t B, int N, T h, const Model<T>& M, const T* xbar,
                            const T* ubar, const T* wind, int64_t wind_sb, T* A, T* Bm,
                            T* xnext, hipStream_t st);
template <class T>
hipError_t launch_sim_step(int64_t B, T h, const Model<T>& M, const T* x, const T* u,
                           const T* wind, int64_t wind_sb, T* xo, hipStream_t st);
template <class T>
hipError_t launch_gen_inputs(int64_t B, int N, T dt, uint64_t seed, uint64_t id_offset,
                             int ref_kind, T* x0, T* xref, int64_t xref_sb, T* uref,
                             int64_t uref_sb, T* wind, hipStream_t st);
hipError_t launch_quat_ops(int64_t B, const double* q1, const double* q2, double* prod, double* inv,
                           double* rot, hipStream_t st);
template <class T>
hipError_t launch_histogram(int64_t B, int nu, const T* u0, double lo, double hi, int nbins,
                            unsigned long long* counts, hipStream_t st);

}  // namespace mpcb
