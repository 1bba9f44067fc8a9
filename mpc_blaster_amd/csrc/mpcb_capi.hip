// mpcb_capi.hip — extern "C" boundary of libmpcblaster.so (declared in include/mpcb.h).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <cxxabi.h>
#include <dlfcn.h>
#include <string>

#include "../../include/mpcb.h"
#include "mpcb_full.h"
#include "mpcb_kernels.h"

using namespace mpcb;

namespace {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) return fail(MPCB_E_HIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

bool inv3(const double* A, double* out) {
  const double d = A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
                   A[2] * (A[3] * A[7] - A[4] * A[6]);
  if (!(std::fabs(d) > 0)) return false;
  out[0] = (A[4] * A[8] - A[5] * A[7]) / d;
  out[1] = (A[2] * A[7] - A[1] * A[8]) / d;
  out[2] = (A[1] * A[5] - A[2] * A[4]) / d;
  out[3] = (A[5] * A[6] - A[3] * A[8]) / d;
  out[4] = (A[0] * A[8] - A[2] * A[6]) / d;
  out[5] = (A[2] * A[3] - A[0] * A[5]) / d;
  out[6] = (A[3] * A[7] - A[4] * A[6]) / d;
  out[7] = (A[1] * A[6] - A[0] * A[7]) / d;
  out[8] = (A[0] * A[4] - A[1] * A[3]) / d;
  return true;
}
}  // namespace

namespace mpcb {
LaunchLog& launch_log() {
  thread_local LaunchLog g{};
  return g;
}
}  // namespace mpcb

struct mpcb_handle {
  mpcb_config cfg;
  const int32_t* as_order_dbg = nullptr;   // (MPCB_AS_ORDER_DBG builds) the active-set kernel's order
  int device;
  int64_t max_batch;
  int grid;              // resident slots (one wavefront of GROUPS instances each)
  void* weights;         // Weights<T>
  void* scratch;          // split: chunk workspace; single-kernel solver: per-slot workspace
  int64_t slot_elems;
  int64_t scratch_bytes;
  int split;              // 1: three-kernel split path; 0: single-kernel solver (boxes)
  int small;              // split path, small unconstrained chunks: cached-[A|B] passes
  int fwd16;              // split path, small chunks: P2 exports [A|B]^T for a 16-lane forward
  int tin;                // split path: the row rollout exports [A|B] (SplitArgs::tin)
  int quad_p1;            // split path, small chunks: rollout with a lane quad per instance
  int64_t chunk;          // split path: instances per chunk
  int64_t chunk_elems;    // elements of the chunk workspace (XU | CC | GP | KR)
  Model<double> Md;
  Model<float> Mf;
  // optional per-phase device timing (mpcb_set_timing): 4 events per split chunk, or ev[0][0..1]
  // around the single launch of the single-kernel solver
  static constexpr int TCHUNKS = 64;
  int timing = 0;
  int timed_chunks = 0;   // chunks recorded by the last solve (0: nothing recorded)
  int timed_split = 0;
  hipEvent_t ev[TCHUNKS][4] = {};
  // full 17/6 model (cfg.nx == 17): per-instance parameters set by mpcb_set_params (nullable:
  // the defaults in the weights block), chunk of instances per launch
  int full = 0;
  const void* params = nullptr;
  int64_t params_sb = 0, params_kb = 0;
  int64_t params_count = 0;   // instance rows behind params (checked against B when params_sb != 0)
  int32_t* qp_stats = nullptr;   // 12/4 input box: per instance [forward passes, masked stages]
  int64_t qp_stats_rows = 0;     // instances of the last boxed solve
  void* u_scratch = nullptr;     // fp32 12/4 input box: U when the caller passes none (the
                                 // refinement kernel restarts from the active set's U, mpcb_as.h)
  const void* last_fn[LOG_SLOTS] = {};   // kernels the last solve launched (mpcb_last_kernels)
};

// A 17/6 call over B instances may only read parameter rows that exist (mpcb_set_params count).
static int check_params(const mpcb_handle* h, int64_t B) {
  if (h->full && h->params && h->params_sb != 0 && B > h->params_count) {
    g_err = "batch " + std::to_string(B) + " exceeds the " + std::to_string(h->params_count) +
            " parameter rows given to mpcb_set_params";
    return MPCB_E_INVALID;
  }
  return MPCB_OK;
}

extern "C" const char* mpcb_last_error(void) { return g_err.c_str(); }
extern "C" int mpcb_abi_version(void) { return MPCB_ABI_VERSION; }

extern "C" int64_t mpcb_workspace_bytes(const mpcb_handle* h) { return h ? h->scratch_bytes : 0; }
extern "C" int mpcb_path(const mpcb_handle* h) { return h ? h->split : -1; }

template <class T>
static void fill_weights(const mpcb_config& c, Weights<T>& w) {
  for (int i = 0; i < NX * NX; ++i) {
    w.Q[i] = (T)c.Q[i];
    w.QN[i] = (T)c.QN[i];
  }
  for (int i = 0; i < NU * NU; ++i) w.R[i] = (T)c.R[i];
  for (int i = 0; i < NU; ++i) {
    w.lbu[i] = (T)c.lbu[i];
    w.ubu[i] = (T)c.ubu[i];
  }
  // constant columns of [A|B] in the ABT2 record layout: slot s <-> direction d = 0,1,2,6,7,8
  const T hv = ((T)c.dt / T(6)) * T(6);
  for (int i = 0; i < NX * ABT2_W; ++i) w.ctab[i] = T(0);
  for (int sl = 0; sl < 6; ++sl) {
    const int d = sl < 3 ? sl : sl + 3;
    w.ctab[d * ABT2_W + sl] = T(1);
    if (d >= 6) w.ctab[(d - 6) * ABT2_W + sl] = hv;
  }
}

template <class T>
static void fill_weights17(const mpcb_config& c, Weights17<T>& w) {
  for (int i = 0; i < NX17 * NX17; ++i) {
    w.Q[i] = (T)c.Q[i];
    w.QN[i] = (T)c.QN[i];
  }
  for (int i = 0; i < NU17 * NU17; ++i) w.R[i] = (T)c.R[i];
  for (int i = 0; i < NU17; ++i) {
    w.lbu[i] = (T)c.lbu[i];
    w.ubu[i] = (T)c.ubu[i];
  }
  for (int i = 0; i < NX17; ++i) {
    w.lbx[i] = (T)c.lbx[i];
    w.ubx[i] = (T)c.ubx[i];
  }
  // acados parameter_values default: every Jacobian block 0, T_blast from the config
  for (int i = 0; i < NP17; ++i) w.p[i] = T(0);
  w.p[24] = (T)c.t_blast;
}

template <class T>
static void fill_model(const mpcb_config& c, const double* Jinv, Model<T>& M) {
  M.minv = (T)(1.0 / c.mass);
  M.g = (T)c.g;
  M.t_blast = (T)c.t_blast;
  M.lx = (T)c.lx;
  M.ly = (T)c.ly;
  M.c = (T)c.c;
  for (int i = 0; i < 9; ++i) {
    M.J[i] = (T)c.J[i];
    M.Jinv[i] = (T)Jinv[i];
  }
}

static int validate_config(const mpcb_config* cfg, int64_t max_batch, double Jinv[9]) {
  const bool full = cfg->nx == NX17 && cfg->nu == NU17;
  if (!(cfg->nx == NX && cfg->nu == NU) && !full)
    return fail(MPCB_E_UNSUPPORTED, "nx=%d nu=%d: implemented models are 12/4 (rigid-body slice) and 17/6 (full)",
                cfg->nx, cfg->nu);
  if (full && cfg->box_u)
    for (int m = 0; m < NU17; ++m)
      if (!(cfg->ubu[m] > cfg->lbu[m]))
        return fail(MPCB_E_INVALID, "17/6 input box needs lbu < ubu (component %d)", m);
  if (cfg->box_x && !(full && cfg->box_u))
    return fail(MPCB_E_UNSUPPORTED, "box_x is implemented for the 17/6 model together with box_u");
  // the state rows' barrier terms (lambda / s up to ~1e12 near the solution) exceed what fp32
  // Riccati factorisations survive: measured 2725 of 4096 random instances failing
  if (cfg->box_x && cfg->dtype != MPCB_F64)
    return fail(MPCB_E_UNSUPPORTED, "box_x needs dtype f64");
  if (cfg->box_x)
    for (int i = 0; i < NX17; ++i)
      if (!(cfg->ubx[i] > cfg->lbx[i]))
        return fail(MPCB_E_INVALID, "17/6 state box needs lbx < ubx (component %d)", i);
  if (cfg->N < 1 || cfg->N > 4096) return fail(MPCB_E_INVALID, "horizon N=%d out of range", cfg->N);
  if (!full && cfg->box_u && cfg->N > 64) return fail(MPCB_E_UNSUPPORTED, "box_u needs N <= 64 (N=%d)", cfg->N);
  if (cfg->dtype != MPCB_F64 && cfg->dtype != MPCB_F32)
    return fail(MPCB_E_INVALID, "dtype=%d", cfg->dtype);
  if (!(cfg->dt > 0) || !(cfg->mass > 0)) return fail(MPCB_E_INVALID, "dt and mass must be > 0");
  if (max_batch < 1) return fail(MPCB_E_INVALID, "max_batch=%lld", (long long)max_batch);
  if (cfg->box_u && cfg->max_as_iter < 1) return fail(MPCB_E_INVALID, "max_as_iter must be >= 1");
  if (!inv3(cfg->J, Jinv)) return fail(MPCB_E_INVALID, "inertia J is singular");
  return MPCB_OK;
}

// LDS of one workgroup at one wave per SIMD: 4 workgroups share a CU's 160 KiB
constexpr size_t LDS_PER_WAVE_SIMD = 160 * 1024 / 4;
// the dynamic LDS a workgroup may ask for without an attribute
constexpr size_t LDS_DYN_MAX = 64 * 1024;

// Kernel variants of a handle: a pure function of the config and max_batch (and MPCB_* switches
// that tests exercise), shared by mpcb_create and the device-free mpcb_plan_kernels.
static void select_path(mpcb_handle* h, const mpcb_config* cfg, int64_t max_batch, int cus) {
  const bool full = cfg->nx == NX17 && cfg->nu == NU17;
  h->cfg = *cfg;
  h->max_batch = max_batch;
  const bool f64 = cfg->dtype == MPCB_F64;
  // resident slots: one 64-thread workgroup per slot, a few per SIMD
  const int64_t waves_needed = (max_batch + GROUPS - 1) / GROUPS;
  int64_t grid = (int64_t)cus * 16;
  if (grid > waves_needed) grid = waves_needed;
  h->grid = (int)grid;
  const size_t esz = f64 ? sizeof(double) : sizeof(float);
  // Path: the split kernels win at every measured batch size (c2: 4096); the single-kernel
  // solver (mpcb_solve.hip) serves, on request, small unconstrained batches
  // (MPCB_SPLIT_MIN_BATCH above the batch) and the first input-box design (MPCB_BOX_IMPL=v1).
  if (full) {
    // one chunk of instances per launch triple; ~N*516 scalars of workspace each
    int64_t chunk = 8192;
    if (const char* e = getenv("MPCB_CHUNK")) chunk = atoll(e);
    if (chunk < 64) chunk = 64;
    if (chunk > max_batch) chunk = max_batch;
    h->full = 1;
    h->split = 1;
    h->chunk = chunk;
    // (+3 instances: a ragged last wavefront of the 16-lane kernel works in private padding slots)
    h->chunk_elems = full17_elems(cfg->N) * ((chunk + 3) / 4 * 4);
    h->scratch_bytes = h->chunk_elems * (int64_t)esz;
    return;
  }
  int64_t split_min = 1;
  if (const char* e = getenv("MPCB_SPLIT_MIN_BATCH")) split_min = atoll(e);
  h->split = (max_batch >= split_min) ? 1 : 0;
  if (const char* e = getenv("MPCB_BOX_IMPL"))   // "v1": the single-kernel active-set solver
    if (cfg->box_u && strcmp(e, "v1") == 0) h->split = 0;
  if (!h->split) {
    h->slot_elems = f64 ? solve_slot_elems<double>(cfg->N, cfg->box_u) : solve_slot_elems<float>(cfg->N, cfg->box_u);
    h->scratch_bytes = h->slot_elems * (int64_t)esz * grid;
    return;
  }
  // chunk of instances whose intermediates (~N*160 scalars each) stay near the 256 MiB
  // Infinity Cache while still giving the Riccati kernel >= 4 wavefronts per SIMD
  int64_t chunk = 65536;
  if (const char* e = getenv("MPCB_CHUNK")) chunk = atoll(e);
  if (chunk < 64) chunk = 64;
  if (chunk > max_batch) chunk = max_batch;
  h->chunk = chunk;
  // optional (MPCB_SMALL_MAX): linearise all stages in parallel and run the Riccati recursion
  // over the cached [A|B].  Measured slower at c2 (lin 62 + passes 172 us vs P2+P3 187 us):
  // the recursion's latency is its LDS exchanges, not the tangents, so it is off by default.
  int64_t small_max = 0;
  if (const char* e = getenv("MPCB_SMALL_MAX")) small_max = atoll(e);
  h->small = (!cfg->box_u && chunk <= small_max) ? 1 : 0;
  // chunks of at most 16384 instances (c2: 4096, one wave per SIMD, latency-bound) use the
  // 16-lane kernels: the forward pass over P2's row-major exports and the row rollout (f split
  // over the 16 lanes of an instance, mpcb_rollout.hip); larger chunks (c3, c5) run the
  // thread-per-instance rollout and forward pass (the lane-quad rollout measured slower there:
  // c3 P1 0.098 vs 0.090 ms, c5 0.38 vs 0.34 ms)
  const bool lat = chunk <= 16384;
  h->fwd16 = (!cfg->box_u && !h->small && lat) ? 1 : 0;
  // the row rollout stages the wave's u / xbar records in dynamic LDS (mpcb_row.h row_lds_bytes,
  // sized here for iterate mode, the larger carve); beyond 64 KiB the lane-quad rollout
  const size_t row_lds = (size_t)GROUPS * ((size_t)cfg->N * NU + (size_t)(cfg->N + 1) * NX) * esz;
  h->quad_p1 = lat ? (row_lds <= LDS_DYN_MAX ? 2 : 1) : 0;
  // the row rollout also integrates the tangents and exports [A|B] (MPCB_P1_TAN: default on in
  // fp64; in fp32 its regrouped tangent algebra doubled the worst U error of the N=60 box test,
  // 3.7e-5 -> 7.3e-5 against the 5e-5 bound, so fp32 keeps the captured scalars); P2 then reads
  // [A|B] instead of integrating it.  Only where a consumer of the row-major exports runs (the
  // 16-lane forward pass or the active-set kernel): the thread-per-instance forward reads the CC
  // record, which the tangent rollout does not write.
  h->tin = (h->quad_p1 == 2 && !h->small && f64 && (cfg->box_u || h->fwd16)) ? 1 : 0;
  if (const char* e = getenv("MPCB_P1_TAN")) if (atoi(e) == 0) h->tin = 0;
  // ... and P2 runs in the same launch (row_riccati_kernel) when the two bodies' LDS still
  // leaves one wave per SIMD resident, unless MPCB_FUSE_P12=0
  if (h->tin && row_lds + RICCATI_F64_STATIC_LDS > LDS_PER_WAVE_SIMD) h->tin = 2;
  if (h->tin)
    if (const char* e = getenv("MPCB_FUSE_P12")) if (atoi(e) == 0) h->tin = 2;
  const int ab = cfg->box_u ? 2 : ((h->small || h->fwd16 || h->tin) ? 1 : 0);
  const int64_t per = f64 ? split_elems_per_instance<double>(cfg->N, 1, ab)
                          : split_elems_per_instance<float>(cfg->N, 1, ab);
  // (+64: the forward's row loads may read up to 4 elements past the last ABT2 row)
  h->chunk_elems = per * ((chunk + 3) / 4 * 4) + 64;
  h->scratch_bytes = h->chunk_elems * (int64_t)esz;
}

// the fp32 refinement list's capacity: the whole batch (c4 lists 252 of 65,536, but on strongly
// constrained draws most instances reach it through the interior-point fallback)
static int64_t ref_cap(int64_t max_batch) { return max_batch; }

extern "C" int mpcb_create(const mpcb_config* cfg, int device, int64_t max_batch, mpcb_handle** out) {
  if (!cfg || !out) return fail(MPCB_E_INVALID, "null argument");
  *out = nullptr;
  double Jinv[9];
  if (int rc = validate_config(cfg, max_batch, Jinv)) return rc;
  const bool full = cfg->nx == NX17 && cfg->nu == NU17;
  const bool f64 = cfg->dtype == MPCB_F64;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MPCB_E_INVALID, "device %d of %d", device, ndev);
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));

  mpcb_handle* h = new mpcb_handle();
  h->device = device;
  select_path(h, cfg, max_batch, prop.multiProcessorCount);
  fill_model(*cfg, Jinv, h->Md);
  fill_model(*cfg, Jinv, h->Mf);
  hipError_t e = hipMalloc(&h->scratch, (size_t)h->scratch_bytes);
  if (e != hipSuccess) {
    delete h;
    return fail(MPCB_E_NOMEM, "workspace %lld bytes: %s", (long long)h->scratch_bytes, hipGetErrorString(e));
  }
  const size_t wbytes = full ? (f64 ? sizeof(Weights17<double>) : sizeof(Weights17<float>))
                             : (f64 ? sizeof(Weights<double>) : sizeof(Weights<float>));
  e = hipMalloc(&h->weights, wbytes);
  if (e != hipSuccess) {
    (void)hipFree(h->scratch);
    delete h;
    return fail(MPCB_E_NOMEM, "weights: %s", hipGetErrorString(e));
  }
  if (full && f64) {
    Weights17<double> w;
    fill_weights17(*cfg, w);
    e = hipMemcpy(h->weights, &w, sizeof(w), hipMemcpyHostToDevice);
  } else if (full) {
    Weights17<float> w;
    fill_weights17(*cfg, w);
    e = hipMemcpy(h->weights, &w, sizeof(w), hipMemcpyHostToDevice);
  } else if (f64) {
    Weights<double> w;
    fill_weights(*cfg, w);
    e = hipMemcpy(h->weights, &w, sizeof(w), hipMemcpyHostToDevice);
  } else {
    Weights<float> w;
    fill_weights(*cfg, w);
    e = hipMemcpy(h->weights, &w, sizeof(w), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    (void)hipFree(h->scratch);
    (void)hipFree(h->weights);
    delete h;
    return fail(MPCB_E_HIP, "weights upload: %s", hipGetErrorString(e));
  }
  if (cfg->box_u && (full || h->split)) {
    // (+ 16: the 12/4 active-set kernel's work counter after the statistics; then its
    // interior-point fallback's list, 2 + max_batch: SplitArgs::as_fb; then the fp32 refinement
    // list, AS_REF_HDR + AS_REF_W ref_cap(max_batch): SplitArgs::as_ref)
    e = hipMalloc((void**)&h->qp_stats,
                  ((size_t)max_batch * 3 + 18 + AS_REF_HDR + (size_t)AS_REF_W * ref_cap(max_batch)) * sizeof(int32_t));
    if (e == hipSuccess && !full && cfg->dtype == MPCB_F32)
      e = hipMalloc(&h->u_scratch, (size_t)max_batch * cfg->N * 4 * sizeof(float));
    if (h->u_scratch) h->scratch_bytes += (int64_t)max_batch * cfg->N * 4 * sizeof(float);
    if (e != hipSuccess) {
      (void)hipFree(h->scratch);
      (void)hipFree(h->weights);
      if (h->qp_stats) (void)hipFree(h->qp_stats);
      delete h;
      return fail(MPCB_E_NOMEM, "qp stats: %s", hipGetErrorString(e));
    }
  }
  *out = h;
  return MPCB_OK;
}

extern "C" int mpcb_destroy(mpcb_handle* h) {
  if (!h) return MPCB_OK;
  (void)hipSetDevice(h->device);
  for (auto& c : h->ev)
    for (auto& e : c)
      if (e) (void)hipEventDestroy(e);
  (void)hipFree(h->scratch);
  (void)hipFree(h->weights);
  if (h->qp_stats) (void)hipFree(h->qp_stats);
  if (h->u_scratch) (void)hipFree(h->u_scratch);
  delete h;
  return MPCB_OK;
}

#ifdef MPCB_AS_ORDER_DBG
// A/B of the active-set kernel's work order: a device array mapping the counter's tickets to
// instances of the first chunk (nullptr: identity)
extern "C" int mpcb_debug_set_as_order(mpcb_handle* h, const int32_t* dev_order) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  h->as_order_dbg = dev_order;
  return MPCB_OK;
}
#endif
// Diagnostic (not part of the ABI header): the last fp32 input-box chunk's refinement list header
// (mpcb_kernels.h AS_REF_*: [0] instances listed, [1] the refinement kernel's counter), read
// synchronously into out[0..1] (tools/c4_full_parity.py).
extern "C" int mpcb_debug_ref_list(mpcb_handle* h, int32_t* out) {
  if (!h || !h->qp_stats || !out) return fail(MPCB_E_INVALID, "no input-box handle");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipMemcpy(out, h->qp_stats + 3 * h->max_batch + 18, 2 * sizeof(int32_t), hipMemcpyDeviceToHost));
  return MPCB_OK;
}
extern "C" int mpcb_qp_stats(mpcb_handle* h, int64_t B, int32_t* out, void* stream) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (!h->qp_stats) return fail(MPCB_E_UNSUPPORTED, "QP statistics are kept by input-box handles");
  if (B < 0 || B > h->qp_stats_rows)
    return fail(MPCB_E_INVALID, "batch %lld exceeds the last boxed solve's %lld instances", (long long)B,
                (long long)h->qp_stats_rows);
  if (B == 0) return MPCB_OK;
  if (!out) return fail(MPCB_E_INVALID, "null array");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipMemcpyAsync(out, h->qp_stats, (size_t)B * 2 * sizeof(int32_t), hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return MPCB_OK;
}

template <class T>
static int solve_body(mpcb_handle* h, int64_t B, int mode, const void* x0, int64_t x0_sb,
                      const void* xbar, const void* ubar, const void* xref, int64_t xref_sb,
                      const void* uref, int64_t uref_sb, const void* wind, int64_t wind_sb,
                      void* u0, void* X, void* U, int32_t* status, void* stream) {
  if (h->full) {
    if (wind) return fail(MPCB_E_UNSUPPORTED, "wind is a 12/4-model extension");
    FullArgs<T> a;
    a.N = h->cfg.N;
    a.mode = mode;
    a.h = (T)h->cfg.dt;
    a.s = (T)h->cfg.cost_scale;
    if constexpr (sizeof(T) == 8) a.M = h->Md; else a.M = h->Mf;
    a.W = reinterpret_cast<const Weights17<T>*>(h->weights);
    a.p = (const T*)h->params; a.p_sb = h->params_sb; a.p_kb = h->params_kb;
    a.x0 = (const T*)x0; a.x0_sb = x0_sb;
    a.xref = (const T*)xref; a.xref_sb = xref_sb;
    a.uref = (const T*)uref; a.uref_sb = uref_sb;
    a.xbar = (const T*)xbar; a.ubar = (const T*)ubar;
    a.u0 = (T*)u0; a.X = (T*)X; a.U = (T*)U; a.status = status;
    a.ws = (T*)h->scratch;
    a.box = h->cfg.box_u;
    a.sbox = h->cfg.box_x;
    a.max_as_iter = h->cfg.max_as_iter;
    a.qp_stats = h->qp_stats;
    int chunk_i = 0;
    for (int64_t b0 = 0; b0 < B; b0 += h->chunk) {
      a.b0 = b0;
      a.nb = (B - b0 < h->chunk) ? B - b0 : h->chunk;
      hipEvent_t* ev = (h->timing && chunk_i < mpcb_handle::TCHUNKS) ? h->ev[chunk_i] : nullptr;
      hipError_t e = launch_full17<T>(a, (hipStream_t)stream, ev);
      if (e != hipSuccess) return fail(MPCB_E_HIP, "full17 launch: %s", hipGetErrorString(e));
      ++chunk_i;
    }
    h->timed_chunks = h->timing ? (chunk_i < mpcb_handle::TCHUNKS ? chunk_i : mpcb_handle::TCHUNKS) : 0;
    h->timed_split = 1;
    if (h->qp_stats) h->qp_stats_rows = B;
    return MPCB_OK;
  }
  if (h->split) {
    SplitArgs<T> a;
    a.N = h->cfg.N;
    a.mode = mode;
    a.h = (T)h->cfg.dt;
    a.s = (T)h->cfg.cost_scale;
    if constexpr (sizeof(T) == 8) a.M = h->Md; else a.M = h->Mf;
    a.W = reinterpret_cast<const Weights<T>*>(h->weights);
    a.x0 = (const T*)x0; a.x0_sb = x0_sb;
    a.xref = (const T*)xref; a.xref_sb = xref_sb;
    a.uref = (const T*)uref; a.uref_sb = uref_sb;
    a.wind = (const T*)wind; a.wind_sb = wind_sb;
    a.xbar = (const T*)xbar; a.ubar = (const T*)ubar;
    a.u0 = (T*)u0; a.X = (T*)X; a.U = (T*)U; a.status = status;
    a.fwd = (X || U || mode == MPCB_MODE_ITERATE || h->cfg.box_u) ? 1 : 0;
    // the active set's pass budget; instances still unconverged go to the interior point
    a.max_as_iter = h->cfg.max_as_iter < AS_IPM_AFTER ? h->cfg.max_as_iter : AS_IPM_AFTER;
    const int N = h->cfg.N;
    int chunk_i = 0;
    for (int64_t b0 = 0; b0 < B; b0 += h->chunk) {
      const int64_t nb = (B - b0 < h->chunk) ? B - b0 : h->chunk;
      T* base = (T*)h->scratch;
      a.b0 = b0;
      a.nb = nb;
      const int64_t nbp = (nb + 3) / 4 * 4;   // quad-blocked layout pads to 4 instances
      a.XU = base;
      a.CC = a.XU + (int64_t)(N + 1) * nbp * XU_REC;
      a.KR = a.CC + (int64_t)N * nbp * CCS_REC;
      a.GP = a.KR + (int64_t)N * nbp * KR2_REC;
      a.small = h->small;
      a.fwd16 = h->fwd16;
      a.quad_p1 = h->quad_p1;
      a.tin = h->tin;
      T* ab = a.GP + (int64_t)N * nbp * GP_REC;
      // row-major exports for the active-set kernel and the 16-lane forward pass; the optional
      // small-batch path (lin_kernel + box_body) keeps its own quad-blocked pair
      a.rm = (h->cfg.box_u || (h->fwd16 && a.fwd)) ? 1 : 0;
      // (box path stage-major: instance-major exports measured no faster at c4 in round 5 --
      // active-set kernel 3.15 vs 3.19 ms, P2 1.06-1.08 vs 1.04 ms -- and round 3)
      a.imajor = h->cfg.box_u ? 0 : 1;
      a.AB = h->small ? ab : nullptr;   // (the small-chunk path's column-ordered [A|B])
      a.ABT = (h->cfg.box_u || h->small || h->tin || (h->fwd16 && a.fwd)) ? ab + (int64_t)N * nbp * AB2_REC : nullptr;
      a.GH = h->cfg.box_u ? a.ABT + (int64_t)N * nbp * ABT2_REC : nullptr;
      a.PS = h->cfg.box_u ? a.GH + (int64_t)N * nbp * GH2_REC : nullptr;
      a.qp_stats = h->qp_stats;
      // the active-set kernel's work counter (MPCB_AS_PERSIST=0: one wave per instance quad)
      a.as_queue = h->qp_stats ? h->qp_stats + 2 * h->max_batch : nullptr;
      if (const char* e = getenv("MPCB_AS_PERSIST")) if (atoi(e) == 0) a.as_queue = nullptr;
      a.as_fb = (h->cfg.box_u && h->qp_stats) ? h->qp_stats + 2 * h->max_batch + 16 : nullptr;
      a.as_ref = (sizeof(T) == 4 && h->cfg.box_u && h->qp_stats) ? h->qp_stats + 3 * h->max_batch + 18 : nullptr;
      if (const char* e = getenv("MPCB_AS_REFINE")) if (atoi(e) == 0) a.as_ref = nullptr;   // (A/B: no refinement)
      a.as_ref_cap = (int)ref_cap(h->max_batch);
      if (a.as_ref && !a.U) a.U = (T*)h->u_scratch;   // (the refinement kernel restarts from U)
      a.as_order = (h->cfg.box_u && b0 == 0) ? h->as_order_dbg : nullptr;
      hipEvent_t* ev = (h->timing && chunk_i < mpcb_handle::TCHUNKS) ? h->ev[chunk_i] : nullptr;
      hipError_t e = launch_split<T>(a, (hipStream_t)stream, ev);
      if (e != hipSuccess) return fail(MPCB_E_HIP, "split launch: %s", hipGetErrorString(e));
      ++chunk_i;
    }
    if (h->timing) {
      h->timed_chunks = chunk_i < mpcb_handle::TCHUNKS ? chunk_i : mpcb_handle::TCHUNKS;
      h->timed_split = 1;
    }
    if (h->qp_stats) h->qp_stats_rows = B;
    return MPCB_OK;
  }
  SolveArgs<T> a;
  a.B = B;
  a.N = h->cfg.N;
  a.mode = mode;
  a.box = h->cfg.box_u;
  a.max_as_iter = h->cfg.max_as_iter;
  a.h = (T)h->cfg.dt;
  a.s = (T)h->cfg.cost_scale;
  if constexpr (sizeof(T) == 8) a.M = h->Md; else a.M = h->Mf;
  a.W = reinterpret_cast<const Weights<T>*>(h->weights);
  a.x0 = (const T*)x0; a.x0_sb = x0_sb;
  a.xref = (const T*)xref; a.xref_sb = xref_sb;
  a.uref = (const T*)uref; a.uref_sb = uref_sb;
  a.wind = (const T*)wind; a.wind_sb = wind_sb;
  a.xbar = (const T*)xbar; a.ubar = (const T*)ubar;
  a.u0 = (T*)u0; a.X = (T*)X; a.U = (T*)U; a.status = status;
  a.scratch = (T*)h->scratch;
  a.slot_elems = h->slot_elems;
  const int64_t waves = (B + GROUPS - 1) / GROUPS;
  const int grid = (int)(waves < h->grid ? waves : h->grid);
  if (h->timing) (void)hipEventRecord(h->ev[0][0], (hipStream_t)stream);
  hipError_t e = launch_solve<T>(a, grid, (hipStream_t)stream);
  if (e != hipSuccess) return fail(MPCB_E_HIP, "solve launch: %s", hipGetErrorString(e));
  if (h->timing) {
    (void)hipEventRecord(h->ev[0][1], (hipStream_t)stream);
    h->timed_chunks = 1;
    h->timed_split = 0;
  }
  return MPCB_OK;
}

// solve_body with the launch log: the kernels this solve launches (or, in a dry run, would launch)
template <class T>
static int solve_impl(mpcb_handle* h, int64_t B, int mode, const void* x0, int64_t x0_sb,
                      const void* xbar, const void* ubar, const void* xref, int64_t xref_sb,
                      const void* uref, int64_t uref_sb, const void* wind, int64_t wind_sb,
                      void* u0, void* X, void* U, int32_t* status, void* stream) {
  LaunchLog& L = launch_log();
  for (auto& f : L.fn) f = nullptr;
  const int rc = solve_body<T>(h, B, mode, x0, x0_sb, xbar, ubar, xref, xref_sb, uref, uref_sb, wind,
                               wind_sb, u0, X, U, status, stream);
  for (int i = 0; i < LOG_SLOTS; ++i) h->last_fn[i] = L.fn[i];
  return rc;
}

// "mpcb::riccati_kernel_f32<false, false, false>": the demangled kernel symbol without its return
// type and parameters, as rocprofv3 names the dispatch (a kernel's host handle is a dynamic symbol
// of this library named like the device function)
static std::string kernel_name(const void* fn) {
  if (!fn) return "";
  Dl_info inf;
  if (!dladdr(fn, &inf) || !inf.dli_sname) return "?";
  int st = 0;
  char* d = abi::__cxa_demangle(inf.dli_sname, nullptr, nullptr, &st);
  std::string s = d ? d : inf.dli_sname;
  free(d);
  if (s.rfind("void ", 0) == 0) s = s.substr(5);
  int depth = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '<') ++depth;
    else if (s[i] == '>') --depth;
    else if (s[i] == '(' && depth == 0) return s.substr(0, i);
  }
  return s;
}

static int write_kernel_names(const void* const fn[LOG_SLOTS], char* buf, int64_t len) {
  std::string out;
  for (int i = 0; i < LOG_SLOTS; ++i) out += kernel_name(fn[i]) + (i + 1 < LOG_SLOTS ? "\n" : "");
  if (!buf || len < (int64_t)out.size() + 1)
    return fail(MPCB_E_INVALID, "kernel names need a buffer of %zu bytes", out.size() + 1);
  memcpy(buf, out.c_str(), out.size() + 1);
  return MPCB_OK;
}

extern "C" int mpcb_plan_kernels(const mpcb_config* cfg, int64_t max_batch, int64_t B, int mode, int want_traj,
                                 char* buf, int64_t len) {
  if (!cfg) return fail(MPCB_E_INVALID, "null config");
  double Jinv[9];
  if (int rc = validate_config(cfg, max_batch, Jinv)) return rc;
  if (B < 1 || B > max_batch) return fail(MPCB_E_INVALID, "batch %lld outside 1..max_batch", (long long)B);
  if (mode != MPCB_MODE_ROLLOUT && mode != MPCB_MODE_ITERATE) return fail(MPCB_E_INVALID, "mode=%d", mode);
  mpcb_handle h;
  h.device = -1;
  select_path(&h, cfg, max_batch, 256);
  fill_model(*cfg, Jinv, h.Md);
  fill_model(*cfg, Jinv, h.Mf);
  // (never dereferenced: a dry run makes no HIP call and launches nothing)
  alignas(16) static double dummy[64];
  void* d = dummy;
  LaunchLog& L = launch_log();
  L.dry = true;
  int rc = cfg->dtype == MPCB_F64
               ? solve_impl<double>(&h, B, mode, d, 0, d, d, d, 0, d, 0, nullptr, 0, d, want_traj ? d : nullptr,
                                    want_traj ? d : nullptr, (int32_t*)d, nullptr)
               : solve_impl<float>(&h, B, mode, d, 0, d, d, d, 0, d, 0, nullptr, 0, d, want_traj ? d : nullptr,
                                   want_traj ? d : nullptr, (int32_t*)d, nullptr);
  L.dry = false;
  if (rc) return rc;
  return write_kernel_names(h.last_fn, buf, len);
}

extern "C" int mpcb_last_kernels(const mpcb_handle* h, char* buf, int64_t len) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  return write_kernel_names(h->last_fn, buf, len);
}

extern "C" int mpcb_set_timing(mpcb_handle* h, int enable) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (enable && !h->ev[0][0]) {
    hipError_t e = hipSetDevice(h->device);
    for (auto& c : h->ev)
      for (auto& ev : c)
        if (e == hipSuccess) e = hipEventCreate(&ev);
    if (e != hipSuccess) return fail(MPCB_E_HIP, "hipEventCreate: %s", hipGetErrorString(e));
  }
  h->timing = enable ? 1 : 0;
  h->timed_chunks = 0;
  return MPCB_OK;
}

extern "C" int mpcb_last_timing(mpcb_handle* h, float* ms) {
  if (!h || !ms) return fail(MPCB_E_INVALID, "null argument");
  ms[0] = ms[1] = ms[2] = 0.f;
  if (!h->timing || h->timed_chunks == 0) return fail(MPCB_E_INVALID, "no timed solve recorded");
  for (int c = 0; c < h->timed_chunks; ++c) {
    const int phases = h->timed_split ? 3 : 1;
    for (int p = 0; p < phases; ++p) {
      float t = 0.f;
      hipError_t e = hipEventSynchronize(h->ev[c][p + 1]);
      if (e == hipSuccess) e = hipEventElapsedTime(&t, h->ev[c][p], h->ev[c][p + 1]);
      if (e != hipSuccess) return fail(MPCB_E_HIP, "event timing: %s", hipGetErrorString(e));
      // 17/6: the phases run nominal17, lin17ws, riccati17 (+ forward); ms[1] stays the Riccati
      const int slot = !h->timed_split ? 1 : (h->full ? (p == 0 ? 0 : (p == 1 ? 2 : 1)) : p);
      ms[slot] += t;
    }
  }
  return MPCB_OK;
}

static int check_solve(mpcb_handle* h, int64_t B, const void* x0, const void* xref, const void* uref,
                       const void* u0, const void* X, const void* U, const int32_t* status) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (B < 0 || B > h->max_batch)
    return fail(MPCB_E_INVALID, "batch %lld exceeds max_batch %lld", (long long)B, (long long)h->max_batch);
  if (B > 0 && (!x0 || !xref || !uref || !u0 || !status))
    return fail(MPCB_E_INVALID, "x0, xref, uref, u0 and status are required");
  // the trajectory outputs are written in 16-byte chunks
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(U)) & 15)
    return fail(MPCB_E_INVALID, "X and U must be 16-byte aligned");
  return MPCB_OK;
}

extern "C" int mpcb_solve(mpcb_handle* h, int64_t B, const void* x0, int64_t x0_sb, const void* xref,
               int64_t xref_sb, const void* uref, int64_t uref_sb, const void* wind, int64_t wind_sb,
               void* u0, void* X, void* U, int32_t* status, void* stream) {
  int rc = check_solve(h, B, x0, xref, uref, u0, X, U, status);
  if (!rc) rc = check_params(h, B);
  if (rc || B == 0) return rc;
  HIP_TRY(hipSetDevice(h->device));
  if (h->cfg.dtype == MPCB_F64)
    return solve_impl<double>(h, B, MPCB_MODE_ROLLOUT, x0, x0_sb, nullptr, nullptr, xref, xref_sb, uref,
                              uref_sb, wind, wind_sb, u0, X, U, status, stream);
  return solve_impl<float>(h, B, MPCB_MODE_ROLLOUT, x0, x0_sb, nullptr, nullptr, xref, xref_sb, uref,
                           uref_sb, wind, wind_sb, u0, X, U, status, stream);
}

extern "C" int mpcb_solve_iterate(mpcb_handle* h, int64_t B, const void* x0, int64_t x0_sb, const void* xbar,
                       const void* ubar, const void* xref, int64_t xref_sb, const void* uref,
                       int64_t uref_sb, const void* wind, int64_t wind_sb, void* u0, void* X, void* U,
                       int32_t* status, void* stream) {
  int rc = check_solve(h, B, x0, xref, uref, u0, X, U, status);
  if (!rc) rc = check_params(h, B);
  if (rc || B == 0) return rc;
  if (!xbar || !ubar) return fail(MPCB_E_INVALID, "xbar and ubar are required");
  HIP_TRY(hipSetDevice(h->device));
  if (h->cfg.dtype == MPCB_F64)
    return solve_impl<double>(h, B, MPCB_MODE_ITERATE, x0, x0_sb, xbar, ubar, xref, xref_sb, uref,
                              uref_sb, wind, wind_sb, u0, X, U, status, stream);
  return solve_impl<float>(h, B, MPCB_MODE_ITERATE, x0, x0_sb, xbar, ubar, xref, xref_sb, uref,
                           uref_sb, wind, wind_sb, u0, X, U, status, stream);
}

extern "C" int mpcb_linearize(mpcb_handle* h, int64_t B, const void* xbar, const void* ubar, const void* wind,
                   int64_t wind_sb, void* A, void* Bm, void* xnext, void* stream) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (B < 0) return fail(MPCB_E_INVALID, "negative batch");
  if (B == 0) return MPCB_OK;
  if (!xbar || !ubar || !A || !Bm || !xnext) return fail(MPCB_E_INVALID, "null array");
  if (int rc = check_params(h, B)) return rc;
  HIP_TRY(hipSetDevice(h->device));
  hipError_t e;
  if (h->full) {
    if (wind) return fail(MPCB_E_UNSUPPORTED, "wind is a 12/4-model extension");
    const int64_t psb = h->params ? h->params_sb : 0, pkb = h->params ? h->params_kb : 0;
    if (h->cfg.dtype == MPCB_F64) {
      const double* p = h->params ? (const double*)h->params : reinterpret_cast<const Weights17<double>*>(h->weights)->p;
      e = launch_linearize17<double>(B, h->cfg.N, h->cfg.dt, h->Md, p, psb, pkb, (const double*)xbar,
                                     (const double*)ubar, (double*)A, (double*)Bm, (double*)xnext,
                                     (hipStream_t)stream);
    } else {
      const float* p = h->params ? (const float*)h->params : reinterpret_cast<const Weights17<float>*>(h->weights)->p;
      e = launch_linearize17<float>(B, h->cfg.N, (float)h->cfg.dt, h->Mf, p, psb, pkb, (const float*)xbar,
                                    (const float*)ubar, (float*)A, (float*)Bm, (float*)xnext,
                                    (hipStream_t)stream);
    }
  } else if (h->cfg.dtype == MPCB_F64)
    e = launch_linearize<double>(B, h->cfg.N, h->cfg.dt, h->Md, (const double*)xbar, (const double*)ubar,
                                 (const double*)wind, wind_sb, (double*)A, (double*)Bm, (double*)xnext,
                                 (hipStream_t)stream);
  else
    e = launch_linearize<float>(B, h->cfg.N, (float)h->cfg.dt, h->Mf, (const float*)xbar, (const float*)ubar,
                                (const float*)wind, wind_sb, (float*)A, (float*)Bm, (float*)xnext,
                                (hipStream_t)stream);
  if (e != hipSuccess) return fail(MPCB_E_HIP, "linearize launch: %s", hipGetErrorString(e));
  return MPCB_OK;
}

extern "C" int mpcb_sim_step(mpcb_handle* h, int64_t B, const void* x, const void* u, const void* wind,
                  int64_t wind_sb, double T, void* x_out, void* stream) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (B < 0) return fail(MPCB_E_INVALID, "negative batch");
  if (B == 0) return MPCB_OK;
  if (!x || !u || !x_out) return fail(MPCB_E_INVALID, "null array");
  if (!(T > 0)) return fail(MPCB_E_INVALID, "T must be > 0");
  if (int rc = check_params(h, B)) return rc;
  HIP_TRY(hipSetDevice(h->device));
  hipError_t e;
  if (h->full) {
    if (wind) return fail(MPCB_E_UNSUPPORTED, "wind is a 12/4-model extension");
    const int64_t psb = h->params ? h->params_sb : 0;
    if (h->cfg.dtype == MPCB_F64) {
      const double* p = h->params ? (const double*)h->params : reinterpret_cast<const Weights17<double>*>(h->weights)->p;
      e = launch_sim_step17<double>(B, T, h->Md, p, psb, (const double*)x, (const double*)u,
                                    (double*)x_out, (hipStream_t)stream);
    } else {
      const float* p = h->params ? (const float*)h->params : reinterpret_cast<const Weights17<float>*>(h->weights)->p;
      e = launch_sim_step17<float>(B, (float)T, h->Mf, p, psb, (const float*)x, (const float*)u,
                                   (float*)x_out, (hipStream_t)stream);
    }
  } else if (h->cfg.dtype == MPCB_F64)
    e = launch_sim_step<double>(B, T, h->Md, (const double*)x, (const double*)u, (const double*)wind,
                                wind_sb, (double*)x_out, (hipStream_t)stream);
  else
    e = launch_sim_step<float>(B, (float)T, h->Mf, (const float*)x, (const float*)u, (const float*)wind,
                               wind_sb, (float*)x_out, (hipStream_t)stream);
  if (e != hipSuccess) return fail(MPCB_E_HIP, "sim_step launch: %s", hipGetErrorString(e));
  return MPCB_OK;
}

extern "C" int mpcb_gen_inputs(mpcb_handle* h, int64_t B, uint64_t seed, uint64_t id_offset, int ref_kind, void* x0,
                    void* xref, int64_t xref_sb, void* uref, int64_t uref_sb, void* wind, void* stream) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (B < 0) return fail(MPCB_E_INVALID, "negative batch");
  if (B == 0) return MPCB_OK;
  if (!x0 || !xref || !uref) return fail(MPCB_E_INVALID, "null array");
  if (ref_kind == 1 && xref_sb == 0) return fail(MPCB_E_INVALID, "sinusoid refs need xref_sb > 0");
  if (h->full) return fail(MPCB_E_UNSUPPORTED, "the synthetic generator covers the 12/4 configs");
  HIP_TRY(hipSetDevice(h->device));
  hipError_t e;
  if (h->cfg.dtype == MPCB_F64)
    e = launch_gen_inputs<double>(B, h->cfg.N, h->cfg.dt, seed, id_offset, ref_kind, (double*)x0,
                                  (double*)xref, xref_sb, (double*)uref, uref_sb, (double*)wind,
                                  (hipStream_t)stream);
  else
    e = launch_gen_inputs<float>(B, h->cfg.N, (float)h->cfg.dt, seed, id_offset, ref_kind, (float*)x0,
                                 (float*)xref, xref_sb, (float*)uref, uref_sb, (float*)wind,
                                 (hipStream_t)stream);
  if (e != hipSuccess) return fail(MPCB_E_HIP, "gen_inputs launch: %s", hipGetErrorString(e));
  return MPCB_OK;
}

extern "C" int mpcb_histogram(mpcb_handle* h, int64_t B, const void* u0, double lo, double hi, int nbins,
                   int64_t* counts, void* stream) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (B < 0 || nbins < 1 || nbins > 4096 || !(hi > lo)) return fail(MPCB_E_INVALID, "bad histogram args");
  if (h->full) return fail(MPCB_E_UNSUPPORTED, "the u0 histogram covers the 12/4 configs");
  if (B == 0) return MPCB_OK;
  if (!u0 || !counts) return fail(MPCB_E_INVALID, "null array");
  HIP_TRY(hipSetDevice(h->device));
  hipError_t e;
  if (h->cfg.dtype == MPCB_F64)
    e = launch_histogram<double>(B, NU, (const double*)u0, lo, hi, nbins, (unsigned long long*)counts,
                                 (hipStream_t)stream);
  else
    e = launch_histogram<float>(B, NU, (const float*)u0, lo, hi, nbins, (unsigned long long*)counts,
                                (hipStream_t)stream);
  if (e != hipSuccess) return fail(MPCB_E_HIP, "histogram launch: %s", hipGetErrorString(e));
  return MPCB_OK;
}

extern "C" int mpcb_quat_ops(int64_t B, const double* q1, const double* q2, double* prod, double* inv,
                             double* rot, void* stream) {
  if (B < 0) return fail(MPCB_E_INVALID, "B=%lld", (long long)B);
  if (B == 0) return MPCB_OK;
  if (!q1 || (prod && !q2)) return fail(MPCB_E_INVALID, "null quaternion array");
  hipError_t e = launch_quat_ops(B, q1, q2, prod, inv, rot, (hipStream_t)stream);
  if (e != hipSuccess) return fail(MPCB_E_HIP, "quat_ops launch: %s", hipGetErrorString(e));
  return MPCB_OK;
}

extern "C" int mpcb_set_params(mpcb_handle* h, int64_t count, const void* params, int64_t params_sb,
                               int64_t params_kb) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (!h->full) return fail(MPCB_E_UNSUPPORTED, "the 12/4 model's only parameter is T_blast (mpcb_set_t_blast)");
  if (params_sb < 0 || params_kb < 0) return fail(MPCB_E_INVALID, "negative parameter stride");
  if (params && count < 1) return fail(MPCB_E_INVALID, "parameter rows count=%lld", (long long)count);
  h->params = params;
  h->params_sb = params ? params_sb : 0;
  h->params_kb = params ? params_kb : 0;
  h->params_count = params ? count : 0;
  return MPCB_OK;
}

extern "C" int mpcb_set_t_blast(mpcb_handle* h, double t_blast) {
  if (!h) return fail(MPCB_E_INVALID, "null handle");
  if (!std::isfinite(t_blast)) return fail(MPCB_E_INVALID, "T_blast must be finite");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());   // kernels in flight may still read the old value
  h->cfg.t_blast = t_blast;
  h->Md.t_blast = t_blast;
  h->Mf.t_blast = (float)t_blast;
  if (h->full) {
    if (h->cfg.dtype == MPCB_F64) {
      const double v = t_blast;
      HIP_TRY(hipMemcpy((char*)h->weights + offsetof(Weights17<double>, p) + 24 * sizeof(double), &v,
                        sizeof(v), hipMemcpyHostToDevice));
    } else {
      const float v = (float)t_blast;
      HIP_TRY(hipMemcpy((char*)h->weights + offsetof(Weights17<float>, p) + 24 * sizeof(float), &v,
                        sizeof(v), hipMemcpyHostToDevice));
    }
  }
  return MPCB_OK;
}
