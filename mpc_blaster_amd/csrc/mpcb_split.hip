// mpcb_split.hip — the unconstrained SQP_RTI step as three specialised kernels per chunk.
//
// Replaces one acados ``ocp_solver.solve()`` per instance (src/scripts/simulation_blaster.py:80;
// OCP of blastermodel.py:214-292): ERK4 + forward sensitivities, Gauss-Newton LINEAR_LS QP,
// Riccati solve, full step.  The work is split by its natural parallel width:
//  * P1 nominal   — a serial RK4 chain per instance: ONE THREAD PER INSTANCE.  Captures the 20
//    linearisation scalars of every RK4 stage (mpcb_model.h f_nom_lin) instead of materialising
//    A_k, B_k (80 vs 192 scalars per interval).
//  * P2 riccati   — 16 independent sensitivity directions per stage: 16 LANES PER INSTANCE
//    (4 instances per wavefront); lane j integrates the tangent seeded with e_j, so column j of
//    [A_k | B_k] lands in lane j; P, [A|B] and the stage Hessian columns meet in LDS; the 4x4
//    input block is factorised redundantly per lane.  P is stored symmetric by construction.
//  * P3 forward   — a serial chain again (dx_{k+1} = dPhi·(dx_k, du_k) + gap): ONE THREAD PER
//    INSTANCE, writing u0, X = xbar + dx, U = ubar + du and the status.
// Intermediates live in a chunk workspace sized to stay in the 256 MiB Infinity Cache.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/mpcb.h"
#include "mpcb_common.h"
#include "mpcb_split.h"
#include "mpcb_dpp_gen.h"

// fp64 Riccati products through DPP row broadcasts (1) or LDS operands (0, the earlier path)
#ifndef MPCB_P2_DPP
#define MPCB_P2_DPP 1
#endif

#ifndef MPCB_P1_ALLW
#define MPCB_P1_ALLW 1
#endif

// P1: broadcast u_ref rows staged in LDS (up to MPCB_P1_UMAX stages)
#ifndef MPCB_P1_ULDS
#define MPCB_P1_ULDS 1
#endif
#ifndef MPCB_P1_UMAX
#define MPCB_P1_UMAX 64
#endif

#ifndef MPCB_P2_WAVES
#define MPCB_P2_WAVES
#endif

#ifndef MPCB_P2_SWT
#define MPCB_P2_SWT 1
#endif
#ifndef MPCB_P2_CPAD
#define MPCB_P2_CPAD 16
#endif

#ifndef MPCB_P2_PCSEL
#define MPCB_P2_PCSEL 0
#endif

#ifndef MPCB_P2_GVAR   // fp64 P2: G's rows at the constant directions without broadcasts
#define MPCB_P2_GVAR 1
#endif
#ifndef MPCB_P2_WAVES_F32
#define MPCB_P2_WAVES_F32 2
#endif
#ifndef MPCB_P2_WAVES_F32_NOEXP   // the export-free fp32 instantiation (c3, c5)
#define MPCB_P2_WAVES_F32_NOEXP 2
#endif

namespace mpcb {
WT_TABLE(g_wt_p1)
}  // namespace mpcb

#include "mpcb_row.h"
#include "mpcb_as.h"

namespace mpcb {

#ifdef MPCB_STAMPS
// Diagnostic build only: per-region cycle counts of the Riccati stage loop of workgroup 0
// (s_memtime deltas, summed over stages), read back with mpcb_debug_stamps().
__device__ unsigned long long g_stamps[16];
#define STAMP_INIT() unsigned long long st_prev = __builtin_amdgcn_s_memtime(), st_acc[16] = {};
#define STAMP(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_prev; st_prev = t_; }
#define STAMP_DONE() if (blockIdx.x == 0 && threadIdx.x == 0) for (int i_ = 0; i_ < 16; ++i_) if (st_acc[i_]) g_stamps[i_] = st_acc[i_];
#else
#define STAMP_INIT()
#define STAMP(i)
#define STAMP_DONE()
#endif

// ---- wave-staged workspace / output traffic of the thread-per-instance passes (P1, P3) ------
// P1 and P3 run one thread per instance in single-wave workgroups: 64 instances = 16 quads.  For
// a fixed stage k the wave's records of any quad-blocked array are ONE contiguous run of
// 16 x REC x 4 elements, but element-per-thread accesses touch 16 cache lines per instruction
// (measured: the CC stores were 2/3 of P1's time at c3, the CC loads 1/3 of P3's at c2, the
// X/U stores another 1/3 of P3's).  So stores are staged in LDS and written as 16-B chunks
// (P1: 1 KiB of contiguous workspace per wave-instruction), and loads arrive by LDS-DMA
// (global_load_lds_dwordx4) one stage ahead into an element-major [REC][64] image that each
// thread reads conflict-free at img[i * 64 + lane].
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int WAVE = 64, WQ = WAVE / SS;

template <class T> __device__ __forceinline__ void copy16(T* dst, const T* src) {
  *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(src);
}

// Chunks t = lane, lane + 64, ... < TOT of an LDS -> global copy, LDS reads issued in batches of
// 8 ahead of their stores so the LDS latency is paid once per batch, not once per chunk.
template <int TOT, class Src, class Dst>
__device__ __forceinline__ void copy_chunks(int lane, Src src, Dst dst) {
  constexpr int NI = (TOT + 63) / 64;
#pragma unroll
  for (int g = 0; g < NI; g += 8) {
    u32x4 r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (g + e < NI && (TOT % 64 == 0 || (g + e) * 64 + lane < TOT))
        r[e] = *reinterpret_cast<const u32x4*>(src((g + e) * 64 + lane));
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (g + e < NI && (TOT % 64 == 0 || (g + e) * 64 + lane < TOT))
        *reinterpret_cast<u32x4*>(dst((g + e) * 64 + lane)) = r[e];
  }
}

// LDS staging of the wave's 16 quad records of a REC-element stage record; the quad stride
// REC*4+4 keeps the per-thread writes bank-conflict free (fp32 and fp64).
template <class T, int REC, int NQ = WQ>
struct QuadStore {
  static constexpr int STRIDE = REC * SS + 4;
  static constexpr int ELEMS = NQ * STRIDE;
  T* buf;
  __device__ __forceinline__ void put(int lane, int i, T v) const {
    buf[(lane >> 2) * STRIDE + i * SS + (lane & 3)] = v;
  }
  // dst = the wave's first quad record (soa(base, k, REC, nb, c0)); nqv quads are valid.  The
  // wave's records are contiguous in the workspace, so chunk t goes to dst + t * V.
  __device__ __forceinline__ void flush(int lane, T* dst, int nqv) const {
    constexpr int V = 16 / sizeof(T), CPQ = REC * SS / V, TOT = NQ * CPQ;
    auto src = [&](int t) { return buf + t * V + (t / CPQ) * 4; };
    if (nqv == NQ) {
      copy_chunks<TOT>(lane, src, [&](int t) { return dst + t * V; });
    } else {
      for (int t = lane; t < nqv * CPQ; t += WAVE) copy16(dst + t * V, src(t));
    }
  }
};

// LDS-DMA of the wave's stage record (REC elements per instance) into img[i * 64 + lane].
// Chunk t of the wave-linear DMA image holds element i = t / CPI of the V = 16/sizeof(T)
// consecutive instances (t % CPI) * V ..; lane l of instruction m therefore always reads the same
// quad column at row i = m * IPI + l / CPI, i.e. src_lane + m * IPI * 4 (``dma_lane_offset``).
typedef __attribute__((address_space(3))) void lds_void;
template <class T> struct Dma {
  static constexpr int V = 16 / sizeof(T), CPI = WAVE / V, IPI = WAVE / CPI;
  // element offset of lane l's first chunk inside a wave's record run; REC = record length
  __device__ static __forceinline__ int lane_offset(int lane, int rec) {
    const int part = lane % CPI;
    return ((part * V) / SS * rec + lane / CPI) * SS + (part * V) % SS;
  }
  __device__ static __forceinline__ bool lane_valid(int lane, int nqv) { return (lane % CPI) * V / SS < nqv; }
};
template <class T, int REC>
__device__ __forceinline__ void dma_record(unsigned img, const T* src_lane) {
  using D = Dma<T>;
  static_assert((REC * D::CPI) % WAVE == 0, "record must fill whole wave-instructions");
#pragma unroll
  for (int m = 0; m < REC * D::CPI / WAVE; ++m)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src_lane + m * D::IPI * SS),
        (lds_void*)(size_t)(img + m * WAVE * 16), 16, 0, 0);
}

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <class T, bool ITER>
__device__ __forceinline__ void nominal_wave(const SplitArgs<T>& a) {
  __shared__ __attribute__((aligned(16))) T lds_cc[QuadStore<T, CCS_REC>::ELEMS];
  __shared__ __attribute__((aligned(16))) T lds_xu[QuadStore<T, XU_REC>::ELEMS];
  __shared__ __attribute__((aligned(16))) T lds_gp[QuadStore<T, GP_REC>::ELEMS];
  const QuadStore<T, CCS_REC> ccs{lds_cc};
  const QuadStore<T, XU_REC> xus{lds_xu};
  const QuadStore<T, GP_REC> gps{lds_gp};
  const int lane = threadIdx.x;
  const int64_t nb = a.nb;
  const int64_t c0 = (int64_t)blockIdx.x * WAVE;
  // tail lanes recompute the chunk's last instance; their slots are quad padding or unflushed
  const int64_t c = (c0 + lane < nb) ? c0 + lane : nb - 1;
  const int64_t nq = (nb + SS - 1) / SS;
  const int nqv = (int)((nq - c0 / SS) < WQ ? nq - c0 / SS : WQ);
  const int64_t b = a.b0 + c;
  const int N = a.N;
  constexpr bool iterate = ITER;   // (see nominal_quad)
  T w[3] = {T(0), T(0), T(0)};
  if (a.wind) {
    w[0] = a.wind[b * a.wind_sb]; w[1] = a.wind[b * a.wind_sb + 1]; w[2] = a.wind[b * a.wind_sb + 2];
  }
  const T* xbp = a.xbar + b * (int64_t)(N + 1) * NX;
  const T* ubp = a.ubar + b * (int64_t)N * NU;
  const T* ur = a.uref + b * a.uref_sb;
  T x[NX], u[NU];
  load_vec<NX>(iterate ? xbp : a.x0 + b * a.x0_sb, x);
  for (int k = 0; k < N; ++k) {
    if (iterate) load_vec<NX>(xbp + (int64_t)k * NX, x);
    load_vec<NU>(iterate ? ubp + (int64_t)k * NU : ur + (int64_t)k * NU, u);
#pragma unroll
    for (int i = 0; i < NX; ++i) xus.put(lane, i, x[i]);
#pragma unroll
    for (int m = 0; m < NU; ++m) xus.put(lane, NX + m, u[m]);
    T xn[NX];
    rk4_nom<T>(x, u, a.h, a.M, w, xn, [&](int stage, const T* cv) {
#pragma unroll
      for (int i = 0; i < LIN_N; ++i) ccs.put(lane, stage * LIN_N + i, cv[i]);
    });
    if (iterate) {
      const T* nx = xbp + (int64_t)(k + 1) * NX;
#pragma unroll
      for (int i = 0; i < NX; ++i) gps.put(lane, i, xn[i] - nx[i]);
    } else {
#pragma unroll
      for (int i = 0; i < NX; ++i) x[i] = xn[i];
    }
    // one wave per workgroup: its LDS operations complete in order, so no barrier (which would
    // also drain the stores) is needed between the per-thread puts and the chunked flush
    xus.flush(lane, soa(a.XU, k, XU_REC, nb, c0), nqv);
    ccs.flush(lane, soa(a.CC, k, CCS_REC, nb, c0), nqv);
    if (iterate) gps.flush(lane, soa(a.GP, k, GP_REC, nb, c0), nqv);
  }
  if (iterate) load_vec<NX>(xbp + (int64_t)N * NX, x);
#pragma unroll
  for (int i = 0; i < NX; ++i) xus.put(lane, i, x[i]);
#pragma unroll
  for (int m = 0; m < NU; ++m) xus.put(lane, NX + m, T(0));
  xus.flush(lane, soa(a.XU, N, XU_REC, nb, c0), nqv);
}

// ---- P1 with a lane quad per instance (small batches) -------------------------------------
// The rollout's serial chain is dominated by the three sin/cos of every f evaluation.  Here the
// four lanes of a quad share one instance: lane g < 3 evaluates the sin/cos of angle g and a
// quad broadcast (DPP quad_perm, no LDS) hands all six values to the four lanes, which then
// finish f redundantly.  16 instances per one-wave workgroup (4 quads of the workspace layout).
template <int SRC> __device__ __forceinline__ float qbcast(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), SRC * 0x55, 0xF, 0xF, true));
}
template <int SRC> __device__ __forceinline__ double qbcast(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, SRC * 0x55, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), SRC * 0x55, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
struct TrigQuad {
  int g;   // lane within the quad
  template <class T>
  __device__ __forceinline__ void operator()(const T* __restrict__ x, T& sf, T& cf, T& st, T& ct,
                                             T& sp, T& cp) const {
    const T ang = sel<3>(x + 3, g);   // bit-tree select: a plain ?: chain becomes scratch
    T s, c;
    sc(ang, &s, &c);
    sf = qbcast<0>(s); cf = qbcast<0>(c);
    st = qbcast<1>(s); ct = qbcast<1>(c);
    sp = qbcast<2>(s); cp = qbcast<2>(c);
  }
};

// The angle a quad lane takes the sin/cos of, carried through the RK4 stages by the lane itself:
// its rate is f[3 + g] = wx + tt·a, b or ict·a (mpcb_model.h f_nom_lin), i.e.
// (β0·tt + β2·ict)·a + α·wx + γ·b with per-lane 0/1 coefficients, so every stage's angle costs
// three FMAs and no lane select (the select rebuilt its lane masks from spilled SGPRs at every
// f evaluation).  The products by 0 and 1 are exact: the angles equal those of the plain stage
// update x + h·k bit for bit.
template <class T> struct ScFor { using type = ScConst; };   // fp32: sc(float) has its own
template <> struct ScFor<double> { using type = ScRegs; };
template <class T>
struct TrigOwn {
  const T* ang;
  const typename ScFor<T>::type* k;
  __device__ __forceinline__ void operator()(const T* __restrict__, T& sf, T& cf, T& st, T& ct,
                                             T& sp, T& cp) const {
    T s, c;
    if constexpr (sizeof(T) == 8) sc(*ang, &s, &c, *k);
    else sc(*ang, &s, &c);
    sf = qbcast<0>(s); cf = qbcast<0>(c);
    st = qbcast<1>(s); ct = qbcast<1>(c);
    sp = qbcast<2>(s); cp = qbcast<2>(c);
  }
};
template <class T>
struct AngRate {
  T al, ga, b0, b2;
  __device__ __forceinline__ explicit AngRate(int g)
      : al(T(g == 0)), ga(T(g == 1)), b0(T(g == 0)), b2(T(g >= 2)) {}
  // rate of the lane's angle from the stage's captured scalars (c[6] = ict, c[7] = tt, c[8] = a,
  // c[17] = wx) and f[4] = b
  __device__ __forceinline__ T operator()(const T* c, T b) const {
    return fma(fma(b0, c[7], b2 * c[6]), c[8], fma(al, c[17], ga * b));
  }
};
// rk4_nom (mpcb_model.h) with the lane's angle ``ang`` (= x[3 + g] on entry) carried separately
template <class T, class Sink>
__device__ __forceinline__ void rk4_nom_own(const T* __restrict__ x, T ang, const T* __restrict__ u,
                                            T h, const Model<T>& M, const T w[3],
                                            T* __restrict__ xn, const AngRate<T>& rate,
                                            const typename ScFor<T>::type& kc, Sink&& sink) {
  constexpr int NX = 12;
  T k[NX], xs[NX], c[LIN_N];
  const T h2 = T(0.5) * h, h6 = h / T(6);
  T a_s = ang;
  const TrigOwn<T> trig{&a_s, &kc};
  f_nom_lin<T>(x, u, M, w, k, c, trig);
  sink(0, c);
  a_s = fma(h2, rate(c, k[4]), ang);
#pragma unroll
  for (int i = 0; i < NX; ++i) { xn[i] = k[i]; if (i < 3 || i > 5) xs[i] = x[i] + h2 * k[i]; }
  f_nom_lin<T>(xs, u, M, w, k, c, trig);
  sink(1, c);
  a_s = fma(h2, rate(c, k[4]), ang);
#pragma unroll
  for (int i = 0; i < NX; ++i) { xn[i] += T(2) * k[i]; if (i < 3 || i > 5) xs[i] = x[i] + h2 * k[i]; }
  f_nom_lin<T>(xs, u, M, w, k, c, trig);
  sink(2, c);
  a_s = fma(h, rate(c, k[4]), ang);
#pragma unroll
  for (int i = 0; i < NX; ++i) { xn[i] += T(2) * k[i]; if (i < 3 || i > 5) xs[i] = x[i] + h * k[i]; }
  f_nom_lin<T>(xs, u, M, w, k, c, trig);
  sink(3, c);
#pragma unroll
  for (int i = 0; i < NX; ++i) xn[i] = x[i] + h6 * (xn[i] + k[i]);
}

#ifndef MPCB_P1_OWNANG
#define MPCB_P1_OWNANG 1   // each quad lane carries its own angle (TrigOwn / AngRate)
#endif
constexpr int QI = WAVE / 4;   // instances per workgroup of the quad rollout
// ITER: iterate mode (a.mode == MPCB_MODE_ITERATE) as a template argument, so that each
// instantiation's stage loop has one shape (no loop-carried select between the rolled-out and the
// loaded state, no mode branches or their exec masks on the serial chain)
template <class T, bool ITER>
__device__ __forceinline__ void nominal_quad(const SplitArgs<T>& a) {
  constexpr int NQ = QI / SS;
  __shared__ __attribute__((aligned(16))) T lds_cc[QuadStore<T, CCS_REC, NQ>::ELEMS];
  __shared__ __attribute__((aligned(16))) T lds_xu[QuadStore<T, XU_REC, NQ>::ELEMS];
  __shared__ __attribute__((aligned(16))) T lds_gp[QuadStore<T, GP_REC, NQ>::ELEMS];
  const QuadStore<T, CCS_REC, NQ> ccs{lds_cc};
  const QuadStore<T, XU_REC, NQ> xus{lds_xu};
  const QuadStore<T, GP_REC, NQ> gps{lds_gp};
  const int lane = threadIdx.x;
  const int g = lane & 3;
  const int ci = lane >> 2;                        // instance within the workgroup
  const int64_t nb = a.nb;
  const int64_t c0 = (int64_t)blockIdx.x * QI;
  const int64_t c = (c0 + ci < nb) ? c0 + ci : nb - 1;
  const int64_t nq = (nb + SS - 1) / SS;
  const int nqv = (int)((nq - c0 / SS) < NQ ? nq - c0 / SS : NQ);
  const int64_t b = a.b0 + c;
  const int N = a.N;
  constexpr bool iterate = ITER;
#if MPCB_P1_ALLW
  // every lane of the quad stages the (identical) values: no exec-masked branches on the chain
  const bool lead = true;
#else
  const bool lead = g == 0;                        // the lane that stages the quad's values
#endif
#if MPCB_P1_OWNANG
  const AngRate<T> rate(g);
  const typename ScFor<T>::type kc;   // once, outside the stage loop
#else
  const TrigQuad trig{g};
#endif
  T w[3] = {T(0), T(0), T(0)};
  if (a.wind) {
    w[0] = a.wind[b * a.wind_sb]; w[1] = a.wind[b * a.wind_sb + 1]; w[2] = a.wind[b * a.wind_sb + 2];
  }
  const T* xbp = a.xbar + b * (int64_t)(N + 1) * NX;
  const T* ubp = a.ubar + b * (int64_t)N * NU;
  const T* ur = a.uref + b * a.uref_sb;
  T x[NX], u[NU];
  load_vec<NX>(iterate ? xbp : a.x0 + b * a.x0_sb, x);
  // a broadcast input reference (uref_sb == 0: c2, c4, c5) is staged in LDS once, so that the
  // chain's only vector-memory operations are the flush stores (no per-stage load waiting
  // behind them on vmcnt)
  __shared__ T lds_u[MPCB_P1_UMAX * NU];
  const bool ubc = MPCB_P1_ULDS && !iterate && a.uref_sb == 0 && N <= MPCB_P1_UMAX;
  if (ubc) {
    for (int e = lane; e < N * NU; e += WAVE) lds_u[e] = a.uref[e];
    wave_lds_sync();
  }
  STAMP_INIT();
  for (int k = 0; k < N; ++k) {
    STAMP(13);
    if (iterate) load_vec<NX>(xbp + (int64_t)k * NX, x);
    if (ubc) {
#pragma unroll
      for (int m = 0; m < NU; ++m) u[m] = lds_u[k * NU + m];
    } else {
      load_vec<NU>(iterate ? ubp + (int64_t)k * NU : ur + (int64_t)k * NU, u);
    }
    if (lead) {
#pragma unroll
      for (int i = 0; i < NX; ++i) xus.put(ci, i, x[i]);
#pragma unroll
      for (int m = 0; m < NU; ++m) xus.put(ci, NX + m, u[m]);
    }
    T xn[NX];
#if MPCB_P1_OWNANG
    rk4_nom_own<T>(x, sel<3>(x + 3, g), u, a.h, a.M, w, xn, rate, kc, [&](int stage, const T* cv) {
#else
    rk4_nom<T>(x, u, a.h, a.M, w, xn, [&](int stage, const T* cv) {
#endif
      if (lead) {
#pragma unroll
        for (int i = 0; i < LIN_N; ++i) ccs.put(ci, stage * LIN_N + i, cv[i]);
      }
#if MPCB_P1_OWNANG
    });
#else
    }, trig);
#endif
    STAMP(14);
    if (iterate) {
      const T* nx = xbp + (int64_t)(k + 1) * NX;
      if (lead) {
#pragma unroll
        for (int i = 0; i < NX; ++i) gps.put(ci, i, xn[i] - nx[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NX; ++i) x[i] = xn[i];
    }
    wave_lds_sync();
    xus.flush(lane, soa(a.XU, k, XU_REC, nb, c0), nqv);
    ccs.flush(lane, soa(a.CC, k, CCS_REC, nb, c0), nqv);
    if (iterate) gps.flush(lane, soa(a.GP, k, GP_REC, nb, c0), nqv);
    wave_lds_sync();
    STAMP(15);
  }
  STAMP_DONE();
  if (iterate) load_vec<NX>(xbp + (int64_t)N * NX, x);
  if (lead) {
#pragma unroll
    for (int i = 0; i < NX; ++i) xus.put(ci, i, x[i]);
#pragma unroll
    for (int m = 0; m < NU; ++m) xus.put(ci, NX + m, T(0));
  }
  wave_lds_sync();
  xus.flush(lane, soa(a.XU, N, XU_REC, nb, c0), nqv);
}

// EXPORT: code for storing column j of [A|B] (a.ABT) and the input rows of the stage
// Hessian (a.GH) for the 16-lane forward / active-set kernels; each store runs only when its
// array is set (a separate export-free fp32 instantiation keeps the plain pass's registers lean)
// ITER: iterate mode as a template argument (MPCB_P2_ITER_T, default on): the rollout-mode
// instantiation carries no gap pointer, gap prefetch or P·gap term, which frees scalar registers
// (the fp64 body spills SGPRs to VGPR lanes).  MPCB_P2_ITER_T=0: one instantiation, mode tested
// at run time as before.
#ifndef MPCB_P2_ITER_T
#define MPCB_P2_ITER_T 1
#endif
#ifndef MPCB_P2_MVGPR
#define MPCB_P2_MVGPR 1
#endif
#ifndef MPCB_P2_R32
#define MPCB_P2_R32 0
#endif
template <int L> __device__ __forceinline__ float rbc32(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + L, 0xF, 0xF, false));
}
// TIN: the row rollout already integrated the tangents (SplitArgs::tin): column j of [A|B] comes
// from its ABT2 rows (variable directions) or is the constant e_j / e_j + hv e_{j-6} (the others),
// prefetched one stage ahead like the captured scalars it replaces
// lane L's value in every lane of its 16-lane row (one v_mov_b64_dpp row_newbcast)
template <int L> __device__ __forceinline__ double rbc64(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + L, 0xF, 0xF, false);
}

WT_TABLE(g_wt_p2)
template <class T, bool EXPORT, bool ITER = false, bool TIN = false>
__device__ __forceinline__ void riccati_body(const SplitArgs<T>& a, const int64_t c_raw) {
  WT(g_wt_p2, 0);
  WT_HW(g_wt_p2);
  // fp64 DPP path: every exchange of the stage by row broadcasts -- Y reads P straight out of
  // the lanes' unsymmetrised columns (lane max(i, l) owns entry (i, l): mpcb_dpp_gen.h ypn_bc),
  // the stage-cost term S v, H_uu and h_u by broadcasts -- so P needs no LDS transpose and the
  // stage no LDS round trip (the box path's snapshots still publish P through LDS)
  constexpr bool D64 = sizeof(T) == 8 && MPCB_P2_DPP;
  // fp32 (MFMA products), export instantiation: the stage cost, h, the input block and the P update
  // by row broadcasts too (MPCB_P2_R32; P's symmetric exchange stays in LDS).  Measured: c4 P2
  // 1.04 -> 1.02-1.03 ms; in the export-free instantiation (c3, c5: two or more waves per SIMD) the
  // broadcasts cost more issue than the LDS exchanges they replace (c3 0.51 -> 0.54 ms, c5 1.86 ->
  // 1.97 ms).  Off by default: in the export instantiation alone it changes the summation order,
  // so u0 would differ in the last bit between want_traj = 0 and 1 (test_u0_only_path_equals_full_path)
  constexpr bool R32 = sizeof(T) == 4 && EXPORT && MPCB_P2_R32;
  constexpr bool DREG = D64 || R32;
  __shared__ GroupLds<T> lds_all[GROUPS];
  const int lane = threadIdx.x;
  const int q = lane >> 4;
  const int j = lane & 15;
  const int jx = j < NX ? j : 0;
  const int ju = j >= NX ? j - NX : 0;
  GroupLds<T>& L = lds_all[q];
  const int N = a.N;
  const T s = a.s;
  const Weights<T>& W = *a.W;
  const bool iterate = MPCB_P2_ITER_T ? ITER : a.mode == MPCB_MODE_ITERATE;
  const bool valid = c_raw < a.nb;
  const int64_t c = valid ? c_raw : a.nb - 1;
  const int64_t b = a.b0 + c;
  const int64_t nb = a.nb;
  const T* xr = a.xref + b * a.xref_sb;
  const T* ur = a.uref + b * a.uref_sb;
  const T hv = (a.h / T(6)) * T(6);   // the RK4 tangent's position entry of a velocity column
  // fp64 and the fp32 export instantiation: the model constants of the tangent (J, Jinv, arm
  // lengths, 1/m) as opaque loop-invariant VGPRs instead of kernel-argument SGPRs (MPCB_P2_MVGPR,
  // default on): scalar registers the body otherwise spills to VGPR lanes and reads back at every
  // stage (fp64 22 -> 0 spills, fp32 export 14 -> 0)
  Model<T> Mv = a.M;
  if constexpr ((sizeof(T) == 8 || EXPORT) && MPCB_P2_MVGPR) {
    asm volatile("" : "+v"(Mv.minv), "+v"(Mv.lx), "+v"(Mv.ly), "+v"(Mv.c));
#pragma unroll
    for (int i = 0; i < 9; ++i) asm volatile("" : "+v"(Mv.J[i]), "+v"(Mv.Jinv[i]));
  }

  // s * blkdiag(Q, R) in LDS: lane j reads column j (= row j), so the stage-cost terms are the
  // same instruction stream in state and input lanes (no divergent branch per stage)
  __shared__ __attribute__((aligned(16))) T SW[NZ * NZ];
  for (int e = lane; e < NZ * NZ; e += 64) {
    const int r = e / NZ, cl = e % NZ;
    const T wq = (r < NX && cl < NX) ? W.Q[r * NX + cl] : T(0);
    const T wr = (r >= NX && cl >= NX) ? W.R[(r - NX) * NU + (cl - NX)] : T(0);
    SW[e] = s * (wq + wr);
  }
  T pj;      // p_{k+1}[j]
  T Pc[NX];  // column j of P_{k+1} (zero in the input lanes: P padded to 16x16)
  {
    const T xN = soa(a.XU, N, XU_REC, nb, c)[jx * SS];
    L.v[j] = (j < NX) ? xN - xr[(int64_t)N * NX + jx] : T(0);
    wave_lds_sync();
    T acc = T(0);
#pragma unroll
    for (int i = 0; i < NX; ++i) acc += W.QN[jx * NX + i] * L.v[i];
    pj = acc;
    if (j < NX) {
#pragma unroll
      for (int i = 0; i < NX; ++i) L.P[j * NX + i] = W.QN[i * NX + j];
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) Pc[i] = (j < NX) ? W.QN[i * NX + jx] : T(0);
    wave_lds_sync();
  }
  bool qp_ok = true;
  T kff0 = T(0);
  // Stage data is prefetched one stage ahead into registers (5 linearisation scalars, the own
  // component of ybar and yref, one gap value per lane) and committed to a double-buffered LDS
  // copy, so the tangent integrates from LDS and no global-load latency sits on the chain.
  // (every lane loads and commits through one address select: no divergent branch)
  // group stride padded so that two groups' broadcast reads of the same scalar fall on different
  // banks (96 elements put them on one bank: a 2-way conflict on every tangent read)
  __shared__ T Cst[2][GROUPS][CCS_REC + NZ + MPCB_P2_CPAD];
  T pc[TIN ? NX : 5], pyb, pyr, pgp = T(0);
  const int tvj = var_index(j);
  const T kvar = T(tvj >= 0);   // TIN: 1 on the variable directions, 0 on the constant ones
  T ce[NX];                     // TIN: the constant column (0 on the variable directions)
#pragma unroll
  for (int i = 0; i < NX; ++i)
    ce[i] = (tvj >= 0) ? T(0) : ((i == j) ? T(1) : (j >= 6 && j < 9 && i == j - 6) ? hv : T(0));
  auto prefetch = [&](int k) {
#ifdef MPCB_P2_EXP_FIXLOAD   // timing experiment only (wrong results): every stage loads stage N - 1
    k = N - 1;
#endif
    if constexpr (TIN) {
      const T* abt = rec2(a.ABT, k, ABT2_REC, nb, c, N, a.imajor) + (tvj >= 0 ? tvj : 0);
#pragma unroll
      for (int i = 0; i < NX; ++i) pc[i] = abt[i * ABT2_W];
    } else {
      const T* cc = soa(a.CC, k, CCS_REC, nb, c);
#pragma unroll
      for (int r = 0; r < 5; ++r) pc[r] = cc[(j + 16 * r) * SS];
    }
    pyb = soa(a.XU, k, XU_REC, nb, c)[j * SS];
    pyr = *((j < NX) ? xr + (int64_t)k * NX + jx : ur + (int64_t)k * NU + ju);
    if (iterate) pgp = soa(a.GP, k, GP_REC, nb, c)[jx * SS];   // input lanes: unused copy
  };
  auto commit = [&](int bufi) {
    if constexpr (!TIN) {
#pragma unroll
      for (int r = 0; r < 5; ++r) Cst[bufi][q][j + 16 * r] = pc[r];
    }
    Cst[bufi][q][CCS_REC + j] = pgp;
  };
  // D64: s blkdiag(Q, R) column j (the G accumulators' initial values) in registers for the
  // whole recursion: 16 LDS reads and their waits less per stage
  T sw[NZ];
  if constexpr (DREG) {
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
      sw[i] = SW[i * NZ + j];
      asm volatile("" : "+v"(sw[i]));
    }
  }
  prefetch(N - 1);
  commit(0);
  T cyb = pyb, cyr = pyr;
  int buf = 0;
  wave_lds_sync();
  STAMP_INIT();
  WT(g_wt_p2, 1);
  for (int k = N - 1; k >= 0; --k) {
    T col[NX];
    T ptr = T(0);   // R32: this lane's entry of p + P gap
    if constexpr (TIN) {
#pragma unroll
      for (int i = 0; i < NX; ++i) col[i] = fma(kvar, pc[i], ce[i]);
    }
    if (k > 0) prefetch(k - 1);
    STAMP(0);
    {
      const T* cc = &Cst[buf][q][0];
      if constexpr (!DREG) L.v[j] = cyb - cyr;
      if constexpr (!TIN) {
        T dx[NX], du[NU];
#pragma unroll
        for (int i = 0; i < NX; ++i) dx[i] = (j == i) ? T(1) : T(0);
#pragma unroll
        for (int m = 0; m < NU; ++m) du[m] = (j == NX + m) ? T(1) : T(0);
        rk4_tan<T>(cc, dx, du, a.h, Mv, col);
      }
      STAMP(1);
      const int tv = tvj;   // exported: the state-dependent columns only
      // row-major ABT2 rows of the variable columns for the 16-lane forward pass / the active-set
      // kernel (a.ABT is set exactly when a row-major consumer runs; TIN: the rollout wrote them)
      if (!TIN && EXPORT && a.ABT && valid && tv >= 0) {
        T* abt = rec2(a.ABT, k, ABT2_REC, nb, c, N, a.imajor);
#pragma unroll
        for (int i = 0; i < NX; ++i) abt[i * ABT2_W + tv] = col[i];
      }
      if constexpr (!D64) {
        T pt = pj;
        if (iterate) {
#pragma unroll
          for (int i = 0; i < NX; ++i) pt += Pc[i] * cc[CCS_REC + i];
        }
        if constexpr (R32) ptr = pt;
        else L.hv[j] = pt;
      }
    }
    if constexpr (sizeof(T) == 8 && !MPCB_P2_DPP) {   // LDS-operand fp64 products
#pragma unroll
      for (int i = 0; i < NX; ++i) L.X[j * XS + i] = col[i];
    }
    wave_lds_sync();
    STAMP(2);
    T hj = T(0);
    T G[NZ];
    if constexpr (sizeof(T) == 8 && MPCB_P2_DPP) {
      // Y = P [A|B], h = [A|B]^T pt and G = [A|B]^T Y with row-broadcast FMAs: lane l supplies
      // column l of P (= row l) and pt_l, lane i supplies column i of [A|B]; no LDS operands
      double y[NX], g[NZ];
#pragma unroll
      for (int i = 0; i < NX; ++i) y[i] = 0.0;
#pragma unroll
      for (int i = 0; i < NZ; ++i) g[i] = sw[i];   // G = [A|B]^T Y + s blkdiag(Q, R)
      // h = [A|B]^T (p + P gap) = col_j . p + Y_j . gap  (P symmetric)
      ypn_all(y, hj, Pc, pj, col);
      {   // stage cost of h: (s blkdiag(Q, R) v)_j, v_i = ybar_i - yref_i broadcast from lane i
        double acc4[4] = {hj, 0.0, 0.0, 0.0};
        dot16_bc(acc4, cyb - cyr, sw);
        hj = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
      }
      if (iterate) {
        const T* cc = &Cst[buf][q][0];
#pragma unroll
        for (int i = 0; i < NX; ++i) hj = fma(y[i], cc[CCS_REC + i], hj);
      }
#if MPCB_P2_GVAR
      // rows of G at the 10 variable directions by broadcasts; the 6 constant ones from Y alone:
      // column e_p of [A|B] gives G[p][j] = Y[p][j], column e_v + hv e_p (hv = the tangent's
      // h/6 * 6) gives G[v][j] = Y[v][j] + hv Y[p][j]
      gvar_all(g, col, y);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        g[p] = y[p] + sw[p];
        g[6 + p] = fma(hv, y[p], y[6 + p]) + sw[6 + p];
      }
#else
#pragma unroll
      for (int l = 0; l < NX; ++l) fmac16_diag(g, col[l], y[l]);
#endif
#pragma unroll
      for (int i = 0; i < NZ; ++i) G[i] = g[i];
    } else if constexpr (R32) {
      // h = [A|B]^T pt with pt_l broadcast from lane l, plus the stage cost's (S v)_j
      T acc4[4] = {T(0), T(0), T(0), T(0)};
      dot12_bc(acc4, ptr, col);
      dot16_bc(acc4, cyb - cyr, sw);
      hj = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
    } else {
#pragma unroll
    for (int l = 0; l < NX; ++l) hj += col[l] * L.hv[l];
    }
    if constexpr (sizeof(T) == 4) {
      // Y = P [A|B] and G = [A|B]^T Y on the matrix cores (24 MFMAs per 4 instances)
      float y[16], g[16];
      to_columns(outer12(Pc, col), y);     // lane (q,j): Y_q[:, j]  (P symmetric: row = column)
      to_columns(outer12(col, y), g);      // lane (q,j): G_q[:, j]
#pragma unroll
      for (int i = 0; i < NZ; ++i) G[i] = R32 ? g[i] + sw[i] : g[i];
    } else if constexpr (!MPCB_P2_DPP) {
      // (measured: v_mfma_f64_16x16x4_f64 for Y and G with an LDS transpose cut this section
      // from 5.6k to 3.8k cycles per stage but cost more elsewhere, 14.6k vs 13.7k in total)
      T y[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) y[i] = T(0);
#pragma unroll
      for (int l = 0; l < NX; ++l) {
        const T cl = col[l];
#pragma unroll
        for (int i = 0; i < NX; ++i) y[i] += L.P[l * NX + i] * cl;
      }
#pragma unroll
      for (int i = 0; i < NZ; ++i) {
        T acc = T(0);
#pragma unroll
        for (int l = 0; l < NX; ++l) acc += L.X[i * XS + l] * y[l];
        G[i] = acc;
      }
    }
    STAMP(3);
    T Huu[NU * NU], hu[NU];
    if constexpr (DREG) {
      // (the stage cost is in G's and h's accumulators already) H_uu and h_u from the input lanes
      STAMP(4);
      static_for<NU>([&](auto n) {
        constexpr int nn = decltype(n)::value;
#pragma unroll
        for (int m = 0; m < NU; ++m) {
          if constexpr (D64) Huu[m * NU + nn] = rbc64<NX + nn>(G[NX + m]);
          else Huu[m * NU + nn] = rbc32<NX + nn>(G[NX + m]);
        }
        if constexpr (D64) hu[nn] = -rbc64<NX + nn>(hj);
        else hu[nn] = -rbc32<NX + nn>(hj);
      });
    } else {
#pragma unroll
      for (int i = 0; i < NZ; ++i) {
        // SW is symmetric: lane j reads column j so the 16 lanes hit 16 consecutive entries (row j
        // put every second lane on the same bank: an 8-way conflict on each of these reads)
        const T w = MPCB_P2_SWT ? SW[i * NZ + j] : SW[j * NZ + i];
        G[i] += w;
        hj += w * L.v[i];
      }
      // (box path: no Hessian rows here -- the active set is empty in this pass, and the first
      // masked backward recomputes every stage and writes the rows its fixed components need)
#pragma unroll
      for (int m = 0; m < NU; ++m) L.Hu[j * HS + m] = G[NX + m];
      wave_lds_sync();
      L.hv[j] = hj;
      wave_lds_sync();
      STAMP(4);
#pragma unroll
      for (int m = 0; m < NU; ++m) {
#pragma unroll
        for (int n = 0; n < NU; ++n) Huu[m * NU + n] = L.Hu[(NX + n) * HS + m];
        hu[m] = -L.hv[NX + m];
      }
    }
    T Lc[10];
    chol4(Huu, Lc);
    // every entry of the factor feeds the last pivot (through l30, l31, l32), and inv_sqrt keeps a
    // NaN: the factor holds a NaN iff its last entry does
    qp_ok = qp_ok && (Lc[9] == Lc[9]);
    T kff[NU], Kj[NU], nh[NU];
    chol4_solve(Lc, hu, kff);
#pragma unroll
    for (int m = 0; m < NU; ++m) nh[m] = -G[NX + m];
    chol4_solve(Lc, nh, Kj);
    STAMP(5);
    T pn = hj;
#pragma unroll
    for (int m = 0; m < NU; ++m) pn += G[NX + m] * kff[m];
    T Pn[NX];
    if constexpr (DREG) {
      // Pn[i] = G[i] + sum_m H_ux[m][i] K[m][j]: lane i owns H_ux[:, i] = its G[NX..]
#pragma unroll
      for (int i = 0; i < NX; ++i) Pn[i] = G[i];
      const T gu[NU] = {G[NX], G[NX + 1], G[NX + 2], G[NX + 3]};
      pn_all(Pn, gu, Kj);
    } else {
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        T acc = G[i];
#pragma unroll
        for (int m = 0; m < NU; ++m) acc += L.Hu[i * HS + m] * Kj[m];
        Pn[i] = acc;
      }
    }
    STAMP(6);
    kff0 = sel<NU>(kff, ju);
    if (D64 && (TIN || a.rm)) {
      // KR2 (TIN: always this layout), four stores from every lane and no lane branch, so the
      // next stage's wait for its prefetched loads counts exactly these stores (a path without
      // them made the compiler wait for every store to complete, vmcnt(0)): state lane j writes
      // K[m][j]; input lane ju k_ju to slot 12 of row ju and its other three stores to the
      // rows' pad slot 13.  Padding groups write the same values as the instance they repeat.
      T* kr = rec2(a.KR, k, KR2_REC, nb, c, N, a.imajor);
#pragma unroll
      for (int m = 0; m < NU; ++m)
        kr[m * KR2_W + (j < NX ? j : (m == ju ? 12 : 13))] = (j < NX) ? Kj[m] : kff0;
    } else if (valid && a.rm) {   // KR2: K[m][j] at KR2_W m + j, k_m at KR2_W m + 12
      T* kr = rec2(a.KR, k, KR2_REC, nb, c, N, a.imajor);
      if (j < NX) {
#pragma unroll
        for (int m = 0; m < NU; ++m) kr[m * KR2_W + j] = Kj[m];
      } else {
        kr[ju * KR2_W + 12] = kff0;
      }
    } else if (valid) {
      // K[m][j] at 4j + m (state lanes), kff[m] at 4*NX + m (input lanes): the first store is
      // common to both kinds of lane
      T* kr = soa(a.KR, k, KR_REC, nb, c);
      kr[((j < NX) ? 4 * j : 4 * NX + ju) * SS] = (j < NX) ? Kj[0] : kff0;
      if (j < NX) {
#pragma unroll
        for (int m = 1; m < NU; ++m) kr[(4 * j + m) * SS] = Kj[m];
      }
    }
    wave_lds_sync();
    STAMP(7);
    // symmetric by construction: entry (r, c) from lane max(r, c) (see mpcb_solve.hip).  Every
    // lane publishes its column and takes the entries below its diagonal from the lanes that
    // own them: uniform code instead of per-entry predicated stores.  (L.X is free: this
    // stage's products are done.)
    const bool publish = !D64 || (EXPORT && a.PS);   // D64: only the box path's snapshots
    if (publish) {
#pragma unroll
      for (int i = 0; i < NX; ++i) L.X[j * XS + i] = Pn[i];
    }
    pj = pn;
    if (k > 0) commit(buf ^ 1);
    wave_lds_sync();
    if (EXPORT && a.PS && valid && j < NX && k > 0) {
      // box path: the value function P_k, p_k packed by symmetry (mpcb_kernels.h PS2), so the
      // active-set kernel's first masked pass restarts above the highest violated stage instead
      // of recomputing the whole horizon; slot d of lane j is P[j][(j + d) % 12], published by
      // lane max(j, o) above
      T ps[PS2_W];
#pragma unroll
      for (int d = 0; d < 7; ++d) {
        const int o = j + d < NX ? j + d : j + d - NX;
        ps[d] = L.X[(o > j ? o : j) * XS + (o > j ? j : o)];
      }
      ps[7] = pn;
      stv<T, PS2_W>(rec2(a.PS, k, PS2_REC, nb, c, N, a.imajor) + j * PS2_W, ps);
    }
    STAMP(8);
    if constexpr (D64) {
#pragma unroll
      for (int i = 0; i < NX; ++i) Pc[i] = Pn[i];   // unsymmetrised: ypn_bc reads the owners
    } else {
#if MPCB_P2_PCSEL
    {   // unconditional LDS reads + lane-mask selects (no exec-masked branch per entry)
      const uint64_t st_lane = lane_mask(j < NX);
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        const T o = L.X[i * XS + jx];
        Pc[i] = csel(st_lane, csel(lane_mask(i <= j), Pn[i], o), T(0));
      }
    }
#else
#pragma unroll
    for (int i = 0; i < NX; ++i) Pc[i] = (j < NX) ? ((i <= j) ? Pn[i] : L.X[i * XS + j]) : T(0);
#endif
    }
    if constexpr (sizeof(T) == 8 && !MPCB_P2_DPP) {   // the LDS fp64 products read P from LDS
      if (j < NX) {
#pragma unroll
        for (int i = 0; i < NX; ++i) L.P[j * NX + i] = Pc[i];
      }
    }
    buf ^= 1;
    cyb = pyb;
    cyr = pyr;
    STAMP(9);
  }
  STAMP_DONE();
  WT(g_wt_p2, 2);
  if (valid && j == NX) a.status[b] = qp_ok ? MPCB_STATUS_OK : MPCB_STATUS_QP_FAIL;
  if (valid && !a.fwd && j >= NX) {
    // rollout mode without trajectories: dx_0 = 0 so u0 = ubar_0 + kff_0
    const T u = cyb + kff0;   // cyb = own component of (xbar_0 | ubar_0)
    a.u0[b * NU + ju] = u;
    const bool fin = isfin(u);
    if (!fin) a.status[b] = MPCB_STATUS_NAN;
  }
  WT(g_wt_p2, 3);
}

// P3 LDS carve (dynamic): two stage images (XU | KR | CC) for the one-stage-ahead DMA, plus the
// output-row staging of S stages x (X row | U row) per instance.  S is the largest that keeps
// the residency each use needs: fp32 large chunks 4 waves/CU (<= 40 KiB), fp64 + CC <= 160 KiB.
template <class T, bool USE_CC>
struct FwdLds {
  static constexpr int IN = (XU_REC + KR_REC + (USE_CC ? CCS_REC : 0)) * WAVE;
  static constexpr int S = (sizeof(T) == 8) == USE_CC ? 1 : 4;
  static constexpr int V = 16 / sizeof(T);
  static constexpr int ROW = NX + NU;
  static constexpr int RSTRIDE = S * ROW + V;
  static constexpr size_t BYTES = (size_t)(2 * IN + WAVE * RSTRIDE) * sizeof(T);
};

// USE_CC: integrate the forward tangent from the captured linearisation scalars (small chunks:
// CC is cache resident) instead of re-evaluating f with sin/cos (large chunks: saves streaming
// 80 scalars per stage back from HBM).
template <class T, bool USE_CC, bool ITER>
__device__ __forceinline__ void forward_wave(const SplitArgs<T>& a) {
  using L = FwdLds<T, USE_CC>;
  constexpr int S = L::S, V = L::V, ROW = L::ROW;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  T* const img0 = reinterpret_cast<T*>(dyn_lds);
  T* const img1 = img0 + L::IN;
  T* const rows = img1 + L::IN;
  const int lane = threadIdx.x;
  const int64_t nb = a.nb;
  const int64_t c0 = (int64_t)blockIdx.x * WAVE;
  const bool valid = c0 + lane < nb;
  const int64_t c = valid ? c0 + lane : nb - 1;
  const int64_t nq = (nb + SS - 1) / SS;
  const int nqv = (int)((nq - c0 / SS) < WQ ? nq - c0 / SS : WQ);
  const int nvalid = (int)((nb - c0) < WAVE ? nb - c0 : WAVE);
  const int64_t b = a.b0 + c;
  const int N = a.N;
  constexpr bool iterate = ITER;   // (see nominal_quad)
  T w[3] = {T(0), T(0), T(0)};
  if (a.wind) {
    w[0] = a.wind[b * a.wind_sb]; w[1] = a.wind[b * a.wind_sb + 1]; w[2] = a.wind[b * a.wind_sb + 2];
  }
  // LDS byte addresses of the two stage images (M0 operands of the DMA)
  const unsigned lds0 = (unsigned)(size_t)(lds_void*)dyn_lds;
  const unsigned lds1 = lds0 + L::IN * (unsigned)sizeof(T);
  const bool dma_lane = Dma<T>::lane_valid(lane, nqv);
  const int off_xu = Dma<T>::lane_offset(lane, XU_REC), off_kr = Dma<T>::lane_offset(lane, KR_REC),
            off_cc = Dma<T>::lane_offset(lane, CCS_REC);
  auto dma = [&](int k, unsigned im) {
    if (dma_lane) {
      dma_record<T, XU_REC>(im, soa(a.XU, k, XU_REC, nb, c0) + off_xu);
      if (k < N) {
        dma_record<T, KR_REC>(im + XU_REC * WAVE * sizeof(T), soa(a.KR, k, KR_REC, nb, c0) + off_kr);
        if constexpr (USE_CC)
          dma_record<T, CCS_REC>(im + (XU_REC + KR_REC) * WAVE * sizeof(T),
                                 soa(a.CC, k, CCS_REC, nb, c0) + off_cc);
      }
    }
  };
  // rows [k0, k0 + NS) of X (and of U where < N) of the wave's valid instances
  auto flush_rows = [&](int k0, auto ns_tag) {
    constexpr int NS = decltype(ns_tag)::value, CX = NX / V, CU = NU / V;
    const int64_t inst0 = a.b0 + c0;
    // chunk t of X: instance t / (NS*CX), row (t % (NS*CX)) / CX, part t % CX
    auto xsrc = [&](int t) {
      const int l = t / (NS * CX), r = t - l * (NS * CX), sr = r / CX;
      return rows + l * L::RSTRIDE + sr * ROW + (r - sr * CX) * V;
    };
    auto xdst = [&](int t) {
      const int l = t / (NS * CX), r = t - l * (NS * CX);
      return a.X + ((inst0 + l) * (N + 1) + k0) * NX + r * V;
    };
    auto usrc = [&](int t) {
      const int l = t / (NS * CU), r = t - l * (NS * CU), sr = r / CU;
      return rows + l * L::RSTRIDE + sr * ROW + NX + (r - sr * CU) * V;
    };
    auto udst = [&](int t) {
      const int l = t / (NS * CU), r = t - l * (NS * CU);
      return a.U + ((inst0 + l) * N + k0) * NU + r * V;
    };
    const bool do_u = a.U && k0 + NS <= N;
    if (nvalid == WAVE) {
      if (a.X) copy_chunks<WAVE * NS * CX>(lane, xsrc, xdst);
      if (do_u) copy_chunks<WAVE * NS * CU>(lane, usrc, udst);
    } else {
      if (a.X)
        for (int t = lane; t < nvalid * NS * CX; t += WAVE) copy16(xdst(t), xsrc(t));
      if (do_u)
        for (int t = lane; t < nvalid * NS * CU; t += WAVE) copy16(udst(t), usrc(t));
    }
  };
  dma(0, lds0);
  wait_vm();
  T dx[NX];
  {
    const T* x0 = a.x0 + b * a.x0_sb;
#pragma unroll
    for (int i = 0; i < NX; ++i) dx[i] = iterate ? x0[i] - img0[i * WAVE + lane] : T(0);
  }
  bool fin = true;
  for (int k = 0; k < N; ++k) {
    T* const cur = (k & 1) ? img1 : img0;
    T* const nxt = (k & 1) ? img0 : img1;
    dma(k + 1, (k & 1) ? lds0 : lds1);
    T gp[NX];
    if (USE_CC && iterate) {
      const T* g = soa(a.GP, k, GP_REC, nb, c);
#pragma unroll
      for (int i = 0; i < NX; ++i) gp[i] = g[i * SS];
    }
    T xb[NX], ub[NU], du[NU];
#pragma unroll
    for (int i = 0; i < NX; ++i) xb[i] = cur[i * WAVE + lane];
#pragma unroll
    for (int m = 0; m < NU; ++m) ub[m] = cur[(NX + m) * WAVE + lane];
    const T* kr = cur + XU_REC * WAVE + lane;
#pragma unroll
    for (int m = 0; m < NU; ++m) du[m] = kr[(4 * NX + m) * WAVE];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
#pragma unroll
      for (int m = 0; m < NU; ++m) du[m] += kr[(4 * i + m) * WAVE] * dx[i];
    }
    T* const row = rows + lane * L::RSTRIDE + (k % S) * ROW;
#pragma unroll
    for (int i = 0; i < NX; ++i) row[i] = xb[i] + dx[i];
    {
      T uo[NU];
#pragma unroll
      for (int m = 0; m < NU; ++m) {
        uo[m] = ub[m] + du[m];
        row[NX + m] = uo[m];
        fin = fin && isfin(uo[m]);
      }
      if (k == 0 && valid) store_vec<NU>(a.u0 + b * NU, uo);
    }
    if (k % S == S - 1) flush_rows(k - (S - 1), std::integral_constant<int, S>());
    T phi[NX], dphi[NX];
    if constexpr (USE_CC) {
      const T* cc = cur + (XU_REC + KR_REC) * WAVE + lane;
      rk4_tan_g<T, false>([&](int i) { return cc[i * WAVE]; }, dx, du, a.h, a.M, dphi);
    } else {
      rk4<T, true>(xb, dx, ub, du, a.h, a.M, w, phi, dphi);
    }
    wait_vm();          // stage k+1 image landed (and this stage's row stores drained)
    if (iterate) {
#pragma unroll
      for (int i = 0; i < NX; ++i)
        dx[i] = USE_CC ? dphi[i] + gp[i] : dphi[i] + (phi[i] - nxt[i * WAVE + lane]);
    } else {
#pragma unroll
      for (int i = 0; i < NX; ++i) dx[i] = dphi[i];
    }
  }
  {
    const T* last = (N & 1) ? img1 : img0;
    T* const row = rows + lane * L::RSTRIDE + (N % S) * ROW;
#pragma unroll
    for (int i = 0; i < NX; ++i) row[i] = last[i * WAVE + lane] + dx[i];
    // rows N - N % S .. N: the terminal row and the unflushed tail, one row at a time
    for (int k0 = N - N % S; k0 <= N; ++k0) {
      if constexpr (S > 1) {
        T* const src = rows + lane * L::RSTRIDE + (k0 % S) * ROW;
        T* const dst = rows + lane * L::RSTRIDE;
        if (k0 % S) {
#pragma unroll
          for (int i = 0; i < ROW; ++i) dst[i] = src[i];
        }
      }
      flush_rows(k0, std::integral_constant<int, 1>());
    }
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) fin = fin && isfin(dx[i]);
  if (valid && !fin) a.status[b] = MPCB_STATUS_NAN;
}

template <class T> int64_t split_elems_per_instance(int N, int iterate, int box) {
  // (KR sized for the larger of its two layouts; box == 1: the old [A|B] pair of the small path or
  // ABT2 of the 16-lane forward)
  return (int64_t)(N + 1) * XU_REC + (int64_t)N * (CCS_REC + KR2_REC + (iterate ? GP_REC : 0)) +
         (box == 2 ? (int64_t)N * (AB2_REC + ABT2_REC + GH2_REC + PS2_REC)
                   : box == 1 ? (int64_t)N * (AB_REC + ABT2_REC) : 0);
}

template <class T, bool ITER>
__global__ void __launch_bounds__(64) nominal_kernel(SplitArgs<T> a) { nominal_wave<T, ITER>(a); }
template <class T, bool ITER>
__global__ void __launch_bounds__(64) nominal_quad_kernel(SplitArgs<T> a) { nominal_quad<T, ITER>(a); }
template <class T, bool USE_CC, bool ITER>
__global__ void __launch_bounds__(64) forward_kernel(SplitArgs<T> a) { forward_wave<T, USE_CC, ITER>(a); }
// register budget: fp32 at 2 waves/SIMD (measured faster than 3 with its small spill); fp64 uncapped
template <bool EXPORT, bool ITER = false, bool TIN = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(EXPORT ? MPCB_P2_WAVES_F32 : MPCB_P2_WAVES_F32_NOEXP, 8)))
riccati_kernel_f32(SplitArgs<float> a) {
  riccati_body<float, EXPORT, ITER, TIN>(a, (int64_t)blockIdx.x * GROUPS + (threadIdx.x >> 4));
}
template <bool EXPORT, bool ITER = false, bool TIN = false>
__global__ void __launch_bounds__(64) MPCB_P2_WAVES riccati_kernel_f64(SplitArgs<double> a) {
  riccati_body<double, EXPORT, ITER, TIN>(a, (int64_t)blockIdx.x * GROUPS + (threadIdx.x >> 4));
}

// c2 (fp64 small chunks with the tangent export): P1 and P2 of a quad in ONE kernel.  Nothing
// crosses quads between them, so the wave that rolled its four instances out runs their Riccati
// recursion straight after, without the kernel boundary (its drain and cache write-back) and the
// second kernel's launch and prologue; its own ABT2 / XU stores are ordered before its loads by
// the workgroup fence (MPCB_FUSE_P12=0 at build or run time: two kernels).
#ifndef MPCB_FUSE_P12
#define MPCB_FUSE_P12 1
#endif
template <bool ITER, bool DJ>
__global__ void __launch_bounds__(64) MPCB_P2_WAVES row_riccati_kernel(SplitArgs<double> a) {
  row_body<double, ITER, DJ, true>(a);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  riccati_body<double, true, ITER, true>(a, (int64_t)blockIdx.x * GROUPS + (threadIdx.x >> 4));
}

template <class T, bool USE_CC, bool ITER>
static hipError_t launch_forward_m(const SplitArgs<T>& a, unsigned grid, hipStream_t st) {
  constexpr size_t bytes = FwdLds<T, USE_CC>::BYTES;
  static_assert(bytes <= 160 * 1024, "P3 LDS carve exceeds the CU's 160 KiB");
  if (!dry_run()) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&forward_kernel<T, USE_CC, ITER>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (attr != hipSuccess) return attr;
  }
  MPCB_LAUNCH(PH_FORWARD, (forward_kernel<T, USE_CC, ITER>), dim3(grid), dim3(WAVE), bytes, st, a);
  return hipSuccess;
}
template <class T, bool USE_CC>
static hipError_t launch_forward(const SplitArgs<T>& a, unsigned grid, hipStream_t st) {
  return a.mode == MPCB_MODE_ITERATE ? launch_forward_m<T, USE_CC, true>(a, grid, st)
                                     : launch_forward_m<T, USE_CC, false>(a, grid, st);
}

template <class T> hipError_t launch_split(const SplitArgs<T>& a, hipStream_t st, hipEvent_t* ev) {
  const unsigned gw = (unsigned)((a.nb + WAVE - 1) / WAVE);
  const unsigned g64 = (unsigned)((a.nb + GROUPS - 1) / GROUPS);
  if (ev) (void)hipEventRecord(ev[0], st);
  const bool fuse = sizeof(T) == 8 && MPCB_FUSE_P12 && a.quad_p1 == 2 && a.tin == 1 && !a.small;
  if (fuse) {
    // (the phase events: "nominal" empty, "riccati" the fused kernel)
    if (ev) (void)hipEventRecord(ev[1], st);
    const dim3 grid((unsigned)((a.nb + SS - 1) / SS));
    const size_t lds = row_lds_bytes(a);
    const bool it = a.mode == MPCB_MODE_ITERATE;   // (the row body's mode is always a template argument)
    if constexpr (sizeof(T) == 8) {
      if (!dry_run()) {
        static const hipError_t lds_ok = [] {
          hipFuncAttributes at;
          hipError_t e = hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&row_riccati_kernel<false, true>));
          if (e == hipSuccess && at.sharedSizeBytes > RICCATI_F64_STATIC_LDS) e = hipErrorInvalidConfiguration;
          return e;
        }();
        if (lds_ok != hipSuccess) return lds_ok;
      }
      if (row_dj(a)) {
        if (it) MPCB_LAUNCH(PH_RICCATI, (row_riccati_kernel<true, true>), grid, dim3(64), lds, st, a);
        else MPCB_LAUNCH(PH_RICCATI, (row_riccati_kernel<false, true>), grid, dim3(64), lds, st, a);
      } else {
        if (it) MPCB_LAUNCH(PH_RICCATI, (row_riccati_kernel<true, false>), grid, dim3(64), lds, st, a);
        else MPCB_LAUNCH(PH_RICCATI, (row_riccati_kernel<false, false>), grid, dim3(64), lds, st, a);
      }
    }
  } else if (a.quad_p1 == 2) {
    const hipError_t e = launch_nominal_row<T>(a, st);
    if (e != hipSuccess) return e;
  } else if (a.quad_p1) {
    const dim3 gq((unsigned)((a.nb + QI - 1) / QI));
    if (a.mode == MPCB_MODE_ITERATE) MPCB_LAUNCH(PH_NOMINAL, (nominal_quad_kernel<T, true>), gq, dim3(WAVE), 0, st, a);
    else MPCB_LAUNCH(PH_NOMINAL, (nominal_quad_kernel<T, false>), gq, dim3(WAVE), 0, st, a);
  }
  else if (a.mode == MPCB_MODE_ITERATE)
    MPCB_LAUNCH(PH_NOMINAL, (nominal_kernel<T, true>), dim3(gw), dim3(WAVE), 0, st, a);
  else
    MPCB_LAUNCH(PH_NOMINAL, (nominal_kernel<T, false>), dim3(gw), dim3(WAVE), 0, st, a);
  if (ev && !fuse) (void)hipEventRecord(ev[1], st);
  if (a.small) {   // linearisation + Riccati + forward over the cached [A|B] (mpcb_box.hip)
    hipError_t e = launch_small<T>(a, st);
    if (ev) (void)hipEventRecord(ev[2], st);
    if (ev) (void)hipEventRecord(ev[3], st);
    return e != hipSuccess ? e : (dry_run() ? hipSuccess : hipGetLastError());
  }
  const bool it = MPCB_P2_ITER_T && a.mode == MPCB_MODE_ITERATE;
  if constexpr (sizeof(T) == 4) {
    if (it) {
      if (a.ABT) MPCB_LAUNCH(PH_RICCATI, (riccati_kernel_f32<true, true>), dim3(g64), dim3(64), 0, st, a);
      else MPCB_LAUNCH(PH_RICCATI, (riccati_kernel_f32<false, true>), dim3(g64), dim3(64), 0, st, a);
    } else {
      if (a.ABT) MPCB_LAUNCH(PH_RICCATI, (riccati_kernel_f32<true>), dim3(g64), dim3(64), 0, st, a);
      else MPCB_LAUNCH(PH_RICCATI, (riccati_kernel_f32<false>), dim3(g64), dim3(64), 0, st, a);
    }
  } else {
    // one fp64 instantiation per mode (export guarded at run time): measured leaner than the
    // export-free one, which LLVM schedules into 368 bytes of scratch spill
    if (fuse) {
      // (P2 ran in row_riccati_kernel)
    } else if (a.tin) {
      if (it) MPCB_LAUNCH(PH_RICCATI, (riccati_kernel_f64<true, true, true>), dim3(g64), dim3(64), 0, st, a);
      else MPCB_LAUNCH(PH_RICCATI, (riccati_kernel_f64<true, false, true>), dim3(g64), dim3(64), 0, st, a);
    } else if (it) {
      MPCB_LAUNCH(PH_RICCATI, (riccati_kernel_f64<true, true>), dim3(g64), dim3(64), 0, st, a);
    } else {
      MPCB_LAUNCH(PH_RICCATI, (riccati_kernel_f64<true>), dim3(g64), dim3(64), 0, st, a);
    }
  }
  if (ev) (void)hipEventRecord(ev[2], st);
  hipError_t e = hipSuccess;
  if (a.GH)   // input boxes: active-set iterations over the exported linearisation (mpcb_as.hip)
    e = launch_as<T>(a, st);
  else if (a.fwd && a.fwd16)   // forward pass from the exported [A|B]^T, 16 lanes per instance
    e = launch_fwd_rm<T>(a, st);
  else if (a.fwd)   // (chunks above 16384: re-evaluates f rather than streaming 80 captured
                    // scalars per stage back from HBM; the variant depends on the handle, not on
                    // this call's batch, so an instance's outputs do not depend on its batch)
    e = launch_forward<T, false>(a, gw, st);
  if (ev) (void)hipEventRecord(ev[3], st);
  return e != hipSuccess ? e : (dry_run() ? hipSuccess : hipGetLastError());
}

template hipError_t launch_split<double>(const SplitArgs<double>&, hipStream_t, hipEvent_t*);
template hipError_t launch_split<float>(const SplitArgs<float>&, hipStream_t, hipEvent_t*);
template int64_t split_elems_per_instance<double>(int, int, int);
template int64_t split_elems_per_instance<float>(int, int, int);

}  // namespace mpcb

#ifdef MPCB_STAMPS
// (same translation unit as g_stamps: the library is built without -fgpu-rdc)
#ifdef MPCB_STAMPS
extern "C" int mpcb_debug_wt_p1f(unsigned long long* out) {   // the row body inside row_riccati_kernel
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::g_wt_p1), sizeof(unsigned long long) * MPCB_WT_MAX * 7) == hipSuccess ? 0 : -2;
}
extern "C" int mpcb_debug_wt_p2(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::g_wt_p2), sizeof(unsigned long long) * MPCB_WT_MAX * 7) == hipSuccess ? 0 : -2;
}
#endif
extern "C" int mpcb_debug_wt_max(void) { return MPCB_WT_MAX; }
extern "C" int mpcb_debug_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::g_stamps), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : -2;
}
#endif
