// mpcb_as.h -- the body of the active-set kernel and of the unconstrained 16-lane forward pass
// (as_body), shared by mpcb_as.hip (their kernels) and mpcb_split.hip (c2's fused kernel).  The
// design notes are at the top of mpcb_as.hip.  Stamp tables live in the owning translation unit
// (MPCB_AS_OWNER, mpcb_as.hip) only: without -fgpu-rdc a device variable cannot be shared.
#pragma once

#if defined(MPCB_STAMPS) && defined(MPCB_AS_OWNER)
#define MPCB_AS_STAMPS 1
#define AS_WT(slot) WT(g_wt_p3, slot)
#else
#define AS_WT(slot)
#endif

#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/mpcb.h"
#include "mpcb_kernels.h"
#include "mpcb_common.h"
#include "mpcb_split.h"

#ifndef MPCB_AS_WAVES
#define MPCB_AS_WAVES 2
#endif
#ifndef MPCB_AS_FDEPTH   // forward-pass prefetch ring (stages): active-set kernel
#define MPCB_AS_FDEPTH 2
#endif
#ifndef MPCB_AS_ITER_T   // the mode as a template argument (as in P1 / P2 / P3)
#define MPCB_AS_ITER_T 1
#endif
#ifndef MPCB_FWD_FDEPTH  // the same for the unconstrained forward pass (fwd_rm_kernel)
#define MPCB_FWD_FDEPTH 2
#endif

namespace mpcb {
namespace asq {

#if defined(MPCB_REF_TRACE) && defined(MPCB_AS_OWNER)
__device__ int g_ref_trace[128][20];
#endif
#if defined(MPCB_REF_STAMPS) && defined(MPCB_AS_OWNER)
// Diagnostic build only: s_memtime cycles of the refinement's sweeps in workgroup 0 of the
// refinement kernel, summed over its calls ([0] re-simulation, [1] adjoint for the correction,
// [2] correction backward, [3] correction forward, [4] deciding adjoint, [5] calls), read by
// mpcb_debug_ref_stamps() (tools/ref_stamps.py)
__device__ unsigned long long g_refst[8];
#define RSTAMP(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); rst[i] += t_ - rst_prev; rst_prev = t_; }
#else
#define RSTAMP(i)
#endif
#ifdef MPCB_AS_STAMPS
// Diagnostic build only: per-region s_memtime cycles of workgroup 0, wave-summed over the whole
// kernel ([0] backward init, [1..3] backward stage parts, [4..6] forward stage parts, [7] forward
// tail + active-set update, [8] iterations, [9] backward stages), read by mpcb_debug_stamps_as()
__device__ unsigned long long g_astamps[12];
#define ASTAMP(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ast_acc[i] += t_ - ast_prev; ast_prev = t_; }
#else
#define ASTAMP(i)
#endif

// ---- DPP row broadcasts (16-lane rows = one instance) ---------------------------------------
// Inline asm: the compiler's hazard recognizer does not look inside, so every block starts with
// s_nop 4 (VALU / EXEC write -> DPP read wait states); no source is written inside a block.
// Every block runs with all 16 lanes of each row active (group-uniform control flow only).
#define ASQ_I(op, d, s, b, l) op " %" #d ", %" #s ", %" #b " row_newbcast:" #l " row_mask:0xf bank_mask:0xf\n\t"
#define ASQ_A(op, d, s, b, l) op " %" #d ", |%" #s "|, |%" #b "| row_newbcast:" #l " row_mask:0xf bank_mask:0xf\n\t"
// acc[l & 3] += bcast_l(%4) * %(5 + l)
#define ASQ_DOT12(M, op)                                                                           \
  M(op, 0, 4, 5, 0) M(op, 1, 4, 6, 1) M(op, 2, 4, 7, 2) M(op, 3, 4, 8, 3) M(op, 0, 4, 9, 4)       \
  M(op, 1, 4, 10, 5) M(op, 2, 4, 11, 6) M(op, 3, 4, 12, 7) M(op, 0, 4, 13, 8) M(op, 1, 4, 14, 9)   \
  M(op, 2, 4, 15, 10) M(op, 3, 4, 16, 11)
#define ASQ_DOT16(M, op) ASQ_DOT12(M, op) M(op, 0, 4, 17, 12) M(op, 1, 4, 18, 13) M(op, 2, 4, 19, 14) M(op, 3, 4, 20, 15)
#define ASQ_OUT4(acc) "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
#define ASQ_IN12(z, r) "v"(z), "v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]), "v"(r[6]), \
                       "v"(r[7]), "v"(r[8]), "v"(r[9]), "v"(r[10]), "v"(r[11])
#define ASQ_IN16(z, r) ASQ_IN12(z, r), "v"(r[12]), "v"(r[13]), "v"(r[14]), "v"(r[15])

// fp32: acc[0] += sum_{l = 0 mod 4} ..., acc[1..3] = (their sums from zero): the first product of
// accumulators 1..3 is a v_mul_f32_dpp instead of a v_fmac into a zeroed register (the zeroing
// moves were ~5 % of a forward stage's instructions).  fp64 has no DPP form of v_mul_f64 (VOP3).
#define ASQ_FIRST(M, mop) M(mop, 1, 4, 6, 1) M(mop, 2, 4, 7, 2) M(mop, 3, 4, 8, 3)
#define ASQ_DOT12Z(M, op, mop)                                                                      \
  M(op, 0, 4, 5, 0) ASQ_FIRST(M, mop) M(op, 0, 4, 9, 4) M(op, 1, 4, 10, 5) M(op, 2, 4, 11, 6)     \
  M(op, 3, 4, 12, 7) M(op, 0, 4, 13, 8) M(op, 1, 4, 14, 9) M(op, 2, 4, 15, 10) M(op, 3, 4, 16, 11)
#define ASQ_DOT16Z(M, op, mop) ASQ_DOT12Z(M, op, mop) M(op, 0, 4, 17, 12) M(op, 1, 4, 18, 13) M(op, 2, 4, 19, 14) M(op, 3, 4, 20, 15)
#define ASQ_OUT4Z(acc) "+v"(acc[0]), "=&v"(acc[1]), "=&v"(acc[2]), "=&v"(acc[3])

// acc[*] += sum_{l<12} bcast_l(z) * r[l]   (fp32: acc[1..3] need not be initialised)
__device__ __forceinline__ void dot12(float (&acc)[4], float z, const float (&r)[12]) {
  asm("s_nop 4\n\t" ASQ_DOT12Z(ASQ_I, "v_fmac_f32_dpp", "v_mul_f32_dpp") : ASQ_OUT4Z(acc) : ASQ_IN12(z, r));
}
__device__ __forceinline__ void dot12(double (&acc)[4], double z, const double (&r)[12]) {
  asm("s_nop 4\n\t" ASQ_DOT12(ASQ_I, "v_fmac_f64_dpp") : ASQ_OUT4(acc) : ASQ_IN12(z, r));
}
// acc[*] += sum_{l<16} bcast_l(z) * r[l]   (fp32: acc[1..3] need not be initialised)
__device__ __forceinline__ void dot16(float (&acc)[4], float z, const float (&r)[16]) {
  asm("s_nop 4\n\t" ASQ_DOT16Z(ASQ_I, "v_fmac_f32_dpp", "v_mul_f32_dpp") : ASQ_OUT4Z(acc) : ASQ_IN16(z, r));
}
__device__ __forceinline__ void dot16(double (&acc)[4], double z, const double (&r)[16]) {
  asm("s_nop 4\n\t" ASQ_DOT16(ASQ_I, "v_fmac_f64_dpp") : ASQ_OUT4(acc) : ASQ_IN16(z, r));
}
// acc[*] += sum_{l<16} |bcast_l(z) * r[l]|   (fp32: acc[1..3] need not be initialised)
__device__ __forceinline__ void dot16abs(float (&acc)[4], float z, const float (&r)[16]) {
  asm("s_nop 4\n\t" ASQ_DOT16Z(ASQ_A, "v_fmac_f32_dpp", "v_mul_f32_dpp") : ASQ_OUT4Z(acc) : ASQ_IN16(z, r));
}
__device__ __forceinline__ void dot16abs(double (&acc)[4], double z, const double (&r)[16]) {
  asm("s_nop 4\n\t" ASQ_DOT16(ASQ_A, "v_fmac_f64_dpp") : ASQ_OUT4(acc) : ASQ_IN16(z, r));
}
// acc[*] += sum_{l<12} |bcast_l(z) * r[l]|
__device__ __forceinline__ void dot12abs(double (&acc)[4], double z, const double (&r)[12]) {
  asm("s_nop 4\n\t" ASQ_DOT12(ASQ_A, "v_fmac_f64_dpp") : ASQ_OUT4(acc) : ASQ_IN12(z, r));
}
// acc[i] += bcast_i(a) * b, i < 12 (lane i's a feeds accumulator i); the fp64 form is
// mpcb_split.h fmac12_diag
#define ASQ_D(d, l) "v_fmac_f32_dpp %" #d ", %12, %13 row_newbcast:" #l " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ void diag12(float (&acc)[12], float a, float b) {
  asm("s_nop 4\n\t" ASQ_D(0, 0) ASQ_D(1, 1) ASQ_D(2, 2) ASQ_D(3, 3) ASQ_D(4, 4) ASQ_D(5, 5) ASQ_D(6, 6)
      ASQ_D(7, 7) ASQ_D(8, 8) ASQ_D(9, 9) ASQ_D(10, 10) ASQ_D(11, 11)
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
        "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11])
      : "v"(a), "v"(b));
}
__device__ __forceinline__ void diag12(double (&acc)[12], double a, double b) { fmac12_diag(acc, a, b); }
#undef ASQ_D

template <class T> __device__ __forceinline__ T sum4(const T (&a)[4]) { return (a[0] + a[1]) + (a[2] + a[3]); }

// lane L's value in every lane of its row (v_mov_b32_dpp row_newbcast:L)
template <int L> __device__ __forceinline__ unsigned bcu(unsigned v) {
  return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x150 + L, 0xF, 0xF, true);
}
template <int L> __device__ __forceinline__ int bc(int v) { return (int)bcu<L>((unsigned)v); }
template <int L> __device__ __forceinline__ float bc(float v) { return __uint_as_float(bcu<L>(__float_as_uint(v))); }
template <int L> __device__ __forceinline__ unsigned bc(unsigned v) { return bcu<L>(v); }
template <int L> __device__ __forceinline__ uint64_t bc(uint64_t v) {
  return ((uint64_t)bcu<L>((unsigned)(v >> 32)) << 32) | bcu<L>((unsigned)v);
}
template <int L> __device__ __forceinline__ double bc(double v) {
  return __builtin_bit_cast(double, bc<L>(__builtin_bit_cast(uint64_t, v)));
}

// stage-invariant addressing of one quad-blocked workspace array (mpcb_split.h soa()):
// element e of the stage-k record of this lane's instance = p0 + k * stride + e * SS
template <class T> struct Arr {
  T* p0;
  int64_t stride;
  __device__ __forceinline__ T* at(int k) const { return p0 + (int64_t)k * stride; }
};
// quad-blocked (soa) array: element e of the record at p0 + k * stride + e * SS
template <class T> __device__ __forceinline__ Arr<T> arr(T* base, int rec, int64_t nq, int64_t c) {
  return Arr<T>{base ? base + ((c >> 2) * rec) * SS + (c & (SS - 1)) : nullptr, nq * rec * SS};
}
// row-major export (rec2): element e of the record at p0 + k * stride + e
template <class T> __device__ __forceinline__ Arr<T> arr2(T* base, int rec, int64_t nq, int64_t c, int N, int imaj) {
  // (mpcb_split.h rec2: instance-major or stage-major)
  if (imaj) return Arr<T>{base ? base + c * N * (int64_t)rec : nullptr, rec};
  return Arr<T>{base ? base + ((c >> 2) * SS + (c & (SS - 1))) * rec : nullptr, nq * SS * rec};
}

// BOX: the active-set iterations; !BOX: one forward pass over P2's gains (unconstrained small
// chunks, SplitArgs::fwd16)
// Output staging: a pass's X / U rows go to LDS (one [(N+1)*12 | N*4] block per instance) and
// leave as 16-B vector stores after the pass.  Stores issued inside the stage loop would sit in
// the same in-order vmcnt queue as the prefetch loads, so every wait for a prefetched row also
// waited for the write acknowledgements of the previous stages' scattered 4/8-B output stores.
constexpr int OUT_NMAX = 64;   // longer horizons store directly
template <class T> __host__ __device__ constexpr int out_elems(int N) { return (N + 1) * NX + N * NU; }
// the refinement kernel's block per instance: the staged rows, then the refinement's N x NU
// feedforward terms and (N + 1) x NX state errors x - xref, then a copy of the staged U and X rows
template <class T> __host__ __device__ constexpr int ref_elems(int N) {
  return 2 * out_elems<T>(N) + N * NU + (N + 1) * NX;   // (+ a copy of the staged rows)
}

// Stage masks (active sets, violations: bit k = stage k) of a horizon N <= 32 in 32-bit registers
// (W32: half the VALU of every mask shift / or in the stage loops), else 64-bit.
template <bool W32> struct Masks {
  using M = std::conditional_t<W32, uint32_t, uint64_t>;
  static constexpr int WB = W32 ? 32 : 64;
  __device__ static __forceinline__ int popc(M v) { if constexpr (W32) return __builtin_popcount(v); else return __popcll(v); }
  __device__ static __forceinline__ int ffs(M v) { if constexpr (W32) return __builtin_ffs((int)v); else return __ffsll((long long)v); }
  __device__ static __forceinline__ int clz(M v) { if constexpr (W32) return __builtin_clz(v); else return __clzll(v); }
};

#ifdef MPCB_AS_STAMPS
WT_TABLE(g_wt_p3)
#endif
// (I <= jj) ? a : b with the lane condition computed at use into VCC (no hoisted lane mask)
template <int I> __device__ __forceinline__ float sel_le(int jj, float a, float b) {
  float r;
  asm("v_cmp_le_i32 vcc, %3, %4\n\tv_cndmask_b32 %0, %2, %1, vcc" : "=v"(r) : "v"(a), "v"(b), "i"(I), "v"(jj) : "vcc");
  return r;
}
template <int I> __device__ __forceinline__ double sel_le(int jj, double a, double b) {
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  unsigned lo, hi;
  asm("v_cmp_le_i32 vcc, %6, %7\n\tv_cndmask_b32 %0, %3, %2, vcc\n\tv_cndmask_b32 %1, %5, %4, vcc"
      : "=&v"(lo), "=&v"(hi)
      : "v"((unsigned)ua), "v"((unsigned)ub), "v"((unsigned)(ua >> 32)), "v"((unsigned)(ub >> 32)), "i"(I), "v"(jj)
      : "vcc");
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// p as an opaque VGPR value that still addresses global memory (the address-space cast keeps the
// loads and stores global_*: through a plain opaque pointer the compiler falls back to flat_*
// accesses, which also count against lgkmcnt)
template <class P> __device__ __forceinline__ P* vglobal(P* p) {
  uint64_t v = reinterpret_cast<uint64_t>(p);
  asm volatile("" : "+v"(v));
  return (P*)(__attribute__((address_space(1))) P*)v;
}

// The fp32 box kernel's refinement + KKT verification of one set (as_body, below, says what and
// why).  Every lane of the wave runs it (wave-uniform: the DPP blocks need whole rows); groups
// with ver = false compute along and write nothing.  Its stage loops are latency chains over a
// few hundred instances, so each keeps its next stage's loads in flight (two register slots, the
// loop unrolled by two, as the active-set kernel's backward pass).
// refinement steps per pass before the verification (up to REF_STEPS_MAX when the verification
// would release a component: one more step before acting on it), the refined passes whose
// multiplier verdicts count, and the verification's tolerance on a multiplier relative to its
// terms' sum
constexpr int REF_STEPS = 1, REF_STEPS_MAX = 1, REF_PASSES = 8;
constexpr double REF_TOL = 0x1p-18;
template <bool W32> struct RefIn {
  using M = typename Masks<W32>::M;
  using T = float;
  const T* x0;   // this instance's x0
  Arr<T> XU, GP, ABT, KR, PS;
  const T* cbase; int64_t cstride;   // the lane's [A|B] column (ABT2 rows or W.ctab)
  const T* refp; int64_t refs;       // the lane's reference component
  const T* xrN;
  const T* QN;
  const T* SW;                       // s blkdiag(Q, R) (LDS)
  T* PX;                             // the group's P block (LDS)
  T* xs; T* us; T* dks;              // the group's staged X rows, U rows, refinement feedforward (LDS)
  T* es;                             // ... and state errors x - xref (LDS)
  T crow[6];
  M lowm, upm;
  T lbm, ubm, tol_u;
  int N;
  bool iterate, ver;
};
template <bool W32> struct RefOut { typename Masks<W32>::M rd, alo, ahi; int sweeps; };

// run body(k, slot) for k = k0, k0 + dir, ... (N stages) with load(k, slot) one stage ahead in two
// register slots (every slot a fixed register set; loads for stages outside [0, N) are clamped)
template <class S, class L, class B>
__device__ __forceinline__ void ring2(int N, bool down, L&& load, B&& body) {
  S s0, s1;
  const int k0 = down ? N - 1 : 0, dir = down ? -1 : 1;
  auto kc = [&](int k) { return k < 0 ? 0 : (k >= N ? N - 1 : k); };
  load(k0, s0);
  for (int i = 0; i < N; i += 2) {
    const int k = k0 + dir * i;
    load(kc(k + dir), s1);
    body(k, s0);
    if (i + 1 >= N) break;
    load(kc(k + 2 * dir), s0);
    body(k + dir, s1);
  }
}

template <bool W32>
__device__ __forceinline__ RefOut<W32> refine_verify(const RefIn<W32>& in) {
  using T = float;
  using Mk = Masks<W32>;
  using M = typename Mk::M;
  const int lane = threadIdx.x;
  const int j = lane & 15;
  const int jx = j < NX ? j : 0;
  const int ju = j >= NX ? j - NX : 0;
  const bool stl = j < NX;
  const uint64_t mst = lane_mask(stl);
  const int N = in.N;
  const bool iterate = in.iterate, ver = in.ver;
  const Arr<T> XU = in.XU, GP = in.GP, ABT = in.ABT, KR = in.KR, PS = in.PS;
  const T* const cbase = in.cbase;
  const int64_t cstride = in.cstride;
  const T* const refp = in.refp;
  const int64_t refs = in.refs;
  const T* const SW = in.SW;
  T* const PX = in.PX;
  T* const xs = in.xs;
  T* const us = in.us;
  T* const dks = in.dks;
  // the adjoint reads the state errors e = x - xref rounded to fp32, not x: rounding x itself
  // (|x| ~ 1, e ~ 1e-2) put ~1e-6 of noise into the multipliers through Q e
  T* const es = in.es;
  const M lowm = in.lowm, upm = in.upm;
  T crow[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) crow[i] = in.crow[i];
  // the lane's row of [A|B] (state lanes: variable columns loaded, constant ones crow), fp64
  auto arow = [&](const T* rv, double (&row)[NZ]) {
#pragma unroll
    for (int t = 0; t < NVAR; ++t) row[var_col(t)] = (double)rv[t];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      row[p] = (double)crow[p];
      row[6 + p] = (double)crow[3 + p];
    }
  };
  M rd = 0, alo = 0, ahi = 0;   // input lanes: released stages, free components beyond a bound
#if defined(MPCB_REF_STAMPS) && defined(MPCB_AS_OWNER)
  unsigned long long rst[8] = {}, rst_prev = __builtin_amdgcn_s_memtime();
#endif

  // (1) the states re-simulated in fp64 from the staged U, x_k into xs
  struct SF { T rv[NVAR]; T yb, gp, rf; };
  {
    double zd = 0.0;   // state lanes dx_i, input lanes du_m
    if (iterate && stl) zd = (double)in.x0[jx] - (double)XU.at(0)[jx * SS];
    ring2<SF>(N, false,
        [&](int k, SF& s) {
          ldv<T, NVAR, 8>(ABT.at(k) + jx * ABT2_W, s.rv);
          s.yb = XU.at(k)[j * SS];
          s.gp = iterate ? GP.at(k)[jx * SS] : T(0);
          s.rf = refp[(int64_t)k * refs];
        },
        [&](int k, const SF& s) {
          double row[NZ];
          arow(s.rv, row);
          if (!stl) {
            zd = (double)us[k * NU + ju] - (double)s.yb;
          } else if (ver) {
            const double xk = (double)s.yb + zd;
            xs[k * NX + jx] = (T)xk;
            es[k * NX + jx] = (T)(xk - (double)s.rf);
          }
          double acc[4] = {(double)s.gp, 0.0, 0.0, 0.0};
          dot16(acc, zd, row);
          if (stl) zd = sum4(acc);
        });
    if (stl && ver) {
      const double xN = (double)XU.at(N)[jx * SS] + zd;
      xs[N * NX + jx] = (T)xN;
      es[N * NX + jx] = (T)(xN - (double)in.xrN[jx]);
    }
  }
  RSTAMP(0);
  struct SA { T cr[NX]; T rf; };
  int sweeps = 1;   // stage loops run (qp_stats counts each as a forward pass)
  for (int r = 0;; ++r) {
    ++sweeps;
    // (2) the adjoint sweep (fp64): lambda_N = QN e_N, g_k = [A|B]_k^T lambda_{k+1} + s blkdiag(Q,
    // R)(e_k, u_k - uref_k); r < REF_STEPS keeps the input lanes' g_k for the correction (dks),
    // r = REF_STEPS decides
    double lam;
    {
      const double eN = stl ? (double)es[N * NX + jx] : 0.0;
      double qn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) qn[i] = stl ? (double)in.QN[i * NX + jx] : 0.0;
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      dot12(acc, eN, qn);
      lam = sum4(acc);
    }
    ring2<SA>(N, true,
        [&](int k, SA& s) {
          const T* rows = cbase + (int64_t)k * cstride;
#pragma unroll
          for (int i = 0; i < NX; ++i) s.cr[i] = rows[i * ABT2_W];
          s.rf = refp[(int64_t)k * refs];
        },
        [&](int k, const SA& s) {
          const double w = stl ? (double)es[k * NX + jx] : (double)us[k * NU + ju] - (double)s.rf;
          double col[NX], swc[NZ];
#pragma unroll
          for (int i = 0; i < NX; ++i) col[i] = (double)s.cr[i];
#pragma unroll
          for (int i = 0; i < NZ; ++i) swc[i] = (double)SW[i * NZ + j];
          double acc[4] = {0.0, 0.0, 0.0, 0.0};
          dot12(acc, lam, col);
          dot16(acc, w, swc);
          const double g = sum4(acc);
          if (stl) {
            lam = g;
          } else {
            if (ver) dks[k * NU + ju] = (T)g;
          }
          if (!stl && r >= REF_STEPS) {
            double aa[4] = {0.0, 0.0, 0.0, 0.0};
            dot12abs(aa, lam, col);
            dot16abs(aa, w, swc);
            const double tolp = REF_TOL * sum4(aa);
            const bool lo = (lowm >> k) & 1u, hi = (upm >> k) & 1u;
            const T uk = us[k * NU + ju];
            rd |= (M)((lo && g < -tolp) || (hi && g > tolp)) << k;
            alo |= (M)(!lo && !hi && uk < in.lbm - in.tol_u) << k;
            ahi |= (M)(!lo && !hi && uk > in.ubm + in.tol_u) << k;
          }
        });
    if (r >= REF_STEPS) {
      RSTAMP(4);
    } else {
      RSTAMP(1);
    }
    // decided, unless a release is pending and another step is left (wave-uniform)
    if (r >= REF_STEPS) {
      if (r == REF_STEPS_MAX || !__builtin_amdgcn_ballot_w64(ver && rd != 0)) break;
      rd = alo = ahi = 0;
    }
    sweeps += 2;
    // (2b) the correction's backward recursion (fp32): the masked Riccati recursion of the set for
    // the linear term alone, d = -H_FF^{-1} g_F (P_{k+1}: QN, else the PS2 snapshot, which holds
    // the current set's value function); dks: g_k in, the feedforward d_k out
    struct SB { T cr[NX]; T ps[PS2_W]; };
    T pc = T(0);   // state lanes: the correction's p_{k+1}
    ring2<SB>(N, true,
        [&](int k, SB& s) {
          const T* rows = cbase + (int64_t)k * cstride;
#pragma unroll
          for (int i = 0; i < NX; ++i) s.cr[i] = rows[i * ABT2_W];
          ldv<T, PS2_W>(PS.at(k + 1 < N ? k + 1 : k) + jx * PS2_W, s.ps);
        },
        [&](int k, const SB& s) {
          const bool lo = !stl && ((lowm >> k) & 1u), hi = !stl && ((upm >> k) & 1u);
          T Pc[NX];
          if (k == N - 1) {
#pragma unroll
            for (int i = 0; i < NX; ++i) Pc[i] = stl ? in.QN[i * NX + jx] : T(0);
          } else {   // (unpacked through the group's LDS block, as at a restart)
            if (stl) {
#pragma unroll
              for (int d = 0; d < PS2_W; ++d) PX[jx * PS2_W + d] = s.ps[d];
            }
            wave_lds_sync();
#pragma unroll
            for (int i = 0; i < NX; ++i) {
              const int dd = (jx - i + NX) % NX;
              Pc[i] = stl ? PX[dd <= 6 ? i * PS2_W + dd : jx * PS2_W + (NX - dd)] : T(0);
            }
            wave_lds_sync();
          }
          // G = [A|B]^T P [A|B] + s blkdiag(Q, R) (lane j: column j), h = [A|B]^T p + (0, g)
          float y[16], gg[16];
          to_columns(outer12(Pc, s.cr), y);
          to_columns(outer12(s.cr, y), gg);
          T G[NZ];
#pragma unroll
          for (int i = 0; i < NZ; ++i) G[i] = gg[i] + SW[i * NZ + j];
          T hj;
          {
            T ac[4] = {T(0), T(0), T(0), T(0)};
            dot12(ac, pc, s.cr);
            hj = sum4(ac) + (stl ? T(0) : dks[k * NU + ju]);
          }
          T Ht[NU * NU], ht[NU], Hux_t[NU];
          static_for<NU>([&](auto mm) {
            constexpr int m = decltype(mm)::value;
            Ht[m * NU + 0] = bc<NX + 0>(G[NX + m]);
            Ht[m * NU + 1] = bc<NX + 1>(G[NX + m]);
            Ht[m * NU + 2] = bc<NX + 2>(G[NX + m]);
            Ht[m * NU + 3] = bc<NX + 3>(G[NX + m]);
            ht[m] = bc<NX + m>(hj);
            Hux_t[m] = G[NX + m];
          });
          {   // fixed components: d = 0 (identity rows and columns, no gradient)
            const int fx_own = (lo || hi) ? 1 : 0;
            int fixed[NU];
            fixed[0] = bc<NX + 0>(fx_own); fixed[1] = bc<NX + 1>(fx_own);
            fixed[2] = bc<NX + 2>(fx_own); fixed[3] = bc<NX + 3>(fx_own);
#pragma unroll
            for (int m = 0; m < NU; ++m) {
              ht[m] = fixed[m] ? T(0) : ht[m];
              Hux_t[m] = fixed[m] ? T(0) : Hux_t[m];
#pragma unroll
              for (int n = 0; n < NU; ++n)
                Ht[m * NU + n] = (fixed[m] || fixed[n]) ? ((m == n) ? T(1) : T(0)) : Ht[m * NU + n];
            }
          }
          T Lc[10], kff[NU], nh[NU];
          chol4(Ht, Lc);
#pragma unroll
          for (int m = 0; m < NU; ++m) nh[m] = -ht[m];
          chol4_solve(Lc, nh, kff);
          T pn = hj;
#pragma unroll
          for (int m = 0; m < NU; ++m) pn += Hux_t[m] * kff[m];
          pc = stl ? pn : T(0);
          if (!stl && ver) dks[k * NU + ju] = sel<NU>(kff, ju);
        });
    RSTAMP(2);
    // (3) the correction's forward pass with the stored gains (KR2), fused with the next
    // re-simulation: u_k += K_k (x_k - x_k^old) + d_k (input lanes), then x_{k+1} in fp64 from the
    // refined u (state lanes; x_k^old: the previous re-simulation in xs)
    struct SC { T pv[KR2_W]; T yb, gp, rf; };
    double zd = 0.0;
    if (iterate && stl) zd = (double)in.x0[jx] - (double)XU.at(0)[jx * SS];
    ring2<SC>(N, false,
        [&](int k, SC& s) {
          ldv<T, KR2_W, 8>(stl ? ABT.at(k) + jx * ABT2_W : KR.at(k) + ju * KR2_W, s.pv);
          s.yb = XU.at(k)[j * SS];
          s.gp = iterate ? GP.at(k)[jx * SS] : T(0);
          s.rf = refp[(int64_t)k * refs];
        },
        [&](int k, const SC& s) {
          // state lanes: the refined x_k minus the previous one (fp32 is enough for the gain product)
          T dxs = T(0);
          if (stl) {
            const double xn = (double)s.yb + zd;
            dxs = (T)(xn - (double)xs[k * NX + jx]);
            if (ver) {
              xs[k * NX + jx] = (T)xn;
              es[k * NX + jx] = (T)(xn - (double)s.rf);
            }
          }
          T ac[4] = {stl ? T(0) : dks[k * NU + ju], T(0), T(0), T(0)};
          T krow[NX];
#pragma unroll
          for (int i = 0; i < NX; ++i) krow[i] = s.pv[i];
          dot12(ac, dxs, krow);
          double zk = zd;
          if (!stl) {
            const T un = us[k * NU + ju] + sum4(ac);
            if (ver) us[k * NU + ju] = un;
            zk = (double)un - (double)s.yb;
          }
          double row[NZ];
          arow(s.pv, row);
          double acc[4] = {(double)s.gp, 0.0, 0.0, 0.0};
          dot16(acc, zk, row);
          if (stl) zd = sum4(acc);
        });
    if (stl && ver) {
      const double xN = (double)XU.at(N)[jx * SS] + zd;
      xs[N * NX + jx] = (T)xN;
      es[N * NX + jx] = (T)(xN - (double)in.xrN[jx]);
    }
    RSTAMP(3);
  }
#if defined(MPCB_REF_STAMPS) && defined(MPCB_AS_OWNER)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    for (int i_ = 0; i_ < 5; ++i_) g_refst[i_] += rst[i_];
    g_refst[5] += 1;
  }
#endif
  return RefOut<W32>{rd, alo, ahi, sweeps};
}

// The refinement list (SplitArgs::as_ref): [0] count, [1] the refinement kernel's work counter,
// then AS_REF_W words per entry -- chunk instance, passes, forward passes, backward stages, and
// per input component m the stage masks of its lower (4 + 2m, + 1 for stages 32..63) and upper
// (12 + 2m, ...) active sets.  Written by the 16 lanes of the instance's group.
template <bool W32, class M>
__device__ __forceinline__ void as_ref_put(int* e, int j, int c, int git, int n_fwd, int n_bst, M lowm, M upm) {
  if (j == 0) {
    e[0] = c;
    e[1] = git;
    e[2] = n_fwd;
    e[3] = n_bst;
  }
  if (j >= NX) {
    const int w = 4 + 2 * (j - NX);
    e[w] = (int)(uint32_t)lowm;
    e[w + 8] = (int)(uint32_t)upm;
    if constexpr (!W32) {
      e[w + 1] = (int)(uint32_t)((uint64_t)lowm >> 32);
      e[w + 9] = (int)(uint32_t)((uint64_t)upm >> 32);
    }
  }
}

// REF: the refinement kernel (as_ref_kernel_f32, mpcb_as.hip): its groups take the instances the
// active-set kernel listed in SplitArgs::as_ref (converged sets with an undecided multiplier),
// restore their active sets and pass counts, redo the final forward pass (the same arithmetic:
// the same U and multipliers) and run the refinement + verification below, iterating on where it
// changes the set.  The active-set kernel itself only lists them: inlined there, the refinement's
// registers spilled its pass loop (c4 kernel 3.44 vs 3.24 ms).
template <class T, bool BOX, bool W32 = false, bool ITER = false, bool REF = false>
__device__ __forceinline__ void as_body(const SplitArgs<T>& args) {
  if constexpr (!BOX) AS_WT(0);
  // box kernel: the workspace and I/O pointers as opaque loop-invariant VGPRs (as P2's model
  // constants): kept in scalar registers they were spilled to VGPR lanes and read back with
  // v_readlane at every pass and instance change
  SplitArgs<T> a = args;
  if constexpr (BOX) {
    a.XU = vglobal(a.XU); a.GP = vglobal(a.GP); a.ABT = vglobal(a.ABT); a.GH = vglobal(a.GH);
    a.KR = vglobal(a.KR); a.PS = vglobal(a.PS); a.xref = vglobal(a.xref); a.uref = vglobal(a.uref);
    a.u0 = vglobal(a.u0); a.X = vglobal(a.X); a.U = vglobal(a.U); a.status = vglobal(a.status);
    a.qp_stats = vglobal(a.qp_stats); a.x0 = vglobal(a.x0); a.as_fb = vglobal(a.as_fb);
    a.as_ref = vglobal(a.as_ref);
  }
  using Mk = Masks<W32>;
  using M = typename Mk::M;
  constexpr int WB = Mk::WB;
  constexpr bool UNC = BOX && sizeof(T) == 4;   // fp32 box: undecided multipliers are flagged
  constexpr bool VER = UNC && REF;               // ... and refined + verified (REF kernel)
  __shared__ T lds_px[GROUPS][NX * NX];   // P_k by columns, for the symmetric transpose
  extern __shared__ __attribute__((aligned(16))) unsigned char as_dyn[];
  const int lane = threadIdx.x;
  const int q = lane >> 4;
  const int j = lane & 15;
  const int jx = j < NX ? j : 0;
  const int ju = j >= NX ? j - NX : 0;
  const bool stl = j < NX;                          // state lane (else input lane ju)
  const uint64_t mst = lane_mask(stl);
  T* const PX = lds_px[q];
  const int64_t nb = a.nb;
  const int N = a.N;
  // the RK4 tangent's position entry of a velocity column, h/6 * (1 + 2 + 2 + 1) as the tangent
  // computes it: the same [A|B] column as P2's (mpcb_split.hip riccati_body hv), whose snapshots
  // the first masked pass restarts from
  const T h = (a.h / T(6)) * T(6);
  const Weights<T>& W = *a.W;
  const bool iterate = MPCB_AS_ITER_T ? ITER : a.mode == MPCB_MODE_ITERATE;   // (see riccati_body)
  const T lbm = W.lbu[ju], ubm = W.ubu[ju];
  constexpr T eps = sizeof(T) == 8 ? T(2.220446049250313e-16) : T(1.1920929e-7);
  const T tol_u = T(16) * eps * (fabs(lbm) + fabs(ubm) + T(1));
  int64_t nq = (nb + SS - 1) / SS;
  // (box kernel, rollout mode: the record strides derived from nq are loop-invariant VGPRs too)
  if constexpr (BOX && !ITER) asm volatile("" : "+v"(nq));   // (iterate: VGPR-bound already)
  // The group's instance and its workspace records.  Box kernel with a work counter (a.as_queue):
  // the grid holds the waves the machine keeps resident, and a group whose instance finished
  // takes the next one from the counter, so a wave does not carry three idle groups while its
  // slowest instance finishes (3.8 active-set passes per instance, 5.2 per wave with fixed quads).
  bool valid;
  int64_t c, b;
  const T *xr, *ur, *xrN;
  Arr<T> XU, GP, ABT, GH, KR, PS;
  const T* cbase;
  int64_t cstride;
  const T* refp;
  const int64_t refs = stl ? NX : NU;
  const int tv = var_index(j);                      // variable column of [A|B] owned by lane j
  // constant directions read their column from W.ctab with the same strided loads (slot 0..5)
  const int cslot = j < 3 ? j : j - 3;
  const int* ent = nullptr;   // REF: the group's list entry (AS_REF_W words, as_ref_put)
  auto bind = [&](int64_t c_raw) {
#ifdef MPCB_AS_ORDER_DBG   // (tools/ab_as_order.py)
    if (a.as_order && c_raw < nb) c_raw = a.as_order[c_raw];
#endif
    if constexpr (REF) {
      valid = c_raw < a.as_ref[0] && c_raw < a.as_ref_cap;
      ent = a.as_ref + AS_REF_HDR + (valid ? c_raw : 0) * AS_REF_W;
      c = valid ? ent[0] : nb - 1;
    } else {
      valid = c_raw < nb;
      c = valid ? c_raw : nb - 1;     // an empty group shadows the last instance
    }
    b = a.b0 + c;
    xr = a.xref + b * a.xref_sb;
    ur = a.uref + b * a.uref_sb;
    xrN = xr + (int64_t)N * NX;
    XU = arr(a.XU, XU_REC, nq, c);
    GP = arr(iterate ? a.GP : (T*)nullptr, GP_REC, nq, c);
    ABT = arr2(a.ABT, ABT2_REC, nq, c, N, a.imajor);
    GH = arr2(BOX ? a.GH : (T*)nullptr, GH2_REC, nq, c, N, a.imajor);
    KR = arr2(a.KR, KR2_REC, nq, c, N, a.imajor);
    PS = arr2(BOX ? a.PS : (T*)nullptr, PS2_REC, nq, c, N, a.imajor);
    // the masked backward's column loads: ABT2 rows (variable directions) or W.ctab (constant
    // ones, stride 0), and the own reference component
    cbase = tv >= 0 ? ABT.p0 + tv : W.ctab + cslot;
    cstride = tv >= 0 ? ABT.stride : 0;
    refp = stl ? xr + jx : ur + ju;
  };
  bind((int64_t)blockIdx.x * GROUPS + q);
  // (Measured and dropped, round 4: stores from every lane with the masked-out ones into a
  // per-lane scratch, so that the waits for the prefetched loads no longer drain the stores --
  // 3.15 -> 4.73 ms, the scratch writes cost more than the drains; prefetching the backward
  // stages for every group: no change.)
  // s * blkdiag(Q, R) in LDS (shared by the wave's 4 instances): lane j reads column j (= row j),
  // the stage cost of direction j, when a backward stage needs it
  __shared__ T SW[NZ * NZ];
  if constexpr (BOX) {   // (the backward pass's; the forward-only instantiation allocates no LDS)
    for (int e = lane; e < NZ * NZ; e += 64) {
      const int r = e / NZ, cl = e % NZ;
      const T wq = (r < NX && cl < NX) ? W.Q[r * NX + cl] : T(0);
      const T wr = (r >= NX && cl >= NX) ? W.R[(r - NX) * NU + (cl - NX)] : T(0);
      SW[e] = a.s * (wq + wr);
    }
    wave_lds_sync();
  }
  // row i of [A|B] at the constant columns (state lanes): position e_p, velocity e_v + h e_p
  // (h: the tangent's h/6 * 6, above)
  T crow[6];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    crow[p] = (jx == p) ? T(1) : T(0);
    crow[3 + p] = ((jx == 6 + p) ? T(1) : T(0)) + ((jx == p) ? h : T(0));
  }

  M lowm = 0, upm = 0;          // input lanes: active sets of component ju, bit k = stage k
  bool done = !valid;           // (box: the group has no instance left)
  int32_t st = MPCB_STATUS_OK;
  int best = 0x7fffffff, pcount = 3;
  int n_fwd = 0, n_bst = 0;
  int kc = -1;                  // highest stage whose active set changed (group-uniform)
  int git = 0;                  // passes of the group's current instance
  int rpass = 0;                // REF: refined passes of the group's current instance
  M relm = 0, pin = 0;          // REF, input lanes: stages released by the refinement; fixed again after
  M lrel = 0;                   // REF, input lanes: the releases the last refined pass applied
  // REF: the listed instance's active set and counts (as_ref_put), and its U (the output the
  // active-set kernel wrote: mpcb_solve passes a U buffer of the handle's when the caller has none)
  auto restore = [&]() {
    rpass = 0;
    relm = pin = lrel = 0;
    if constexpr (REF) {
      if (valid) {
        T* const us0 = reinterpret_cast<T*>(as_dyn) + q * ref_elems<T>(N) + (N + 1) * NX;
        const T* const ub = a.U + b * (int64_t)N * NU;
        for (int e = j; e < N * NU; e += NZ) us0[e] = ub[e];
        wave_lds_sync();
        git = ent[1];
        n_fwd = ent[2];
        n_bst = ent[3];
        kc = ent[AS_REF_KC];   // (an interior-point instance: the full backward pass first)
        const int w = 4 + 2 * ju;
        if (!stl) {
          lowm = (M)(uint32_t)ent[w];
          upm = (M)(uint32_t)ent[w + 8];
          if constexpr (!W32) {
            lowm |= (M)(uint32_t)ent[w + 1] << 32;
            upm |= (M)(uint32_t)ent[w + 9] << 32;
          }
          // the set's fixed components at their bounds: an interior-point instance (crossover,
          // mpcb_asipm.h) left them ~sqrt(mu) inside, and the refinement corrects the free
          // components only, so those offsets stayed in U (up to 4.8e-4 normwise on the sweep's
          // wind draws); an active-set instance has them there already
          for (int k = 0; k < N; ++k)
            if (((lowm | upm) >> k) & 1u) us0[k * NU + ju] = ((lowm >> k) & 1u) ? lbm : ubm;
        }
        wave_lds_sync();
      }
    }
  };
  restore();
  bool u0fin = true;           // u0 of the flushed (final) pass is finite (staged outputs)
  // (the box kernel: always -- mpcb_create refuses box_u beyond N = 64 and mpcb_solve X / U that
  // are not 16-B aligned -- so its stage loop carries no direct-store path)
  const bool stage_out = BOX || (N <= OUT_NMAX && ((((uintptr_t)a.X) | ((uintptr_t)a.U)) & 15) == 0);
  // an instance's outcome: the QP status of the unconstrained pass (P2 wrote it) carries over
  auto finish = [&](bool write_status) {
    if (valid && j == NX) {
      bool fin = u0fin;
      if (!stage_out) {   // direct stores
        T u0c[NU];
        load_vec<NU>(a.u0 + b * NU, u0c);
#pragma unroll
        for (int m = 0; m < NU; ++m) fin = fin && isfin(u0c[m]);
      }
      const int32_t st0 = a.status[b];
      if (write_status) a.status[b] = !fin ? MPCB_STATUS_NAN : (st0 != MPCB_STATUS_OK ? st0 : st);
      if (BOX && a.qp_stats) {
        a.qp_stats[2 * b] = n_fwd;
        a.qp_stats[2 * b + 1] = n_bst;
      }
    }
  };
#ifdef MPCB_AS_STAMPS
  unsigned long long ast_prev = __builtin_amdgcn_s_memtime(), ast_acc[12] = {};
#endif
  for (;;) {
#ifdef MPCB_AS_STAMPS
    ast_acc[8] += 1;
#endif
    int kmax = kc;
#pragma unroll
    for (int g = 0; g < GROUPS; ++g) {
      const int o = __builtin_amdgcn_readlane(kc, g * 16);
      kmax = o > kmax ? o : kmax;
    }
    if (git > 0 && !done && kc >= 0) n_bst += kc + 1;
    if (!done && !REF) ++n_fwd;
    // ------------------------------------------------ masked Riccati over the cached [A|B]
    ASTAMP(7);
    if (BOX && kmax >= 0) {   // (a group in its first pass has kc = -1)
#ifdef MPCB_AS_STAMPS
      ast_acc[9] += kmax + 1;
#endif
      T Pc[NX], pj;
      {
        const T vN = stl ? XU.at(N)[jx * SS] - xrN[jx] : T(0);
        T qn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) qn[i] = stl ? W.QN[i * NX + jx] : T(0);
        T acc[4] = {T(0), T(0), T(0), T(0)};
        dot12(acc, vN, qn);
        pj = stl ? sum4(acc) : T(0);
#pragma unroll
        for (int i = 0; i < NX; ++i) Pc[i] = qn[i];
        if (kc >= 0 && kc < N - 1 && stl) {   // restart: the value function stored at kc + 1
          // P[i][j] sits with lane i at slot (j - i) % 12 when that is <= 6, else with lane j at
          // slot (i - j) % 12 (the packed PS2 record, mpcb_kernels.h)
          // (unpacked through the group's LDS block: per-lane LDS offsets instead of 12 global
          // addresses, which the compiler kept live into a spill)
          T ps[PS2_W];
          ldv<T, PS2_W>(PS.at(kc + 1) + jx * PS2_W, ps);
#pragma unroll
          for (int d = 0; d < PS2_W; ++d) PX[jx * PS2_W + d] = ps[d];
          wave_lds_sync();
#pragma unroll
          for (int i = 0; i < NX; ++i) {
            const int dd = (jx - i + NX) % NX;
            Pc[i] = PX[dd <= 6 ? i * PS2_W + dd : jx * PS2_W + (NX - dd)];
          }
          pj = ps[7];
        }
        wave_lds_sync();   // the stages' PX writes follow the reads
      }
      bool qp_ok = true;
      // Stage data one stage ahead (column j of [A|B], own ybar and yref components, own gap
      // component) in two register slots, the stage loop unrolled by two (each slot a fixed register set: the
      // copy of a one-slot prefetch into the stage's operands was 14 moves and 14 separate waits
      // per stage).  Every group loads at every stage the wave visits, so no exec mask guards the
      // loads: a group above its own restart stage (k > kc) reloads its stage kc, a cache hit,
      // and discards the result.  (The prefetch keeps the raw loaded values: forming e = ybar - yref inside it made the
      // compiler wait for the loads it had just issued, vmcnt(0), at every backward stage)
      T rcol[2][NX], rref[2], ryb[2], rgp[2] = {T(0), T(0)};
      const int kcl = kc >= 0 ? kc : 0;
      auto bload = [&](int k, auto slot_tag) {
        constexpr int sl = decltype(slot_tag)::value;
        const int kk = k <= kc ? k : kcl;
        // column tv of the stage's ABT2 rows, or (constant directions) of W.ctab: one load
        // pattern for every lane (no lane branch)
        const T* rows = cbase + (int64_t)kk * cstride;
#pragma unroll
        for (int i = 0; i < NX; ++i) rcol[sl][i] = rows[i * ABT2_W];
        ryb[sl] = XU.at(kk)[j * SS];
        rref[sl] = refp[(int64_t)kk * refs];
        if (iterate) rgp[sl] = GP.at(kk)[jx * SS];   // (input lanes: unused)
      };
      auto bstage = [&](int k, auto slot_tag) {
        constexpr int sl = decltype(slot_tag)::value;
        const bool act = k <= kc;   // this group's stage is recomputed
        T col[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) col[i] = rcol[sl][i];
        const T e = ryb[sl] - rref[sl], yb = ryb[sl], gpo = rgp[sl];
        // pt = p + P gap (component j), h = [A|B]^T pt
        T pt = pj;
        if (iterate) {
          T acc[4] = {T(0), T(0), T(0), T(0)};
          dot12(acc, gpo, Pc);
          pt += stl ? sum4(acc) : T(0);
        }
        T hj;
        T G[NZ];
        if constexpr (sizeof(T) == 4) {
          T acc[4] = {T(0), T(0), T(0), T(0)};
          dot12(acc, pt, col);
          hj = sum4(acc);
          float y[16], g[16];
          to_columns(outer12(Pc, col), y);   // lane (q,j): Y_q[:, j]  (P symmetric: row = column)
          to_columns(outer12(col, y), g);    // lane (q,j): G_q[:, j]
#pragma unroll
          for (int i = 0; i < NZ; ++i) G[i] = g[i];
        } else {
          double y[NX], g[NZ];
          double hh = 0.0;
#pragma unroll
          for (int i = 0; i < NX; ++i) y[i] = 0.0;
#pragma unroll
          for (int i = 0; i < NZ; ++i) g[i] = 0.0;
          static_for<NX>([&](auto l) { fmac13_bc<decltype(l)::value>(y, hh, Pc, pt, col[l]); });
#pragma unroll
          for (int l = 0; l < NX; ++l) fmac16_diag(g, col[l], y[l]);
          hj = hh;
#pragma unroll
          for (int i = 0; i < NZ; ++i) G[i] = g[i];
        }
        // stage cost: G += s blkdiag(Q, R), h += s blkdiag(Q, R) (ybar - yref)
        {
          T swc[NZ];
#pragma unroll
          for (int i = 0; i < NZ; ++i) swc[i] = SW[i * NZ + j];
          T acc[4] = {hj, T(0), T(0), T(0)};
          dot16(acc, e, swc);
          hj = sum4(acc);
#pragma unroll
          for (int i = 0; i < NZ; ++i) G[i] += swc[i];
        }
        ASTAMP(1);
        // unmasked input row of a component fixed at this stage: the forward's multiplier.  (Where
        // the component is free the forward never reads the row, and a stage whose fixed set
        // changes is recomputed -- and its row written -- before the next forward pass.)
        {
          T gr[20];
#pragma unroll
          for (int i = 0; i < NZ; ++i) gr[i] = G[i];
          gr[NZ] = hj;
          gr[17] = gr[18] = gr[19] = T(0);
          if (act && valid && !stl && (((lowm | upm) >> k) & 1u)) stv<T, 20>(GH.at(k) + ju * 20, gr);
        }
        // the 4x4 input block and h_u from the input lanes; masking of the fixed components
        T Ht[NU * NU], ht[NU], Hux_t[NU];
        static_for<NU>([&](auto mm) {
          constexpr int m = decltype(mm)::value;
          Ht[m * NU + 0] = bc<NX + 0>(G[NX + m]);
          Ht[m * NU + 1] = bc<NX + 1>(G[NX + m]);
          Ht[m * NU + 2] = bc<NX + 2>(G[NX + m]);
          Ht[m * NU + 3] = bc<NX + 3>(G[NX + m]);
          ht[m] = bc<NX + m>(hj);
          Hux_t[m] = G[NX + m];
        });
        {
          const bool lo = (lowm >> k) & 1u, hi = (upm >> k) & 1u;
          const bool fx = !stl && (lo || hi);
          // (a stage at which no group of the wave fixes a component: the masking is the identity)
          if (__builtin_amdgcn_ballot_w64(fx)) {
            const int fx_own = fx ? 1 : 0;
            // input lanes (yb = ubar): the fixed value's offset, 0 where the component is free
            const T dl_own = lo ? (lbm - yb) : (hi ? (ubm - yb) : T(0));
            int fixed[NU];
            T delta[NU];
            fixed[0] = bc<NX + 0>(fx_own); fixed[1] = bc<NX + 1>(fx_own);
            fixed[2] = bc<NX + 2>(fx_own); fixed[3] = bc<NX + 3>(fx_own);
            delta[0] = bc<NX + 0>(dl_own); delta[1] = bc<NX + 1>(dl_own);
            delta[2] = bc<NX + 2>(dl_own); delta[3] = bc<NX + 3>(dl_own);
            T hn[NU];
#pragma unroll
            for (int m = 0; m < NU; ++m) {
              // h_F += H_FA delta_A (delta = 0 on the free components: no select)
              T acc = ht[m];
#pragma unroll
              for (int n = 0; n < NU; ++n) acc = fma(Ht[m * NU + n], delta[n], acc);
              hn[m] = fixed[m] ? -delta[m] : acc;
              Hux_t[m] = fixed[m] ? T(0) : Hux_t[m];
            }
#pragma unroll
            for (int m = 0; m < NU; ++m) {
              ht[m] = hn[m];
#pragma unroll
              for (int n = 0; n < NU; ++n) {
                const bool f = fixed[m] || fixed[n];
                Ht[m * NU + n] = f ? ((m == n) ? T(1) : T(0)) : Ht[m * NU + n];
              }
            }
          }
        }
        T Lc[10];
        chol4(Ht, Lc);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 10; ++i) ok = ok && (Lc[i] == Lc[i]);
        qp_ok = qp_ok && (ok || !act);
        T kff[NU], Kj[NU], nh[NU];
#pragma unroll
        for (int m = 0; m < NU; ++m) nh[m] = -ht[m];
        chol4_solve(Lc, nh, kff);
#pragma unroll
        for (int m = 0; m < NU; ++m) nh[m] = -Hux_t[m];
        chol4_solve(Lc, nh, Kj);
        T pn = hj;
#pragma unroll
        for (int m = 0; m < NU; ++m) pn += G[NX + m] * kff[m];
        // Pn[i] = G[i] + sum_m H_xu[i][m] K[m][j]; lane i owns H_xu[i][:] = its (unmasked) G[NX..]
        T Pn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) Pn[i] = G[i];
#pragma unroll
        for (int m = 0; m < NU; ++m) diag12(Pn, G[NX + m], Kj[m]);
        {   // KR2: K[m][j] at KR2_W m + j, k_m at KR2_W m + 12
          if (act && valid) {
            T* kr = KR.at(k);
            if (stl) {
#pragma unroll
              for (int m = 0; m < NU; ++m) kr[m * KR2_W + j] = Kj[m];
            } else {
              kr[ju * KR2_W + 12] = sel<NU>(kff, ju);
            }
          }
        }
        ASTAMP(2);
        // symmetric by construction: entry (r, c) from lane max(r, c) (see mpcb_split.hip): lane j
        // publishes its column as row j of PX and takes the entries below its diagonal from the
        // rows of the lanes that own them.  The lane-class select computes its condition at use
        // (v_cmp into VCC): the twelve hoisted 64-bit masks of a plain select were spilled scalar
        // registers, and per-lane LDS addresses instead of selects (measured) put 44 % of the
        // kernel's LDS cycles into bank conflicts
        if (stl) {
#pragma unroll
          for (int i = 0; i < NX; ++i) PX[j * NX + i] = Pn[i];
        }
        wave_lds_sync();
        {
          // (the input lanes' Pc and pj are never read -- P's rows 12..15 of the products and
          // the broadcasts from lanes >= 12 are not summed -- so they take whatever comes)
          const uint64_t ma = lane_mask(act);
          static_for<NX>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            Pc[i] = csel(ma, sel_le<i>(jx, Pn[i], PX[i * NX + jx]), Pc[i]);
          });
          pj = csel(ma, pn, pj);
        }
        // packed snapshot of P_k, p_k for a later restart: slot d of lane j is P[j][(j + d) % 12],
        // the entry lane max(j, o) published above
        {
          T ps[PS2_W];
#pragma unroll
          for (int d = 0; d < 7; ++d) {
            const int o = jx + d < NX ? jx + d : jx + d - NX;
            ps[d] = PX[(o > jx ? o : jx) * NX + (o > jx ? jx : o)];
          }
          ps[7] = pj;
          if (act && valid && stl && k > 0) stv<T, PS2_W>(PS.at(k) + j * PS2_W, ps);
        }
        wave_lds_sync();
        ASTAMP(3);
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      bload(kmax, I0{});
      ASTAMP(0);
      for (int k = kmax; k >= 0; k -= 2) {
        if (k > 0) bload(k - 1, I1{});
        bstage(k, I0{});
        if (k == 0) break;
        if (k > 1) bload(k - 2, I0{});
        bstage(k - 1, I1{});
      }
      if (!qp_ok) st = MPCB_STATUS_QP_FAIL;
    }

    // ------------------------------------------------ forward pass, multipliers, violations
    M vlo = 0, vhi = 0, vfl = 0, vfu = 0;   // input lanes: violation sets of component ju
    // (fp32 box) input lanes: a fixed component's multiplier lies within its rounding bound
    // tol_mu, so the pass's KKT test cannot decide its sign (verified below)
    bool unc = false;
    const bool write = valid && !done;
    // LDS staging of this pass's outputs (launch_*: dynamic LDS when N <= OUT_NMAX)
    T* const xs = reinterpret_cast<T*>(as_dyn) + q * (REF ? ref_elems<T>(N) : out_elems<T>(N));   // X rows, then U rows
    T* const us = xs + (N + 1) * NX;
    T zj = T(0);   // state lanes: dx_j; input lanes: du_ju
    if (iterate && stl) zj = a.x0[b * a.x0_sb + jx] - XU.at(0)[jx * SS];
    // Stage data FD stages ahead in a ring of register slots (the stage loop is unrolled by FD so
    // every slot is a fixed register set, loaded at the end of the stage that consumed it and used
    // FD - 1 stages later): own ybar component; one row (a state lane's ABT2 row: the variable
    // columns of row jx of [A|B] and the gap; an input lane's KR2 row: row ju of K and k_ju);
    // input lanes whose component is fixed
    // at the stage: row ju of the stage Hessian with h_u.  The raw vectors stay in the slot until
    // use: moving them on arrival would make the compiler wait for the loads right away.
    // (The Hessian rows, needed at few stages, come one stage ahead through a single slot.)
    constexpr int FD = BOX ? MPCB_AS_FDEPTH : MPCB_FWD_FDEPTH;
    constexpr int FL = KR2_W;
    T pv[FD][FL], pyb[FD], pgp[FD], pg[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) pg[i] = T(0);   // (a free component's row is never loaded)
    auto rload = [&](int k, auto slot_tag) {
      constexpr int sl = decltype(slot_tag)::value;
      pyb[sl] = XU.at(k)[j * SS];
      // one load for both kinds of lane, from a per-lane address: an input lane's KR2 row (13
      // elements used), a state lane's 10-element ABT2 row followed by the next row or record,
      // or by the workspace padding; 8-B vectors in fp32 (rows start 8-B aligned), 16-B in fp64
      ldv<T, FL, sizeof(T) == 8 ? 16 : 8>(stl ? ABT.at(k) + jx * ABT2_W : KR.at(k) + ju * KR2_W, pv[sl]);
      if (iterate) pgp[sl] = GP.at(k)[jx * SS];   // state lanes: gap_jx (input lanes: unused)
    };
    auto gload = [&](int k) {
      // (the 17 used elements only: loading the row's 3 pad elements too left registers the
      // compiler reused as temporaries while the load was in flight -- a vmcnt(0) wait per stage)
      if (BOX && (((lowm | upm) >> k) & 1u)) {
        ldv<T, 16>(GH.at(k) + ju * 20, pg);
        pg[NZ] = GH.at(k)[ju * 20 + NZ];
      }
    };
    // a converged group rides along with its wave's other groups: its loads are skipped and its
    // results (garbage) neither written nor used
    const bool fetch = !BOX || !done;
    if constexpr (!REF) {   // (the refinement kernel has no fp32 forward pass: the refinement's
                            // correction from the previous point is this set's Newton step)
      if (fetch) gload(0);
      static_for<FD>([&](auto s) { rload(decltype(s)::value < N ? decltype(s)::value : N - 1, s); });
    }
    auto stage = [&](int k, auto slot_tag) {
      constexpr int sl = decltype(slot_tag)::value;
      // the lane's row of the dot below: a state lane's row of [A|B] (variable columns loaded,
      // constant ones crow); an input lane's row of the stage Hessian with h_u (box), loaded where
      // its component is fixed -- elsewhere the multiplier it yields is never read, so the row
      // is whatever the slot held (no select on the fixed set), and without the box the input
      // lanes' dot result is not used at all (no selects)
      T row[NZ];
      if constexpr (BOX) {
#pragma unroll
        for (int t = 0; t < NVAR; ++t) row[var_col(t)] = csel(mst, pv[sl][t], pg[var_col(t)]);
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          row[p] = csel(mst, crow[p], pg[p]);
          row[6 + p] = csel(mst, crow[3 + p], pg[6 + p]);
        }
      } else {
#pragma unroll
        for (int t = 0; t < NVAR; ++t) row[var_col(t)] = pv[sl][t];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          row[p] = crow[p];
          row[6 + p] = crow[3 + p];
        }
      }
      const T r0 = csel(mst, iterate ? pgp[sl] : T(0), BOX ? pg[NZ] : T(0));
      const T yb = pyb[sl];
      ASTAMP(4);
      // du = k + K dx (input lanes; dx_i broadcast from state lane i)
      {
        T acc[4] = {pv[sl][NX], T(0), T(0), T(0)};
        T krow[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) krow[i] = pv[sl][i];
        dot12(acc, zj, krow);
        zj = csel(mst, zj, sum4(acc));
      }
      const T yo = yb + zj;   // state lanes: x_k = xbar_k + dx_k; input lanes: u_k
      // (Measured and dropped, round 6: a projected first pass -- a component beyond its bound
      // clamped as the pass goes -- cut c4's forward passes 3.83 -> 3.48 per instance and its
      // backward stages 1 %, the kernel time not at all (3.19 vs 3.20 ms), and its fuller first
      // violation sets sent 120 instead of 26 of the 192 hard wind + sine draws to the fallback.)
      if (stage_out) {
        if (stl) xs[k * NX + jx] = yo;
        else us[k * NU + ju] = yo;
      } else if (write) {
        if (stl) {
          if (a.X) a.X[(b * (N + 1) + k) * NX + jx] = yo;
        } else {
          if (a.U) a.U[(b * N + k) * NU + ju] = yo;
          if (k == 0) a.u0[b * NU + ju] = yo;
        }
      }
      ASTAMP(5);
      // every lane: r0 + row . z  (state lanes dx_{k+1}; input lanes the multiplier mu)
      T acc[4] = {r0, T(0), T(0), T(0)};
      dot16(acc, zj, row);
      const T v = sum4(acc);
      const bool lo = !stl && ((lowm >> k) & 1u), hi = !stl && ((upm >> k) & 1u);
      T tol_mu = T(0);
      // the rounding bound of mu matters only where its sign is wrong for its side (elsewhere
      // the test below fails whatever the tolerance): computed only when some lane of the wave
      // has such a multiplier (wave-uniform: the DPP block needs whole rows).  fp32: wherever a
      // component is fixed, since a right-sign multiplier within the bound is undecided too (the
      // fp32 Riccati form carries errors of 0.35 tol_mu by stage 2 of 30)
      if (BOX && __builtin_amdgcn_ballot_w64(UNC ? (lo || hi) : ((lo && v < T(0)) || (hi && v > T(0))))) {
        T aa[4] = {T(fabs(r0)), T(0), T(0), T(0)};
        dot16abs(aa, zj, row);
        tol_mu = T(64) * eps * sum4(aa);
      }
      if (!stl) {
        const bool fr = !(lo || hi);
        const T mu = v;
        // violations beyond the rounding noise of u and mu (see mpcb_box.hip)
        vlo |= (M)(fr && yo < lbm - tol_u) << k;
        vhi |= (M)(fr && yo > ubm + tol_u) << k;
        vfl |= (M)(lo && mu < -tol_mu) << k;
        vfu |= (M)(hi && mu > tol_mu) << k;
        if constexpr (UNC) unc = unc || ((lo || hi) && fabs(mu) <= tol_mu);
      } else {
        zj = v;
      }
      // the next stage's Hessian rows (fixed components only), then this slot's refill FD stages
      // ahead from every lane (the tail reloads stage N - 1, unused): in this order the waits for
      // both stay exact
      if (k + 1 < N && fetch) gload(k + 1);
      rload(k + FD < N ? k + FD : N - 1, slot_tag);
      ASTAMP(6);
    };
    if constexpr (!BOX) AS_WT(1);
    for (int k0 = 0; k0 < (REF ? 0 : N); k0 += FD) {
      static_for<FD>([&](auto s) {
        if (k0 + decltype(s)::value < N) stage(k0 + decltype(s)::value, s);
      });
    }
    if constexpr (!BOX) AS_WT(2);
    // outputs of this pass: staged rows leave as 16-B vectors once the pass is known to be final
    // (the unconstrained pass; the active-set pass that converged or used the last iteration)
    if (!REF && stage_out && stl) xs[N * NX + jx] = XU.at(N)[jx * SS] + zj;
    auto flush_out = [&]() {
      wave_lds_sync();
      constexpr int V = 16 / sizeof(T);
      typedef T Vec __attribute__((ext_vector_type(V)));
      const int nx = (N + 1) * NX, nu = N * NU;
      if (a.X) {
        Vec* dst = reinterpret_cast<Vec*>(a.X + b * nx);
        const Vec* src = reinterpret_cast<const Vec*>(xs);
        for (int t = j; t < nx / V; t += NZ) dst[t] = src[t];
      }
      if (a.U) {
        Vec* dst = reinterpret_cast<Vec*>(a.U + b * nu);
        const Vec* src = reinterpret_cast<const Vec*>(us);
        for (int t = j; t < nu / V; t += NZ) dst[t] = src[t];
      }
      if (!stl) a.u0[b * NU + ju] = us[ju];
      u0fin = true;
#pragma unroll
      for (int m = 0; m < NU; ++m) u0fin = u0fin && isfin(us[m]);
    };
    if (!stage_out && write && a.X && stl) a.X[(b * (N + 1) + N) * NX + jx] = XU.at(N)[jx * SS] + zj;
    if (!BOX && stage_out && write) flush_out();
    if constexpr (!BOX) break;

    // ------------------------------------------------ fp64-residual refinement + KKT verification (fp32 box)
    // (REF kernel: every pass.)  A converged fp32 pass with a fixed component whose multiplier lies
    // within its rounding bound tol_mu = 64 eps sum|terms| has not decided that component: the Riccati-form multiplier
    // h_u + G_ux dx + G_uu du sums terms ~10 that cancel to ~1e-4, while the component's curvature
    // can be as small as s R (1.7e-3 at the last stage), so an undecided multiplier of -8e-5 leaves
    // u 0.03 N off the minimiser.  c4 (tools/c4_full_parity.py): 24 of 65,536 instances beyond 5e-5
    // in U, each with one component fixed at a bound that the exact solution leaves free.  Neither
    // the fp32 data nor the rollout is the cause (the exact QP on the device's fp32 [A|B] is 1.8e-7
    // off; an fp64 rollout changes nothing: tools/box_verify_debug.py): the fp32 solve's own error
    // in the free components (~1e-3 N) moves the gradient at the fixed ones by ~8e-5.  So:
    //   r = 0  refinement: the objective's exact gradient g at the pass's U in fp64 over the same
    //          fp32 stage data (states re-simulated from U, then the adjoint sweep
    //          lambda_N = QN e_N, g_k = [A|B]_k^T lambda_{k+1} + s blkdiag(Q, R)(e_k, u_k - uref_k)),
    //          then the correction d = -H_FF^{-1} g_F on the free components by the fp32 Riccati
    //          recursion of the same set (P_{k+1} from the PS2 snapshots, which hold the current
    //          set's value function: the linear-term recursion only, no gap, d x_0 = 0) and a
    //          forward pass with the stored gains (KR2): U += d;
    //   r = 1  verification: g again at the refined U.  Fixed components whose multiplier has the
    //          wrong sign beyond 2^-20 of its terms' sum (~0.3) and free components beyond their
    //          bound by more than tol_u are this pass's violation sets, in place of the fp32
    //          forward pass's (which is what cannot decide them: after a release the fp32 pass
    //          put the released component back below its bound, and 27 of 157 c4 instances
    //          cycled), and the Kim-Park update below proceeds on them.
    // The active-set kernel lists the instances whose converged set has an undecided multiplier
    // (as_ref_put); the refinement kernel restores each set, redoes its final forward pass and runs
    // every further pass this way.  Each refinement is counted as five forward passes (its sweeps) in qp_stats.
    // The output X of a refined instance is the fp64 re-simulation of its U.
    // Oracle: oracle.ocp.pdas_solve (the exact-arithmetic active set).
    if constexpr (VER) {
      const bool ver = write;
      if (__builtin_amdgcn_ballot_w64(ver)) {   // (wave-uniform: the DPP blocks need whole rows)
        // the refinement's stage loops read their records one stage at a time (no prefetch ring):
        // bring the group's records into L2 first, all loads in flight at once (lane j touches
        // stages j, j + 16, ...: one dword per 128-B line), so those loops wait on L2, not HBM
        if (ver) {
          T acc = T(0);
          for (int k = j; k <= N; k += 16) {
            T v[16];
            const int kk = k < N ? k : N - 1;
            const T* ab = ABT.at(kk);
            const T* kr = KR.at(kk);
            const T* ps = PS.at(kk);
            const T* xu = XU.at(k);
            v[0] = ab[0]; v[1] = ab[32]; v[2] = ab[64]; v[3] = ab[96]; v[4] = ab[ABT2_REC - 1];
            v[5] = kr[0]; v[6] = kr[32]; v[7] = kr[KR2_REC - 1];
            v[8] = ps[0]; v[9] = ps[32]; v[10] = ps[64]; v[11] = ps[PS2_REC - 1];
            v[12] = xu[0]; v[13] = xu[32];
            v[14] = iterate ? GP.at(kk)[0] : T(0);
            v[15] = xr[(int64_t)k * NX];
#pragma unroll
            for (int i = 0; i < 16; ++i) acc += v[i];
          }
          asm volatile("" ::"v"(acc));
        }
        RefIn<W32> in{a.x0 + b * a.x0_sb, XU, GP, ABT, KR, PS, cbase, cstride, refp, refs, xrN, W.QN,
                      SW, PX, xs, us, us + N * NU, us + 2 * N * NU,
                      {crow[0], crow[1], crow[2], crow[3], crow[4], crow[5]},
                      lowm, upm, lbm, ubm, tol_u, N, iterate, ver};
        const RefOut<W32> ro = refine_verify<W32>(in);
        // after REF_PASSES refined passes the multiplier verdicts are dropped: a component whose
        // release and re-fix alternate (a 2-cycle on 20 of 157 c4 instances: the exact multiplier
        // +1.7e-6, within the refinement's accuracy on fp32 data) stays at its bound, which moves
        // the solution by |mu| / s R ~ 1e-3 N at most
        // a component released and then found beyond its bound again is pinned at it (the 2-cycle)
        const M rd = (rpass < REF_PASSES ? ro.rd : M(0)) & ~pin, alo = ro.alo, ahi = ro.ahi;
        ++rpass;
        pin |= (alo | ahi) & relm;
        relm |= rd;
        // the previous pass's releases all came back (beyond their bounds) and nothing else
        // changed: the set is the one before them, whose refined rows were kept -- finish with
        // those instead of refactoring the set once more (the slowest c4 instances' third pass)
        {
          T* const ubk = us + 2 * N * NU + (N + 1) * NX;
          T* const xbk = ubk + N * NU;
          const int mine = (stl || (rd == 0 && (alo | ahi) == lrel)) ? 1 : 0;
          const int anyr = (!stl && lrel != 0) ? 1 : 0;
          const bool undo = ((bc<NX + 0>(mine) & bc<NX + 1>(mine)) & (bc<NX + 2>(mine) & bc<NX + 3>(mine))) &&
                            ((bc<NX + 0>(anyr) | bc<NX + 1>(anyr)) | (bc<NX + 2>(anyr) | bc<NX + 3>(anyr)));
          const int rel_o = (!stl && rd != 0) ? 1 : 0;
          const bool releases = (bc<NX + 0>(rel_o) | bc<NX + 1>(rel_o)) | (bc<NX + 2>(rel_o) | bc<NX + 3>(rel_o));
          wave_lds_sync();
          if (ver && undo) {
            for (int e = j; e < N * NU; e += NZ) us[e] = ubk[e];
            for (int e = j; e < (N + 1) * NX; e += NZ) xs[e] = xbk[e];
            lowm |= alo;
            upm |= ahi;
          } else if (ver && releases) {
            for (int e = j; e < N * NU; e += NZ) ubk[e] = us[e];
            for (int e = j; e < (N + 1) * NX; e += NZ) xbk[e] = xs[e];
          }
          wave_lds_sync();
          lrel = (ver && releases && !undo) ? rd : M(0);
          if (ver && undo) rpass = -1;   // (marker: converged by the undo, below)
        }
#if defined(MPCB_REF_TRACE) && defined(MPCB_AS_OWNER)   // (diagnostic builds: the passes of chunk instance MPCB_REF_TRACE)
        if (ver && c == MPCB_REF_TRACE && git < 128) {
          if (!stl) {
            int* t = g_ref_trace[git] + 5 * ju;
            t[0] = (int)(uint32_t)lowm; t[1] = (int)(uint32_t)upm;
            t[2] = (int)(uint32_t)rd; t[3] = (int)(uint32_t)alo; t[4] = (int)(uint32_t)ahi;
          }
        }
#endif
        if (ver) {
          n_fwd += ro.sweeps;
          const bool und = rpass < 0;
          if (und) rpass = REF_PASSES;
          vlo = und ? M(0) : alo;
          vhi = und ? M(0) : ahi;
          vfl = und ? M(0) : rd & lowm;
          vfu = und ? M(0) : rd & upm;
        }
      }
    }
    // ------------------------------------------------ active-set update (Kim-Park)
    const M V = vlo | vhi | vfl | vfu;
    const int cnt = stl ? 0 : Mk::popc(V);
    const int firstk = (!stl && V) ? Mk::ffs(V) - 1 : WB;
    int nV, first;
    {
      const int c0 = bc<NX + 0>(cnt), c1 = bc<NX + 1>(cnt), c2 = bc<NX + 2>(cnt), c3 = bc<NX + 3>(cnt);
      nV = (c0 + c1) + (c2 + c3);
      const int f0 = bc<NX + 0>(firstk) * NU + 0, f1 = bc<NX + 1>(firstk) * NU + 1;
      const int f2 = bc<NX + 2>(firstk) * NU + 2, f3 = bc<NX + 3>(firstk) * NU + 3;
      const int fa = f0 < f1 ? f0 : f1, fb = f2 < f3 ? f2 : f3;
      first = fa < fb ? fa : fb;
    }
    const bool gconv = nV == 0;
    const bool full = (nV < best) || (pcount > 0);
    pcount = (nV < best) ? 3 : (full ? pcount - 1 : pcount);
    best = nV < best ? nV : best;
    const M selm = full ? V : ((first < WB * NU && (first % NU) == ju && !stl) ? (M(1) << (first / NU)) : M(0));
    const M nlow = (lowm | (selm & vlo)) & ~(selm & vfl);
    const M nup = (upm | (selm & vhi)) & ~(selm & vfu);
    const M diff = stl ? M(0) : ((nlow ^ lowm) | (nup ^ upm));
    M changed = (bc<NX + 0>(diff) | bc<NX + 1>(diff)) | (bc<NX + 2>(diff) | bc<NX + 3>(diff));
    if (!done && !gconv) {
      if constexpr (REF) {   // the refinement starts the next set from this point: fixed at the bounds
        if (!stl) {
          const M nf = (nlow | nup) & ~(lowm | upm);
          for (int k = 0; k < N; ++k)
            if ((nf >> k) & 1u) us[k * NU + ju] = ((nlow >> k) & 1u) ? lbm : ubm;
        }
      }
      lowm = nlow;
      upm = nup;
    } else {
      changed = 0;
    }
    // restart at kc + 1 from the snapshot there: the last pass that recomputed that stage, or
    // (never recomputed: its active set is still empty) P2's unconstrained pass
    kc = changed ? WB - 1 - Mk::clz(changed) : -1;
    const bool cvd = gconv;   // converged (the refinement kernel: on the refined violation sets)
    // the instance is finished: converged, or the pass cap
    // (or, with the fallback, the first pass violates more than 7/20 of the horizon's input
    // components: oracle.ocp.AS_IPM_NV_NUM / _DEN, a strongly constrained QP)
    const bool crowded = BOX && a.as_fb && git == 0 && nV * AS_IPM_NV_DEN > AS_IPM_NV_NUM * N * NU;
    const bool fin_now = write && (cvd || git + 1 >= a.max_as_iter || crowded);
    if (stage_out && fin_now) flush_out();
    wave_lds_sync();   // the next pass's staging writes follow the flush's LDS reads
    ++git;
    if (fin_now) {
      // not converged within the pass budget (min(max_as_iter, AS_IPM_AFTER), mpcb_capi.hip): the
      // interior point takes the instance over (mpcb_asipm.h, oracle.ocp.pdas_solve) unless a
      // factorisation failed; the status is then the fallback's to write
      const bool to_ipm = BOX && !REF && !cvd && st == MPCB_STATUS_OK && a.as_fb;
      if (to_ipm) {
        if (j == 0) a.as_fb[2 + atomicAdd(a.as_fb, 1)] = (int)c;
      } else if (!cvd) {
        st = (st == MPCB_STATUS_OK) ? MPCB_STATUS_MAXITER : st;
      }
      if constexpr (UNC && !REF) {
        // a converged set with an undecided multiplier: listed for the refinement kernel (its
        // outputs are written here as well, and overwritten there)
        // ... or whose first-stage controls are all below AS_REF_U0 (the test's normwise error of
        // u0 divides by max(|u0|, 1): there fp32's ~1e-4 N absolute error counts in full -- 6 of
        // c4's 65,536 instances beyond 5e-5, all with |u0| < 1.5 N; 95 have |u0| < 2 N)
        const int so = (!stl && fabs(us[ju]) < T(AS_REF_U0)) ? 1 : 0;
        const bool small = (bc<NX + 0>(so) & bc<NX + 1>(so)) & (bc<NX + 2>(so) & bc<NX + 3>(so));
        const int un = unc ? 1 : 0;
        // ... or that took AS_REF_PASSES passes or more: the hard QPs, where the fp32 solve's own
        // error grows (the hard wind + sine draws: 10-34-pass instances 6e-5 to 1.2e-4 off at an
        // fp32 data sensitivity of 4e-6 to 9e-6; listing from 6 passes on instead -- 4,544 of
        // c4's 65,536 -- took the refinement kernel from 0.33 to 0.47 ms)
        // ... or whose converged set fixes AS_REF_FIX_NUM / AS_REF_FIX_DEN of the horizon's input
        // components or more: a strongly constrained QP, on which the fp32 solve's error in the
        // free components grows (sweep cases 65 / 112, sine references: 4-9 passes, 32-68 % fixed,
        // 5.1e-5 to 1.4e-4 off; no c4 instance fixes more than 24 %)
        const int nf = stl ? 0 : Mk::popc(lowm | upm);
        const bool crowdf = ((bc<NX + 0>(nf) + bc<NX + 1>(nf)) + (bc<NX + 2>(nf) + bc<NX + 3>(nf))) * AS_REF_FIX_DEN >=
                            AS_REF_FIX_NUM * N * NU;
        const bool lst = cvd && a.as_ref &&
                         (small || crowdf || git >= AS_REF_PASSES ||
                          ((bc<NX + 0>(un) | bc<NX + 1>(un)) | (bc<NX + 2>(un) | bc<NX + 3>(un))));
        if (lst) {   // (group-uniform: the row broadcast below has its 16 lanes)
          int t = 0;
          if (j == 0) t = atomicAdd(a.as_ref, 1);
          t = bc<0>(t);
          if (t < a.as_ref_cap) {
            int* const e = a.as_ref + AS_REF_HDR + (int64_t)t * AS_REF_W;
            as_ref_put<W32>(e, j, (int)c, git, n_fwd, n_bst, lowm, upm);
            if (j == 0) e[AS_REF_KC] = -1;   // (its factorisation is the converged pass's)
          }

        }
      }
      finish(!to_ipm);
      // the next instance of the chunk (lane 0 of the group draws it), else the group stays empty
      int nxt = (int)nb;
      if constexpr (REF) {
        if (j == 0) nxt = (int)gridDim.x * GROUPS + atomicAdd(a.as_ref + 1, 1);
        nxt = bc<0>(nxt);
      } else if (a.as_queue) {
        if (j == 0) nxt = (int)gridDim.x * GROUPS + atomicAdd(a.as_queue, 1);
        nxt = bc<0>(nxt);
      }
      bind(nxt);
      lowm = upm = 0;
      st = MPCB_STATUS_OK;
      best = 0x7fffffff;
      pcount = 3;
      n_fwd = n_bst = 0;
      kc = -1;
      git = 0;
      restore();
      u0fin = true;
      done = !valid;
    } else if (!valid) {
      done = true;
    }
    if (__all(done)) break;
  }
#ifdef MPCB_AS_STAMPS
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int i_ = 0; i_ < 12; ++i_) g_astamps[i_] = ast_acc[i_];
#endif
  if constexpr (!BOX) finish(true);   // (the box kernel finishes each instance as it converges)
  if constexpr (!BOX) AS_WT(3);
}

}  // namespace asq
}  // namespace mpcb
