// mpcb_common.h — device helpers shared by the solve kernels (internal).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "mpcb_kernels.h"

namespace mpcb {

// Row strides of the per-lane LDS rows written by all 16 lanes of a group at once: NX + 1 and
// NU + 1 put the 16 rows on distinct bank pairs (ds_write_b64 / ds_write_b32 bank = dword mod 32;
// the unpadded 12- and 4-element rows were 4-way conflicts: SQ_LDS_BANK_CONFLICT 54 % of P2's
// LDS cycles at c2, profiles/pmc_c2.json).
constexpr int XS = NX + 1, HS = NU + 1;
template <class T>
struct GroupLds {
  T P[NX * NX];   // value-function Hessian, P[l*NX + i] = column l (symmetric)
  T X[NZ * XS];   // X[j*XS + i] = ([A|B])_{i j} (split path; the other kernels use stride NX)
  T Hu[NZ * HS];  // Hu[j*HS + m] = G_{NX+m, j}   (H_ux columns, then H_uu; split path stride)
  T v[NZ];        // vector exchange (e = ybar - yref, then pt = p + P b)
  T hv[NZ];       // gradient h = [h_x; h_u]
};

// Per-lane record in the workspace, per stage: 4 gain values (+ box-mode extras).
template <int BOX> struct Rec { static constexpr int n = BOX ? 24 : 4; };

// LDS ordering inside a single-wavefront workgroup.  A wave's LDS instructions execute and return
// in issue order, so a later ds_read sees every earlier ds_write of the same wave with no barrier
// and no lgkmcnt(0) drain; only the compiler must keep the program order of the LDS accesses,
// which this (code-free) memory clobber does.  __syncthreads() would drain every outstanding LDS
// operation at each exchange.  Valid only for 64-thread (one-wave) workgroups.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("" ::: "memory"); }

// Diagnostic builds only (-DMPCB_STAMPS): per-wave timeline of a kernel in its translation unit's
// table, s_memrealtime (100 MHz, one clock for the whole chip) at slot 0 entry, 1 loop start,
// 2 loop end, 3 exit; lane 0 of each of the first 4096 workgroups writes it (a vector store).
#ifdef MPCB_STAMPS
// waves recorded per kernel (c3 / c5 P2: 16384 / 32768 one-wave workgroups)
#ifndef MPCB_WT_MAX
#define MPCB_WT_MAX 32768
#endif
// slots 5, 6 (entries MPCB_WT_MAX * (4 + slot) + wg): s_memtime, the shader-clock counter, at loop
// start and end, so a wave's clock is (slot-6 - slot-5 cycles) / (its loop's realtime)
#define WT_TABLE(name) __device__ unsigned long long name[MPCB_WT_MAX * 7];
// slot 4 of the table (entries MPCB_WT_MAX * 4 + wg): the wave's HW_ID (SIMD, CU, SE) and XCC_ID
#define WT_HW(name)                                                                 \
  {                                                                                 \
    const unsigned hw_ = __builtin_amdgcn_s_getreg(63492), xcc_ = __builtin_amdgcn_s_getreg(63508); \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < MPCB_WT_MAX)                        \
      name[MPCB_WT_MAX * 4 + blockIdx.x] = ((unsigned long long)xcc_ << 32) | hw_; \
  }
#define WT(name, slot)                                                              \
  {                                                                                 \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                 \
    const unsigned long long c_ = __builtin_amdgcn_s_memtime();                     \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < MPCB_WT_MAX) {                      \
      name[blockIdx.x * 4 + (slot)] = t_;                                           \
      if ((slot) == 1 || (slot) == 2) name[MPCB_WT_MAX * (4 + (slot)) + blockIdx.x] = c_; \
    }                                                                               \
  }
#else
#define WT_TABLE(name)
#define WT(name, slot)
#define WT_HW(name)
#endif

// f(std::integral_constant<int, i>{}) for i = 0 .. n-1 (compile-time lane indices for DPP)
template <int n, class F, int i = 0> __device__ __forceinline__ void static_for(F&& f) {
  if constexpr (i < n) {
    f(std::integral_constant<int, i>{});
    static_for<n, F, i + 1>(static_cast<F&&>(f));
  }
}

// Identity that LLVM cannot see through (keeps selects of array elements as selects).
template <class T> __device__ __forceinline__ T opq(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Per-lane m ? a : b for a lane mask m held in SGPRs (m = ballot of the condition): one
// v_cndmask_b32 per dword.  A C++ ?: on values the compiler cannot speculate (the results of
// asm statements) becomes exec-masked branches; on array elements InstCombine may fold it into a
// load from a selected address (a dynamically indexed scratch array).  This is neither.
__device__ __forceinline__ unsigned cnd32(uint64_t m, unsigned a, unsigned b) {
  unsigned r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
  return r;
}
template <class T> __device__ __forceinline__ T csel(uint64_t m, T a, T b) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "csel: 32- or 64-bit values");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, cnd32(m, __builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b)));
  } else {
    const unsigned long long ua = __builtin_bit_cast(unsigned long long, a);
    const unsigned long long ub = __builtin_bit_cast(unsigned long long, b);
    const unsigned lo = cnd32(m, (unsigned)ua, (unsigned)ub);
    const unsigned hi = cnd32(m, (unsigned)(ua >> 32), (unsigned)(ub >> 32));
    return __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
  }
}
__device__ __forceinline__ uint64_t lane_mask(bool c) { return __builtin_amdgcn_ballot_w64(c); }

// x is finite (one v_cmp_class).  Not (x - x) == 0: when x is a product formed in the same
// expression, FMA contraction turns x - x into fma(a, b, -x) = the product's rounding error, and
// a finite x then reads as non-finite (it did, in the 17/6 interior point's step test).
template <class T> __device__ __forceinline__ bool isfin(T x) { return __builtin_isfinite(x); }

// a[j] (0 <= j < n <= 16) for a register array: a bit-tree of csel on the bits of j.
template <int n, int bit, class T> __device__ __forceinline__ T sel_level(const T* a, int j) {
  if constexpr (n == 1) {
    return a[0];
  } else {
    constexpr int w = (n + 1) / 2;
    const uint64_t m = lane_mask((j >> bit) & 1);
    T l[w];
#pragma unroll
    for (int i = 0; i < w; ++i) l[i] = csel(m, a[(2 * i + 1 < n) ? 2 * i + 1 : n - 1], a[2 * i]);
    return sel_level<w, bit + 1>(l, j);
  }
}
template <int n, class T> __device__ __forceinline__ T sel(const T* a, int j) {
  static_assert(n >= 1 && n <= 16, "sel: 1..16 elements");
  return sel_level<n, 0>(a, j);
}

// 1 / sqrt(x) from the hardware estimate v_rsq refined by Newton steps: fp32 one (~1 ulp; sqrtf and
// an IEEE division were ~13 instructions per pivot), fp64 two (~1 ulp, a fraction of the
// instructions of sqrt + an IEEE division).  A non-positive pivot still yields NaN/inf, which the
// callers' status checks catch.  MPCB_IEEE_DIV=1 restores sqrt + division in fp32.
#ifndef MPCB_IEEE_DIV
#define MPCB_IEEE_DIV 0
#endif
__device__ __forceinline__ float inv_sqrt(float x) {
#if MPCB_IEEE_DIV
  return 1.0f / sqrtf(x);
#else
  const float r = __builtin_amdgcn_rsqf(x);
  return r * fmaf(-0.5f * x * r, r, 1.5f);
#endif
}
__device__ __forceinline__ double inv_sqrt(double x) {
  double r = __builtin_amdgcn_rsq(x);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double e = fma(-x * r, r, 1.0);   // 1 - x r^2
    r = fma(0.5 * r, e, r);
  }
  return r;
}

template <class T>
__device__ __forceinline__ void chol4(const T H[16], T L[10]) {
  // L packed lower: L00 L10 L11 L20 L21 L22 L30 L31 L32 L33 (diagonal holds 1/L_ii)
  T i00 = inv_sqrt(H[0]);
  T l10 = H[4] * i00, l20 = H[8] * i00, l30 = H[12] * i00;
  T i11 = inv_sqrt(H[5] - l10 * l10);
  T l21 = (H[9] - l20 * l10) * i11, l31 = (H[13] - l30 * l10) * i11;
  T i22 = inv_sqrt(H[10] - l20 * l20 - l21 * l21);
  T l32 = (H[14] - l30 * l20 - l31 * l21) * i22;
  T i33 = inv_sqrt(H[15] - l30 * l30 - l31 * l31 - l32 * l32);
  L[0] = i00; L[1] = l10; L[2] = i11; L[3] = l20; L[4] = l21; L[5] = i22;
  L[6] = l30; L[7] = l31; L[8] = l32; L[9] = i33;
}

template <class T>
__device__ __forceinline__ void chol4_solve(const T L[10], const T b[4], T x[4]) {
  // forward L y = b, backward L^T x = y
  T y0 = b[0] * L[0];
  T y1 = (b[1] - L[1] * y0) * L[2];
  T y2 = (b[2] - L[3] * y0 - L[4] * y1) * L[5];
  T y3 = (b[3] - L[6] * y0 - L[7] * y1 - L[8] * y2) * L[9];
  x[3] = y3 * L[9];
  x[2] = (y2 - L[8] * x[3]) * L[5];
  x[1] = (y1 - L[4] * x[2] - L[7] * x[3]) * L[2];
  x[0] = (y0 - L[1] * x[1] - L[3] * x[2] - L[6] * x[3]) * L[0];
}

template <int n, class T>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const T* v) {
#pragma unroll
  for (int i = 0; i < n; ++i) p[i] = v[i];
}

// per (interval, instance) record: 80 linearisation scalars, 12 gap values, 4 pad
constexpr int CC_REC = LIN_STAGE + 16;

template <int n, class T>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, T* out) {
#pragma unroll
  for (int i = 0; i < n; ++i) out[i] = p[i];
}

}  // namespace mpcb
