// mpcb_split.h — pieces shared by the split-path kernels (mpcb_split.hip, mpcb_box.hip): the
// fp32 MFMA block contractions of the 16-lane Riccati layout and the quad-blocked workspace.
#pragma once
#include <hip/hip_runtime.h>

#include "mpcb_common.h"

namespace mpcb {

// ---- fp32 MFMA block contractions (gfx950 v_mfma_f32_16x16x1_4b_f32) -------------------------
// With 4 instances per wave and lane (q, j) owning column j of instance q's 16x16 tiles, the
// 4-block outer-product MFMA computes C_q += a_q (x) b_q for all four instances at once, where
// lane (q, i) supplies a_q[i] and lane (q, j) supplies b_q[j]: a K=12 contraction is 12 MFMAs
// and needs NO operand movement.  The accumulator comes back in the standard 16x16 layout per
// block (lane 16g+jj, register 4b+r  <->  C_b[4g+r][jj]); ``to_columns`` transposes (lane group,
// register block) with permlane32/16 swaps so lane (q, j) again holds column j of C_q.
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void swap32(float& x, float& y) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  x = __uint_as_float(r[0]);
  y = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& x, float& y) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  x = __uint_as_float(r[0]);
  y = __uint_as_float(r[1]);
}

// acc (MFMA layout) -> out[i] = C_q[i][j] in lane (q, j), i = 0..15
__device__ __forceinline__ void to_columns(const v16f& acc, float out[16]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float R0 = acc[r], R1 = acc[4 + r], R2 = acc[8 + r], R3 = acc[12 + r];
    swap32(R0, R2);
    swap32(R1, R3);
    swap16(R0, R1);
    swap16(R2, R3);
    out[r] = R0;
    out[4 + r] = R1;
    out[8 + r] = R2;
    out[12 + r] = R3;
  }
}

// C_q = sum_{l<12} a_q[:, l] (x) b_q[l, :]   (a, b: this lane's 12 values of row/col l)
__device__ __forceinline__ v16f outer12(const float a[12], const float b[12]) {
  v16f acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int l = 0; l < 12; ++l) acc = __builtin_amdgcn_mfma_f32_16x16x1f32(a[l], b[l], acc, 0, 0, 0);
  return acc;
}

// ---- fp64 row-broadcast FMAs (gfx950 DPP64: v_fmac_f64_dpp ... row_newbcast:L) -------------
// Lane L of every 16-lane row (= one instance of the Riccati layout) broadcasts its src0 to the
// whole row inside the FMA itself, so the fp64 block contractions read their operands from the
// owning lanes' registers instead of LDS (the LDS products were bound by the CU's LDS bandwidth:
// every lane read all of P and [A|B] each stage).  One asm block per broadcast pattern; the
// leading s_nop covers the VALU-write -> DPP-read and EXEC-write -> DPP wait states that the
// compiler's hazard recognizer does not insert for inline asm (DPP sources are never written
// inside a block).
#define MPCB_BC(d, s, b, l) \
  "v_fmac_f64_dpp %" #d ", %" #s ", %" #b " row_newbcast:" l " row_mask:0xf bank_mask:0xf\n\t"

// acc[i] += bcast_L(a[i]) * b  (i < 12) and acc12 += bcast_L(a12) * b
template <int L>
__device__ __forceinline__ void fmac13_bc(double (&acc)[12], double& acc12, const double (&a)[12],
                                          double a12, double b) {
  asm("s_nop 4\n\t"
      MPCB_BC(0, 13, 26, "%c27") MPCB_BC(1, 14, 26, "%c27") MPCB_BC(2, 15, 26, "%c27")
      MPCB_BC(3, 16, 26, "%c27") MPCB_BC(4, 17, 26, "%c27") MPCB_BC(5, 18, 26, "%c27")
      MPCB_BC(6, 19, 26, "%c27") MPCB_BC(7, 20, 26, "%c27") MPCB_BC(8, 21, 26, "%c27")
      MPCB_BC(9, 22, 26, "%c27") MPCB_BC(10, 23, 26, "%c27") MPCB_BC(11, 24, 26, "%c27")
      MPCB_BC(12, 25, 26, "%c27")
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
        "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]),
        "+v"(acc12)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
        "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(a12), "v"(b), "i"(L));
}

// acc[i] += bcast_i(a) * b  (i < 16): lane i's a feeds accumulator i
__device__ __forceinline__ void fmac16_diag(double (&acc)[16], double a, double b) {
  asm("s_nop 4\n\t"
      MPCB_BC(0, 16, 17, "0") MPCB_BC(1, 16, 17, "1") MPCB_BC(2, 16, 17, "2")
      MPCB_BC(3, 16, 17, "3") MPCB_BC(4, 16, 17, "4") MPCB_BC(5, 16, 17, "5")
      MPCB_BC(6, 16, 17, "6") MPCB_BC(7, 16, 17, "7") MPCB_BC(8, 16, 17, "8")
      MPCB_BC(9, 16, 17, "9") MPCB_BC(10, 16, 17, "10") MPCB_BC(11, 16, 17, "11")
      MPCB_BC(12, 16, 17, "12") MPCB_BC(13, 16, 17, "13") MPCB_BC(14, 16, 17, "14")
      MPCB_BC(15, 16, 17, "15")
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
        "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]),
        "+v"(acc[12]), "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15])
      : "v"(a), "v"(b));
}

// acc[i] += bcast_i(a) * b for the 10 variable directions i = 3..5, 9..15 (mpcb_kernels.h var_col):
// the rows of G = [A|B]^T Y whose [A|B] column depends on the linearisation point
__device__ __forceinline__ void fmac10_var(double (&acc)[16], double a, double b) {
  asm("s_nop 4\n\t"
      MPCB_BC(0, 10, 11, "3") MPCB_BC(1, 10, 11, "4") MPCB_BC(2, 10, 11, "5")
      MPCB_BC(3, 10, 11, "9") MPCB_BC(4, 10, 11, "10") MPCB_BC(5, 10, 11, "11")
      MPCB_BC(6, 10, 11, "12") MPCB_BC(7, 10, 11, "13") MPCB_BC(8, 10, 11, "14")
      MPCB_BC(9, 10, 11, "15")
      : "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]),
        "+v"(acc[12]), "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15])
      : "v"(a), "v"(b));
}

// acc[i] += bcast_i(a) * b  (i < 12)
__device__ __forceinline__ void fmac12_diag(double (&acc)[12], double a, double b) {
  asm("s_nop 4\n\t"
      MPCB_BC(0, 12, 13, "0") MPCB_BC(1, 12, 13, "1") MPCB_BC(2, 12, 13, "2")
      MPCB_BC(3, 12, 13, "3") MPCB_BC(4, 12, 13, "4") MPCB_BC(5, 12, 13, "5")
      MPCB_BC(6, 12, 13, "6") MPCB_BC(7, 12, 13, "7") MPCB_BC(8, 12, 13, "8")
      MPCB_BC(9, 12, 13, "9") MPCB_BC(10, 12, 13, "10") MPCB_BC(11, 12, 13, "11")
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
        "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11])
      : "v"(a), "v"(b));
}
#undef MPCB_BC

// Quad-blocked SoA chunk layouts: instances are grouped in quads (the 4 instances of one P2
// wavefront); element i of the stage-k record of chunk instance c lives at
//   base[((k * nquad + c / 4) * REC + i) * 4 + c % 4],   element stride SS = 4.
// P2 reads a wavefront's whole stage record as one contiguous REC x 16 B tile (its 5-element
// prefetch per lane is 64 consecutive floats per instruction).  P1/P3 (thread per instance)
// touch 16 lines per instruction that the next 7 elements reuse from L1.  A plain [k][i][nb]
// SoA put every element on its own page and a 64-instance blocking spread each line over the
// 8 XCDs' L2s (measured 2.7 % L2 hit rate, ~10x over-fetch).
constexpr int SS = 4;
template <class T>
__device__ __forceinline__ T* soa(T* base, int k, int rec, int64_t nb, int64_t c) {
  const int64_t nq = (nb + SS - 1) / SS;
  return base + (((int64_t)k * nq + (c >> 2)) * rec) * SS + (c & (SS - 1));
}

// Row-major export records (mpcb_kernels.h AB2_REC ...): record of chunk instance c at stage k,
// instance-major (imaj: an instance's N records contiguous, so a 16-lane group walks one region
// stage by stage) or stage-major (stage k of every instance, then stage k + 1): SplitArgs::imajor.
template <class T>
__device__ __forceinline__ T* rec2(T* base, int k, int rec, int64_t nb, int64_t c, int N, int imaj) {
  const int64_t nq = (nb + SS - 1) / SS;
  return base + (imaj ? c * N + k : ((int64_t)k * nq + (c >> 2)) * SS + (c & (SS - 1))) * (int64_t)rec;
}

// n contiguous elements through VB-byte vector accesses (p VB-byte aligned, n * sizeof(T) % VB == 0)
template <class T, int n, int VB = 16> __device__ __forceinline__ void ldv(const T* __restrict__ p, T* v) {
  constexpr int W = VB / sizeof(T);
  static_assert(W >= 1 && (n % W) == 0, "ldv: whole vectors");
  typedef T V __attribute__((ext_vector_type(W)));
  const V* vp = reinterpret_cast<const V*>(p);
#pragma unroll
  for (int c = 0; c < n / W; ++c) {
    const V x = vp[c];
#pragma unroll
    for (int e = 0; e < W; ++e) v[c * W + e] = x[e];
  }
}
template <class T, int n> __device__ __forceinline__ void stv(T* __restrict__ p, const T* v) {
  constexpr int W = 16 / sizeof(T);
  static_assert((n % W) == 0, "stv: whole 16-B vectors");
  typedef T V __attribute__((ext_vector_type(W)));
  V* vp = reinterpret_cast<V*>(p);
#pragma unroll
  for (int c = 0; c < n / W; ++c) {
    V x;
#pragma unroll
    for (int e = 0; e < W; ++e) x[e] = v[c * W + e];
    vp[c] = x;
  }
}

}  // namespace mpcb
