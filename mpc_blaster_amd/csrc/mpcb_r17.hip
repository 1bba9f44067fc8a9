// mpcb_r17.hip — the 17/6 Riccati pass and its interior point in a 16-lane DPP layout
// (blastermodel.py:214-292, acados_ocp_blasterModel.json: N = 60, nx = 17,
// nu = 6).
//
// Layout.  Four instances per wavefront, 16 lanes each (one DPP row per instance), so every
// operand exchange inside an instance is a row broadcast folded into the consuming FMA
// (v_fmac_f{32,64}_dpp ... row_newbcast:L) — no LDS operands in the products.  The 23 columns of
// [A|B] do not fit 16 lanes, but 9 of them are structural (f17 does not depend on the position
// or POC states and is linear in the velocity, mpcb_full.hip lin17ws):
//   identity columns  AB[:, c] = e_c                 c in {0,1,2, 14,15,16}
//   shear columns     AB[:, 6+c] = e_{6+c} + h e_c + h Jp[:, c] e_poc
// Lane t holds column z(t) of [A|B]: the 14 dense columns (Euler angles 3-5, body rates 9-11,
// swivel angles 12-13, inputs 17-22) and the shear columns 6, 7; the third shear column (8) is
// implicit (its five nonzeros are read from the cached [A|B]).  Lane t also owns column s(t) of
// the value-function Hessian P: s = z for the state-column lanes 0-7, 14, 15, and the identity
// states 0,1,2,14,15,16 for the input lanes 8-13.  P's 17th column (state 8) is never held as an
// array: by symmetry it is the set of entries P[8, s(t)] across the lanes, plus P[8,8].
//
// Per stage (backward), for the four instances of a wave:
//   Y = P [A|B]_z          16 row-broadcast passes of a P column (+ the distributed column 8)
//   G_z = [A|B]^T Y_z      16 row-broadcast passes of [A|B] columns; identity rows are Y rows
//   Huu, h_u               input lanes' columns through a small LDS block
//   G for identity states  rows gathered from the other lanes' Y (LDS), the rest from P
//   K, k                   6x6 Cholesky per lane (redundant), own column of K
//   P_new = G + Hxu K      6 row-broadcast passes, then the symmetric exchange (LDS)
// Dense flop count per stage (tools/bench_full17.py): 39,316; the structural columns make the
// executed count about 60 % of that.
#include <hip/hip_runtime.h>

#include "../../include/mpcb.h"
#include "mpcb_common.h"
#include "mpcb_full.h"

// forward-pass ring depths (stages of row loads in flight): the unconstrained pass, the interior
// point's Newton-step pass
#ifndef MPCB_Q17_FD
#define MPCB_Q17_FD 3
#endif
#ifndef MPCB_Q17_FD_STEP
#define MPCB_Q17_FD_STEP 3
#endif

namespace mpcb {
namespace q17 {

constexpr int LN = 16, GR = 64 / LN;   // lanes per instance, instances per wavefront
#ifdef MPCB_Q17_STAMPS
// Diagnostic build only: per-region s_memtime deltas of workgroup 0, printed at the end.
#define QSTAMP_INIT() unsigned long long qs_prev = __builtin_amdgcn_s_memtime(), qs_acc[12] = {};
#define QSTAMP(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); qs_acc[i] += t_ - qs_prev; qs_prev = t_; }
#define QSTAMP_DONE(tag) if (blockIdx.x == 0 && threadIdx.x == 0) printf("QSTAMP %s %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", tag, \
    qs_acc[0], qs_acc[1], qs_acc[2], qs_acc[3], qs_acc[4], qs_acc[5], qs_acc[6], qs_acc[7], qs_acc[8], qs_acc[9], qs_acc[10], qs_acc[11]);
#else
#define QSTAMP_INIT()
#define QSTAMP(i)
#define QSTAMP_DONE(tag)
#endif
constexpr int OM = 8;                  // the state whose P column is held distributed

// lane t -> z column of [A|B] it holds, state column of P it owns; state i -> owning lane
__host__ __device__ constexpr int zcol(int t) { return t < 3 ? 3 + t : t < 8 ? 6 + t : t < 14 ? 9 + t : t - 8; }
__host__ __device__ constexpr int sown(int t) { return t < 8 ? zcol(t) : t < 11 ? t - 8 : t < 14 ? t + 3 : t - 8; }
__host__ __device__ constexpr int tstate(int i) {
  return i < 3 ? 8 + i : i < 6 ? i - 3 : i < 8 ? i + 8 : i == 8 ? -1 : i < 14 ? i - 6 : i - 3;
}
// identity states held by the input lanes, in lane order (lane 8 + ci owns IDS[ci])
__host__ __device__ constexpr int ids(int ci) { return ci < 3 ? ci : ci + 11; }
// nonzero rows of the implicit shear column 8: AB[8,8] = 1, AB[2,8] = h, AB[14+m,8] = h Jp[m][2]
__host__ __device__ constexpr int c8row(int r) { return r == 0 ? 8 : r == 1 ? 2 : 12 + r; }

// ---- row-broadcast FMAs ----------------------------------------------------------------------
// The leading s_nop covers the VALU-write -> DPP-read wait states the hazard recognizer does not
// insert for inline asm (no DPP source is written inside a block); see mpcb_split.h.
#define Q17_BC(op, d, s, b, l) op " %" #d ", %" #s ", %" #b " row_newbcast:" l " row_mask:0xf bank_mask:0xf\n\t"

// y[i] += bcast_L(a[i]) * b (i < 17), h += bcast_L(ah) * b
#define Q17_BC18(OP)                                                                                        \
  asm("s_nop 4\n\t" Q17_BC(OP, 0, 18, 36, "%c37") Q17_BC(OP, 1, 19, 36, "%c37") Q17_BC(OP, 2, 20, 36, "%c37") \
      Q17_BC(OP, 3, 21, 36, "%c37") Q17_BC(OP, 4, 22, 36, "%c37") Q17_BC(OP, 5, 23, 36, "%c37")               \
      Q17_BC(OP, 6, 24, 36, "%c37") Q17_BC(OP, 7, 25, 36, "%c37") Q17_BC(OP, 8, 26, 36, "%c37")               \
      Q17_BC(OP, 9, 27, 36, "%c37") Q17_BC(OP, 10, 28, 36, "%c37") Q17_BC(OP, 11, 29, 36, "%c37")             \
      Q17_BC(OP, 12, 30, 36, "%c37") Q17_BC(OP, 13, 31, 36, "%c37") Q17_BC(OP, 14, 32, 36, "%c37")            \
      Q17_BC(OP, 15, 33, 36, "%c37") Q17_BC(OP, 16, 34, 36, "%c37") Q17_BC(OP, 17, 35, 36, "%c37")            \
      : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]),       \
        "+v"(y[8]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]), "+v"(y[12]), "+v"(y[13]), "+v"(y[14]),              \
        "+v"(y[15]), "+v"(y[16]), "+v"(h)                                                                     \
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]),  \
        "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(a[12]), "v"(a[13]), "v"(a[14]), "v"(a[15]), "v"(a[16]),       \
        "v"(ah), "v"(b), "i"(L))
template <int L, class T>
__device__ __forceinline__ void bc18(T (&y)[NX17], T& h, const T (&a)[NX17], T ah, T b) {
  if constexpr (sizeof(T) == 8) Q17_BC18("v_fmac_f64_dpp"); else Q17_BC18("v_fmac_f32_dpp");
}

// acc_t += bcast_t(a) * b for the 16 lanes t of the row; acc_t = g[t] (DIAG) or y[sown(t)]
#define Q17_D16(OP, ...)                                                                                  \
  asm("s_nop 4\n\t" Q17_BC(OP, 0, 16, 17, "0") Q17_BC(OP, 1, 16, 17, "1") Q17_BC(OP, 2, 16, 17, "2")      \
      Q17_BC(OP, 3, 16, 17, "3") Q17_BC(OP, 4, 16, 17, "4") Q17_BC(OP, 5, 16, 17, "5")                    \
      Q17_BC(OP, 6, 16, 17, "6") Q17_BC(OP, 7, 16, 17, "7") Q17_BC(OP, 8, 16, 17, "8")                    \
      Q17_BC(OP, 9, 16, 17, "9") Q17_BC(OP, 10, 16, 17, "10") Q17_BC(OP, 11, 16, 17, "11")                \
      Q17_BC(OP, 12, 16, 17, "12") Q17_BC(OP, 13, 16, 17, "13") Q17_BC(OP, 14, 16, 17, "14")              \
      Q17_BC(OP, 15, 16, 17, "15")                                                                        \
      : __VA_ARGS__                                                                                       \
      : "v"(a), "v"(b))
#define Q17_G16 "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), "+v"(g[6]), \
    "+v"(g[7]), "+v"(g[8]), "+v"(g[9]), "+v"(g[10]), "+v"(g[11]), "+v"(g[12]), "+v"(g[13]),         \
    "+v"(g[14]), "+v"(g[15])
#define Q17_YS16 "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]), "+v"(y[12]), \
    "+v"(y[13]), "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[14]), "+v"(y[15]), "+v"(y[16]),            \
    "+v"(y[6]), "+v"(y[7])
template <class T> __device__ __forceinline__ void diag16(T (&g)[LN], T a, T b) {
  if constexpr (sizeof(T) == 8) Q17_D16("v_fmac_f64_dpp", Q17_G16); else Q17_D16("v_fmac_f32_dpp", Q17_G16);
}
template <class T> __device__ __forceinline__ void diag16_sown(T (&y)[NX17], T a, T b) {
  static_assert(sown(0) == 3 && sown(8) == 0 && sown(11) == 14 && sown(14) == 6, "Q17_YS16 order");
  if constexpr (sizeof(T) == 8) Q17_D16("v_fmac_f64_dpp", Q17_YS16); else Q17_D16("v_fmac_f32_dpp", Q17_YS16);
}

// acc += sum_t bcast_t(a) * w[t] over the 16 lanes t of the row: four interleaved partial sums
// (a single dependent chain of 16 DPP FMAs costs the forward pass its latency)
#define Q17_C16(OP)                                                                                      \
  asm("s_nop 4\n\t" Q17_BC(OP, 0, 4, 5, "0") Q17_BC(OP, 1, 4, 6, "1") Q17_BC(OP, 2, 4, 7, "2")           \
      Q17_BC(OP, 3, 4, 8, "3") Q17_BC(OP, 0, 4, 9, "4") Q17_BC(OP, 1, 4, 10, "5") Q17_BC(OP, 2, 4, 11, "6") \
      Q17_BC(OP, 3, 4, 12, "7") Q17_BC(OP, 0, 4, 13, "8") Q17_BC(OP, 1, 4, 14, "9")                       \
      Q17_BC(OP, 2, 4, 15, "10") Q17_BC(OP, 3, 4, 16, "11") Q17_BC(OP, 0, 4, 17, "12")                   \
      Q17_BC(OP, 1, 4, 18, "13") Q17_BC(OP, 2, 4, 19, "14") Q17_BC(OP, 3, 4, 20, "15")                   \
      : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)                                                            \
      : "v"(a), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]),  \
        "v"(w[8]), "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]), "v"(w[14]), "v"(w[15]))
template <class T> __device__ __forceinline__ void chain16(T& acc, T a, const T (&w)[LN]) {
  T p0 = acc, p1 = T(0), p2 = T(0), p3 = T(0);
  if constexpr (sizeof(T) == 8) Q17_C16("v_fmac_f64_dpp"); else Q17_C16("v_fmac_f32_dpp");
  acc = (p0 + p1) + (p2 + p3);
}

// sum over the 16 lanes of the row of v (every lane gets it): four interleaved DPP partial sums
#define Q17_S16(OP)                                                                                      \
  asm("s_nop 4\n\t" Q17_BC(OP, 0, 4, 5, "0") Q17_BC(OP, 1, 4, 5, "1") Q17_BC(OP, 2, 4, 5, "2")           \
      Q17_BC(OP, 3, 4, 5, "3") Q17_BC(OP, 0, 4, 5, "4") Q17_BC(OP, 1, 4, 5, "5") Q17_BC(OP, 2, 4, 5, "6")  \
      Q17_BC(OP, 3, 4, 5, "7") Q17_BC(OP, 0, 4, 5, "8") Q17_BC(OP, 1, 4, 5, "9")                        \
      Q17_BC(OP, 2, 4, 5, "10") Q17_BC(OP, 3, 4, 5, "11") Q17_BC(OP, 0, 4, 5, "12")                     \
      Q17_BC(OP, 1, 4, 5, "13") Q17_BC(OP, 2, 4, 5, "14") Q17_BC(OP, 3, 4, 5, "15")                     \
      : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)                                                          \
      : "v"(v), "v"(one))
template <class T> __device__ __forceinline__ T sum16(T v, T init = T(0)) {
  T p0 = init, p1 = T(0), p2 = T(0), p3 = T(0);
  const T one = T(1);
  if constexpr (sizeof(T) == 8) Q17_S16("v_fmac_f64_dpp"); else Q17_S16("v_fmac_f32_dpp");
  return (p0 + p1) + (p2 + p3);
}
#undef Q17_S16

// lane L's v in every lane of the row (0 + bcast_L(v) * 1: exact)
template <int L, class T> __device__ __forceinline__ T bcast(T v) {
  T r = T(0);
  const T one = T(1);
  if constexpr (sizeof(T) == 8)
    asm("s_nop 4\n\t" Q17_BC("v_fmac_f64_dpp", 0, 1, 2, "%c3") : "+v"(r) : "v"(v), "v"(one), "i"(L));
  else
    asm("s_nop 4\n\t" Q17_BC("v_fmac_f32_dpp", 0, 1, 2, "%c3") : "+v"(r) : "v"(v), "v"(one), "i"(L));
  return r;
}
#undef Q17_BC18
#undef Q17_D16
#undef Q17_C16

// sum / min / max over the 16 lanes of the row (DPP broadcasts of every lane: 16 instructions)
template <class T> __device__ __forceinline__ T row_sum(T v) {
  T s = T(0);
  static_for<LN>([&](auto l) { s += bcast<decltype(l)::value>(v); });
  return s;
}
template <class T> __device__ __forceinline__ T row_min(T v) {
  T s = v;
  static_for<LN>([&](auto l) { s = fmin(s, bcast<decltype(l)::value>(v)); });
  return s;
}
template <class T> __device__ __forceinline__ T row_max(T v) {
  T s = v;
  static_for<LN>([&](auto l) { s = fmax(s, bcast<decltype(l)::value>(v)); });
  return s;
}
__device__ __forceinline__ int row_or(int v) {
  const float f = row_max((float)v);
  return f > 0.f ? 1 : 0;
}

// per-instance LDS block.  Bank layout (MI355X_MICROARCH.md §LDS: ds_read_b64 banks (a/4) mod 64
// over 32-lane halves = two instances; ds_write_b64 banks (a/4) mod 32 over 16-lane groups):
//  - the block is 32 dwords mod 64 long (fp64; 16 mod 32 in fp32), so the two instances of a half
//    read opposite halves of the bank row;
//  - X's columns are stored at xpos(s): the 16 columns the exchange reads are contiguous (32
//    dwords), state 8's (never read back) last -- stored by s they spanned 34 dwords and wrapped
//    onto the sibling instance's banks;
//  - HU rows are 9 long: the six input lanes' stores of one entry hit distinct bank pairs (rows of
//    8 put lanes m and m + 2 on one bank, 3-way);
//  - V and the rows of s Q hold the states at xpos too (by s, lanes s = 0 and 16 shared a bank:
//    the compiler pairs the Q reads as ds_read2_b64, banked (a/4) mod 32).
__host__ __device__ constexpr int xpos(int s) { return s < OM ? s : s == OM ? NX17 - 1 : s - 1; }
template <class T> struct Lds {
  T V[24];            // cost residual (ybar + iterate - yref): state i at xpos(i), input n at 17 + n
  T HU[NU17][9];      // input lane m: G[17+n, 17+m] (n < 6), h_u[m], G[8, 17+m]
  T YC[6][17];        // lane t: Y[c, z(t)] for the identity states c = ids(0..5) (stride 17: banks)
  T X[LN][NX17];      // P_new columns (symmetric exchange), entry i of lane t's column at xpos(i)
  T pad[12];
};
static_assert(sizeof(Lds<double>) / 4 % 64 == 32 && sizeof(Lds<float>) / 4 % 32 == 16, "Lds bank layout");

template <class T>
struct Ctx {
  const FullArgs<T>& a;
  Ws17<T> w;
  WsM17<T> wm;        // Mehrotra arrays (riccati17q_kernel<T, true, true>)
  const T* xr;
  const T* ur;
  Lds<T>& L;
  const T* sQ;        // s * Q (row-major 17 x 17, Q[i][j] at i * 17 + xpos(j): banks), LDS
  const T* sR;        // s * R (6 x 6), LDS
  int t, s, z, m;     // lane in the row, owned state, z column, input index (input lanes; else 0)
  bool in, valid;
  int ks;             // 1; 0 once the group is parked (finished, outputs written): every stage-indexed
                      // workspace access then goes to stage 0, so a finished group riding along with
                      // its wave's others moves no HBM traffic
};

// state-box row (k, i): dx-coordinate bounds, the iterate and its slacks / multipliers
template <class T>
struct SRow {
  T y, lb, ub, sl, su, ll, lu, rl, ru;
  __device__ __forceinline__ SRow(T y_, T xb, T lbx, T ubx, T sl_, T su_, T ll_, T lu_)
      : y(y_), lb(lbx - xb), ub(ubx - xb), sl(sl_), su(su_), ll(ll_), lu(lu_) {
    rl = y - lb - sl;
    ru = ub - y - su;
  }
  __device__ __forceinline__ SRow(const Ctx<T>& r, int k, int i)
      : SRow(r.w.DX[(int64_t)k * NX17 + i], r.w.XB[(int64_t)k * NX17 + i], r.a.W->lbx[i], r.a.W->ubx[i],
             r.w.IX[(int64_t)k * 4 * NX17 + i], r.w.IX[(int64_t)k * 4 * NX17 + NX17 + i],
             r.w.IX[(int64_t)k * 4 * NX17 + 2 * NX17 + i], r.w.IX[(int64_t)k * 4 * NX17 + 3 * NX17 + i]) {}
  __device__ __forceinline__ void barrier(T smu, T& D, T& d) const {
    const T isl = recip(sl), isu = recip(su);
    D = ll * isl + lu * isu;
    d = -smu * (isl - isu) + (ll * isl) * rl - (lu * isu) * ru;
  }
};

// Stage data loaded one stage ahead, as raw loads: every value is consumed a stage later (any
// arithmetic or select on a load here would wait for it on the spot).
template <class T>
struct Pre {
  T ab[NX17];      // column z of [A_k | B_k]
  T a8[5];         // the nonzeros of the implicit column 8 (rows c8row(0..4))
  T xs, x8, xrs, xr8, ub, urm;          // xbar_k[s], xbar_k[8], xref_k[s], xref_k[8], ubar_k[m], uref_k[m]
};

template <class T>
__device__ __forceinline__ void prefetch(const Ctx<T>& r, int k, Pre<T>& p) {
  k *= r.ks;
  const T* ABk = r.w.AB + (int64_t)k * NZ17 * NX17;
#pragma unroll
  for (int i = 0; i < NX17; ++i) p.ab[i] = ABk[r.z * NX17 + i];
#pragma unroll
  for (int q = 0; q < 5; ++q) p.a8[q] = ABk[OM * NX17 + c8row(q)];
  const int64_t kx = (int64_t)k * NX17;
  p.xs = r.w.XB[kx + r.s];
  p.x8 = r.w.XB[kx + OM];
  p.xrs = r.xr[kx + r.s];
  p.xr8 = r.xr[kx + OM];
  p.ub = r.w.UB[(int64_t)k * NU17 + r.m];
  p.urm = r.ur[(int64_t)k * NU17 + r.m];
}

// The interior point's iterate, multipliers and state-row slacks of the current stage: loaded at
// the top of the stage and consumed after the two product passes (they are not carried a stage
// ahead: that register set pushed the fp64 interior-point kernel into scratch)
template <class T>
struct Cur {
  T dxs, dx8, du, ll, lu;               // dx_k[s], dx_k[8], (du, lambda_l, lambda_u)_k[m]
  T ddxs, ddx8;                         // the last Newton step of dx_k[s], dx_k[8] (pending)
  T ixs[4], ix8[4];                     // state rows (s_l, s_u, lambda_l, lambda_u) of s and 8
};
template <class T, bool SBX = true>
__device__ __forceinline__ void load_cur(const Ctx<T>& r, int k, Cur<T>& p) {
  k *= r.ks;
  const int64_t kx = (int64_t)k * NX17;
  p.dxs = r.w.DX[kx + r.s];
  p.dx8 = r.w.DX[kx + OM];
  p.ddxs = r.w.DDX[kx + r.s];
  p.ddx8 = r.w.DDX[kx + OM];
  const T* ip = r.w.IP + (int64_t)k * 18;
  p.du = ip[r.m];
  p.ll = ip[6 + r.m];
  p.lu = ip[12 + r.m];
  if constexpr (SBX) {   // the state rows (SBX: the kernel can have a state box)
    const T* ix = r.w.IX + (int64_t)k * 4 * NX17;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      p.ixs[e] = ix[e * NX17 + r.s];
      p.ix8[e] = ix[e * NX17 + OM];
    }
  }
}

// Riccati backward over the cached [A|B] (+ gaps in iterate mode, + the interior point's barrier
// terms and the iterate shift when r.a.box).  Writes K (row-major 6 x 17) and k to KR.  With the
// box, the previous iteration's step of the state trajectory, dx += apend ddx, is applied here
// stage by stage (written back to DX) instead of in a pass of its own.
// POLC (the fp64 state-box kernel): with pol (this group polishes, oracle.ocp.al_polish) every
// row takes the augmented-Lagrangian terms of its active side instead of the barrier: D = rho and
// d = nu + rho (y - b) on an active row (side != 0), nothing on an inactive one.  The rows then hold
// (nu, side) where the multipliers (lambda_l, lambda_u) were: IP[6 + m], IP[12 + m] and IX rows 2, 3.
// SBX: the kernel instantiation can carry state rows (the fp64 state-box kernel); the others
// (the input box alone: Mehrotra in fp64, fp32) compile the state-row code and its registers out.
template <class T, bool MEH = false, bool POLC = false, bool SBX = true>
__device__ __forceinline__ bool backward(const Ctx<T>& r, T smu, T apend = T(0), bool pol = false) {
  const FullArgs<T>& a = r.a;
  const bool ipm = a.box != 0;
  const bool gaps = !ipm && a.mode == MPCB_MODE_ITERATE;
  const bool sbox = SBX && ipm && a.sbox != 0;
  Lds<T>& L = r.L;
  const int t = r.t, s = r.s, N = a.N;
  const bool in = r.in;
  const Weights17<T>& W = *a.W;
  constexpr int KR_N = Ws17<T>::KR_N;
  const uint64_t m_in = lane_mask(in);
  // terminal cost: P_N = QN, p_N = QN (x_N - xref_N)
  T Pc[NX17], P88, pj, p8;
  {
    const int Nq = N * r.ks;   // (a parked group: stage 0)
    T xs = r.w.XB[(int64_t)Nq * NX17 + s], x8 = r.w.XB[(int64_t)Nq * NX17 + OM];
    if (ipm) {
      T* dxn = r.w.DX + (int64_t)Nq * NX17;
      const T* ddn = r.w.DDX + (int64_t)Nq * NX17;
      // (a select, not a product with apend = 0: DDX is not yet written before the first step)
      const T ys = (apend != T(0)) ? dxn[s] + apend * ddn[s] : dxn[s];
      const T y8 = (apend != T(0)) ? dxn[OM] + apend * ddn[OM] : dxn[OM];
      dxn[s] = ys;
      dxn[OM] = y8;
      xs += ys;
      x8 += y8;
    }
    L.V[xpos(s)] = xs - r.xr[(int64_t)Nq * NX17 + s];
    L.V[xpos(OM)] = x8 - r.xr[(int64_t)Nq * NX17 + OM];
    wave_lds_sync();
    pj = T(0);
    p8 = T(0);
#pragma unroll
    for (int i = 0; i < NX17; ++i) {
      const T vi = L.V[xpos(i)];
      pj += W.QN[s * NX17 + i] * vi;
      p8 += W.QN[OM * NX17 + i] * vi;
      Pc[i] = W.QN[i * NX17 + s];
    }
    P88 = W.QN[OM * NX17 + OM];
    wave_lds_sync();
    if constexpr (MEH) {   // p_N for the corrector's vector pass
      T* gv = r.wm.GV + (int64_t)Nq * 24;
      gv[s] = pj;
      gv[OM] = p8;
    }
  }
  // box constants in registers (a load consumed on the spot would wait inside the stage loop)
  const T lbm = W.lbu[r.m], ubm = W.ubu[r.m];
  const T lbs = W.lbx[s], ubs = W.ubx[s], lb8 = W.lbx[OM], ub8 = W.ubx[OM];
  bool qp_ok = true;
  Pre<T> nx;
  prefetch(r, N - 1, nx);
  QSTAMP_INIT();
  for (int k = N - 1; k >= 0; --k) {
    const Pre<T> cu = nx;
    prefetch(r, k > 0 ? k - 1 : 0, nx);   // (unconditional: no branch join on the loads)
    const int kq = k * r.ks;   // workspace stage (a parked group: 0)
    Cur<T> ic;
    if (ipm) load_cur<T, SBX>(r, k, ic);
    // pt = p + P gap (iterate mode)
    T pt = pj, pt8 = p8;
    if (gaps) {
      const T* gk = r.w.GP + (int64_t)kq * NX17;
      T prow = Pc[OM] * gk[s];   // P[8, s] gap[s]: summed over the row below
#pragma unroll
      for (int i = 0; i < NX17; ++i) pt += Pc[i] * gk[i];
      pt8 += P88 * gk[OM] + row_sum(prow);
    }
    QSTAMP(0);
    // ---- Y = P [A|B]_z and h_AB = [A|B]_z^T pt
    T y[NX17], hab = T(0);
#pragma unroll
    for (int i = 0; i < NX17; ++i) y[i] = T(0);
    static_for<LN>([&](auto l) {
      constexpr int tl = decltype(l)::value;
      bc18<tl>(y, hab, Pc, pt, cu.ab[sown(tl)]);
    });
    diag16_sown(y, Pc[OM], cu.ab[OM]);
    y[OM] += P88 * cu.ab[OM];
    hab += pt8 * cu.ab[OM];
    QSTAMP(1);
    // ---- G_z = [A|B]^T Y_z: rows z(t') by row broadcasts of [A|B] columns, identity rows = Y rows,
    // row 8 by the shear column
    T g[LN];
#pragma unroll
    for (int i = 0; i < LN; ++i) g[i] = T(0);
#pragma unroll
    for (int l = 0; l < NX17; ++l) diag16(g, cu.ab[l], y[l]);
    T g8 = T(0);
#pragma unroll
    for (int q = 0; q < 5; ++q) g8 += cu.a8[q] * y[c8row(q)];
    QSTAMP(2);
    if (ipm) {   // the pending step of this stage's iterate (unconditional stores)
      ic.dxs = (apend != T(0)) ? ic.dxs + apend * ic.ddxs : ic.dxs;
      ic.dx8 = (apend != T(0)) ? ic.dx8 + apend * ic.ddx8 : ic.dx8;
      r.w.DX[(int64_t)kq * NX17 + s] = ic.dxs;
      r.w.DX[(int64_t)kq * NX17 + OM] = ic.dx8;
    }
    // cost residual (ybar [+ iterate] - yref) into LDS (general Q, R)
    L.V[xpos(s)] = (ipm ? cu.xs + ic.dxs : cu.xs) - cu.xrs;
    L.V[xpos(OM)] = (ipm ? cu.x8 + ic.dx8 : cu.x8) - cu.xr8;
    if (in) L.V[NX17 + r.m] = (ipm ? cu.ub + ic.du : cu.ub) - cu.urm;
    // identity rows of this lane's Y for the identity-state lanes (their G column, by symmetry)
#pragma unroll
    for (int ci = 0; ci < 6; ++ci) L.YC[ci][t] = y[ids(ci)];
    wave_lds_sync();
    // ---- input lanes: their column G[:, 17+m] (+ s R, + barrier) -> Huu, h_u, Hux[:, 8]
    T gu_own = T(0);   // (MEH) the input's gradient without the p term
    if (in) {
      const int m = r.m;
      T hu = hab;
      T gu = T(0);
#pragma unroll
      for (int n = 0; n < NU17; ++n) {
        const T wr = r.sR[n * NU17 + m];
        if constexpr (MEH) gu += wr * L.V[NX17 + n];
        else hu += wr * L.V[NX17 + n];
        L.HU[m][n] = g[8 + n] + wr;
      }
      if constexpr (MEH) {
        gu_own = gu;
        hu = hab + gu;
      }
      if (ipm) {
        const T sl = ic.du - (lbm - cu.ub), su = (ubm - cu.ub) - ic.du;
        const T isl = recip(sl), isu = recip(su);
        T D = ic.ll * isl + ic.lu * isu, d = -smu * (isl - isu);
        if constexpr (POLC) {
          const bool act = ic.lu != T(0);
          const T bnd = ic.lu < T(0) ? lbm - cu.ub : ubm - cu.ub;
          D = pol ? (act ? T(POL17_RHO) : T(0)) : D;
          d = pol ? (act ? ic.ll + T(POL17_RHO) * (ic.du - bnd) : T(0)) : d;
        }
        L.HU[m][m] += D;
        hu += d;
      }
      L.HU[m][6] = hu;
      L.HU[m][7] = g8;
    }
    wave_lds_sync();
    QSTAMP(3);
    // ---- this lane's state column Gs = G[:, s] (23 rows by z index) and gradient h_s
    T Gs[NZ17];
    {
      // column lanes: (g, Y rows, g8); identity lanes: rows z(t') from the lanes' Y (YC), identity
      // rows from P (AB[:, c] = e_c), row 8 by the shear column applied to P's column
      const int ci = in ? r.m : 0;
      T spc = T(0);
#pragma unroll
      for (int q = 0; q < 5; ++q) spc += cu.a8[q] * Pc[c8row(q)];
#pragma unroll
      for (int tp = 0; tp < LN; ++tp) Gs[zcol(tp)] = csel(m_in, L.YC[ci][tp], g[tp]);
#pragma unroll
      for (int q = 0; q < 6; ++q) Gs[ids(q)] = csel(m_in, Pc[ids(q)], y[ids(q)]);
      Gs[OM] = csel(m_in, spc, g8);
    }
    T hs = in ? pt : hab;   // AB[:, c]^T pt = pt_c for an identity state
    T gs = T(0);            // (MEH) the state's gradient without the p term
#pragma unroll
    for (int i = 0; i < NX17; ++i) {
      const T wq = r.sQ[i * NX17 + xpos(s)];
      Gs[i] += wq;
      if constexpr (MEH) gs += wq * L.V[xpos(i)];
      else hs += wq * L.V[xpos(i)];
    }
    if constexpr (MEH) hs = hs + gs;
    // row 8 of every lane's G column is needed as the distributed column 8 of G; G[8,8] itself:
    // a^T P a with a = AB[:, 8] (rows 8, 2, 14..16) from P88, the lanes' P[8, .] and (P a)
    T spc_own = T(0);
#pragma unroll
    for (int q = 0; q < 5; ++q) spc_own += cu.a8[q] * Pc[c8row(q)];   // (P a)_s
    T pa8 = P88 * cu.a8[0];                                             // (P a)_8
    T G88 = T(0), h8 = T(0);
    {
      const T pc8 = Pc[OM];
      pa8 += bcast<tstate(2)>(pc8) * cu.a8[1] + bcast<tstate(14)>(pc8) * cu.a8[2] +
             bcast<tstate(15)>(pc8) * cu.a8[3] + bcast<tstate(16)>(pc8) * cu.a8[4];
      G88 = cu.a8[0] * pa8 + cu.a8[1] * bcast<tstate(2)>(spc_own) + cu.a8[2] * bcast<tstate(14)>(spc_own) +
            cu.a8[3] * bcast<tstate(15)>(spc_own) + cu.a8[4] * bcast<tstate(16)>(spc_own);
      h8 = cu.a8[0] * pt8 + cu.a8[1] * bcast<tstate(2)>(pt) + cu.a8[2] * bcast<tstate(14)>(pt) +
           cu.a8[3] * bcast<tstate(15)>(pt) + cu.a8[4] * bcast<tstate(16)>(pt);
      T gr8 = T(0);
#pragma unroll
      for (int i = 0; i < NX17; ++i) {
        if constexpr (MEH) gr8 += r.sQ[OM * NX17 + xpos(i)] * L.V[xpos(i)];
        else h8 += r.sQ[OM * NX17 + xpos(i)] * L.V[xpos(i)];
      }
      if constexpr (MEH) {   // (no state rows in the Mehrotra kernel: the gradients are complete)
        h8 = h8 + gr8;
        T* gv = r.wm.GV + (int64_t)kq * 24;
        gv[s] = gs;
        gv[OM] = gr8;
        gv[in ? NX17 + r.m : 23] = gu_own;
      }
      G88 += r.sQ[OM * NX17 + xpos(OM)];
    }
    if (sbox && k > 0) {   // state-box rows of this stage: barrier terms on the state diagonals
      T D, d;
      auto rowterms = [&](T y, T xb, T lb, T ub, const T (&ix)[4]) {
        SRow<T>(y, xb, lb, ub, ix[0], ix[1], ix[2], ix[3]).barrier(smu, D, d);
        if constexpr (POLC) {   // (nu, side) in rows 2, 3; bounds in dx coordinates
          const bool act = ix[3] != T(0);
          const T bnd = (ix[3] < T(0) ? lb : ub) - xb;
          D = pol ? (act ? T(POL17_RHO) : T(0)) : D;
          d = pol ? (act ? ix[2] + T(POL17_RHO) * (y - bnd) : T(0)) : d;
        }
      };
      rowterms(ic.dxs, cu.xs, lbs, ubs, ic.ixs);
#pragma unroll
      for (int i = 0; i < NX17; ++i) Gs[i] += (i == s) ? D : T(0);
      hs += d;
      rowterms(ic.dx8, cu.x8, lb8, ub8, ic.ix8);
      G88 += D;
      h8 += d;
    }
    QSTAMP(4);
    // ---- Huu (lower triangle from the column owners), Cholesky, k, K columns
    T H[NU17 * NU17], hu[NU17], hx8[NU17];
#pragma unroll
    for (int i = 0; i < NU17; ++i) {
#pragma unroll
      for (int j = 0; j <= i; ++j) H[i * NU17 + j] = L.HU[j][i];
      hu[i] = L.HU[i][6];
      hx8[i] = L.HU[i][7];
    }
    T Lc[NU17 * NU17];
    chol_n<T, NU17>(H, Lc);
    if constexpr (MEH) {   // packed lower triangle (row i at i(i+1)/2): lane t stores entries t and 16 + t % 5
      T pk[21];
#pragma unroll
      for (int i = 0; i < NU17; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) pk[i * (i + 1) / 2 + j] = Lc[i * NU17 + j];
      T* lc = r.wm.LC + (int64_t)kq * WsM17<T>::LC_N;
      lc[t] = sel<16>(pk, t);
      lc[16 + t % 5] = sel<5>(pk + 16, t % 5);
    }
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NU17; ++i) ok = ok && (Lc[i * NU17 + i] == Lc[i * NU17 + i]);
    qp_ok = qp_ok && ok;
    T kff[NU17], Ks[NU17], K8[NU17], nb[NU17];
#pragma unroll
    for (int i = 0; i < NU17; ++i) nb[i] = -hu[i];
    chol_n_solve<T, NU17>(Lc, nb, kff);
#pragma unroll
    for (int i = 0; i < NU17; ++i) nb[i] = -Gs[NX17 + i];
    chol_n_solve<T, NU17>(Lc, nb, Ks);
#pragma unroll
    for (int i = 0; i < NU17; ++i) nb[i] = -hx8[i];
    chol_n_solve<T, NU17>(Lc, nb, K8);
    QSTAMP(5);
    {   // KR: K row-major [6][17], then k[6].  Unconditional stores (a padding group owns its slot):
        // the K column of state 8 and k are the same in every lane (each lane solved the same
        // 6x6 systems), so every lane writes them to a fixed or its own input's slot
      T* kr = r.w.KR + (int64_t)kq * KR_N;
#pragma unroll
      for (int i = 0; i < NU17; ++i) {
        kr[i * NX17 + s] = Ks[i];
        kr[i * NX17 + OM] = K8[i];
      }
      kr[NU17 * NX17 + r.m] = sel<NU17>(kff, r.m);
    }
    QSTAMP(6);
    // ---- P_new[:, s] = G_xx[:, s] + Hxu K[:, s]; p_new; the 8 entries
    T Pn[NX17];
#pragma unroll
    for (int i = 0; i < NX17; ++i) Pn[i] = Gs[i];
#pragma unroll
    for (int n = 0; n < NU17; ++n) {
      diag16_sown(Pn, Gs[NX17 + n], Ks[n]);
      Pn[OM] += hx8[n] * Ks[n];
    }
    T pn = hs, pn8 = h8, P88n = G88;
#pragma unroll
    for (int n = 0; n < NU17; ++n) {
      pn += Gs[NX17 + n] * kff[n];
      pn8 += hx8[n] * kff[n];
      P88n += hx8[n] * K8[n];
    }
#ifdef MPCB_Q17_DEBUG
    if (blockIdx.x == 0 && threadIdx.x < LN && k >= N - 2) {
      printf("QG %d %d %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", k, t, s, (double)Gs[0], (double)Gs[1], (double)Gs[2], (double)Gs[3], (double)Gs[4], (double)Gs[5], (double)Gs[6], (double)Gs[7], (double)Gs[8], (double)Gs[9], (double)Gs[10], (double)Gs[11], (double)Gs[12], (double)Gs[13], (double)Gs[14], (double)Gs[15], (double)Gs[16], (double)Gs[17], (double)Gs[18], (double)Gs[19], (double)Gs[20], (double)Gs[21], (double)Gs[22]);
      printf("QH %d %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", k, t, (double)hs, (double)h8, (double)G88, (double)pt, (double)Ks[0], (double)Ks[1], (double)Ks[2], (double)Ks[3], (double)Ks[4], (double)Ks[5], (double)kff[0], (double)kff[1], (double)kff[2], (double)kff[3], (double)kff[4], (double)kff[5]);
      printf("QP %d %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", k, t, (double)Pn[0], (double)Pn[1], (double)Pn[2], (double)Pn[3], (double)Pn[4], (double)Pn[5], (double)Pn[6], (double)Pn[7], (double)Pn[8], (double)Pn[9], (double)Pn[10], (double)Pn[11], (double)Pn[12], (double)Pn[13], (double)Pn[14], (double)Pn[15], (double)Pn[16]);
      printf("QY %d %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", k, t, (double)y[0], (double)y[1], (double)y[2], (double)y[3], (double)y[4], (double)y[5], (double)y[6], (double)y[7], (double)y[8], (double)y[9], (double)y[10], (double)y[11], (double)y[12], (double)y[13], (double)y[14], (double)y[15], (double)y[16]);
    }
#endif
    // symmetric by construction: entry (i, s) from the lane max(own, owner of i)
#pragma unroll
    for (int i = 0; i < NX17; ++i) L.X[t][xpos(i)] = Pn[i];
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < NX17; ++i) {
      if (i == OM) {
        Pc[i] = Pn[i];
      } else {
        const T o = L.X[tstate(i)][xpos(s)];
        Pc[i] = csel(lane_mask(tstate(i) > t), o, Pn[i]);
      }
    }
    P88 = P88n;
    pj = pn;
    p8 = pn8;
    wave_lds_sync();
    QSTAMP(7);
  }
  QSTAMP_DONE("bwd");
  return qp_ok;
}

// Mehrotra's corrector: its LQ problem has the predictor's matrices (same iterate, same D) and a
// gradient that differs only by the rows' target terms
//   Delta d = -(t_l/s_l - t_u/s_u),  t = sigma mu - Delta s_a Delta lambda_a,   = c - sigma mu w
// (w, c per row in DC).  This pass is the vector half of the Riccati recursion for the corrector's
// gradient (the predictor's stage gradients without the p terms in GV, plus Delta d) over the
// stored factor (LC) and gains (KR):
//   h_u = B^T p + g_u + Delta d_u,   k = -Huu^{-1} h_u,   p' = A^T p + g_x + Delta d_x + K^T h_u
// (K^T h_u = Hxu k), from p_N, and overwrites k.  (The full gradient, not the difference alone:
// near the conditioning limit, lambda / s ~ 1e16, predictor k + correction k cancelled to ~1e-6.)
// Uniform stage values (the factor, K's column of state 8) are loaded spread over the lanes and
// taken by row broadcasts.
template <class T>
struct PreC {
  T ab[NX17];      // column z of [A_k | B_k]
  T a8[5];         // the nonzeros of column 8
  T ks[NU17];      // K[:, s]
  T k8;            // K[t % 6, 8]
  T gs, g8, gu;    // the predictor's gradients without the p terms
  T lc0, lc1;      // packed factor entries t and 16 + t % 5
  T ws, cs, w8, c8, wu, cu;
};

template <class T>
__device__ __forceinline__ void prefetch_c(const Ctx<T>& r, int k, PreC<T>& p) {
  k *= r.ks;
  const T* ABk = r.w.AB + (int64_t)k * NZ17 * NX17;
#pragma unroll
  for (int i = 0; i < NX17; ++i) p.ab[i] = ABk[r.z * NX17 + i];
#pragma unroll
  for (int q = 0; q < 5; ++q) p.a8[q] = ABk[OM * NX17 + c8row(q)];
  const T* kr = r.w.KR + (int64_t)k * Ws17<T>::KR_N;
#pragma unroll
  for (int n = 0; n < NU17; ++n) p.ks[n] = kr[n * NX17 + r.s];
  p.k8 = kr[(r.t % NU17) * NX17 + OM];
  const T* gv = r.wm.GV + (int64_t)k * 24;
  p.gs = gv[r.s];
  p.g8 = gv[OM];
  p.gu = gv[NX17 + r.m];
  const T* lc = r.wm.LC + (int64_t)k * WsM17<T>::LC_N;
  p.lc0 = lc[r.t];
  p.lc1 = lc[16 + r.t % 5];
  const T* dc = r.wm.DC + (int64_t)k * WsM17<T>::DC_N;
  p.ws = dc[r.s];
  p.cs = dc[24 + r.s];
  p.w8 = dc[OM];
  p.c8 = dc[24 + OM];
  p.wu = dc[NX17 + r.m];
  p.cu = dc[24 + NX17 + r.m];
}

template <class T>
__device__ __forceinline__ void backward_corr(const Ctx<T>& r, T smu) {
  const int s = r.s, N = r.a.N;
  const bool in = r.in;
  T pc = r.wm.GV[(int64_t)N * r.ks * 24 + s], pc8 = r.wm.GV[(int64_t)N * r.ks * 24 + OM];
  PreC<T> nx;
  prefetch_c(r, N - 1, nx);
  for (int k = N - 1; k >= 0; --k) {
    const PreC<T> cu = nx;
    prefetch_c(r, k > 0 ? k - 1 : 0, nx);
    // [A|B]_z^T p (B^T p at input m on the input lanes)
    T hab = pc8 * cu.ab[OM];
    static_for<LN>([&](auto l) {
      constexpr int tl = decltype(l)::value;
      hab += bcast<tl>(pc) * cu.ab[sown(tl)];
    });
    const T hu = hab + cu.gu + (cu.cu - smu * cu.wu);
    T h6[NU17];
    static_for<NU17>([&](auto n) { h6[decltype(n)::value] = bcast<8 + decltype(n)::value>(hu); });
    const T hs = (in ? pc : hab) + cu.gs + (cu.cs - smu * cu.ws);
    const T h8 = cu.a8[0] * pc8 + cu.a8[1] * bcast<tstate(2)>(pc) + cu.a8[2] * bcast<tstate(14)>(pc) +
                 cu.a8[3] * bcast<tstate(15)>(pc) + cu.a8[4] * bcast<tstate(16)>(pc) + cu.g8 + (cu.c8 - smu * cu.w8);
    // the factor from the lanes' packed entries
    T Lc[NU17 * NU17];
    static_for<21>([&](auto pp) {
      constexpr int p_ = decltype(pp)::value;
      constexpr int i = p_ < 1 ? 0 : p_ < 3 ? 1 : p_ < 6 ? 2 : p_ < 10 ? 3 : p_ < 15 ? 4 : 5;
      constexpr int j = p_ - i * (i + 1) / 2;
      if constexpr (p_ < 16) Lc[i * NU17 + j] = bcast<p_>(cu.lc0);
      else Lc[i * NU17 + j] = bcast<p_ - 16>(cu.lc1);
    });
    T nb[NU17], kc[NU17];
#pragma unroll
    for (int n = 0; n < NU17; ++n) nb[n] = -h6[n];
    chol_n_solve<T, NU17>(Lc, nb, kc);
    r.w.KR[(int64_t)k * r.ks * Ws17<T>::KR_N + NU17 * NX17 + r.m] = sel<NU17>(kc, r.m);
    T pn = hs, pn8 = h8;
    static_for<NU17>([&](auto n) {
      constexpr int n_ = decltype(n)::value;
      pn += cu.ks[n_] * h6[n_];
      pn8 += bcast<n_>(cu.k8) * h6[n_];
    });
    pc = pn;
    pc8 = pn8;
  }
}

// complementarity targets of a row for Mehrotra's corrector: t = sigma mu - Delta s_a Delta lambda_a
template <class T>
__device__ __forceinline__ void targets(T smu, T sl, T su, T ll, T lu, T dsl_a, T dsu_a, T& tl, T& tu,
                                        T isl, T isu) {
  const T dll_a = (-ll * sl - ll * dsl_a) * isl, dlu_a = (-lu * su - lu * dsu_a) * isu;
  tl = smu - dsl_a * dll_a;
  tu = smu - dsu_a * dlu_a;
}

// Forward pass over K, k.  GAIN: du = K dx + k; else du from the interior point's iterate (the
// starting trajectory).  STEP: the Newton step (zero gaps, dx_0 = 0) into DDX / DDU; !STEP and
// !OUT: the iterate into DX.  OUT: X = xbar + dx, U = ubar + du, u0 (when write).  Returns this
// lane's finiteness.
template <class T, bool GAIN, bool STEP, bool OUT>
__device__ __forceinline__ bool forward(const Ctx<T>& r, T dxs, T dx8, bool write, T* ddx = nullptr, T* ddu = nullptr) {
  // (STEP: the direction's arrays, DDX / DDU unless given: the predictor's DAX / DAU)
  if (!ddx) ddx = r.w.DDX;
  if (!ddu) ddu = r.w.DDU;
  const FullArgs<T>& a = r.a;
  const int t = r.t, s = r.s, N = a.N;
  const bool in = r.in;
  constexpr int KR_N = Ws17<T>::KR_N;
  const bool gaps = !STEP && a.mode == MPCB_MODE_ITERATE;   // (the starting trajectory of the interior point too)
  const int64_t b = a.b0 + (r.w.XB - a.ws) / full17_elems(N);
  const uint64_t m_in = lane_mask(in), m_id = m_in;   // identity-state lanes = input lanes
  bool fin = true;
  // Stage rows FD stages ahead in a ring of register slots, the stage loop unrolled by FD so every
  // slot is a fixed register set (a copy of a slot would wait for its loads on the spot): K row m
  // and k_m (input lanes), row s of [A|B] at the lanes' z columns, the own entry of row 8
  constexpr int FD = STEP ? MPCB_Q17_FD_STEP : MPCB_Q17_FD;
  struct Row { T kr[LN], k8, kf, du, ab[LN], ab8o, c8s, c88, gs, g8, xbs, xb8, ubm; };
  auto load = [&](int k, Row& o) {
    k *= r.ks;
    const T* ABk = r.w.AB + (int64_t)k * NZ17 * NX17;
    if constexpr (GAIN) {
      const T* Kk = r.w.KR + (int64_t)k * KR_N;
#pragma unroll
      for (int tp = 0; tp < LN; ++tp) o.kr[tp] = Kk[r.m * NX17 + sown(tp)];
      o.k8 = Kk[r.m * NX17 + OM];
      o.kf = Kk[NU17 * NX17 + r.m];
    } else {
      o.du = r.w.IP[(int64_t)k * 18 + r.m];
    }
#pragma unroll
    for (int tp = 0; tp < LN; ++tp) o.ab[tp] = ABk[zcol(tp) * NX17 + s];
    o.ab8o = ABk[r.z * NX17 + OM];
    o.c8s = ABk[OM * NX17 + s];
    o.c88 = ABk[OM * NX17 + OM];
    o.gs = r.w.GP[(int64_t)k * NX17 + s];   // (raw: selected at use)
    o.g8 = r.w.GP[(int64_t)k * NX17 + OM];
    o.xbs = r.w.XB[(int64_t)k * NX17 + s];
    o.xb8 = r.w.XB[(int64_t)k * NX17 + OM];
    o.ubm = r.w.UB[(int64_t)k * NU17 + r.m];
  };
  Row ring[FD];
  T u0v = T(0);   // u_0 (OUT: written once after the pass)
  static_for<FD>([&](auto sl) {
    if (decltype(sl)::value < N) load(decltype(sl)::value, ring[decltype(sl)::value]);
  });
  QSTAMP_INIT();
  auto stage = [&](int k, Row& cr) {
    QSTAMP(0);
    T du;
    if constexpr (GAIN) {
      du = cr.kf + cr.k8 * dx8;
      chain16(du, dxs, cr.kr);
    } else {
      du = cr.du;
    }
    if (!in) du = T(0);
    // stores without lane-divergent branches (a branch around a store makes the vmcnt count of
    // the ring's loads dynamic and every wait a vmcnt(0)): each lane stores its own state, and the
    // input lanes' du or (every other lane, the same value) the state-8 entry
    if constexpr (STEP || !OUT) {
      T* base = STEP ? ddx : r.w.DX;
      const int kq = k * r.ks;
      base[(int64_t)kq * NX17 + s] = dxs;
      T* p2 = (STEP && in) ? ddu + (int64_t)kq * NU17 + r.m : base + (int64_t)kq * NX17 + OM;
      *p2 = (STEP && in) ? du : dx8;
    }
    if constexpr (OUT) {
      // caller arrays for valid groups that asked for them, else this lane's own DDX slot
      const bool wx = write && a.X, wu = write && a.U;
      T* p1 = wx ? a.X + (b * (int64_t)(N + 1) + k) * NX17 + s : r.w.DDX + (int64_t)k * NX17 + s;
      *p1 = cr.xbs + dxs;
      T* p2 = in ? (wu ? a.U + (b * (int64_t)N + k) * NU17 + r.m : r.w.DDU + (int64_t)k * NU17 + r.m)
                 : (wx ? a.X + (b * (int64_t)(N + 1) + k) * NX17 + OM : r.w.DDX + (int64_t)k * NX17 + OM);
      *p2 = in ? cr.ubm + du : cr.xb8 + dx8;
      if (k == 0) u0v = cr.ubm + du;
    }
    if (in) {
      const T uo = cr.ubm + du;
      fin = fin && isfin(uo);
    }
    // dx' = [A|B] (dx, du) + gap: lanes broadcast their z value (du on input lanes); row 8 as a
    // row sum of the lanes' own terms
    const T zb = csel(m_in, du, dxs);
    T acc = (gaps ? cr.gs : T(0)) + cr.c8s * dx8 + csel(m_id, dxs, T(0));
    chain16(acc, zb, cr.ab);
    const T acc8 = sum16(cr.ab8o * zb, (gaps ? cr.g8 : T(0)) + cr.c88 * dx8);
    dxs = acc;
    dx8 = acc8;
    fin = fin && isfin(dxs) && isfin(dx8);
    // refill this slot FD stages ahead, unconditionally (a clamped stage index past the end): a
    // refill under a branch makes the count of loads in flight path-dependent, and the
    // compiler then waits for every load (vmcnt(1)) at the top of each stage
    load(k + FD < N ? k + FD : N - 1, cr);
    QSTAMP(1);
  };
  // whole groups of FD stages without guards (a guarded stage makes the loads in flight
  // path-dependent as well), then the N % FD remaining stages
  int k0 = 0;
  for (; k0 + FD <= N; k0 += FD) {
    static_for<FD>([&](auto sl) { stage(k0 + decltype(sl)::value, ring[decltype(sl)::value]); });
  }
  static_for<FD>([&](auto sl) {
    if (k0 + decltype(sl)::value < N) stage(k0 + decltype(sl)::value, ring[decltype(sl)::value]);
  });
  QSTAMP_DONE("fwd");
  if constexpr (STEP || !OUT) {
    T* base = STEP ? ddx : r.w.DX;
    base[(int64_t)N * r.ks * NX17 + s] = dxs;
    base[(int64_t)N * r.ks * NX17 + OM] = dx8;
  }
  if constexpr (OUT) {
    if (write && a.X) {
      T* xo = a.X + (b * (int64_t)(N + 1) + N) * NX17;
      xo[s] = r.w.XB[(int64_t)N * NX17 + s] + dxs;
      if (t == 0) xo[OM] = r.w.XB[(int64_t)N * NX17 + OM] + dx8;
    }
    if (write && in) a.u0[b * NU17 + r.m] = u0v;
  }
  return fin;
}

// The interior point (the iteration of oracle.ocp.ipm_box_solve) in this layout: input rows owned by the input lanes, state rows by the
// owner of the state, the rows of state 8 spread over the lanes by stage (k = 1 + t, 1 + t + 16 ..).
// MEH (fp64, the input box alone): Mehrotra's predictor-corrector (oracle.ocp._ipm_box_mehrotra)
// instead of the adaptive centring.
template <class T, bool BOX, bool MEH>
__global__ void __launch_bounds__(64) riccati17q_kernel(FullArgs<T> a) {
  __shared__ Lds<T> lds_all[GR];
  __shared__ T sQ[NX17 * NX17];
  __shared__ T sR[NU17 * NU17];
  const int lane = threadIdx.x;
  const int q = lane / LN;
  const int t = lane % LN;
  const int64_t c_raw = (int64_t)blockIdx.x * GR + q;
  const bool valid = c_raw < a.nb;
  // A ragged last wave's extra groups (!valid) run on private padding slots of the workspace
  // (mpcb_create sizes it to whole wavefronts), so every workspace store is unconditional.  Those
  // slots are never filled (nominal17q / lin17ws write valid instances only): a padding group
  // iterates on garbage, which is harmless because (1) every reduction and exchange is row-local
  // (DPP row broadcasts, the group's own LDS block), so nothing flows into a valid group, (2) its
  // outputs are never written (valid guards) and (3) the loop exit ignores it (__all(... || !valid)).
  // Its x0 / xref / uref reads use the last instance's (b is clamped).
  const int64_t c = c_raw;
  const int64_t b = a.b0 + (valid ? c : a.nb - 1);
  const int N = a.N;
  const Weights17<T>& W = *a.W;
  const bool iterate = a.mode == MPCB_MODE_ITERATE;
  const bool in = t >= 8 && t < 14;
  const int s = sown(t);
  const int m = in ? t - 8 : 0;
  for (int e = lane; e < NX17 * NX17; e += 64) sQ[e / NX17 * NX17 + xpos(e % NX17)] = a.s * W.Q[e];
  for (int e = lane; e < NU17 * NU17; e += 64) sR[e] = a.s * W.R[e];
  __syncthreads();
  Ctx<T> r{a, Ws17<T>(a.ws + c * full17_elems(N), N), WsM17<T>(Ws17<T>(a.ws + c * full17_elems(N), N), N), a.xref + b * a.xref_sb, a.uref + b * a.uref_sb,
           lds_all[q], sQ, sR, t, s, zcol(t), m, in, valid, 1};
  Lds<T>& L = r.L;
  const T* x0 = a.x0 + b * a.x0_sb;
  const T dx0s = iterate ? x0[s] - r.w.XB[s] : T(0);
  const T dx08 = iterate ? x0[OM] - r.w.XB[OM] : T(0);
  int32_t st = MPCB_STATUS_OK;
  bool fin;
  if constexpr (!BOX) {
    if (!backward<T, false, false, false>(r, T(0))) st = MPCB_STATUS_QP_FAIL;
    __syncthreads();   // K and k are read back across lanes
    fin = forward<T, true, false, true>(r, dx0s, dx08, valid);
  } else {
    const T lbm = W.lbu[m], ubm = W.ubu[m];
    // start: du strictly inside the box, lambda = 1; dx by the dynamics
    if (valid && in) {
      for (int k = 0; k < N; ++k) {
        const T ubk = r.w.UB[(int64_t)k * NU17 + m];
        const T lb = lbm - ubk, ub = ubm - ubk, wd = ub - lb;
        T* ip = r.w.IP + (int64_t)k * 18;
        ip[m] = fmin(fmax(T(0), lb + T(IPM17_THETA) * wd), ub - T(IPM17_THETA) * wd);
        ip[6 + m] = T(1);
        ip[12 + m] = T(1);
      }
    }
    __syncthreads();
    forward<T, false, false, false>(r, dx0s, dx08, false);   // DX of the starting point
    __syncthreads();
    // (a state box exists only with fp64 and without Mehrotra: launch_riccati17q, mpcb_create)
    constexpr bool SBX = !MEH && sizeof(T) == 8;
    const bool sbox = SBX && a.sbox != 0;
    // state rows: s = max(distance to the bound, theta w), lambda = 1
    auto srow_init = [&](int k, int i) {
      const T xb = r.w.XB[(int64_t)k * NX17 + i], y = r.w.DX[(int64_t)k * NX17 + i];
      const T lb = W.lbx[i] - xb, ub = W.ubx[i] - xb, tw = T(IPM17_THETA) * (ub - lb);
      T* ix = r.w.IX + (int64_t)k * 4 * NX17 + i;
      ix[0] = fmax(y - lb, tw);
      ix[NX17] = fmax(ub - y, tw);
      ix[2 * NX17] = T(1);
      ix[3 * NX17] = T(1);
    };
    if (valid && sbox) {
      for (int k = 1; k < N; ++k) srow_init(k, s);
      for (int k = 1 + t; k < N; k += LN) srow_init(k, OM);
    }
    __syncthreads();
    const T rows = T(N * NU17 + (sbox ? (N - 1) * NX17 : 0));
    // the fp64 state-box polish (oracle.ocp.al_polish, mpcb_full.h POL17_*): once a group's interior
    // point has converged (pst 0 -> 1) its rows are classified and it runs up to POL17_ITERS
    // augmented-Lagrangian passes through the same backward / forward call sites as the interior
    // point, while the other groups of the wave may still iterate; 2 = polished (the group keeps
    // re-solving its frozen last pass, which reproduces its direction bit for bit), 3 = finished
    // without a polished point (failure, the iteration cap, or a polish that did not certify)
    constexpr bool POLC = sizeof(T) == 8 && !MEH;
    const bool polish = POLC && sbox;
    int pst = 0, npass = 0, nit = 0;   // (nit: this group's interior-point iterations)
    bool early = false;    // stopped at the conditioning limit (breakdown / collapsed step)
    const int it_max = a.max_as_iter + (polish ? POL17_ITERS : 0);
    auto classify = [&]() {   // side = -1 (lower) / +1 (upper) / 0 by lambda > 100 s, nu = lambda_u - lambda_l
      auto cl = [&](T sl, T su, T ll, T lu, T& nu, T& side) {
        side = ll > T(POL17_ACT) * sl ? T(-1) : (lu > T(POL17_ACT) * su ? T(1) : T(0));
        nu = side != T(0) ? lu - ll : T(0);
      };
      if (in) {
        for (int k = 0; k < N; ++k) {
          const T ubk = r.w.UB[(int64_t)k * NU17 + m];
          T* ip = r.w.IP + (int64_t)k * 18;
          cl(ip[m] - (lbm - ubk), (ubm - ubk) - ip[m], ip[6 + m], ip[12 + m], ip[6 + m], ip[12 + m]);
        }
      }
      auto clrow = [&](int k, int i) {
        T* ix = r.w.IX + (int64_t)k * 4 * NX17 + i;
        cl(ix[0], ix[NX17], ix[2 * NX17], ix[3 * NX17], ix[2 * NX17], ix[3 * NX17]);
      };
      for (int k = 1; k < N; ++k) clrow(k, s);
      for (int k = 1 + t; k < N; k += LN) clrow(k, OM);
    };
    bool done = false;
    T prev_alpha = T(1);
    int nshort = 0;
    T mu = T(0), res = T(0);       // duality measure, state-row residual (of the current iterate)
    T part_n = T(0), res_n = T(0); // their partial sums over the lane's rows after an update
    T apend = T(0);                // the last step length, not yet applied to DX
    // outputs of a finished group: X = xbar + dx, U = ubar + du of its final iterate (with the last
    // step when it is still pending, + the polish's Delta); written when the group finishes, after
    // which it is parked (Ctx::ks)
    bool parked = false;
    auto emit = [&]() {
      fin = true;
      for (int k = 0; k <= N; ++k) {   // (with the last step, when it is still pending)
        T xs = r.w.DX[(int64_t)k * NX17 + s], x8 = r.w.DX[(int64_t)k * NX17 + OM];
        if (apend != T(0)) {
          xs = xs + apend * r.w.DDX[(int64_t)k * NX17 + s];
          x8 = x8 + apend * r.w.DDX[(int64_t)k * NX17 + OM];
        }
        if (POLC && pst == 2) {
          xs = xs + r.w.DDX[(int64_t)k * NX17 + s];
          x8 = x8 + r.w.DDX[(int64_t)k * NX17 + OM];
        }
        if (valid && a.X) {
          T* xo = a.X + (b * (int64_t)(N + 1) + k) * NX17;
          xo[s] = r.w.XB[(int64_t)k * NX17 + s] + xs;
          if (t == 0) xo[OM] = r.w.XB[(int64_t)k * NX17 + OM] + x8;
        }
        fin = fin && isfin(xs) && isfin(x8);
        if (in && k < N) {
          T duk = r.w.IP[(int64_t)k * 18 + m];
          if (POLC && pst == 2) duk = duk + r.w.DDU[(int64_t)k * NU17 + m];
          const T uo = r.w.UB[(int64_t)k * NU17 + m] + duk;
          fin = fin && isfin(uo);
          if (valid && a.U) a.U[(b * (int64_t)N + k) * NU17 + m] = uo;
          if (valid && k == 0) a.u0[b * NU17 + m] = uo;
        }
      }
    };
    constexpr bool F64 = sizeof(T) == 8;
    const T ipm_tol = T(F64 ? IPM17_TOL : IPM17_TOL_F32), ipm_brk = T(F64 ? IPM17_BREAK : IPM17_BREAK_F32);
    const T ipm_res = T(F64 ? IPM17_RES : IPM17_RES_F32);
    QSTAMP_INIT();
    for (int it = 0; it < it_max; ++it) {
      QSTAMP(6);
      // duality measure mu = mean(lambda s), primal residual of the state rows: a pass over the
      // rows at the start, afterwards summed by the update pass of the previous iteration (same
      // rows, same order, same arithmetic); an instance that did not move keeps its values
      if (it > 0) {
        const T mu_n = row_sum(part_n) / (T(2) * rows), res_nr = row_max(res_n);
        if (apend != T(0)) {
          mu = mu_n;
          res = sbox ? res_nr : T(0);
        }
      } else {
      T part = T(0);
      res = T(0);
      if (in) {
#pragma unroll 4
        for (int k = 0; k < N; ++k) {
          const T ubk = r.w.UB[(int64_t)k * NU17 + m];
          const T* ip = r.w.IP + (int64_t)k * 18;
          part += ip[6 + m] * (ip[m] - (lbm - ubk)) + ip[12 + m] * ((ubm - ubk) - ip[m]);
        }
      }
      if (sbox) {
        auto acc_row = [&](int k, int i) {
          const SRow<T> sr(r, k, i);
          part += sr.ll * sr.sl + sr.lu * sr.su;
          res = fmax(res, fmax(fabs(sr.rl), fabs(sr.ru)));
        };
#pragma unroll 4
        for (int k = 1; k < N; ++k) acc_row(k, s);
        for (int k = 1 + t; k < N; k += LN) acc_row(k, OM);
      }
      mu = row_sum(part) / (T(2) * rows);
      if (sbox) res = row_max(res);
      }
      done = done || (!(mu > ipm_tol) && !(res > ipm_res));
      if (polish) {
        if (it == a.max_as_iter && !done) {   // the interior point's own cap
          done = true;
          st = (st == MPCB_STATUS_OK) ? MPCB_STATUS_MAXITER : st;
        }
        if (pst == 0 && done) {
          if (st == MPCB_STATUS_OK && valid) {
            classify();
            pst = 1;
          } else {
            pst = 3;
          }
        }
        __syncthreads();   // the rows of state 8 are read by every lane of the next backward
      }
      const bool finished = polish ? pst >= 2 : done;
      if (finished && !parked) {
        emit();
        parked = true;
        r.ks = 0;
      }
      if (__all(finished || !valid)) break;
      QSTAMP(0);
      T smu;
      if constexpr (!MEH) {
      // centring follows the previous step: sigma = clip(1 - alpha, 0.05, 0.9)
      nit += (pst == 0 && !done) ? 1 : 0;
      smu = fmin(T(IPM17_SIGMA_MAX), fmax(T(IPM17_SIGMA_MIN), T(1) - prev_alpha)) * mu;
      const bool ok_b = backward<T, false, POLC, SBX>(r, smu, apend, pst == 1 || pst == 2);
      apend = T(0);
      if (!ok_b && !done) {
        // a Newton system that lost positive definiteness near the solution: keep the current
        // iterate as converged; earlier it is a failure
        if (!(mu > ipm_brk) && !(res > ipm_res)) {
          done = true;
          early = true;
        } else {
          st = MPCB_STATUS_QP_FAIL;
        }
      }
      __syncthreads();
      QSTAMP(1);
      const bool ffin = forward<T, true, true, false>(r, T(0), T(0), false);   // the Newton step -> DDX, DDU
      __syncthreads();
      QSTAMP(2);
      if (polish && __any(pst == 1)) {
        // one polish pass: rows at z0 + Delta, nu <- nu + rho (y - b) on the active rows, and one
        // active-set change per group (the release of the most negative signed multiplier, else
        // the fix of the inactive row furthest outside its bound)
        const bool pfail = row_or((ok_b && ffin) ? 0 : 1) != 0;
        const bool live = pst == 1 && !pfail;
        T eq_l = T(0), w_l = T(INFINITY), v_l = T(-INFINITY), vside = T(0);
        int wk = 0, wkind = 0, vk = 0, vkind = 0;
        auto prow = [&](int k, int kind, T y, T lb, T ub, T* nup, T side) {
          if (side != T(0)) {
            const T e = y - (side < T(0) ? lb : ub);
            eq_l = fmax(eq_l, fabs(e));
            const T nun = *nup + T(POL17_RHO) * e;
            if (side * nun < w_l) {
              w_l = side * nun;
              wk = k;
              wkind = kind;
            }
            if (live) *nup = nun;
          } else {
            const T v = fmax(lb - y, y - ub);
            if (v > v_l) {
              v_l = v;
              vk = k;
              vkind = kind;
              vside = y < lb ? T(-1) : T(1);
            }
          }
        };
        if (in && pst == 1) {
          for (int k = 0; k < N; ++k) {
            const T ubk = r.w.UB[(int64_t)k * NU17 + m];
            T* ip = r.w.IP + (int64_t)k * 18;
            prow(k, 0, ip[m] + r.w.DDU[(int64_t)k * NU17 + m], lbm - ubk, ubm - ubk, ip + 6 + m, ip[12 + m]);
          }
        }
        auto srow = [&](int k, int i, int kind) {
          const int64_t kx = (int64_t)k * NX17 + i;
          const T xb = r.w.XB[kx];
          T* ix = r.w.IX + (int64_t)k * 4 * NX17 + i;
          prow(k, kind, r.w.DX[kx] + r.w.DDX[kx], W.lbx[i] - xb, W.ubx[i] - xb, ix + 2 * NX17, ix[3 * NX17]);
        };
        if (pst == 1) {
          for (int k = 1; k < N; ++k) srow(k, s, 1);
          for (int k = 1 + t; k < N; k += LN) srow(k, OM, 2);
        }
        const T eq = row_max(eq_l), wmin = row_min(w_l), vmax = row_max(v_l);
        const bool rel = wmin < T(0);
        const bool add = !rel && vmax > T(POL17_FEAS);
        // the lowest lane holding the extreme row makes the change
        const bool cand = rel ? (w_l == wmin) : (add && v_l == vmax);
        const bool win = live && (rel || add) && row_min(cand ? T(t) : T(LN)) == T(t);
        if (win) {
          const int k = rel ? wk : vk, kind = rel ? wkind : vkind;
          const T side = rel ? T(0) : vside;
          T* slot = kind == 0 ? r.w.IP + (int64_t)k * 18 + 6 + m
                              : r.w.IX + (int64_t)k * 4 * NX17 + 2 * NX17 + (kind == 1 ? s : OM);
          slot[0] = T(0);                              // nu
          slot[kind == 0 ? 6 : NX17] = side;           // side
        }
        if (pst == 1) {
          ++npass;
          pst = pfail ? 3 : (!rel && !add && !(eq > T(POL17_EQ))) ? 2 : (npass >= POL17_ITERS ? 3 : 1);
        }
        __syncthreads();
      }
      } else {
      // predictor: targets 0 -> the affine direction into DAX / DAU (K, k, the factor of Huu and
      // the stage gradients stay in KR / LC / GV)
      nit += !done ? 1 : 0;
      const bool ok_b = backward<T, true, false, false>(r, T(0), apend);
      apend = T(0);
      if (!ok_b && !done) {
        if (!(mu > ipm_brk)) {
          done = true;
          early = true;
        } else {
          st = MPCB_STATUS_QP_FAIL;
        }
      }
      __syncthreads();
      QSTAMP(1);
      forward<T, true, true, false>(r, T(0), T(0), false, r.wm.DAX, r.wm.DAU);
      __syncthreads();
      QSTAMP(2);
      // the affine step to the boundary alpha_a, mu_a = (S0 + alpha_a S1 + alpha_a^2 S2) / (2 rows),
      // and per input row w = 1/s_l - 1/s_u, c = Delta s_a Delta lambda_a / s_l - (upper) into DC
      // (the state entries zero: no state rows here)
      // (ratio tests as the largest -dv / v over the rows, by the rows' reciprocals: aa = 1 /
      // max(1, that), no division per row)
      T raa = T(1), S0 = T(0), S1 = T(0), S2 = T(0);
      if (in && !parked) {
#pragma unroll 4
        for (int k = 0; k < N; ++k) {
          const T ubk = r.w.UB[(int64_t)k * NU17 + m];
          const T* ip = r.w.IP + (int64_t)k * 18;
          const T d = r.wm.DAU[(int64_t)k * NU17 + m];
          const T sl = ip[m] - (lbm - ubk), su = (ubm - ubk) - ip[m], ll = ip[6 + m], lu = ip[12 + m];
          const T isl = recip(sl), isu = recip(su);
          const T dsl = d, dsu = -d;
          const T dll = (-ll * sl - ll * dsl) * isl, dlu = (-lu * su - lu * dsu) * isu;
          raa = fmax(raa, fmax(fmax(-dsl * isl, -dsu * isu), fmax(-dll * recip(ll), -dlu * recip(lu))));
          S0 += sl * ll + su * lu;
          S1 += sl * dll + ll * dsl + su * dlu + lu * dsu;
          S2 += dsl * dll + dsu * dlu;
          T* dc = r.wm.DC + (int64_t)k * WsM17<T>::DC_N + NX17 + m;
          dc[0] = isl - isu;
          dc[24] = dsl * dll * isl - dsu * dlu * isu;
        }
      }
      if (!parked) {
        for (int k = 0; k < N; ++k) {
          T* dc = r.wm.DC + (int64_t)k * WsM17<T>::DC_N;
          dc[s] = T(0);
          dc[24 + s] = T(0);
        }
        for (int k = t; k < N; k += LN) {
          T* dc = r.wm.DC + (int64_t)k * WsM17<T>::DC_N;
          dc[OM] = T(0);
          dc[24 + OM] = T(0);
        }
      }
      const T aa = T(1) / row_max(raa);
      const T mu_a = (row_sum(S0) + aa * row_sum(S1) + aa * aa * row_sum(S2)) / (T(2) * rows);
      const T ratio = mu_a / mu;
      const T sig3 = ratio * ratio * ratio;
      const T sig = (sig3 != sig3) ? T(1) : fmin(fmax(sig3, T(0)), T(1));
      smu = sig * mu;
      __syncthreads();
      QSTAMP(7);
      // corrector: the vector Riccati pass for the corrector's gradient (new k), then its direction
      backward_corr<T>(r, smu);
      __syncthreads();
      QSTAMP(8);
      forward<T, true, true, false>(r, T(0), T(0), false);   // -> DDX, DDU
      __syncthreads();
      QSTAMP(9);
      }
      // step length: fraction tau to the boundary, primal and dual, common to the instance
      // (the ratio tests as in the predictor: the largest -dv / v, from tau; amax = 1 / that)
      T ram = T(IPM17_TAU);
      bool dfin = true;   // a finite direction from strictly positive slacks and multipliers
      if (in && !parked) {
#pragma unroll 4
        for (int k = 0; k < N; ++k) {
          const T ubk = r.w.UB[(int64_t)k * NU17 + m];
          const T* ip = r.w.IP + (int64_t)k * 18;
          const T d = r.w.DDU[(int64_t)k * NU17 + m];
          const T sl = ip[m] - (lbm - ubk), su = (ubm - ubk) - ip[m];
          const T ll = ip[6 + m], lu = ip[12 + m];
          const T isl = recip(sl), isu = recip(su);
          T tl = smu, tu = smu;
          if constexpr (MEH) {
            const T da = r.wm.DAU[(int64_t)k * NU17 + m];
            targets(smu, sl, su, ll, lu, da, -da, tl, tu, isl, isu);
          }
          const T dll = (tl - ll * sl - ll * d) * isl, dlu = (tu - lu * su + lu * d) * isu;
          // (recip() is NaN at 0, which fmax would drop from the ratio test: a multiplier that
          // reached 0 is a breakdown, not an unlimited step -- ADVICE r3)
          dfin = dfin && sl > T(0) && su > T(0) && ll > T(0) && lu > T(0) && isfin(d) && isfin(dll) && isfin(dlu);
          ram = fmax(ram, fmax(fmax(-d * isl, d * isu), fmax(-dll * recip(ll), -dlu * recip(lu))));
        }
      }
      if (sbox && !parked) {
        auto step_row = [&](int k, int i) {
          const SRow<T> sr(r, k, i);
          const T dy = r.w.DDX[(int64_t)k * NX17 + i];
          const T dsl = dy + sr.rl, dsu = sr.ru - dy;
          const T isl = recip(sr.sl), isu = recip(sr.su);
          const T dll = (smu - sr.ll * sr.sl - sr.ll * dsl) * isl;
          const T dlu = (smu - sr.lu * sr.su - sr.lu * dsu) * isu;
          dfin = dfin && sr.sl > T(0) && sr.su > T(0) && sr.ll > T(0) && sr.lu > T(0) && isfin(dsl) &&
                 isfin(dsu) && isfin(dll) && isfin(dlu);
          ram = fmax(ram, fmax(fmax(-dsl * isl, -dsu * isu), fmax(-dll * recip(sr.ll), -dlu * recip(sr.lu))));
        };
#pragma unroll 4
        for (int k = 1; k < N; ++k) step_row(k, s);
        for (int k = 1 + t; k < N; k += LN) step_row(k, OM);
      }
      const T amax = T(1) / row_max(ram);
      QSTAMP(3);
      const int dbad = row_or(dfin ? 0 : 1);
      // (a finished instance skips the updates: its Newton step may be non-finite)
      const T alpha = fmin(T(1), T(IPM17_TAU) * amax);
      prev_alpha = alpha;
      if (!done && dbad) {   // no usable direction: converged near the solution, else a failure
        if (mu > ipm_brk || res > ipm_res) st = MPCB_STATUS_QP_FAIL;
        else early = true;
        done = true;
      }
      nshort = (alpha < T(sbox ? IPM17_SBOX_SHORT : IPM17_SHORT)) ? nshort + 1 : 0;
      if (!done && (alpha < T(IPM17_STALL) || nshort >= (sbox ? IPM17_SBOX_SHORT_RUN : IPM17_SHORT_RUN))) {
        // collapsed step, or a run of short ones: converged near the solution (conditioning
        // limit), else an infeasible QP
        if (mu > ipm_brk || res > ipm_res) st = MPCB_STATUS_QP_FAIL;
        else early = true;
        done = true;
      }
      part_n = T(0);
      res_n = T(0);
      if (!done && valid && in) {
#pragma unroll 4
        for (int k = 0; k < N; ++k) {
          const T ubk = r.w.UB[(int64_t)k * NU17 + m];
          T* ip = r.w.IP + (int64_t)k * 18;
          const T d = r.w.DDU[(int64_t)k * NU17 + m];
          const T sl = ip[m] - (lbm - ubk), su = (ubm - ubk) - ip[m];
          const T ll = ip[6 + m], lu = ip[12 + m];
          const T isl = recip(sl), isu = recip(su);
          T tl = smu, tu = smu;
          if constexpr (MEH) {
            const T da = r.wm.DAU[(int64_t)k * NU17 + m];
            targets(smu, sl, su, ll, lu, da, -da, tl, tu, isl, isu);
          }
          const T dll = (tl - ll * sl - ll * d) * isl, dlu = (tu - lu * su + lu * d) * isu;
          const T dun = ip[m] + alpha * d, lln = ll + alpha * dll, lun = lu + alpha * dlu;
          ip[m] = dun;
          ip[6 + m] = lln;
          ip[12 + m] = lun;
          part_n += lln * (dun - (lbm - ubk)) + lun * ((ubm - ubk) - dun);
        }
      }
      if (!done && valid && sbox) {   // state-row slacks and multipliers (before DX moves)
        auto upd_row = [&](int k, int i) {
          const SRow<T> sr(r, k, i);
          const T dy = r.w.DDX[(int64_t)k * NX17 + i];
          const T dsl = dy + sr.rl, dsu = sr.ru - dy;
          const T dll = (smu - sr.ll * sr.sl - sr.ll * dsl) * recip(sr.sl);
          const T dlu = (smu - sr.lu * sr.su - sr.lu * dsu) * recip(sr.su);
          T* ix = r.w.IX + (int64_t)k * 4 * NX17 + i;
          SRow<T> nr = sr;   // the row after the step (dx moves by alpha ddx in the next backward)
          nr.y = sr.y + alpha * dy;
          nr.sl = sr.sl + alpha * dsl;
          nr.su = sr.su + alpha * dsu;
          nr.ll = sr.ll + alpha * dll;
          nr.lu = sr.lu + alpha * dlu;
          nr.rl = nr.y - nr.lb - nr.sl;
          nr.ru = nr.ub - nr.y - nr.su;
          ix[0] = nr.sl;
          ix[NX17] = nr.su;
          ix[2 * NX17] = nr.ll;
          ix[3 * NX17] = nr.lu;
          part_n += nr.ll * nr.sl + nr.lu * nr.su;
          res_n = fmax(res_n, fmax(fabs(nr.rl), fabs(nr.ru)));
        };
#pragma unroll 4
        for (int k = 1; k < N; ++k) upd_row(k, s);
        for (int k = 1 + t; k < N; k += LN) upd_row(k, OM);
      }
      __syncthreads();   // the rows of state 8 are read by every lane of the next backward
      QSTAMP(4);
      apend = (!done && valid) ? alpha : T(0);
    }
    QSTAMP(5);
    QSTAMP_DONE("ipm");
    if (!done) st = (st == MPCB_STATUS_OK) ? MPCB_STATUS_MAXITER : st;
    // an fp64 stop at the conditioning limit that no polish certified: reduced accuracy, acados'
    // MINSTEP (the fp32 interior point stops there by design: its tolerances are scaled)
    if (sizeof(T) == 8 && st == MPCB_STATUS_OK && early && pst != 2) st = MPCB_STATUS_MINSTEP;
    if (valid && t == 0 && a.qp_stats) {
      a.qp_stats[2 * b] = nit;
      a.qp_stats[2 * b + 1] = npass;
    }
    if (!parked) emit();
  }
  // instance status: any lane's non-finite value marks the instance
  const int bad = row_or(fin ? 0 : 1);
  if (valid && t == 0) a.status[b] = bad ? MPCB_STATUS_NAN : st;
}

}  // namespace q17

template <class T> hipError_t launch_riccati17q(const FullArgs<T>& a, hipStream_t st) {
  const dim3 grid((unsigned)((a.nb + q17::GR - 1) / q17::GR));
  if (a.box && !a.sbox && sizeof(T) == 8)
    MPCB_LAUNCH(PH_RICCATI, (q17::riccati17q_kernel<T, true, true>), grid, dim3(64), 0, st, a);
  else if (a.box)
    MPCB_LAUNCH(PH_RICCATI, (q17::riccati17q_kernel<T, true, false>), grid, dim3(64), 0, st, a);
  else
    MPCB_LAUNCH(PH_RICCATI, (q17::riccati17q_kernel<T, false, false>), grid, dim3(64), 0, st, a);
  return dry_run() ? hipSuccess : hipGetLastError();
}
template hipError_t launch_riccati17q<double>(const FullArgs<double>&, hipStream_t);
template hipError_t launch_riccati17q<float>(const FullArgs<float>&, hipStream_t);

}  // namespace mpcb
