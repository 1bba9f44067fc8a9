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

#include "../../include/mpcb.h"
#include "mpcb_common.h"

#ifndef MPCB_P2_WAVES
#define MPCB_P2_WAVES
#endif

#ifndef MPCB_P2_WAVES_F32
#define MPCB_P2_WAVES_F32 2
#endif

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

template <class T>
__device__ __forceinline__ void nominal_body(const SplitArgs<T>& a, const int64_t c) {
  const int64_t nb = a.nb;
  if (c >= nb) return;
  const int64_t b = a.b0 + c;
  const int N = a.N;
  const bool iterate = a.mode == MPCB_MODE_ITERATE;
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
    T* xu = soa(a.XU, k, XU_REC, nb, c);
#pragma unroll
    for (int i = 0; i < NX; ++i) xu[i * SS] = x[i];
#pragma unroll
    for (int m = 0; m < NU; ++m) xu[(NX + m) * SS] = u[m];
    T* cc = soa(a.CC, k, CCS_REC, nb, c);
    T xn[NX];
    rk4_nom<T>(x, u, a.h, a.M, w, xn, [&](int stage, const T* cv) {
#pragma unroll
      for (int i = 0; i < LIN_N; ++i) cc[(stage * LIN_N + i) * SS] = cv[i];
    });
    if (iterate) {
      const T* nx = xbp + (int64_t)(k + 1) * NX;
      T* gp = soa(a.GP, k, GP_REC, nb, c);
#pragma unroll
      for (int i = 0; i < NX; ++i) gp[i * SS] = xn[i] - nx[i];
    } else {
#pragma unroll
      for (int i = 0; i < NX; ++i) x[i] = xn[i];
    }
  }
  if (iterate) load_vec<NX>(xbp + (int64_t)N * NX, x);
  T* xu = soa(a.XU, N, XU_REC, nb, c);
#pragma unroll
  for (int i = 0; i < NX; ++i) xu[i * SS] = x[i];
#pragma unroll
  for (int m = 0; m < NU; ++m) xu[(NX + m) * SS] = T(0);
}

template <class T>
__device__ __forceinline__ void riccati_body(const SplitArgs<T>& a, const int64_t c_raw) {
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
  const bool iterate = a.mode == MPCB_MODE_ITERATE;
  const bool valid = c_raw < a.nb;
  const int64_t c = valid ? c_raw : a.nb - 1;
  const int64_t b = a.b0 + c;
  const int64_t nb = a.nb;
  const T* xr = a.xref + b * a.xref_sb;
  const T* ur = a.uref + b * a.uref_sb;

  T pj;      // p_{k+1}[j]
  T Pc[NX];  // column j of P_{k+1} (zero in the input lanes: P padded to 16x16)
  {
    const T xN = soa(a.XU, N, XU_REC, nb, c)[jx * SS];
    L.v[j] = (j < NX) ? xN - xr[(int64_t)N * NX + jx] : T(0);
    __syncthreads();
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
    __syncthreads();
  }
  bool qp_ok = true;
  T kff0 = T(0);
  // Stage data is prefetched one stage ahead into registers (5 linearisation scalars, the own
  // component of ybar and yref, one gap value per lane) and committed to a double-buffered LDS
  // copy, so the tangent integrates from LDS and no global-load latency sits on the chain.
  __shared__ T Cst[2][GROUPS][CCS_REC + GP_REC];
  T pc[5], pyb, pyr, pgp = T(0);
  auto prefetch = [&](int k) {
    const T* cc = soa(a.CC, k, CCS_REC, nb, c);
#pragma unroll
    for (int r = 0; r < 5; ++r) pc[r] = cc[(j + 16 * r) * SS];
    pyb = soa(a.XU, k, XU_REC, nb, c)[j * SS];
    pyr = (j < NX) ? xr[(int64_t)k * NX + jx] : ur[(int64_t)k * NU + ju];
    if (iterate && j < NX) pgp = soa(a.GP, k, GP_REC, nb, c)[j * SS];
  };
  auto commit = [&](int bufi) {
#pragma unroll
    for (int r = 0; r < 5; ++r) Cst[bufi][q][j + 16 * r] = pc[r];
    if (j < NX) Cst[bufi][q][CCS_REC + j] = pgp;
  };
  prefetch(N - 1);
  commit(0);
  T cyb = pyb, cyr = pyr;
  int buf = 0;
  __syncthreads();
  for (int k = N - 1; k >= 0; --k) {
    if (k > 0) prefetch(k - 1);
    T col[NX];
    {
      const T* cc = &Cst[buf][q][0];
      L.v[j] = cyb - cyr;
      T dx[NX], du[NU];
#pragma unroll
      for (int i = 0; i < NX; ++i) dx[i] = (j == i) ? T(1) : T(0);
#pragma unroll
      for (int m = 0; m < NU; ++m) du[m] = (j == NX + m) ? T(1) : T(0);
      rk4_tan<T>(cc, dx, du, a.h, a.M, col);
      T pt = pj;
      if (iterate) {
#pragma unroll
        for (int i = 0; i < NX; ++i) pt += Pc[i] * cc[CCS_REC + i];
      }
      L.hv[j] = pt;
    }
    if constexpr (sizeof(T) == 8) {   // fp64 path contracts through LDS; fp32 uses MFMA
#pragma unroll
      for (int i = 0; i < NX; ++i) L.X[j * NX + i] = col[i];
    }
    __syncthreads();
    T hj = T(0);
#pragma unroll
    for (int l = 0; l < NX; ++l) hj += col[l] * L.hv[l];
    T G[NZ];
    if constexpr (sizeof(T) == 4) {
      // Y = P [A|B] and G = [A|B]^T Y on the matrix cores (24 MFMAs per 4 instances)
      float y[16], g[16];
      to_columns(outer12(Pc, col), y);     // lane (q,j): Y_q[:, j]  (P symmetric: row = column)
      to_columns(outer12(col, y), g);      // lane (q,j): G_q[:, j]
#pragma unroll
      for (int i = 0; i < NZ; ++i) G[i] = g[i];
    } else {
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
        for (int l = 0; l < NX; ++l) acc += L.X[i * NX + l] * y[l];
        G[i] = acc;
      }
    }
    {
      T acc = T(0);
      if (j < NX) {
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          G[i] += s * W.Q[i * NX + jx];
          acc += W.Q[jx * NX + i] * L.v[i];
        }
      } else {
#pragma unroll
        for (int n = 0; n < NU; ++n) {
          G[NX + n] += s * W.R[n * NU + ju];
          acc += W.R[ju * NU + n] * L.v[NX + n];
        }
      }
      hj += s * acc;
    }
#pragma unroll
    for (int m = 0; m < NU; ++m) L.Hu[j * NU + m] = G[NX + m];
    __syncthreads();
    L.hv[j] = hj;
    __syncthreads();
    T Huu[NU * NU], hu[NU];
#pragma unroll
    for (int m = 0; m < NU; ++m) {
#pragma unroll
      for (int n = 0; n < NU; ++n) Huu[m * NU + n] = L.Hu[(NX + n) * NU + m];
      hu[m] = -L.hv[NX + m];
    }
    T Lc[10];
    chol4(Huu, Lc);
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 10; ++i) ok = ok && (Lc[i] == Lc[i]);
    qp_ok = qp_ok && ok;
    T kff[NU], Kj[NU], nh[NU];
    chol4_solve(Lc, hu, kff);
#pragma unroll
    for (int m = 0; m < NU; ++m) nh[m] = -G[NX + m];
    chol4_solve(Lc, nh, Kj);
    T pn = hj;
#pragma unroll
    for (int m = 0; m < NU; ++m) pn += G[NX + m] * kff[m];
    T Pn[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      T acc = G[i];
#pragma unroll
      for (int m = 0; m < NU; ++m) acc += L.Hu[i * NU + m] * Kj[m];
      Pn[i] = acc;
    }
    if (valid) {
      T* kr = soa(a.KR, k, KR_REC, nb, c);
      if (j < NX) {
#pragma unroll
        for (int m = 0; m < NU; ++m) kr[(4 * j + m) * SS] = Kj[m];
      } else {
        kr[(4 * NX + ju) * SS] = sel<NU>(kff, ju);
      }
    }
    kff0 = sel<NU>(kff, ju);
    __syncthreads();
    // symmetric by construction: entry (r, c) from lane max(r, c) (see mpcb_solve.hip)
    if (j < NX) {
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        if (i <= j) L.P[j * NX + i] = Pn[i];
        if (i < j) L.P[i * NX + j] = Pn[i];
      }
    }
    pj = pn;
    if (k > 0) commit(buf ^ 1);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NX; ++i) Pc[i] = (j < NX) ? L.P[jx * NX + i] : T(0);
    buf ^= 1;
    cyb = pyb;
    cyr = pyr;
  }
  if (valid && j == NX) a.status[b] = qp_ok ? MPCB_STATUS_OK : MPCB_STATUS_QP_FAIL;
  if (valid && !a.fwd && j >= NX) {
    // rollout mode without trajectories: dx_0 = 0 so u0 = ubar_0 + kff_0
    const T u = cyb + kff0;   // cyb = own component of (xbar_0 | ubar_0)
    a.u0[b * NU + ju] = u;
    const bool fin = (u - u) == T(0);
    if (!fin) a.status[b] = MPCB_STATUS_NAN;
  }
}

// USE_CC: integrate the tangent from the captured linearisation scalars (fused small-batch
// path: CC is slot-local and L2-resident) instead of re-evaluating f with sin/cos per stage
// (split path: saves re-reading 80 scalars per stage from HBM).
template <class T, bool USE_CC = false>
__device__ __forceinline__ void forward_body(const SplitArgs<T>& a, const int64_t c) {
  // Recomputes the nominal RK4 stages (one fused value+tangent pass, mpcb_model.h rk4<T,true>)
  // instead of re-reading the 80 captured scalars: per stage it streams only xbar/ubar (16)
  // and the gains (52), prefetched one stage ahead.
  const int64_t nb = a.nb;
  if (c >= nb) return;
  const int64_t b = a.b0 + c;
  const int N = a.N;
  const bool iterate = a.mode == MPCB_MODE_ITERATE;
  T w[3] = {T(0), T(0), T(0)};
  if (a.wind) {
    w[0] = a.wind[b * a.wind_sb]; w[1] = a.wind[b * a.wind_sb + 1]; w[2] = a.wind[b * a.wind_sb + 2];
  }
  T xb[NX], ub[NU], kr[KR_REC];
  {
    const T* xu = soa(a.XU, 0, XU_REC, nb, c);
#pragma unroll
    for (int i = 0; i < XU_REC; ++i) (i < NX ? xb[i] : ub[i - NX]) = xu[i * SS];
    const T* k0 = soa(a.KR, 0, KR_REC, nb, c);
#pragma unroll
    for (int i = 0; i < KR_REC; ++i) kr[i] = k0[i * SS];
  }
  T dx[NX];
  {
    const T* x0 = a.x0 + b * a.x0_sb;
#pragma unroll
    for (int i = 0; i < NX; ++i) dx[i] = iterate ? x0[i] - xb[i] : T(0);
  }
  bool fin = true;
  for (int k = 0; k < N; ++k) {
    // prefetch stage k+1
    T xn[NX], un[NU], krn[KR_REC];
    {
      const T* xu = soa(a.XU, k + 1, XU_REC, nb, c);
#pragma unroll
      for (int i = 0; i < XU_REC; ++i) (i < NX ? xn[i] : un[i - NX]) = xu[i * SS];
      if (k + 1 < N) {
        const T* kp = soa(a.KR, k + 1, KR_REC, nb, c);
#pragma unroll
        for (int i = 0; i < KR_REC; ++i) krn[i] = kp[i * SS];
      }
    }
    T du[NU];
#pragma unroll
    for (int m = 0; m < NU; ++m) du[m] = kr[4 * NX + m];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
#pragma unroll
      for (int m = 0; m < NU; ++m) du[m] += kr[4 * i + m] * dx[i];
    }
    if (a.X) {
      T* Xo = a.X + (b * (N + 1) + k) * NX;
#pragma unroll
      for (int i = 0; i < NX; ++i) Xo[i] = xb[i] + dx[i];
    }
    if (a.U || k == 0) {
      T uo[NU];
#pragma unroll
      for (int m = 0; m < NU; ++m) { uo[m] = ub[m] + du[m]; fin = fin && (uo[m] - uo[m] == T(0)); }
      if (a.U) store_vec<NU>(a.U + (b * N + k) * NU, uo);
      if (k == 0) store_vec<NU>(a.u0 + b * NU, uo);
    }
    T phi[NX], dphi[NX];
    if constexpr (USE_CC) {
      rk4_tan<T, false>(soa(a.CC, k, CCS_REC, nb, c), dx, du, a.h, a.M, dphi, SS);
      if (iterate) {
        const T* gp = soa(a.GP, k, GP_REC, nb, c);
#pragma unroll
        for (int i = 0; i < NX; ++i) phi[i] = gp[i * SS] + xn[i];
      }
    } else {
      rk4<T, true>(xb, dx, ub, du, a.h, a.M, w, phi, dphi);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) dx[i] = iterate ? dphi[i] + (phi[i] - xn[i]) : dphi[i];
#pragma unroll
    for (int i = 0; i < NX; ++i) xb[i] = xn[i];
#pragma unroll
    for (int m = 0; m < NU; ++m) ub[m] = un[m];
#pragma unroll
    for (int i = 0; i < KR_REC; ++i) kr[i] = krn[i];
  }
  if (a.X) {
    T* Xo = a.X + (b * (N + 1) + N) * NX;
#pragma unroll
    for (int i = 0; i < NX; ++i) Xo[i] = xb[i] + dx[i];
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) fin = fin && (dx[i] - dx[i] == T(0));
  if (!fin) a.status[b] = MPCB_STATUS_NAN;
}

template <class T> int64_t split_elems_per_instance(int N, int iterate) {
  return (int64_t)(N + 1) * XU_REC + (int64_t)N * (CCS_REC + KR_REC + (iterate ? GP_REC : 0));
}

template <class T>
__global__ void __launch_bounds__(256) nominal_kernel(SplitArgs<T> a) {
  nominal_body<T>(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}
template <class T, bool USE_CC>
__global__ void __launch_bounds__(256) forward_kernel(SplitArgs<T> a) {
  forward_body<T, USE_CC>(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}
// register budget: fp32 at 2 waves/SIMD (measured faster than 3 with its small spill); fp64 uncapped
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MPCB_P2_WAVES_F32, 8)))
riccati_kernel_f32(SplitArgs<float> a) { riccati_body<float>(a, (int64_t)blockIdx.x * GROUPS + (threadIdx.x >> 4)); }
__global__ void __launch_bounds__(64) MPCB_P2_WAVES riccati_kernel_f64(SplitArgs<double> a) {
  riccati_body<double>(a, (int64_t)blockIdx.x * GROUPS + (threadIdx.x >> 4));
}

// Small batches: the same three bodies run back to back inside ONE wavefront per 4 instances
// (grid-stride over the batch), on a per-wavefront slot of the workspace.  A 4096-instance
// batch is 1024 wavefronts = one per SIMD, so this launch is latency-bound either way; fusing
// removes the two dependent launch boundaries and keeps the workspace L2-resident.
template <class T>
__global__ void __launch_bounds__(64) fused_kernel(SplitArgs<T> a, int64_t B, int64_t slot_elems) {
  const int lane = threadIdx.x, q = lane >> 4, j = lane & 15;
  T* slot = a.XU + (int64_t)blockIdx.x * slot_elems;
  SplitArgs<T> s = a;
  const int N = a.N;
  s.XU = slot;
  s.CC = s.XU + (int64_t)(N + 1) * GROUPS * XU_REC;
  s.KR = s.CC + (int64_t)N * GROUPS * CCS_REC;
  s.GP = s.KR + (int64_t)N * GROUPS * KR_REC;
  for (int64_t wave = blockIdx.x; wave * GROUPS < B; wave += gridDim.x) {
    s.b0 = wave * GROUPS;
    s.nb = (B - s.b0 < GROUPS) ? B - s.b0 : GROUPS;
    if (j == 0) nominal_body<T>(s, q);
    __syncthreads();
    riccati_body<T>(s, q);
    __syncthreads();
    if (s.fwd && j == 0) forward_body<T, true>(s, q);
    __syncthreads();
  }
}

template <class T> int64_t fused_slot_elems(int N) {
  return split_elems_per_instance<T>(N, 1) * GROUPS;
}

template <class T>
hipError_t launch_fused(const SplitArgs<T>& a, int64_t B, int grid, hipStream_t st) {
  hipLaunchKernelGGL((fused_kernel<T>), dim3(grid), dim3(64), 0, st, a, B, fused_slot_elems<T>(a.N));
  return hipGetLastError();
}

template <class T> hipError_t launch_split(const SplitArgs<T>& a, hipStream_t st, hipEvent_t* ev) {
  const unsigned g256 = (unsigned)((a.nb + 255) / 256);
  const unsigned g64 = (unsigned)((a.nb + GROUPS - 1) / GROUPS);
  if (ev) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL((nominal_kernel<T>), dim3(g256), dim3(256), 0, st, a);
  if (ev) (void)hipEventRecord(ev[1], st);
  if constexpr (sizeof(T) == 4)
    hipLaunchKernelGGL(riccati_kernel_f32, dim3(g64), dim3(64), 0, st, a);
  else
    hipLaunchKernelGGL(riccati_kernel_f64, dim3(g64), dim3(64), 0, st, a);
  if (ev) (void)hipEventRecord(ev[2], st);
  // Small chunks keep the captured scalars cache-resident: integrate the forward tangent from
  // them (no sin/cos).  Large chunks re-evaluate f instead of streaming 80 scalars per stage
  // back from HBM.
  if (a.fwd) {
    if (a.nb <= 16384)
      hipLaunchKernelGGL((forward_kernel<T, true>), dim3(g256), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((forward_kernel<T, false>), dim3(g256), dim3(256), 0, st, a);
  }
  if (ev) (void)hipEventRecord(ev[3], st);
  return hipGetLastError();
}

template hipError_t launch_fused<double>(const SplitArgs<double>&, int64_t, int, hipStream_t);
template hipError_t launch_fused<float>(const SplitArgs<float>&, int64_t, int, hipStream_t);
template int64_t fused_slot_elems<double>(int);
template int64_t fused_slot_elems<float>(int);
template hipError_t launch_split<double>(const SplitArgs<double>&, hipStream_t, hipEvent_t*);
template hipError_t launch_split<float>(const SplitArgs<float>&, hipStream_t, hipEvent_t*);
template int64_t split_elems_per_instance<double>(int, int);
template int64_t split_elems_per_instance<float>(int, int);

}  // namespace mpcb
