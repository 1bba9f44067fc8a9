// mpcb_full.hip — one SQP_RTI step of the reference's full 17-state / 6-input OCP
// (blastermodel.py:70-292, acados_ocp_blasterModel.json: N = 60, Tf = 2,
// W = diag(Q17, R6), W_e = 10 Q17, 25 parameters).
//
// Three launches per chunk:
//   nominal17  one thread per instance: the RK4 rollout of u_ref from x0 (or a copy of the
//              persistent iterate) into the workspace;
//   lin17ws    stage-parallel linearisation, 16 lanes per (instance, stage): lanes 0..13
//              integrate the RK4 tangents seeded with e_j of the 14 dense directions, so column j of
//              [A_k | B_k] lands in a lane (what acados' forward VDE computes); lanes 14 / 15 write
//              the 9 structural columns; gaps in iterate mode (lin17_packed, also behind
//              mpcb_linearize);
//   riccati    the Riccati pass, its forward pass and the interior point of the boxes:
//              riccati17q_kernel (mpcb_r17.hip, 16 lanes per instance, the default) or, with
//              MPCB_R17=0, riccati17_kernel below (32 lanes per instance, two per one-wave
//              workgroup, lane j owning column j of the stage Hessian: P, [A|B] and the Hessian
//              columns meet in LDS, the 6x6 input block is factorised redundantly per lane, P is
//              symmetric by construction), each ending with the forward pass (du = K dx + k,
//              dx' = [A|B] (dx, du) + gap) that writes u0, X = xbar + dx, U = ubar + du, status.
// The 12/4 slice has its own MI355X-tuned kernels (mpcb_split.hip); this path carries the full
// model at the reference's own dimensions and is not on the BASELINE benchmark configs.
#include <hip/hip_runtime.h>

#include "../../include/mpcb.h"
#include "mpcb_common.h"
#include "mpcb_full.h"

namespace mpcb {

constexpr int L17 = 32;            // lanes per instance
constexpr int G17 = 64 / L17;      // instances per wavefront

template <class T>
struct FullLds {
  T P[NX17 * NX17];   // P[l*17 + i] = column l of P_{k+1}
  T X[L17 * NX17];    // X[j*17 + i] = [A|B]_{i j}; reused for P's symmetric exchange
  T Hu[L17 * NU17];   // Hu[j*6 + m] = G_{17+m, j}
  T v[L17];           // e = ybar - yref (own component per lane)
  T hv[L17];          // p + P b, then the gradient h
  T z[L17];           // forward pass exchange (dx | du)
  T gp[NX17];         // gap of this stage
};

// ---- phase 0: nominal trajectory, one thread per instance (a serial RK4 chain) ---------------
template <class T>
__global__ void __launch_bounds__(64) nominal17_kernel(FullArgs<T> a) {
  const int64_t c = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (c >= a.nb) return;
  const int64_t b = a.b0 + c;
  const int N = a.N;
  const bool iterate = a.mode == MPCB_MODE_ITERATE;
  Ws17<T> w(a.ws + c * full17_elems(N), N);
  if (iterate) {   // the persistent iterate (X/U may alias xbar/ubar: copy it first)
    for (int i = 0; i < (N + 1) * NX17; ++i) w.XB[i] = a.xbar[b * (int64_t)(N + 1) * NX17 + i];
    for (int i = 0; i < N * NU17; ++i) w.UB[i] = a.ubar[b * (int64_t)N * NU17 + i];
    return;
  }
  P17<T> P;
  const T* pb = a.p ? a.p + b * a.p_sb : a.W->p;
  const int64_t pkb = a.p ? a.p_kb : 0;   // stage-varying parameters (acados set(k, 'p'))
  unpack_p17(pb, P);
  const T* ur = a.uref + b * a.uref_sb;
  T x[NX17], u[NU17];
#pragma unroll
  for (int i = 0; i < NX17; ++i) {
    x[i] = a.x0[b * a.x0_sb + i];
    w.XB[i] = x[i];
  }
  for (int k = 0; k < N; ++k) {
#pragma unroll
    for (int m = 0; m < NU17; ++m) {
      u[m] = ur[(int64_t)k * NU17 + m];
      w.UB[(int64_t)k * NU17 + m] = u[m];
    }
    T xn[NX17];
    if (pkb && k) unpack_p17(pb + k * pkb, P);
    rk4_17<T, false>(x, nullptr, u, nullptr, a.h, a.M, P, xn, nullptr);
#pragma unroll
    for (int i = 0; i < NX17; ++i) {
      x[i] = xn[i];
      w.XB[(int64_t)(k + 1) * NX17 + i] = xn[i];
    }
  }
}

// The same rollout with 16 lanes per instance (4 instances per wavefront): the serial chain's
// cost is the five sin/cos of every f evaluation, so lane t < 5 evaluates the pair of angle t and
// a DPP row broadcast (v_mov_b32_dpp row_newbcast) hands the ten values to the row; the rest of
// f17 runs redundantly in the 16 lanes (one instruction stream).  1024 wavefronts at B = 4096
// instead of 64.
template <int L> __device__ __forceinline__ float rowbc(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + L, 0xF, 0xF, true));
}
template <int L> __device__ __forceinline__ double rowbc(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x150 + L, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x150 + L, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
struct Trig17Row {
  int t;   // lane in the 16-lane row
  template <class T>
  __device__ __forceinline__ void operator()(const T* __restrict__ x, T (&sn)[5], T (&cs)[5]) const {
    const uint64_t m1 = lane_mask(t == 1), m2 = lane_mask(t == 2), m3 = lane_mask(t == 3), m4 = lane_mask(t == 4);
    T ang = csel(m1, x[4], x[3]);
    ang = csel(m2, x[5], ang);
    ang = csel(m3, x[12], ang);
    ang = csel(m4, x[13], ang);
    T s0, c0;
    sc(ang, &s0, &c0);
    sn[0] = rowbc<0>(s0); cs[0] = rowbc<0>(c0);
    sn[1] = rowbc<1>(s0); cs[1] = rowbc<1>(c0);
    sn[2] = rowbc<2>(s0); cs[2] = rowbc<2>(c0);
    sn[3] = rowbc<3>(s0); cs[3] = rowbc<3>(c0);
    sn[4] = rowbc<4>(s0); cs[4] = rowbc<4>(c0);
  }
};

template <class T>
__global__ void __launch_bounds__(64) nominal17q_kernel(FullArgs<T> a) {
  const int lane = threadIdx.x;
  const int t = lane & 15;
  const int64_t c_raw = (int64_t)blockIdx.x * 4 + (lane >> 4);
  const bool valid = c_raw < a.nb;
  const int64_t c = valid ? c_raw : a.nb - 1;   // a ragged last wave recomputes the last instance
  const int64_t b = a.b0 + c;
  const int N = a.N;
  Ws17<T> w(a.ws + c * full17_elems(N), N);
  if (a.mode == MPCB_MODE_ITERATE) {   // the persistent iterate (X/U may alias xbar/ubar: copy it first)
    if (valid) {
      for (int i = t; i < (N + 1) * NX17; i += 16) w.XB[i] = a.xbar[b * (int64_t)(N + 1) * NX17 + i];
      for (int i = t; i < N * NU17; i += 16) w.UB[i] = a.ubar[b * (int64_t)N * NU17 + i];
    }
    return;
  }
  const bool wr = valid && t == 0;
  P17<T> P;
  const T* pb = a.p ? a.p + b * a.p_sb : a.W->p;
  const int64_t pkb = a.p ? a.p_kb : 0;   // stage-varying parameters (acados set(k, 'p'))
  unpack_p17(pb, P);
  const T* ur = a.uref + b * a.uref_sb;
  const Trig17Row trig{t};
  T x[NX17], u[NU17];
#pragma unroll
  for (int i = 0; i < NX17; ++i) {
    x[i] = a.x0[b * a.x0_sb + i];
    if (wr) w.XB[i] = x[i];
  }
  for (int k = 0; k < N; ++k) {
#pragma unroll
    for (int m = 0; m < NU17; ++m) {
      u[m] = ur[(int64_t)k * NU17 + m];
      if (wr) w.UB[(int64_t)k * NU17 + m] = u[m];
    }
    T xn[NX17];
    if (pkb && k) unpack_p17(pb + k * pkb, P);
    rk4_17<T, false>(x, nullptr, u, nullptr, a.h, a.M, P, xn, nullptr, trig);
#pragma unroll
    for (int i = 0; i < NX17; ++i) {
      x[i] = xn[i];
      if (wr) w.XB[(int64_t)(k + 1) * NX17 + i] = xn[i];
    }
  }
}

// ---- the linearisation of every interval, stage-parallel: 16 lanes per (instance, stage) -----
constexpr int LQ17 = 16, GQ17 = 64 / LQ17;

// One (instance, stage) of the packed linearisation, lane t < 16: column j of [A_k | B_k] into
// col(j, v[17]) and, on lane 0, the RK4 successor into succ(xn[17]).  Shared by the workspace
// kernel (lin17ws_kernel) and the dense debug export (linearize17_kernel, mpcb_linearize), so the
// parity test of mpcb_linearize covers the arithmetic the solver runs.
template <class T, class Col, class Succ>
__device__ __forceinline__ void lin17_packed(int t, const T* pb, T h, const Model<T>& M, const T* xk,
                                             const T* uk, Col&& colf, Succ&& succ) {
  if (t >= 14) {
    if (t == 14) {   // position and POC-state directions
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const int jj = q < 3 ? q : 11 + q;
        T v[NX17];
#pragma unroll
        for (int i = 0; i < NX17; ++i) v[i] = (i == jj) ? T(1) : T(0);
        colf(jj, v);
      }
    } else {         // velocity directions
      P17<T> P;
      unpack_p17(pb, P);
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        const int jj = 6 + cc;
        T v[NX17];
#pragma unroll
        for (int i = 0; i < NX17; ++i) {
          v[i] = (i == jj) ? T(1) : T(0);
          if (i == cc) v[i] = h;
          if (i >= 14) v[i] = h * P.Jp[(i - 14) * 3 + cc];
        }
        colf(jj, v);
      }
    }
    return;
  }
  const int j = t < 3 ? 3 + t : (t < 8 ? 6 + t : 9 + t);   // 3..5, 9..13, 17..22
  P17<T> P;
  unpack_p17(pb, P);
  T x[NX17], u[NU17], dx[NX17], du[NU17], xn[NX17], col[NX17];
#pragma unroll
  for (int i = 0; i < NX17; ++i) {
    x[i] = xk[i];
    dx[i] = (j == i) ? T(1) : T(0);
  }
#pragma unroll
  for (int m = 0; m < NU17; ++m) {
    u[m] = uk[m];
    du[m] = (j == NX17 + m) ? T(1) : T(0);
  }
  // the five sin/cos of the nominal point: lane t < 5 of the row evaluates one (Trig17Row)
  rk4_17<T, true>(x, dx, u, du, h, M, P, xn, col, Trig17Row{t});
  colf(j, col);
  if (t == 0) succ(xn);
}

// The workspace linearisation packs 4 (instance, stage) pairs per wavefront, 16 lanes each:
// lanes 0..13 integrate the tangents that need the RK4 (Euler angles, body rates, swivel
// angles, the six inputs); lanes 14 / 15 write the 9 constant columns.  f does not depend on
// the position or POC states (column e_j), and it is linear in the velocity with a constant
// Jacobian (dk_1 = .. = dk_4 = c = e_pos + Jp e_v in the POC rows, so RK4 gives e_j + h c).
template <class T>
__global__ void __launch_bounds__(64) lin17ws_kernel(FullArgs<T> a) {
  const int lane = threadIdx.x;
  const int t = lane % LQ17;
  const int N = a.N;
  const int64_t idx = (int64_t)blockIdx.x * GQ17 + lane / LQ17;   // (instance, stage) pair
  if (idx >= a.nb * N) return;
  const int64_t c = idx / N;
  const int k = (int)(idx % N);
  const int64_t b = a.b0 + c;
  const T* pb = a.p ? a.p + b * a.p_sb + k * a.p_kb : a.W->p;
  Ws17<T> w(a.ws + c * full17_elems(N), N);
  T* ABk = w.AB + (int64_t)k * NZ17 * NX17;
  const T* xk = w.XB + (int64_t)k * NX17;
  lin17_packed<T>(t, pb, a.h, a.M, xk, w.UB + (int64_t)k * NU17,
                  [&](int j, const T* v) {
#pragma unroll
                    for (int i = 0; i < NX17; ++i) ABk[j * NX17 + i] = v[i];
                  },
                  [&](const T* xn) {   // gap Phi(xbar_k, ubar_k) - xbar_{k+1}; the rollout is gap-free
#pragma unroll
                    for (int i = 0; i < NX17; ++i)
                      w.GP[(int64_t)k * NX17 + i] = (a.mode == MPCB_MODE_ITERATE) ? xn[i] - xk[NX17 + i] : T(0);
                  });
}

// ---- phases 1 + 2: Riccati backward over the cached [A|B], then the forward pass -------------
// Shared by the unconstrained step and the interior-point iterations of the input box.  The
// backward pass computes K_k, k_k (workspace KR) for the LQ problem around the nominal
// trajectory shifted by (SHIFT: the current IPM iterate dx, du; else 0), with the gaps (IPM: 0)
// and, for IPM, the barrier terms D_k (added to the diagonal of H_uu) and d_k (added to h_u).
// compiler fences inside the two LDS product loops of the backward pass (every YS columns of
// Y = P [A|B], every GS rows of G): they bound how many LDS reads the scheduler hoists
#ifndef MPCB_R17_YS
#define MPCB_R17_YS 4
#endif
#ifndef MPCB_R17_GS
#define MPCB_R17_GS 2
#endif
template <class T>
struct R17 {
  FullLds<T>& L;
  const T* SW;
  const FullArgs<T>& a;
  Ws17<T> w;
  const T* xr;
  const T* ur;
  int j, jd, jx, ju, N;
  bool dir, valid;
};

// One state-box row (stage k, state lane j): dx-coordinate bounds, the iterate y = dx_k[j], its
// slacks / multipliers and the residuals r_l = y - lb - s_l, r_u = ub - y - s_u (the state rows
// start infeasible: oracle.ocp.ipm_box_solve).
template <class T>
struct SRow17 {
  T y, lb, ub, sl, su, ll, lu, rl, ru;
  __device__ __forceinline__ SRow17(const R17<T>& r, int k) {
    const int j = r.j;
    const T xb = r.w.XB[(int64_t)k * NX17 + j];
    y = r.w.DX[(int64_t)k * NX17 + j];
    lb = r.a.W->lbx[j] - xb;
    ub = r.a.W->ubx[j] - xb;
    const T* ix = r.w.IX + (int64_t)k * 4 * NX17 + j;
    sl = ix[0];
    su = ix[NX17];
    ll = ix[2 * NX17];
    lu = ix[3 * NX17];
    rl = y - lb - sl;
    ru = ub - y - su;
  }
};

// The IPM switch is the launch's box flag read at run time, on purpose: the compile-time
// specialisation of the unconstrained pass scheduled the stage loop into 527 spilled VGPRs
// (1976 B scratch per lane in fp64); with the flag opaque to the compiler it spills nothing.
template <class T>
__device__ __forceinline__ bool riccati17_backward(const R17<T>& r, T smu) {
  const bool IPM = r.a.box != 0;
  FullLds<T>& L = r.L;
  const int j = r.j, jd = r.jd, jx = r.jx, ju = r.ju, N = r.N;
  const Weights17<T>& W = *r.a.W;
  constexpr int KR_N = Ws17<T>::KR_N;
  T pj;
  T Pc[NX17];   // column j of P_{k+1} (zero outside the state lanes)
  {
    T xN = (j < NX17) ? r.w.XB[(int64_t)N * NX17 + jx] : T(0);
    if (IPM && j < NX17) xN += r.w.DX[(int64_t)N * NX17 + jx];
    L.v[j] = (j < NX17) ? xN - r.xr[(int64_t)N * NX17 + jx] : T(0);
    wave_lds_sync();
    T acc = T(0);
#pragma unroll
    for (int i = 0; i < NX17; ++i) acc += W.QN[jx * NX17 + i] * L.v[i];
    pj = (j < NX17) ? acc : T(0);
#pragma unroll
    for (int i = 0; i < NX17; ++i) {
      Pc[i] = (j < NX17) ? W.QN[i * NX17 + jx] : T(0);
      if (j < NX17) L.P[j * NX17 + i] = Pc[i];
    }
    wave_lds_sync();
  }
  bool qp_ok = true;
  // stage data one stage ahead (column jd of [A|B], the gap, the own y - yref component): the
  // loads of stage k - 1 are in flight while stage k computes (without it 59 % of the wave time
  // sat in s_waitcnt: PMC)
  T ncol[NX17], ngp, ne;
  auto prefetch = [&](int k) {
    const T* ABk = r.w.AB + ((int64_t)k * NZ17 + jd) * NX17;
#pragma unroll
    for (int i = 0; i < NX17; ++i) ncol[i] = ABk[i];
    ngp = (j < NX17 && !IPM) ? r.w.GP[(int64_t)k * NX17 + jx] : T(0);
    T yb = (j < NX17) ? r.w.XB[(int64_t)k * NX17 + jx] : r.w.UB[(int64_t)k * NU17 + ju];
    if (IPM) yb += (j < NX17) ? r.w.DX[(int64_t)k * NX17 + jx] : r.w.IP[(int64_t)k * 18 + ju];
    const T yr = (j < NX17) ? r.xr[(int64_t)k * NX17 + jx] : r.ur[(int64_t)k * NU17 + ju];
    ne = r.dir ? yb - yr : T(0);
  };
  prefetch(N - 1);
  for (int k = N - 1; k >= 0; --k) {
    T col[NX17];
#pragma unroll
    for (int i = 0; i < NX17; ++i) col[i] = ncol[i];
    if (j < NX17) L.gp[j] = ngp;
    L.v[j] = ne;
    if (k > 0) prefetch(k - 1);
#pragma unroll
    for (int i = 0; i < NX17; ++i) L.X[j * NX17 + i] = col[i];
    wave_lds_sync();
    T pt = pj;
#pragma unroll
    for (int i = 0; i < NX17; ++i) pt += Pc[i] * L.gp[i];
    L.hv[j] = (j < NX17) ? pt : T(0);
    wave_lds_sync();
    T hj = T(0);
#pragma unroll
    for (int l = 0; l < NX17; ++l) hj += col[l] * L.hv[l];
    T y[NX17];
#pragma unroll
    for (int i = 0; i < NX17; ++i) y[i] = T(0);
#pragma unroll
    for (int l = 0; l < NX17; ++l) {
      const T cl = col[l];
#pragma unroll
      for (int i = 0; i < NX17; ++i) y[i] += L.P[l * NX17 + i] * cl;
      if (l % MPCB_R17_YS == MPCB_R17_YS - 1) wave_lds_sync();
    }
    T G[NZ17];
#pragma unroll
    for (int i = 0; i < NZ17; ++i) {
      T acc = T(0);
#pragma unroll
      for (int l = 0; l < NX17; ++l) acc += L.X[i * NX17 + l] * y[l];
      const T wgt = r.SW[jd * NZ17 + i];
      G[i] = acc + wgt;
      hj += wgt * L.v[i];
      if (i % MPCB_R17_GS == MPCB_R17_GS - 1) wave_lds_sync();
    }
    if (IPM) {   // state-box rows of this stage: barrier terms on the state lane's diagonal
      if (r.a.sbox && j < NX17 && k > 0) {
        const SRow17<T> sr(r, k);
        const T Dj = sr.ll / sr.sl + sr.lu / sr.su;
        hj += -smu * (T(1) / sr.sl - T(1) / sr.su) + (sr.ll / sr.sl) * sr.rl - (sr.lu / sr.su) * sr.ru;
#pragma unroll
        for (int i = 0; i < NX17; ++i) G[i] += (i == j) ? Dj : T(0);
      }
    }
#pragma unroll
    for (int m = 0; m < NU17; ++m) L.Hu[j * NU17 + m] = G[NX17 + m];
    wave_lds_sync();
    L.hv[j] = hj;
    wave_lds_sync();
    T Huu[NU17 * NU17], ht[NU17], Lc[NU17 * NU17];
#pragma unroll
    for (int m = 0; m < NU17; ++m) {
#pragma unroll
      for (int n = 0; n < NU17; ++n) Huu[m * NU17 + n] = L.Hu[(NX17 + n) * NU17 + m];
      ht[m] = L.hv[NX17 + m];
    }
    if (IPM) {   // barrier terms of this stage (instance-uniform values)
      const T* ip = r.w.IP + (int64_t)k * 18;
#pragma unroll
      for (int m = 0; m < NU17; ++m) {
        const T ubk = r.w.UB[(int64_t)k * NU17 + m];
        const T sl = ip[m] - (W.lbu[m] - ubk), su = (W.ubu[m] - ubk) - ip[m];
        Huu[m * NU17 + m] += ip[6 + m] / sl + ip[12 + m] / su;
        ht[m] -= smu * (T(1) / sl - T(1) / su);
      }
    }
    chol_n<T, NU17>(Huu, Lc);
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NU17; ++i) ok = ok && (Lc[i * NU17 + i] == Lc[i * NU17 + i]);
    qp_ok = qp_ok && ok;
    T kff[NU17], Kj[NU17], nh[NU17];
#pragma unroll
    for (int m = 0; m < NU17; ++m) nh[m] = -ht[m];
    chol_n_solve<T, NU17>(Lc, nh, kff);
#pragma unroll
    for (int m = 0; m < NU17; ++m) nh[m] = -G[NX17 + m];
    chol_n_solve<T, NU17>(Lc, nh, Kj);
    T pn = hj;
#pragma unroll
    for (int m = 0; m < NU17; ++m) pn += G[NX17 + m] * kff[m];
    T Pn[NX17];
#pragma unroll
    for (int i = 0; i < NX17; ++i) {
      T acc = G[i];
#pragma unroll
      for (int m = 0; m < NU17; ++m) acc += L.Hu[i * NU17 + m] * Kj[m];
      Pn[i] = acc;
    }
    if (r.valid && j < NX17) {
#pragma unroll
      for (int m = 0; m < NU17; ++m) r.w.KR[(int64_t)k * KR_N + j * NU17 + m] = Kj[m];
    }
    if (r.valid && j >= NX17 && r.dir) r.w.KR[(int64_t)k * KR_N + NU17 * NX17 + ju] = sel<NU17>(kff, ju);
    wave_lds_sync();
    // symmetric by construction: entry (r, c) from lane max(r, c)
#pragma unroll
    for (int i = 0; i < NX17; ++i) L.X[j * NX17 + i] = Pn[i];
    pj = (j < NX17) ? pn : T(0);
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < NX17; ++i) {
      Pc[i] = (j < NX17) ? ((i <= j) ? Pn[i] : L.X[i * NX17 + jx]) : T(0);
      if (j < NX17) L.P[j * NX17 + i] = Pc[i];
    }
    wave_lds_sync();
  }
  return qp_ok;
}

// Forward pass over K, k.  GAIN: du = K dx + k; else du from the IPM iterate (the initial
// trajectory).  STEP: the Newton step (zero gaps, dx_0 = 0) into the workspace DDX / DDU.
// Returns this lane's finiteness; writes X / U / u0 when OUT.
template <class T, bool GAIN, bool STEP, bool OUT>
__device__ __forceinline__ bool forward17(const R17<T>& r, T dxj, bool write) {
  FullLds<T>& L = r.L;
  const int j = r.j, ju = r.ju, N = r.N;
  const FullArgs<T>& a = r.a;
  constexpr int KR_N = Ws17<T>::KR_N;
  const bool ilane = j >= NX17 && r.dir;
  const int64_t b = a.b0 + (r.w.XB - a.ws) / full17_elems(N);
  bool fin = true;
  // the stage's row data one stage ahead: state lanes row j of [A_k | B_k] and the gap, input
  // lanes row ju of (K_k | k_k) (or the iterate's du)
  T nr[NZ17 + 1];
  auto prefetch = [&](int k) {
    if (j < NX17) {
      const T* ABk = r.w.AB + (int64_t)k * NZ17 * NX17;
#pragma unroll
      for (int l = 0; l < NZ17; ++l) nr[l] = ABk[l * NX17 + j];
      nr[NZ17] = STEP ? T(0) : r.w.GP[(int64_t)k * NX17 + j];
    } else if (ilane) {
      if constexpr (GAIN) {
        const T* Kk = r.w.KR + (int64_t)k * KR_N;
#pragma unroll
        for (int i = 0; i < NX17; ++i) nr[i] = Kk[i * NU17 + ju];
        nr[NX17] = Kk[NU17 * NX17 + ju];
      } else {
        nr[0] = r.w.IP[(int64_t)k * 18 + ju];
      }
    }
  };
  prefetch(0);
  for (int k = 0; k < N; ++k) {
    T cr[NZ17 + 1];
#pragma unroll
    for (int i = 0; i <= NZ17; ++i) cr[i] = nr[i];
    if (k + 1 < N) prefetch(k + 1);
    if (j < NX17) L.z[j] = dxj;
    wave_lds_sync();
    T duj = T(0);
    if (ilane) {
      if constexpr (GAIN) {
        T acc = cr[NX17];
#pragma unroll
        for (int i = 0; i < NX17; ++i) acc += cr[i] * L.z[i];
        duj = acc;
      } else {
        duj = cr[0];
      }
      L.z[j] = duj;
    }
    wave_lds_sync();
    if (STEP && r.valid && j < NX17) r.w.DDX[(int64_t)k * NX17 + j] = dxj;
    if (STEP && r.valid && ilane) r.w.DDU[(int64_t)k * NU17 + ju] = duj;
    if (!STEP && !OUT && r.valid && j < NX17) r.w.DX[(int64_t)k * NX17 + j] = dxj;
    if (OUT && write && j < NX17 && a.X) a.X[(b * (int64_t)(N + 1) + k) * NX17 + j] = r.w.XB[(int64_t)k * NX17 + j] + dxj;
    if (ilane) {
      const T uo = r.w.UB[(int64_t)k * NU17 + ju] + duj;
      fin = fin && ((uo - uo) == T(0));
      if (OUT && write && a.U) a.U[(b * (int64_t)N + k) * NU17 + ju] = uo;
      if (OUT && write && k == 0) a.u0[b * NU17 + ju] = uo;
    }
    if (j < NX17) {
      T acc = cr[NZ17];
#pragma unroll
      for (int l = 0; l < NZ17; ++l) acc += cr[l] * L.z[l];
      dxj = acc;
    }
    fin = fin && ((dxj - dxj) == T(0));
    wave_lds_sync();
  }
  if (STEP && r.valid && j < NX17) r.w.DDX[(int64_t)N * NX17 + j] = dxj;
  if (!STEP && !OUT && r.valid && j < NX17) r.w.DX[(int64_t)N * NX17 + j] = dxj;
  if (OUT && write && j < NX17 && a.X) a.X[(b * (int64_t)(N + 1) + N) * NX17 + j] = r.w.XB[(int64_t)N * NX17 + j] + dxj;
  return fin;
}

// BOX: the input box lbu <= u <= ubu of the reference OCP (blastermodel.py:259-264; thrust
// [0, 65] N, swivel rate +-0.0873 rad/s) by a primal-dual interior point over the Riccati
// recursion (acados uses HPIPM's; oracle.ocp.ipm_box_solve is the same iteration, incl. the
// adaptive centring sigma = clip(1 - previous step, 0.05, 0.9) and the stall test): Newton steps
// of the barrier-perturbed KKT system linearised at the current iterate (input Hessian + D,
// gradient - sigma mu (1/s_l - 1/s_u)), a common primal/dual step length tau to the boundary,
// until mu = mean(lambda s) <= 1e-12 (or a breakdown of the Newton system once mu <= 1e-8).  (The exact active set of the 12/4 path needs thousands of
// exchanges on this model: the swivel-rate weight is 1e-5.)  With a.sbox also the state box
// lbx <= x_k <= ubx on stages 1..N-1 (blastermodel.py:268-270): explicit slacks and multipliers
// per row (workspace IX, owned by the state lane), an infeasible start, barrier terms on the
// diagonal of H_xx, and convergence also needs max |r| <= 1e-9.
template <class T, bool BOX>
__global__ void __launch_bounds__(64) riccati17_kernel(FullArgs<T> a) {
  __shared__ FullLds<T> lds_all[G17];
  __shared__ T SW[NZ17 * NZ17];   // s * blkdiag(Q, R)
  const int lane = threadIdx.x;
  const int q = lane / L17;
  const int j = lane % L17;
  const int64_t c_raw = (int64_t)blockIdx.x * G17 + q;
  const bool valid = c_raw < a.nb;
  const int64_t c = valid ? c_raw : a.nb - 1;  // a ragged last wave shadows the last instance
  const int64_t b = a.b0 + c;
  const int N = a.N;
  const Weights17<T>& W = *a.W;
  const bool iterate = a.mode == MPCB_MODE_ITERATE;
  const bool dir = j < NZ17;
  const R17<T> r{lds_all[q], SW, a, Ws17<T>(a.ws + c * full17_elems(N), N), a.xref + b * a.xref_sb,
                 a.uref + b * a.uref_sb, j, dir ? j : 0, j < NX17 ? j : 0,
                 (j >= NX17 && dir) ? j - NX17 : 0, N, dir, valid};
  FullLds<T>& L = r.L;
  const bool ilane = j >= NX17 && dir;
  const int ju = r.ju;
  for (int e = lane; e < NZ17 * NZ17; e += 64) {
    const int rr = e / NZ17, cl = e % NZ17;
    const T wq = (rr < NX17 && cl < NX17) ? W.Q[rr * NX17 + cl] : T(0);
    const T wr = (rr >= NX17 && cl >= NX17) ? W.R[(rr - NX17) * NU17 + (cl - NX17)] : T(0);
    SW[e] = a.s * (wq + wr);
  }
  __syncthreads();
  const T* x0 = a.x0 + b * a.x0_sb;
  const T dx0 = (iterate && j < NX17) ? x0[r.jx] - r.w.XB[r.jx] : T(0);
  int32_t st = MPCB_STATUS_OK;
  bool fin;
  if constexpr (!BOX) {
    if (!riccati17_backward<T>(r, T(0))) st = MPCB_STATUS_QP_FAIL;
    __syncthreads();   // K and k are read back across lanes
    fin = forward17<T, true, false, true>(r, dx0, valid);
  } else {
    const T lbm = W.lbu[ju], ubm = W.ubu[ju];
    // start: du strictly inside the box, lambda = 1; dx by the dynamics
    if (valid && ilane) {
      for (int k = 0; k < N; ++k) {
        const T ubk = r.w.UB[(int64_t)k * NU17 + ju];
        const T lb = lbm - ubk, ub = ubm - ubk, wd = ub - lb;
        T* ip = r.w.IP + (int64_t)k * 18;
        ip[ju] = fmin(fmax(T(0), lb + T(IPM17_THETA) * wd), ub - T(IPM17_THETA) * wd);
        ip[6 + ju] = T(1);
        ip[12 + ju] = T(1);
      }
    }
    __syncthreads();
    forward17<T, false, false, false>(r, dx0, false);   // DX of the starting point
    const bool sbox = a.sbox != 0;
    const bool xlane = sbox && j < NX17;
    if (valid && xlane) {   // state rows: s = max(distance to the bound, theta w), lambda = 1
      for (int k = 1; k < N; ++k) {
        const T xb = r.w.XB[(int64_t)k * NX17 + j], y = r.w.DX[(int64_t)k * NX17 + j];
        const T lb = W.lbx[j] - xb, ub = W.ubx[j] - xb, tw = T(IPM17_THETA) * (ub - lb);
        T* ix = r.w.IX + (int64_t)k * 4 * NX17 + j;
        ix[0] = fmax(y - lb, tw);
        ix[NX17] = fmax(ub - y, tw);
        ix[2 * NX17] = T(1);
        ix[3 * NX17] = T(1);
      }
    }
    __syncthreads();
    const T rows = T(N * NU17 + (sbox ? (N - 1) * NX17 : 0));
    bool done = false;
    T prev_alpha = T(1);
    int nshort = 0;
    constexpr bool F64 = sizeof(T) == 8;
    const T ipm_tol = T(F64 ? IPM17_TOL : IPM17_TOL_F32), ipm_brk = T(F64 ? IPM17_BREAK : IPM17_BREAK_F32);
    const T ipm_res = T(F64 ? IPM17_RES : IPM17_RES_F32);
    for (int it = 0; it < a.max_as_iter; ++it) {
      // duality measure mu = mean(lambda s) (input lanes sum over stages, then over components)
      T part = T(0);
      if (ilane) {
#pragma unroll 4
        for (int k = 0; k < N; ++k) {
          const T ubk = r.w.UB[(int64_t)k * NU17 + ju];
          const T* ip = r.w.IP + (int64_t)k * 18;
          part += ip[6 + ju] * (ip[ju] - (lbm - ubk)) + ip[12 + ju] * ((ubm - ubk) - ip[ju]);
        }
      }
      T res = T(0);
      if (xlane) {
#pragma unroll 4
        for (int k = 1; k < N; ++k) {
          const SRow17<T> sr(r, k);
          part += sr.ll * sr.sl + sr.lu * sr.su;
          res = fmax(res, fmax(fabs(sr.rl), fabs(sr.ru)));
        }
      }
      T mu = T(0);
#pragma unroll
      for (int m = 0; m < NZ17; ++m) mu += __shfl(part, q * L17 + m);
      mu /= T(2) * rows;
      if (sbox) {
#pragma unroll
        for (int m = 0; m < NX17; ++m) res = fmax(res, __shfl(res, q * L17 + m));
      }
      done = done || (!(mu > ipm_tol) && !(res > ipm_res));
      if (__all(done || !valid)) break;
      // centring follows the previous step: sigma = clip(1 - alpha, 0.05, 0.9)
      const T smu = fmin(T(IPM17_SIGMA_MAX), fmax(T(IPM17_SIGMA_MIN), T(1) - prev_alpha)) * mu;
      if (!riccati17_backward<T>(r, smu) && !done) {
        // a Newton system that lost positive definiteness near the solution (lambda / s ~ 1e18 on
        // an active row): keep the current iterate as converged; earlier it is a failure
        if (!(mu > ipm_brk) && !(res > ipm_res)) done = true;
        else st = MPCB_STATUS_QP_FAIL;
      }
      __syncthreads();
      forward17<T, true, true, false>(r, T(0), false);   // the Newton step -> DDX, DDU
      __syncthreads();
      // step length: fraction tau to the boundary, primal and dual, common to the instance
      T amax = T(1) / T(IPM17_TAU);
      bool dfin = true;   // a finite direction from strictly positive slacks (fp32 can lose both)
      if (ilane) {
#pragma unroll 4
        for (int k = 0; k < N; ++k) {
          const T ubk = r.w.UB[(int64_t)k * NU17 + ju];
          const T* ip = r.w.IP + (int64_t)k * 18;
          const T d = r.w.DDU[(int64_t)k * NU17 + ju];
          const T sl = ip[ju] - (lbm - ubk), su = (ubm - ubk) - ip[ju];
          const T ll = ip[6 + ju], lu = ip[12 + ju];
          const T dll = (smu - ll * sl - ll * d) / sl, dlu = (smu - lu * su + lu * d) / su;
          dfin = dfin && sl > T(0) && su > T(0) && (d - d) == T(0) && (dll - dll) == T(0) && (dlu - dlu) == T(0);
          if (d < T(0)) amax = fmin(amax, -sl / d);
          if (d > T(0)) amax = fmin(amax, su / d);
          if (dll < T(0)) amax = fmin(amax, -ll / dll);
          if (dlu < T(0)) amax = fmin(amax, -lu / dlu);
        }
      }
      if (xlane) {
#pragma unroll 4
        for (int k = 1; k < N; ++k) {
          const SRow17<T> sr(r, k);
          const T dy = r.w.DDX[(int64_t)k * NX17 + j];
          const T dsl = dy + sr.rl, dsu = sr.ru - dy;
          const T dll = (smu - sr.ll * sr.sl - sr.ll * dsl) / sr.sl;
          const T dlu = (smu - sr.lu * sr.su - sr.lu * dsu) / sr.su;
          dfin = dfin && (dsl - dsl) == T(0) && (dsu - dsu) == T(0) && (dll - dll) == T(0) && (dlu - dlu) == T(0);
          if (dsl < T(0)) amax = fmin(amax, -sr.sl / dsl);
          if (dsu < T(0)) amax = fmin(amax, -sr.su / dsu);
          if (dll < T(0)) amax = fmin(amax, -sr.ll / dll);
          if (dlu < T(0)) amax = fmin(amax, -sr.lu / dlu);
        }
      }
      int dbad = dfin ? 0 : 1;
#pragma unroll
      for (int m = 0; m < NZ17; ++m) {
        amax = fmin(amax, __shfl(amax, q * L17 + m));
        dbad |= __shfl(dbad, q * L17 + m);
      }
      // (a finished instance skips the updates: its Newton step may be non-finite)
      const T alpha = fmin(T(1), T(IPM17_TAU) * amax);
      prev_alpha = alpha;
      if (!done && dbad) {   // no usable direction: converged near the solution, else a failure
        if (mu > ipm_brk || res > ipm_res) st = MPCB_STATUS_QP_FAIL;
        done = true;
      }
      nshort = (alpha < T(IPM17_SHORT)) ? nshort + 1 : 0;
      if (!done && (alpha < T(IPM17_STALL) || nshort >= IPM17_SHORT_RUN)) {
        // collapsed step, or a run of short ones: converged near the solution (conditioning
        // limit), else an infeasible QP
        if (mu > ipm_brk || res > ipm_res) st = MPCB_STATUS_QP_FAIL;
        done = true;
      }
      if (!done && valid && ilane) {
#pragma unroll 4
        for (int k = 0; k < N; ++k) {
          const T ubk = r.w.UB[(int64_t)k * NU17 + ju];
          T* ip = r.w.IP + (int64_t)k * 18;
          const T d = r.w.DDU[(int64_t)k * NU17 + ju];
          const T sl = ip[ju] - (lbm - ubk), su = (ubm - ubk) - ip[ju];
          const T ll = ip[6 + ju], lu = ip[12 + ju];
          const T dll = (smu - ll * sl - ll * d) / sl, dlu = (smu - lu * su + lu * d) / su;
          ip[ju] += alpha * d;
          ip[6 + ju] = ll + alpha * dll;
          ip[12 + ju] = lu + alpha * dlu;
        }
      }
      if (!done && valid && xlane) {   // state-row slacks and multipliers (before DX moves: the residuals use it)
#pragma unroll 4
        for (int k = 1; k < N; ++k) {
          const SRow17<T> sr(r, k);
          const T dy = r.w.DDX[(int64_t)k * NX17 + j];
          const T dsl = dy + sr.rl, dsu = sr.ru - dy;
          const T dll = (smu - sr.ll * sr.sl - sr.ll * dsl) / sr.sl;
          const T dlu = (smu - sr.lu * sr.su - sr.lu * dsu) / sr.su;
          T* ix = r.w.IX + (int64_t)k * 4 * NX17 + j;
          ix[0] = sr.sl + alpha * dsl;
          ix[NX17] = sr.su + alpha * dsu;
          ix[2 * NX17] = sr.ll + alpha * dll;
          ix[3 * NX17] = sr.lu + alpha * dlu;
        }
      }
      if (!done && valid && j < NX17) {
        for (int k = 0; k <= N; ++k) r.w.DX[(int64_t)k * NX17 + j] += alpha * r.w.DDX[(int64_t)k * NX17 + j];
      }
      __syncthreads();
    }
    if (!done) st = (st == MPCB_STATUS_OK) ? MPCB_STATUS_MAXITER : st;
    // outputs: X = xbar + dx, U = ubar + du of the final iterate
    fin = true;
    for (int k = 0; k <= N; ++k) {
      if (valid && j < NX17 && a.X)
        a.X[(b * (int64_t)(N + 1) + k) * NX17 + j] = r.w.XB[(int64_t)k * NX17 + j] + r.w.DX[(int64_t)k * NX17 + j];
      if (ilane && k < N) {
        const T uo = r.w.UB[(int64_t)k * NU17 + ju] + r.w.IP[(int64_t)k * 18 + ju];
        fin = fin && ((uo - uo) == T(0));
        if (valid && a.U) a.U[(b * (int64_t)N + k) * NU17 + ju] = uo;
        if (valid && k == 0) a.u0[b * NU17 + ju] = uo;
      }
      if (j < NX17) {
        const T xo = r.w.DX[(int64_t)k * NX17 + j];
        fin = fin && ((xo - xo) == T(0));
      }
    }
  }
  // instance status: lane 0 of the instance collects its lanes' finiteness through LDS
  L.v[j] = fin ? T(0) : T(1);
  wave_lds_sync();
  if (valid && j == 0) {
    bool all = true;
    for (int i = 0; i < L17; ++i) all = all && (L.v[i] == T(0));
    a.status[b] = !all ? MPCB_STATUS_NAN : st;
  }
}

// [A|B] of every shooting interval into dense arrays (debug / parity, mpcb_linearize), by the
// solver's own packed linearisation (lin17_packed): 16 lanes per (instance, stage).
template <class T>
__global__ void __launch_bounds__(64) linearize17_kernel(int64_t B, int N, T h, Model<T> M,
                                                         const T* p, int64_t p_sb, int64_t p_kb,
                                                         const T* xbar, const T* ubar, T* A, T* Bm,
                                                         T* xnext) {
  const int lane = threadIdx.x;
  const int t = lane % LQ17;
  const int64_t o = (int64_t)blockIdx.x * GQ17 + lane / LQ17;   // (instance, stage) = b * N + k
  if (o >= B * N) return;
  const int64_t b = o / N;
  const int k = (int)(o % N);
  lin17_packed<T>(t, p + b * p_sb + k * p_kb, h, M, xbar + (b * (N + 1) + k) * NX17, ubar + o * NU17,
                  [&](int j, const T* v) {
#pragma unroll
                    for (int i = 0; i < NX17; ++i) {
                      if (j < NX17) A[(o * NX17 + i) * NX17 + j] = v[i];
                      else Bm[(o * NX17 + i) * NU17 + (j - NX17)] = v[i];
                    }
                  },
                  [&](const T* xn) {
                    if (xnext) {
#pragma unroll
                      for (int i = 0; i < NX17; ++i) xnext[o * NX17 + i] = xn[i];
                    }
                  });
}

template <class T>
__global__ void __launch_bounds__(64) sim17_kernel(int64_t B, T h, Model<T> M, const T* p, int64_t p_sb,
                                                   const T* x, const T* u, T* xo) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  P17<T> P;
  unpack_p17(p + b * p_sb, P);
  T xv[NX17], uv[NU17], xn[NX17];
#pragma unroll
  for (int i = 0; i < NX17; ++i) xv[i] = x[b * NX17 + i];
#pragma unroll
  for (int m = 0; m < NU17; ++m) uv[m] = u[b * NU17 + m];
  rk4_17<T, false>(xv, nullptr, uv, nullptr, h, M, P, xn, nullptr);
#pragma unroll
  for (int i = 0; i < NX17; ++i) xo[b * NX17 + i] = xn[i];
}

template <class T> hipError_t launch_full17(const FullArgs<T>& a, hipStream_t st, hipEvent_t* ev) {
  if (ev) (void)hipEventRecord(ev[0], st);
  if (a.q17)   // 16 lanes per instance (the lane-parallel trig); the thread-per-instance rollout otherwise
    hipLaunchKernelGGL(nominal17q_kernel<T>, dim3((unsigned)((a.nb + 3) / 4)), dim3(64), 0, st, a);
  else
    hipLaunchKernelGGL(nominal17_kernel<T>, dim3((unsigned)((a.nb + 63) / 64)), dim3(64), 0, st, a);
  if (ev) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(lin17ws_kernel<T>, dim3((unsigned)((a.nb * a.N + GQ17 - 1) / GQ17)), dim3(64), 0, st, a);
  if (ev) (void)hipEventRecord(ev[2], st);
  if (a.q17) {
    const hipError_t e = launch_riccati17q<T>(a, st);
    if (e != hipSuccess) return e;
  } else if (a.box) {
    hipLaunchKernelGGL((riccati17_kernel<T, true>), dim3((unsigned)((a.nb + G17 - 1) / G17)), dim3(64), 0, st, a);
  } else {
    hipLaunchKernelGGL((riccati17_kernel<T, false>), dim3((unsigned)((a.nb + G17 - 1) / G17)), dim3(64), 0, st, a);
  }
  if (ev) (void)hipEventRecord(ev[3], st);
  return hipGetLastError();
}
template <class T>
hipError_t launch_linearize17(int64_t B, int N, T h, const Model<T>& M, const T* p, int64_t p_sb,
                              int64_t p_kb, const T* xbar, const T* ubar, T* A, T* Bm, T* xnext,
                              hipStream_t st) {
  const unsigned grid = (unsigned)((B * N + GQ17 - 1) / GQ17);
  hipLaunchKernelGGL(linearize17_kernel<T>, dim3(grid), dim3(64), 0, st, B, N, h, M, p, p_sb, p_kb, xbar,
                     ubar, A, Bm, xnext);
  return hipGetLastError();
}
template <class T>
hipError_t launch_sim_step17(int64_t B, T h, const Model<T>& M, const T* p, int64_t p_sb,
                             const T* x, const T* u, T* xo, hipStream_t st) {
  hipLaunchKernelGGL(sim17_kernel<T>, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, st, B, h, M, p,
                     p_sb, x, u, xo);
  return hipGetLastError();
}

template hipError_t launch_full17<double>(const FullArgs<double>&, hipStream_t, hipEvent_t*);
template hipError_t launch_full17<float>(const FullArgs<float>&, hipStream_t, hipEvent_t*);
template hipError_t launch_linearize17<double>(int64_t, int, double, const Model<double>&, const double*,
                                               int64_t, int64_t, const double*, const double*, double*, double*,
                                               double*, hipStream_t);
template hipError_t launch_linearize17<float>(int64_t, int, float, const Model<float>&, const float*,
                                              int64_t, int64_t, const float*, const float*, float*, float*,
                                              float*, hipStream_t);
template hipError_t launch_sim_step17<double>(int64_t, double, const Model<double>&, const double*, int64_t,
                                              const double*, const double*, double*, hipStream_t);
template hipError_t launch_sim_step17<float>(int64_t, float, const Model<float>&, const float*, int64_t,
                                             const float*, const float*, float*, hipStream_t);

}  // namespace mpcb
