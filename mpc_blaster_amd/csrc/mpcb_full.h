// mpcb_full.h — the full 17-state / 6-input BLASTER model on the device.
//
// Restates f_expl_expr of src/scripts/blastermodel.py:70-201 with every state and parameter:
//   x = [p(3), eta = (phi, theta, psi), v(3), omega(3), alpha(2), poc(3)]      (:171-190)
//   u = [T0..T3, alpha1_dot, alpha2_dot]                                       (:191-193)
//   p = vec(J_angles 3x2) | vec(J_euler 3x3) | vec(J_p 3x3) | T_blast (column-major, :203-210)
//   p_dot     = v
//   eta_dot   = inv(R_to_omega(phi, theta)) omega                              (:128-141, :162)
//   v_dot     = R (e3 sum T + R_gimbal e3 T_blast) / m - g e3                   (:143-163)
//               R = Rz Ry Rx (:103-122), R_gimbal e3 = Ry(a1) Rx(a2) e3 = [s1 c2, -s2, c1 c2]
//   omega_dot = inv(J) (M(T) - omega x J omega)                                (:95-101, :164)
//   alpha_dot = u[4:6]
//   poc_dot   = J_p v + J_euler eta_dot + J_angles alpha_dot                   (:165-167)
// ``f17_tan`` evaluates f and one directional derivative J_f (dx, du) in the same pass
// (forward-mode dual numbers: each lane of an instance seeds one of the 23 directions).
#pragma once
#include <hip/hip_runtime.h>

#include "mpcb_common.h"
#include "mpcb_model.h"

namespace mpcb {

constexpr int NX17 = 17, NU17 = 6, NZ17 = NX17 + NU17, NP17 = 25;

// per-instance parameters unpacked from the 25-vector (row-major blocks)
template <class T>
struct P17 {
  T Ja[6];   // J_angles 3x2
  T Je[9];   // J_euler  3x3
  T Jp[9];   // J_p      3x3
  T tb;      // T_blast
};

template <class T>
__device__ __forceinline__ void unpack_p17(const T* __restrict__ p, P17<T>& P) {
  // column-major vec (blastermodel.py:203-210): block[i][j] = p[off + j*3 + i]
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) P.Ja[i * 2 + j] = p[j * 3 + i];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      P.Je[i * 3 + j] = p[6 + j * 3 + i];
      P.Jp[i * 3 + j] = p[15 + j * 3 + i];
    }
  }
  P.tb = p[24];
}

// sin/cos of the five angles of f17 (Euler angles x[3..5], swivel angles x[12..13]), one thread
struct Trig17Serial {
  template <class T>
  __device__ __forceinline__ void operator()(const T* __restrict__ x, T (&s)[5], T (&c)[5]) const {
    sc(x[3], &s[0], &c[0]);
    sc(x[4], &s[1], &c[1]);
    sc(x[5], &s[2], &c[2]);
    sc(x[12], &s[3], &c[3]);
    sc(x[13], &s[4], &c[4]);
  }
};

template <class T, bool TAN, class Trig = Trig17Serial>
__device__ __forceinline__ void f17_tan(const T* __restrict__ x, const T* __restrict__ dx,
                                        const T* __restrict__ u, const T* __restrict__ du,
                                        const Model<T>& M, const P17<T>& P, T* __restrict__ f,
                                        T* __restrict__ df, const Trig& trig = Trig()) {
  T tsn[5], tcs[5];
  trig(x, tsn, tcs);
  const T sf = tsn[0], cf = tcs[0], st = tsn[1], ct = tcs[1], sp = tsn[2], cp = tcs[2];
  const T s1 = tsn[3], c1 = tcs[3], s2 = tsn[4], c2 = tcs[4];
  const T ict = recip(ct);
  const T tt = st * ict;
  const T wx = x[9], wy = x[10], wz = x[11];
  f[0] = x[6]; f[1] = x[7]; f[2] = x[8];
  const T a = sf * wy + cf * wz;
  const T b = cf * wy - sf * wz;
  const T ed0 = wx + tt * a, ed1 = b, ed2 = a * ict;
  f[3] = ed0; f[4] = ed1; f[5] = ed2;
  // R = Rz(psi) Ry(theta) Rx(phi)
  const T cpst = cp * st, spst = sp * st;
  const T R00 = cp * ct, R01 = cpst * sf - sp * cf, R02 = cpst * cf + sp * sf;
  const T R10 = sp * ct, R11 = spst * sf + cp * cf, R12 = spst * cf - cp * sf;
  const T R20 = -st, R21 = ct * sf, R22 = ct * cf;
  // body force: motors along e3 plus the swivelled blaster thrust
  const T Tsum = (u[0] + u[1]) + (u[2] + u[3]);
  const T fb0 = P.tb * (s1 * c2), fb1 = -P.tb * s2, fb2 = Tsum + P.tb * (c1 * c2);
  f[6] = (R00 * fb0 + R01 * fb1 + R02 * fb2) * M.minv;
  f[7] = (R10 * fb0 + R11 * fb1 + R12 * fb2) * M.minv;
  f[8] = (R20 * fb0 + R21 * fb1 + R22 * fb2) * M.minv - M.g;
  const T jw0 = M.J[0] * wx + M.J[1] * wy + M.J[2] * wz;
  const T jw1 = M.J[3] * wx + M.J[4] * wy + M.J[5] * wz;
  const T jw2 = M.J[6] * wx + M.J[7] * wy + M.J[8] * wz;
  const T k0 = wy * jw2 - wz * jw1;
  const T k1 = wz * jw0 - wx * jw2;
  const T k2 = wx * jw1 - wy * jw0;
  const T m0 = (u[1] + u[3] - u[0] - u[2]) * M.ly - k0;
  const T m1 = (u[1] + u[2] - u[0] - u[3]) * M.lx - k1;
  const T m2 = (u[2] + u[3] - u[0] - u[1]) * M.c - k2;
  f[9] = M.Jinv[0] * m0 + M.Jinv[1] * m1 + M.Jinv[2] * m2;
  f[10] = M.Jinv[3] * m0 + M.Jinv[4] * m1 + M.Jinv[5] * m2;
  f[11] = M.Jinv[6] * m0 + M.Jinv[7] * m1 + M.Jinv[8] * m2;
  f[12] = u[4];
  f[13] = u[5];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    f[14 + i] = P.Jp[i * 3] * x[6] + P.Jp[i * 3 + 1] * x[7] + P.Jp[i * 3 + 2] * x[8] +
                P.Je[i * 3] * ed0 + P.Je[i * 3 + 1] * ed1 + P.Je[i * 3 + 2] * ed2 +
                P.Ja[i * 2] * u[4] + P.Ja[i * 2 + 1] * u[5];
  if constexpr (TAN) {
    const T dphi = dx[3], dth = dx[4], dpsi = dx[5];
    const T dwx = dx[9], dwy = dx[10], dwz = dx[11];
    const T dsf = cf * dphi, dcf = -sf * dphi;
    const T dst = ct * dth, dct = -st * dth;
    const T dsp = cp * dpsi, dcp = -sp * dpsi;
    const T ds1 = c1 * dx[12], dc1 = -s1 * dx[12];
    const T ds2 = c2 * dx[13], dc2 = -s2 * dx[13];
    const T dict = -ict * ict * dct;
    const T dtt = dst * ict + st * dict;
    df[0] = dx[6]; df[1] = dx[7]; df[2] = dx[8];
    const T da = dsf * wy + sf * dwy + dcf * wz + cf * dwz;
    const T db = dcf * wy + cf * dwy - dsf * wz - sf * dwz;
    const T ded0 = dwx + dtt * a + tt * da, ded1 = db, ded2 = da * ict + a * dict;
    df[3] = ded0; df[4] = ded1; df[5] = ded2;
    const T dcpst = dcp * st + cp * dst, dspst = dsp * st + sp * dst;
    const T dR00 = dcp * ct + cp * dct;
    const T dR01 = dcpst * sf + cpst * dsf - dsp * cf - sp * dcf;
    const T dR02 = dcpst * cf + cpst * dcf + dsp * sf + sp * dsf;
    const T dR10 = dsp * ct + sp * dct;
    const T dR11 = dspst * sf + spst * dsf + dcp * cf + cp * dcf;
    const T dR12 = dspst * cf + spst * dcf - dcp * sf - cp * dsf;
    const T dR20 = -dst, dR21 = dct * sf + ct * dsf, dR22 = dct * cf + ct * dcf;
    const T dTsum = (du[0] + du[1]) + (du[2] + du[3]);
    const T dfb0 = P.tb * (ds1 * c2 + s1 * dc2), dfb1 = -P.tb * ds2;
    const T dfb2 = dTsum + P.tb * (dc1 * c2 + c1 * dc2);
    df[6] = (dR00 * fb0 + dR01 * fb1 + dR02 * fb2 + R00 * dfb0 + R01 * dfb1 + R02 * dfb2) * M.minv;
    df[7] = (dR10 * fb0 + dR11 * fb1 + dR12 * fb2 + R10 * dfb0 + R11 * dfb1 + R12 * dfb2) * M.minv;
    df[8] = (dR20 * fb0 + dR21 * fb1 + dR22 * fb2 + R20 * dfb0 + R21 * dfb1 + R22 * dfb2) * M.minv;
    const T djw0 = M.J[0] * dwx + M.J[1] * dwy + M.J[2] * dwz;
    const T djw1 = M.J[3] * dwx + M.J[4] * dwy + M.J[5] * dwz;
    const T djw2 = M.J[6] * dwx + M.J[7] * dwy + M.J[8] * dwz;
    const T dk0 = dwy * jw2 + wy * djw2 - dwz * jw1 - wz * djw1;
    const T dk1 = dwz * jw0 + wz * djw0 - dwx * jw2 - wx * djw2;
    const T dk2 = dwx * jw1 + wx * djw1 - dwy * jw0 - wy * djw0;
    const T dm0 = (du[1] + du[3] - du[0] - du[2]) * M.ly - dk0;
    const T dm1 = (du[1] + du[2] - du[0] - du[3]) * M.lx - dk1;
    const T dm2 = (du[2] + du[3] - du[0] - du[1]) * M.c - dk2;
    df[9] = M.Jinv[0] * dm0 + M.Jinv[1] * dm1 + M.Jinv[2] * dm2;
    df[10] = M.Jinv[3] * dm0 + M.Jinv[4] * dm1 + M.Jinv[5] * dm2;
    df[11] = M.Jinv[6] * dm0 + M.Jinv[7] * dm1 + M.Jinv[8] * dm2;
    df[12] = du[4];
    df[13] = du[5];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      df[14 + i] = P.Jp[i * 3] * dx[6] + P.Jp[i * 3 + 1] * dx[7] + P.Jp[i * 3 + 2] * dx[8] +
                   P.Je[i * 3] * ded0 + P.Je[i * 3 + 1] * ded1 + P.Je[i * 3 + 2] * ded2 +
                   P.Ja[i * 2] * du[4] + P.Ja[i * 2 + 1] * du[5];
  }
}

// One classic RK4 step (acados sim_erk: 4 stages, 1 step) of f17 with an optional tangent.
template <class T, bool TAN, class Trig = Trig17Serial>
__device__ __forceinline__ void rk4_17(const T* __restrict__ x, const T* __restrict__ dx,
                                       const T* __restrict__ u, const T* __restrict__ du, T h,
                                       const Model<T>& M, const P17<T>& P, T* __restrict__ xn,
                                       T* __restrict__ dxn, const Trig& trig = Trig()) {
  T k[NX17], dk[NX17], xs[NX17], dxs[NX17];
  const T h2 = T(0.5) * h, h6 = h / T(6);
  f17_tan<T, TAN>(x, dx, u, du, M, P, k, dk, trig);
#pragma unroll
  for (int i = 0; i < NX17; ++i) {
    xn[i] = k[i];
    xs[i] = x[i] + h2 * k[i];
    if constexpr (TAN) { dxn[i] = dk[i]; dxs[i] = dx[i] + h2 * dk[i]; }
  }
  f17_tan<T, TAN>(xs, dxs, u, du, M, P, k, dk, trig);
#pragma unroll
  for (int i = 0; i < NX17; ++i) {
    xn[i] += T(2) * k[i];
    xs[i] = x[i] + h2 * k[i];
    if constexpr (TAN) { dxn[i] += T(2) * dk[i]; dxs[i] = dx[i] + h2 * dk[i]; }
  }
  f17_tan<T, TAN>(xs, dxs, u, du, M, P, k, dk, trig);
#pragma unroll
  for (int i = 0; i < NX17; ++i) {
    xn[i] += T(2) * k[i];
    xs[i] = x[i] + h * k[i];
    if constexpr (TAN) { dxn[i] += T(2) * dk[i]; dxs[i] = dx[i] + h * dk[i]; }
  }
  f17_tan<T, TAN>(xs, dxs, u, du, M, P, k, dk, trig);
#pragma unroll
  for (int i = 0; i < NX17; ++i) {
    xn[i] = x[i] + h6 * (xn[i] + k[i]);
    if constexpr (TAN) dxn[i] = dx[i] + h6 * (dxn[i] + dk[i]);
  }
}

// Device-resident weights of the 17/6 OCP (row-major) and the default parameter vector.
template <class T>
struct Weights17 {
  T Q[NX17 * NX17];
  T R[NU17 * NU17];
  T QN[NX17 * NX17];
  T lbu[NU17], ubu[NU17];
  T lbx[NX17], ubx[NX17];   // state box on stages 1..N-1 (FullArgs::sbox)
  T p[NP17];
};

template <class T>
struct FullArgs {
  int64_t b0, nb;    // first global instance of the chunk, instances in the chunk
  int N, mode;
  T h, s;
  Model<T> M;
  const Weights17<T>* W;
  const T* p; int64_t p_sb, p_kb;   // parameters [B|1][N|1][25] (instance / stage strides, 0 =
                                   // broadcast); nullptr -> W->p
  const T* x0; int64_t x0_sb;
  const T* xref; int64_t xref_sb;
  const T* uref; int64_t uref_sb;
  const T* xbar; const T* ubar;
  T* u0; T* X; T* U; int32_t* status;
  T* ws;             // chunk workspace: per instance full17_elems(N) elements
  int box;           // input box lbu <= u <= ubu (interior-point iterations)
  int sbox;          // with box: state box lbx <= x_k <= ubx on stages 1..N-1
  int max_as_iter;   // iteration cap
  int32_t* qp_stats; // boxes: per instance [interior-point iterations, polish passes] (mpcb_qp_stats)
};

__host__ __device__ constexpr int64_t full17_elems(int N) {
  // XB (N+1)x17 | UB Nx6 | AB N x 23 columns x 17 | KR N x (6x17 + 6) | GP N x 17 |
  // boxes: DX, DDX (N+1)x17 | IP N x 18 | DDU N x 6 | IX (N+1) x 4 x 17 | LC N x 24 | DAX (N+1)x17 | DAU N x 6 | DC N x 48 | GV (N+1) x 24
  return (int64_t)(N + 1) * NX17 + (int64_t)N * (NU17 + NZ17 * NX17 + NU17 * NX17 + NU17 + NX17) +
         2 * (int64_t)(N + 1) * NX17 + (int64_t)N * (18 + NU17) + 4 * (int64_t)(N + 1) * NX17 +
         (int64_t)N * 24 + (int64_t)(N + 1) * NX17 + (int64_t)N * NU17 + (int64_t)N * 48 + (int64_t)(N + 1) * 24;
}

// n x n Cholesky (row-major H, lower L with 1/L_ii on the diagonal) and the solve L L^T x = b
template <class T, int n>
__device__ __forceinline__ void chol_n(const T* __restrict__ H, T* __restrict__ L) {
#pragma unroll
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      T acc = H[i * n + j];
#pragma unroll
      for (int k = 0; k < j; ++k) acc -= L[i * n + k] * L[j * n + k];
      if (i == j) L[i * n + i] = inv_sqrt(acc);
      else L[i * n + j] = acc * L[j * n + j];
    }
  }
}
template <class T, int n>
__device__ __forceinline__ void chol_n_solve(const T* __restrict__ L, const T* __restrict__ b,
                                             T* __restrict__ x) {
  T y[n];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    T acc = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) acc -= L[i * n + k] * y[k];
    y[i] = acc * L[i * n + i];
  }
#pragma unroll
  for (int i = n - 1; i >= 0; --i) {
    T acc = y[i];
#pragma unroll
    for (int k = i + 1; k < n; ++k) acc -= L[k * n + i] * x[k];
    x[i] = acc * L[i * n + i];
  }
}

// x[i] for a lane-dependent i < 17 without dynamic register indexing
template <class T> __device__ __forceinline__ T sel17(const T* x, int i) {
  const T lo = sel<16>(x, i & 15);
  return (i == 16) ? x[16] : lo;
}

// Per-instance workspace carve (FullArgs::ws, full17_elems(N) elements per instance).
template <class T>
struct Ws17 {
  T *XB, *UB, *AB, *KR, *GP;
  T *DX, *DDX, *IP, *DDU, *IX;
  static constexpr int KR_N = NU17 * NX17 + NU17;
  __device__ __forceinline__ Ws17(T* ws, int N) {
    XB = ws;                                     // [N+1][17] nominal states
    UB = XB + (int64_t)(N + 1) * NX17;           // [N][6]    nominal inputs
    AB = UB + (int64_t)N * NU17;                 // [N][23][17] column j of [A_k|B_k] at j*17
    KR = AB + (int64_t)N * NZ17 * NX17;          // [N][6*17 + 6]: K[m][i] at i*6 + m, then k
    GP = KR + (int64_t)N * KR_N;                 // [N][17] gaps
    // input box (interior point): iterate dx, step, (du, lambda_l, lambda_u), step du
    DX = GP + (int64_t)N * NX17;                 // [N+1][17]
    DDX = DX + (int64_t)(N + 1) * NX17;          // [N+1][17]
    IP = DDX + (int64_t)(N + 1) * NX17;          // [N][18]: du | lambda_l | lambda_u
    DDU = IP + (int64_t)N * 18;                  // [N][6]
    // state box: slacks and multipliers s_l | s_u | lambda_l | lambda_u of the rows of stage k
    IX = DDU + (int64_t)N * NU17;                // [N+1][4][17]
  }
};

// The Mehrotra arrays after IX (mpcb_r17.hip; a separate carve so the other 17/6 kernels keep
// their register footprint): the packed Cholesky factor of Huu per stage (21 of 24), the
// predictor's (affine) direction, and per row (z index: states, then 17 + m) w = 1/s_l - 1/s_u at
// [0, 24), c = Delta s_a Delta lambda_a / s_l - (upper) at [24, 48): the corrector's gradient
// change is c - sigma mu w.  GV: the predictor's stage gradients without the p terms (cost and
// barrier: states at [0, 17), inputs at [17, 23)), and p_N at stage N.
template <class T>
struct WsM17 {
  T *LC, *DAX, *DAU, *DC, *GV;
  static constexpr int LC_N = 24, DC_N = 48;
  __device__ __forceinline__ WsM17(const Ws17<T>& w, int N) {
    LC = w.IX + (int64_t)(N + 1) * 4 * NX17;     // [N][24]
    DAX = LC + (int64_t)N * LC_N;                // [N+1][17]
    DAU = DAX + (int64_t)(N + 1) * NX17;         // [N][6]
    DC = DAU + (int64_t)N * NU17;                // [N][48]
    GV = DC + (int64_t)N * DC_N;                 // [N+1][24]
  }
};

constexpr double IPM17_SIGMA_MIN = 0.05, IPM17_SIGMA_MAX = 0.9, IPM17_TAU = 0.995, IPM17_THETA = 0.1;
// (IPM17_BREAK: oracle.ocp.IPM_BREAK_TOL, where the choice of 1e-5 is explained: an fp64 exit
// there that the polish below does not certify ends MPCB_STATUS_MINSTEP, not OK)
constexpr double IPM17_TOL = 1e-12, IPM17_BREAK = 1e-5, IPM17_STALL = 1e-6, IPM17_RES = 1e-9;
// the fp64 state-box polish (oracle.ocp.al_polish): augmented-Lagrangian passes over the
// interior point's active set with one active-set change per pass
constexpr double POL17_RHO = 1e10, POL17_EQ = 1e-10, POL17_FEAS = 1e-10, POL17_ACT = 100.0;
constexpr int POL17_ITERS = 12;
constexpr double IPM17_SHORT = 1e-2;   // IPM17_SHORT_RUN steps in a row below it: a stalled QP
constexpr int IPM17_SHORT_RUN = 10;
// with the state box (the only QPs here that can be infeasible; oracle.ocp IPM_SBOX_SHORT): 7
// steps in a row below 0.05 away from the solution.  On the 4096 bench draws (N = 60) no
// LP-feasible instance takes more than 3 such steps in a row, the 68 LP-infeasible ones stop
// after at most 69 iterations instead of 115 (the launch's tail: feasible ones need <= 62)
constexpr double IPM17_SBOX_SHORT = 5e-2;
constexpr int IPM17_SBOX_SHORT_RUN = 7;
// fp32: the duality measure stops near 1e-6 (lambda / s reaches the fp32 conditioning limit
// long before 1e-12), so the tolerances scale with the precision; the result is checked
// against the fp64 oracle in tests/test_gpu_full17.py
constexpr double IPM17_TOL_F32 = 1e-6, IPM17_BREAK_F32 = 1e-3, IPM17_RES_F32 = 1e-5;

// ev (nullable): 4 events recorded before nominal17, after it, after lin17ws and after riccati17.
template <class T> hipError_t launch_full17(const FullArgs<T>& a, hipStream_t st, hipEvent_t* ev = nullptr);
template <class T> hipError_t launch_riccati17q(const FullArgs<T>& a, hipStream_t st);
template <class T>
hipError_t launch_linearize17(int64_t B, int N, T h, const Model<T>& M, const T* p, int64_t p_sb,
                              int64_t p_kb, const T* xbar, const T* ubar, T* A, T* Bm, T* xnext, hipStream_t st);
template <class T>
hipError_t launch_sim_step17(int64_t B, T h, const Model<T>& M, const T* p, int64_t p_sb,
                             const T* x, const T* u, T* xo, hipStream_t st);

}  // namespace mpcb
