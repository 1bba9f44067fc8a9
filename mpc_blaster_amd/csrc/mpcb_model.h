// mpcb_model.h — BLASTER rigid-body dynamics on the device, value + one forward tangent.
//
// Restates f_expl_expr of src/scripts/blastermodel.py:95-201 for the 12-state/4-input slice
// (x = [p, phi, theta, psi, v, omega], u = 4 motor thrusts, swivel alpha = 0 so
// R_gimbal = I):
//   p_dot     = v                                              (:124)
//   eta_dot   = inv(R_to_omega(phi, theta)) @ omega           (:128-141, :162) closed form
//   v_dot     = (R e3 (sum T) + R e3 T_blast) / m + [0,0,-g]   (:163), R = Rz Ry Rx (:103-122)
//   omega_dot = inv(J) (M(T) - omega x J omega)               (:95-101, :164)
// plus an optional world-frame wind force / m in v_dot (c5 build extension).
//
// ``f_tan`` evaluates f and its directional derivative J_f(x,u)·(dx,du) in one pass
// (forward-mode dual numbers).  Each lane of an instance's 16-lane group seeds one
// direction, so the RK4 sensitivity columns of [A|B] come out one per lane without ever
// forming the Jacobian (what acados' forward VDE does symbolically).
#pragma once
#include <hip/hip_runtime.h>

namespace mpcb {

template <class T>
struct Model {
  T minv, g, t_blast, lx, ly, c;
  T J[9], Jinv[9];
};

// sin/cos for the attitude angles: Cody-Waite reduction by pi/2 + fdlibm / Cephes minimax
// kernels (<= 1-2 ulp for |a| < 2^19).  The library sincos carries a Payne-Hanek large-argument
// path that costs ~4x the instructions and registers on every call; here it is only the
// (never taken in practice) fallback.  Three calls per f evaluation make this the dominant
// cost of the nominal passes.
// Horner step t * z + c as a three-address v_fma_f64 (MPCB_SC_ASM, default on).  Left to itself the
// compiler turns each step into v_fmac_f64 (the addend is the destination) and so copies the
// loop-invariant coefficient first: one v_mov per step, ~14 per call, 56 per RK4 interval of the
// issue-bound P1 rollout.
#ifndef MPCB_SC_ASM
#define MPCB_SC_ASM 1
#endif
__device__ __forceinline__ double hstep(double t, double z, double c) {
#if MPCB_SC_ASM
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(t), "v"(z), "v"(c));
  return r;
#else
  return fma(t, z, c);
#endif
}
// sin/cos polynomial coefficients (fdlibm __kernel_sin / __kernel_cos), highest degree first
struct ScConst {
  __device__ static constexpr double s(int i) {
    constexpr double t[6] = {1.58969099521155010221e-10, -2.50507602534068634195e-08,
                             2.75573137070700676789e-06, -1.98412698298579493134e-04,
                             8.33333333332248946124e-03, -1.66666666666666324348e-01};
    return t[i];
  }
  __device__ static constexpr double c(int i) {
    constexpr double t[6] = {-1.13596475577881948265e-11, 2.08757232129817482790e-09,
                             -2.75573143513906633035e-07, 2.48015872894767294178e-05,
                             -1.38888888888741095749e-03, 4.16666666666666019037e-02};
    return t[i];
  }
};
// The same coefficients as loop-invariant registers the compiler cannot see into: used by the
// serial P1 rollout, where the compiler otherwise re-assembles some constant pairs from copied
// halves at every call (7 v_mov_b32 per sin/cos).  Identical values, identical results.
struct ScRegs {
  double vs[6], vc[6];
  __device__ __forceinline__ ScRegs() {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      vs[i] = ScConst::s(i); vc[i] = ScConst::c(i);
      asm volatile("" : "+v"(vs[i]));
      asm volatile("" : "+v"(vc[i]));
    }
  }
  __device__ __forceinline__ double s(int i) const { return vs[i]; }
  __device__ __forceinline__ double c(int i) const { return vc[i]; }
};
// MPCB_SC_FALLBACK=0: no large-argument fallback (instruction counting of the fast path only:
// tools/isa_loop.py; never a shipped build)
#ifndef MPCB_SC_FALLBACK
#define MPCB_SC_FALLBACK 1
#endif
// sc_core: the reduction and kernels alone, valid for |a| < 2^19 (the caller checks the domain)
template <class K>
__device__ __forceinline__ void sc_core(double a, double* s, double* c, const K& k) {
  const double n = rint(a * 6.36619772367581382433e-01);           // 2/pi
  double r = fma(-n, 1.57079632673412561417e+00, a);              // pio2_1 (33 bits)
  r = fma(-n, 6.07710050650619224932e-11, r);                     // pio2_1t
  const double z = r * r;
  double ps = hstep(k.s(0), z, k.s(1));
  ps = hstep(ps, z, k.s(2));
  ps = hstep(ps, z, k.s(3));
  ps = hstep(ps, z, k.s(4));
  ps = hstep(ps, z, k.s(5));
  const double sr = fma(r * z, ps, r);
  double pc = hstep(k.c(0), z, k.c(1));
  pc = hstep(pc, z, k.c(2));
  pc = hstep(pc, z, k.c(3));
  pc = hstep(pc, z, k.c(4));
  pc = hstep(pc, z, k.c(5));
  pc = z * pc;
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  const double cr = w + (((1.0 - w) - hz) + z * pc);
  const int q = (int)n & 3;
  const double s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
  *s = (q & 2) ? -s0 : s0;
  *c = ((q + 1) & 2) ? -c0 : c0;
}
template <class K>
__device__ __forceinline__ void sc(double a, double* s, double* c, const K& k) {
#if MPCB_SC_FALLBACK
  if (!(fabs(a) < 524288.0)) { sincos(a, s, c); return; }
#endif
  sc_core(a, s, c, k);
}
__device__ __forceinline__ void sc(double a, double* s, double* c) { sc(a, s, c, ScConst{}); }
// fp32: |a| < 8192
__device__ __forceinline__ void sc_core(float a, float* s, float* c) {
  const float n = rintf(a * 0.636619772367581343f);
  float r = fmaf(-n, 1.57079637050628662109375f, a);              // pio2 hi
  r = fmaf(-n, -4.37113900018624283e-08f, r);                     // pio2 lo
  const float z = r * r;
  const float sr = fmaf(r * z, -1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f), r);
  const float cr = fmaf(z * z, 4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f),
                        fmaf(-0.5f, z, 1.0f));
  const int q = (int)n & 3;
  const float s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
  *s = (q & 2) ? -s0 : s0;
  *c = ((q + 1) & 2) ? -c0 : c0;
}
__device__ __forceinline__ void sc(float a, float* s, float* c) {
#if MPCB_SC_FALLBACK
  if (!(fabsf(a) < 8192.0f)) { sincosf(a, s, c); return; }
#endif
  sc_core(a, s, c);
}

// 1/x by the hardware reciprocal and two Newton steps (fp64: v_rcp_f64 + 4 FMAs, ~1 ulp; the
// IEEE division sequence is ~11 instructions with its scale / fixup steps).  Domain: normal, finite,
// non-zero x -- cos(theta) of a flying attitude, and the 17/6 interior point's strictly positive
// slacks and multipliers (mpcb_r17.hip, which keeps them >= a positive floor before taking
// reciprocals).  recip(0) is NaN, not inf (fma(-0, inf, 1) = NaN): callers whose argument can
// reach 0 or a denormal must use safe_recip.  MPCB_IEEE_DIV=1 restores the division.
#ifndef MPCB_IEEE_DIV
#define MPCB_IEEE_DIV 0
#endif
__device__ __forceinline__ double recip(double x) {
#if MPCB_IEEE_DIV
  return 1.0 / x;
#else
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
#endif
}
// 1/x that keeps IEEE semantics at 0 / denormals / inf (the division) for arguments outside
// recip()'s domain
template <class T> __device__ __forceinline__ T safe_recip(T x) { return T(1) / x; }
__device__ __forceinline__ float recip(float x) {
#if MPCB_IEEE_DIV
  return 1.0f / x;
#else
  const float r = __builtin_amdgcn_rcpf(x);
  return fmaf(fmaf(-x, r, 1.0f), r, r);
#endif
}

// f and (optionally) its tangent.  wind may be nullptr-equivalent (w0=w1=w2=0).
template <class T, bool TAN>
__device__ __forceinline__ void f_tan(const T* __restrict__ x, const T* __restrict__ dx,
                                      const T* __restrict__ u, const T* __restrict__ du,
                                      const Model<T>& M, const T w[3],
                                      T* __restrict__ f, T* __restrict__ df) {
  T sf, cf, st, ct, sp, cp;
  sc(x[3], &sf, &cf);
  sc(x[4], &st, &ct);
  sc(x[5], &sp, &cp);
  const T ict = recip(ct);
  const T tt = st * ict;
  const T wx = x[9], wy = x[10], wz = x[11];
  // ---- p_dot = v
  f[0] = x[6]; f[1] = x[7]; f[2] = x[8];
  // ---- eta_dot = W^-1 omega
  const T a = sf * wy + cf * wz;
  const T b = cf * wy - sf * wz;
  f[3] = wx + tt * a;
  f[4] = b;
  f[5] = a * ict;
  // ---- v_dot
  const T Ttot = (u[0] + u[1]) + (u[2] + u[3]) + M.t_blast;
  const T s = Ttot * M.minv;
  const T cfst = cf * st;
  const T r0 = cp * cfst + sp * sf;
  const T r1 = sp * cfst - cp * sf;
  const T r2 = cf * ct;
  f[6] = r0 * s + w[0] * M.minv;
  f[7] = r1 * s + w[1] * M.minv;
  f[8] = r2 * s - M.g + w[2] * M.minv;
  // ---- omega_dot = Jinv (Mom - w x J w)
  const T jw0 = M.J[0] * wx + M.J[1] * wy + M.J[2] * wz;
  const T jw1 = M.J[3] * wx + M.J[4] * wy + M.J[5] * wz;
  const T jw2 = M.J[6] * wx + M.J[7] * wy + M.J[8] * wz;
  const T c0 = wy * jw2 - wz * jw1;
  const T c1 = wz * jw0 - wx * jw2;
  const T c2 = wx * jw1 - wy * jw0;
  const T m0 = (u[1] + u[3] - u[0] - u[2]) * M.ly - c0;
  const T m1 = (u[1] + u[2] - u[0] - u[3]) * M.lx - c1;
  const T m2 = (u[2] + u[3] - u[0] - u[1]) * M.c - c2;
  f[9] = M.Jinv[0] * m0 + M.Jinv[1] * m1 + M.Jinv[2] * m2;
  f[10] = M.Jinv[3] * m0 + M.Jinv[4] * m1 + M.Jinv[5] * m2;
  f[11] = M.Jinv[6] * m0 + M.Jinv[7] * m1 + M.Jinv[8] * m2;
  if constexpr (TAN) {
    const T dphi = dx[3], dth = dx[4], dpsi = dx[5];
    const T dwx = dx[9], dwy = dx[10], dwz = dx[11];
    const T dsf = cf * dphi, dcf = -sf * dphi;
    const T dst = ct * dth, dct = -st * dth;
    const T dsp = cp * dpsi, dcp = -sp * dpsi;
    const T dict = -ict * ict * dct;
    const T dtt = dst * ict + st * dict;
    df[0] = dx[6]; df[1] = dx[7]; df[2] = dx[8];
    const T da = dsf * wy + sf * dwy + dcf * wz + cf * dwz;
    const T db = dcf * wy + cf * dwy - dsf * wz - sf * dwz;
    df[3] = dwx + dtt * a + tt * da;
    df[4] = db;
    df[5] = da * ict + a * dict;
    const T dT = (du[0] + du[1]) + (du[2] + du[3]);
    const T ds = dT * M.minv;
    const T dcfst = dcf * st + cf * dst;
    const T dr0 = dcp * cfst + cp * dcfst + dsp * sf + sp * dsf;
    const T dr1 = dsp * cfst + sp * dcfst - dcp * sf - cp * dsf;
    const T dr2 = dcf * ct + cf * dct;
    df[6] = dr0 * s + r0 * ds;
    df[7] = dr1 * s + r1 * ds;
    df[8] = dr2 * s + r2 * ds;
    const T djw0 = M.J[0] * dwx + M.J[1] * dwy + M.J[2] * dwz;
    const T djw1 = M.J[3] * dwx + M.J[4] * dwy + M.J[5] * dwz;
    const T djw2 = M.J[6] * dwx + M.J[7] * dwy + M.J[8] * dwz;
    const T dc0 = dwy * jw2 + wy * djw2 - dwz * jw1 - wz * djw1;
    const T dc1 = dwz * jw0 + wz * djw0 - dwx * jw2 - wx * djw2;
    const T dc2 = dwx * jw1 + wx * djw1 - dwy * jw0 - wy * djw0;
    const T dm0 = (du[1] + du[3] - du[0] - du[2]) * M.ly - dc0;
    const T dm1 = (du[1] + du[2] - du[0] - du[3]) * M.lx - dc1;
    const T dm2 = (du[2] + du[3] - du[0] - du[1]) * M.c - dc2;
    df[9] = M.Jinv[0] * dm0 + M.Jinv[1] * dm1 + M.Jinv[2] * dm2;
    df[10] = M.Jinv[3] * dm0 + M.Jinv[4] * dm1 + M.Jinv[5] * dm2;
    df[11] = M.Jinv[6] * dm0 + M.Jinv[7] * dm1 + M.Jinv[8] * dm2;
  }
}

// One classic RK4 step (acados sim_erk, 4 stages, 1 step) with an optional forward tangent.
// xn = Phi(x, u); dxn = dPhi/d(x,u) · (dx, du).
template <class T, bool TAN>
__device__ __forceinline__ void rk4(const T* __restrict__ x, const T* __restrict__ dx,
                                    const T* __restrict__ u, const T* __restrict__ du, T h,
                                    const Model<T>& M, const T w[3], T* __restrict__ xn,
                                    T* __restrict__ dxn) {
  constexpr int NX = 12;
  T k[NX], dk[NX], xs[NX], dxs[NX];
  const T h2 = T(0.5) * h, h6 = h / T(6);
  f_tan<T, TAN>(x, dx, u, du, M, w, k, dk);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    xn[i] = k[i];
    xs[i] = x[i] + h2 * k[i];
    if constexpr (TAN) { dxn[i] = dk[i]; dxs[i] = dx[i] + h2 * dk[i]; }
  }
  f_tan<T, TAN>(xs, dxs, u, du, M, w, k, dk);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    xn[i] += T(2) * k[i];
    xs[i] = x[i] + h2 * k[i];
    if constexpr (TAN) { dxn[i] += T(2) * dk[i]; dxs[i] = dx[i] + h2 * dk[i]; }
  }
  f_tan<T, TAN>(xs, dxs, u, du, M, w, k, dk);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    xn[i] += T(2) * k[i];
    xs[i] = x[i] + h * k[i];
    if constexpr (TAN) { dxn[i] += T(2) * dk[i]; dxs[i] = dx[i] + h * dk[i]; }
  }
  f_tan<T, TAN>(xs, dxs, u, du, M, w, k, dk);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    xn[i] = x[i] + h6 * (xn[i] + k[i]);
    if constexpr (TAN) dxn[i] = dx[i] + h6 * (dxn[i] + dk[i]);
  }
}

}  // namespace mpcb

namespace mpcb {

// ---------------------------------------------------------------------------------------------
// Split evaluation used by the fused solve kernel.  The nominal pass evaluates f once per RK4
// stage and captures the 20 scalars the tangent needs (trig values, rotation column, thrust
// scale, angular momentum, body rates): ``Lin``.  The tangent passes then apply J_f(x_i,u)·(dx,du)
// from those scalars with ~70 FMAs and no transcendental, so every direction lane carries only
// tangent vectors (register diet: the 16 lanes of an instance no longer recompute the shared
// nominal trajectory, its sin/cos, or hold it live).
// ---------------------------------------------------------------------------------------------
constexpr int LIN_N = 20;      // scalars per RK4 stage
constexpr int LIN_STAGE = 80;  // per shooting interval (4 stages)

// sin/cos of the three attitude angles (the default: one thread evaluates all three)
struct TrigSerial {
  template <class T>
  __device__ __forceinline__ void operator()(const T* __restrict__ x, T& sf, T& cf, T& st, T& ct,
                                             T& sp, T& cp) const {
    sc(x[3], &sf, &cf);
    sc(x[4], &st, &ct);
    sc(x[5], &sp, &cp);
  }
};

template <class T, class Trig = TrigSerial>
__device__ __forceinline__ void f_nom_lin(const T* __restrict__ x, const T* __restrict__ u,
                                          const Model<T>& M, const T w[3], T* __restrict__ f,
                                          T* __restrict__ c, const Trig& trig = Trig()) {
  T sf, cf, st, ct, sp, cp;
  trig(x, sf, cf, st, ct, sp, cp);
  const T ict = recip(ct);
  const T tt = st * ict;
  const T wx = x[9], wy = x[10], wz = x[11];
  f[0] = x[6]; f[1] = x[7]; f[2] = x[8];
  const T a = sf * wy + cf * wz;
  const T b = cf * wy - sf * wz;
  f[3] = wx + tt * a;
  f[4] = b;
  f[5] = a * ict;
  const T Ttot = (u[0] + u[1]) + (u[2] + u[3]) + M.t_blast;
  const T s = Ttot * M.minv;
  const T cfst = cf * st;
  const T r0 = cp * cfst + sp * sf;
  const T r1 = sp * cfst - cp * sf;
  const T r2 = cf * ct;
  f[6] = r0 * s + w[0] * M.minv;
  f[7] = r1 * s + w[1] * M.minv;
  f[8] = r2 * s - M.g + w[2] * M.minv;
  const T jw0 = M.J[0] * wx + M.J[1] * wy + M.J[2] * wz;
  const T jw1 = M.J[3] * wx + M.J[4] * wy + M.J[5] * wz;
  const T jw2 = M.J[6] * wx + M.J[7] * wy + M.J[8] * wz;
  const T c0 = wy * jw2 - wz * jw1;
  const T c1 = wz * jw0 - wx * jw2;
  const T c2 = wx * jw1 - wy * jw0;
  const T m0 = (u[1] + u[3] - u[0] - u[2]) * M.ly - c0;
  const T m1 = (u[1] + u[2] - u[0] - u[3]) * M.lx - c1;
  const T m2 = (u[2] + u[3] - u[0] - u[1]) * M.c - c2;
  f[9] = M.Jinv[0] * m0 + M.Jinv[1] * m1 + M.Jinv[2] * m2;
  f[10] = M.Jinv[3] * m0 + M.Jinv[4] * m1 + M.Jinv[5] * m2;
  f[11] = M.Jinv[6] * m0 + M.Jinv[7] * m1 + M.Jinv[8] * m2;
  c[0] = sf; c[1] = cf; c[2] = st; c[3] = ct; c[4] = sp; c[5] = cp; c[6] = ict; c[7] = tt;
  c[8] = a; c[9] = cfst; c[10] = s; c[11] = r0; c[12] = r1; c[13] = r2;
  c[14] = jw0; c[15] = jw1; c[16] = jw2; c[17] = wx; c[18] = wy; c[19] = wz;
}

// df = J_f(x_i, u) · (dx, du) from the captured scalars c (same algebra as f_tan's TAN branch).
template <class T>
__device__ __forceinline__ void f_tan_lin(const T* __restrict__ c, const T* __restrict__ dx,
                                          const T* __restrict__ du, const Model<T>& M,
                                          T* __restrict__ df) {
  const T sf = c[0], cf = c[1], st = c[2], ct = c[3], sp = c[4], cp = c[5], ict = c[6], tt = c[7];
  const T a = c[8], cfst = c[9], s = c[10], r0 = c[11], r1 = c[12], r2 = c[13];
  const T jw0 = c[14], jw1 = c[15], jw2 = c[16], wx = c[17], wy = c[18], wz = c[19];
  const T dphi = dx[3], dth = dx[4], dpsi = dx[5];
  const T dwx = dx[9], dwy = dx[10], dwz = dx[11];
  const T dsf = cf * dphi, dcf = -sf * dphi;
  const T dst = ct * dth, dct = -st * dth;
  const T dsp = cp * dpsi, dcp = -sp * dpsi;
  const T dict = -ict * ict * dct;
  const T dtt = dst * ict + st * dict;
  df[0] = dx[6]; df[1] = dx[7]; df[2] = dx[8];
  const T da = dsf * wy + sf * dwy + dcf * wz + cf * dwz;
  const T db = dcf * wy + cf * dwy - dsf * wz - sf * dwz;
  df[3] = dwx + dtt * a + tt * da;
  df[4] = db;
  df[5] = da * ict + a * dict;
  const T dT = (du[0] + du[1]) + (du[2] + du[3]);
  const T ds = dT * M.minv;
  const T dcfst = dcf * st + cf * dst;
  const T dr0 = dcp * cfst + cp * dcfst + dsp * sf + sp * dsf;
  const T dr1 = dsp * cfst + sp * dcfst - dcp * sf - cp * dsf;
  const T dr2 = dcf * ct + cf * dct;
  df[6] = dr0 * s + r0 * ds;
  df[7] = dr1 * s + r1 * ds;
  df[8] = dr2 * s + r2 * ds;
  const T djw0 = M.J[0] * dwx + M.J[1] * dwy + M.J[2] * dwz;
  const T djw1 = M.J[3] * dwx + M.J[4] * dwy + M.J[5] * dwz;
  const T djw2 = M.J[6] * dwx + M.J[7] * dwy + M.J[8] * dwz;
  const T dc0 = dwy * jw2 + wy * djw2 - dwz * jw1 - wz * djw1;
  const T dc1 = dwz * jw0 + wz * djw0 - dwx * jw2 - wx * djw2;
  const T dc2 = dwx * jw1 + wx * djw1 - dwy * jw0 - wy * djw0;
  const T dm0 = (du[1] + du[3] - du[0] - du[2]) * M.ly - dc0;
  const T dm1 = (du[1] + du[2] - du[0] - du[3]) * M.lx - dc1;
  const T dm2 = (du[2] + du[3] - du[0] - du[1]) * M.c - dc2;
  df[9] = M.Jinv[0] * dm0 + M.Jinv[1] * dm1 + M.Jinv[2] * dm2;
  df[10] = M.Jinv[3] * dm0 + M.Jinv[4] * dm1 + M.Jinv[5] * dm2;
  df[11] = M.Jinv[6] * dm0 + M.Jinv[7] * dm1 + M.Jinv[8] * dm2;
}

// Nominal RK4 step that hands each stage's captured scalars to ``sink(stage, c)``.
template <class T, class Sink, class Trig = TrigSerial>
__device__ __forceinline__ void rk4_nom(const T* __restrict__ x, const T* __restrict__ u, T h,
                                        const Model<T>& M, const T w[3], T* __restrict__ xn,
                                        Sink&& sink, const Trig& trig = Trig()) {
  constexpr int NX = 12;
  T k[NX], xs[NX], c[LIN_N];
  const T h2 = T(0.5) * h, h6 = h / T(6);
  f_nom_lin<T>(x, u, M, w, k, c, trig);
  sink(0, c);
#pragma unroll
  for (int i = 0; i < NX; ++i) { xn[i] = k[i]; xs[i] = x[i] + h2 * k[i]; }
  f_nom_lin<T>(xs, u, M, w, k, c, trig);
  sink(1, c);
#pragma unroll
  for (int i = 0; i < NX; ++i) { xn[i] += T(2) * k[i]; xs[i] = x[i] + h2 * k[i]; }
  f_nom_lin<T>(xs, u, M, w, k, c, trig);
  sink(2, c);
#pragma unroll
  for (int i = 0; i < NX; ++i) { xn[i] += T(2) * k[i]; xs[i] = x[i] + h * k[i]; }
  f_nom_lin<T>(xs, u, M, w, k, c, trig);
  sink(3, c);
#pragma unroll
  for (int i = 0; i < NX; ++i) xn[i] = x[i] + h6 * (xn[i] + k[i]);
}

// Tangent of the RK4 step along (dx, du) from the 4 captured stages (LIN_STAGE values; ``get(i)``
// returns captured scalar i).  FENCE keeps each RK stage's scalars from being loaded up front
// (register diet when they sit in LDS next to a register-heavy Riccati body); without it all 80
// loads issue together (one memory round trip per interval, for latency-bound callers).
template <class T, bool FENCE = true, class Get>
__device__ __forceinline__ void rk4_tan_g(Get get, const T* __restrict__ dx,
                                          const T* __restrict__ du, T h, const Model<T>& M,
                                          T* __restrict__ dxn) {
  constexpr int NX = 12;
  T dk[NX], dxs[NX], c[LIN_N];
  const T h2 = T(0.5) * h, h6 = h / T(6);
#pragma unroll
  for (int i = 0; i < LIN_N; ++i) c[i] = get(i);
  f_tan_lin<T>(c, dx, du, M, dk);
#pragma unroll
  for (int i = 0; i < NX; ++i) { dxn[i] = dk[i]; dxs[i] = dx[i] + h2 * dk[i]; }
  if constexpr (FENCE) asm volatile("" ::: "memory");  // load each stage's scalars just before use
#pragma unroll
  for (int i = 0; i < LIN_N; ++i) c[i] = get(LIN_N + i);
  f_tan_lin<T>(c, dxs, du, M, dk);
#pragma unroll
  for (int i = 0; i < NX; ++i) { dxn[i] += T(2) * dk[i]; dxs[i] = dx[i] + h2 * dk[i]; }
  if constexpr (FENCE) asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < LIN_N; ++i) c[i] = get(2 * LIN_N + i);
  f_tan_lin<T>(c, dxs, du, M, dk);
#pragma unroll
  for (int i = 0; i < NX; ++i) { dxn[i] += T(2) * dk[i]; dxs[i] = dx[i] + h * dk[i]; }
  if constexpr (FENCE) asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < LIN_N; ++i) c[i] = get(3 * LIN_N + i);
  f_tan_lin<T>(c, dxs, du, M, dk);
#pragma unroll
  for (int i = 0; i < NX; ++i) dxn[i] = dx[i] + h6 * (dxn[i] + dk[i]);
}

// The same from a strided record ``C`` (``cs`` = element stride: 1 for AoS, 4 for quad-blocked).
template <class T, bool FENCE = true>
__device__ __forceinline__ void rk4_tan(const T* __restrict__ C, const T* __restrict__ dx,
                                        const T* __restrict__ du, T h, const Model<T>& M,
                                        T* __restrict__ dxn, int64_t cs = 1) {
  rk4_tan_g<T, FENCE>([&](int i) { return C[i * cs]; }, dx, du, h, M, dxn);
}

}  // namespace mpcb
