// mpcb_row.h -- P1 with a 16-lane row per instance (small chunks: c2), as a device body: the
// kernel of mpcb_rollout.hip and the fused rollout + Riccati kernel of mpcb_split.hip run it.
//
// The nominal RK4 rollout of the linearisation point (acados sim_erk on the OCP of
// blastermodel.py:214-292; dynamics f_expl_expr, blastermodel.py:95-201) is a serial chain of
// 4·N evaluations of f per instance.  At c2 (4096 instances) the lane-quad rollout
// (nominal_quad_kernel, mpcb_split.hip) fills 256 wavefronts — one SIMD in four — and each of
// them issues the whole of f for 16 instances, because the quad's lanes only split the sin/cos.
// Here the 16 lanes of a row SPLIT f itself, so a wavefront carries 4 instances (one workspace
// quad) and c2 runs 1024 wavefronts, one per SIMD, each with a chain about half as long:
//
//   lane t < 12 holds state x_t and computes f_t; lanes 12..15 hold u_{t-12} (f = 0 there);
//   every lane takes sin/cos of its own state (lanes 3, 4, 5: phi, theta, psi) and lane 4 the
//   reciprocal 1/cos(theta); row broadcasts (v_mov_b64_dpp row_newbcast) give every lane the
//   eleven scalars the row shares (sin/cos of the three angles, 1/cos(theta), tan(theta), the
//   body rates); the few products of f that several rows share (a, b, the rotation column
//   R e3) are formed once per lane; then lane t's row of f is assembled from them by FMAs with
//   loop-invariant per-lane 0/1 coefficients (and, for the body rates, the per-lane quadratic
//   form of -J^-1 (w x J w) plus the per-interval J^-1 M(u));
//   the RK4 stage update of x_t is lane-local.
//
// The captured linearisation scalars (mpcb_model.h f_nom_lin: 20 per RK stage) are stored from
// the lanes that hold them into the same quad-blocked CC record the other P1 variants write, so
// P2 is unchanged; likewise XU (x_k, u_k) and, in iterate mode, the gaps GP.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "../../include/mpcb.h"
#include "mpcb_common.h"
#include "mpcb_kernels.h"
#include "mpcb_split.h"

namespace mpcb {

namespace {

// lane L's value in every lane of its 16-lane row (fp64: one v_mov_b64_dpp)
template <int L, class T> __device__ __forceinline__ T rbc(T v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + L, 0xF, 0xF, false);   // (no old value to zero)
}
// lane t + 6's value in lane t of the row (row_shl:6; lanes 10..15 read 0)
template <class T> __device__ __forceinline__ T shl6(T v) {
  return __builtin_amdgcn_mov_dpp(v, 0x106, 0xF, 0xF, true);
}

// Taylor coefficients of the stage angle offsets (MPCB_ROW_SC_ADD) as opaque loop-invariant
// registers (fp64 constants are not encodable as literals): sin d = d + d^3 (v0 d^6 + v1 d^4 +
// v2 d^2 + v3), cos d - 1 = d^2 (v4 d^8 + v5 d^6 + v6 d^4 + v7 d^2 + v8)
#ifndef MPCB_ROW_SC_ADD
#define MPCB_ROW_SC_ADD 1
#endif
struct SaRegs {
  double v[9];
  __device__ __forceinline__ SaRegs() {
    v[0] = 1.0 / 362880.0; v[1] = -1.0 / 5040.0; v[2] = 1.0 / 120.0; v[3] = -1.0 / 6.0;
    v[4] = -1.0 / 3628800.0; v[5] = 1.0 / 40320.0; v[6] = -1.0 / 720.0; v[7] = 1.0 / 24.0; v[8] = -0.5;
#pragma unroll
    for (int i = 0; i < 9; ++i) asm volatile("" : "+v"(v[i]));
  }
};

struct SaNone {};

template <class T> struct ScOf { using type = ScConst; using sa = SaNone; };
template <> struct ScOf<double> { using type = ScRegs; using sa = std::conditional_t<MPCB_ROW_SC_ADD != 0, SaRegs, SaNone>; };

}  // namespace

// Tangent of one RK stage along the lane's direction (TAN): dk = J_f(x_s, u)·(dS, e_u) from the
// stage's scalars, which every lane of the row already holds after the broadcasts (the algebra of
// mpcb_model.h f_tan_lin, regrouped around the products the nominal f shares: with the lane's input
// direction a constant, dT·minv and J^-1 M(du) are loop-invariant per lane).  DJ: diagonal J, so
// (w x Jw)' is (J_a - J_b)(w_b dw_c + dw_b w_c) per component.
template <class T> struct StageSc {
  T sf, cf, st, ct, sp, cp, ict, tt, a, b, cfst, s, r0, r1, r2, wx, wy, wz, jw0, jw1, jw2;
};
template <class T> struct TanConst {
  T dsl;             // dT · minv of the lane's input direction (0 on state lanes)
  T Ju[3];           // J^-1 M(e_u) of the lane's input direction
  T kd[3];           // DJ: -Jinv_ii (J_a - J_b)
  T J[9], Ji[9];     // general J
};
template <class T, bool DJ>
__device__ __forceinline__ void tan_stage(const StageSc<T>& c, const T* __restrict__ dS,
                                          const TanConst<T>& K, T* __restrict__ dk) {
  const T dphi = dS[3], dth = dS[4], dpsi = dS[5];
  const T dwx = dS[9], dwy = dS[10], dwz = dS[11];
  const T ict2st = c.ict * c.ict * c.st;                 // d(1/ct)/dth
  const T dict = ict2st * dth;
  const T dtt = fma(c.ct * c.ict, dth, c.st * dict);     // dst ict + st dict
  const T da = fma(dphi, c.b, fma(c.sf, dwy, c.cf * dwz));
  const T db = fma(-dphi, c.a, fma(c.cf, dwy, -c.sf * dwz));
  dk[0] = dS[6]; dk[1] = dS[7]; dk[2] = dS[8];
  dk[3] = fma(dtt, c.a, fma(c.tt, da, dwx));
  dk[4] = db;
  dk[5] = fma(da, c.ict, c.a * dict);
  const T dcfst = fma(c.r2, dth, -(c.sf * c.st) * dphi);   // dcf st + cf dst
  const T dr0 = fma(-dpsi, c.r1, fma(c.cp, dcfst, (c.sp * c.cf) * dphi));
  const T dr1 = fma(dpsi, c.r0, fma(c.sp, dcfst, -(c.cp * c.cf) * dphi));
  const T dr2 = -fma(c.sf * c.ct, dphi, c.cfst * dth);
  dk[6] = fma(dr0, c.s, c.r0 * K.dsl);
  dk[7] = fma(dr1, c.s, c.r1 * K.dsl);
  dk[8] = fma(dr2, c.s, c.r2 * K.dsl);
  if constexpr (DJ) {
    dk[9] = fma(K.kd[0], fma(dwy, c.wz, c.wy * dwz), K.Ju[0]);
    dk[10] = fma(K.kd[1], fma(dwz, c.wx, c.wz * dwx), K.Ju[1]);
    dk[11] = fma(K.kd[2], fma(dwx, c.wy, c.wx * dwy), K.Ju[2]);
  } else {
    const T djw0 = fma(K.J[0], dwx, fma(K.J[1], dwy, K.J[2] * dwz));
    const T djw1 = fma(K.J[3], dwx, fma(K.J[4], dwy, K.J[5] * dwz));
    const T djw2 = fma(K.J[6], dwx, fma(K.J[7], dwy, K.J[8] * dwz));
    const T dc0 = fma(dwy, c.jw2, c.wy * djw2) - fma(dwz, c.jw1, c.wz * djw1);
    const T dc1 = fma(dwz, c.jw0, c.wz * djw0) - fma(dwx, c.jw2, c.wx * djw2);
    const T dc2 = fma(dwx, c.jw1, c.wx * djw1) - fma(dwy, c.jw0, c.wy * djw0);
    dk[9] = K.Ju[0] - fma(K.Ji[0], dc0, fma(K.Ji[1], dc1, K.Ji[2] * dc2));
    dk[10] = K.Ju[1] - fma(K.Ji[3], dc0, fma(K.Ji[4], dc1, K.Ji[5] * dc2));
    dk[11] = K.Ju[2] - fma(K.Ji[6], dc0, fma(K.Ji[7], dc1, K.Ji[8] * dc2));
  }
}

// DJ: diagonal inertia (the reference's J, simulation_blaster.py:13-15): the gyroscopic term of
// body rate t is one product (w_{t+1} w_{t+2}); otherwise the general six-product quadratic form.
// TAN: the row also integrates the RK4 tangent of direction e_t (lane t; state lanes e_x, input
// lanes e_u) through the same four stages and exports the variable columns of [A_k | B_k] as the
// ABT2 rows (mpcb_kernels.h) that P2 then reads instead of integrating them (SplitArgs::tin).  The
// tangent of stage s is independent of the nominal stage s + 1, so the two chains interleave in
// one basic block; no captured-scalar record (CC) is written.
// The body of P1 (nominal_row_kernel, and the first half of the fused row_riccati_kernel of
// mpcb_split.hip).  The including translation unit declares WT_TABLE(g_wt_p1).
template <class T, bool ITER, bool DJ, bool TAN>
__device__ __forceinline__ void row_body(const SplitArgs<T>& a) {
  WT(g_wt_p1, 0);
  const int lane = threadIdx.x;
  const int t = lane & 15;                 // row lane
  const int q = lane >> 4;                 // instance within the wavefront's quad
  const int64_t nb = a.nb;
  const int64_t nq = (nb + SS - 1) / SS;
  const int64_t qd = blockIdx.x;           // the wavefront's workspace quad
  const int64_t c_raw = qd * SS + q;
  const int64_t c = c_raw < nb ? c_raw : nb - 1;   // ragged quad: recompute the last instance
  const int64_t b = a.b0 + c;
  const int N = a.N;
  const Model<T>& M = a.M;
  const T h = a.h, h2 = T(0.5) * a.h, h6 = a.h / T(6);

  // ---- loop-invariant per-lane coefficients (0/1 row selectors, J-dependent forms) ----------
  const T kv = T(t < 3);                   // f_t = v_t (t < 3), from lane t + 6
  const T k1 = T(t == 3);                  // f_3 = wx + tt a
  const T k2 = T(t == 3), k3 = T(t == 5);  // f_5 = ict a
  const T k4 = T(t == 4);                  // f_4 = b
  const T kr0 = T(t == 6), kr1 = T(t == 7), kr2 = T(t == 8);   // f_{6+i} = s r_i + const
  // body rates t = 9..11: f = J^-1 M(u) - J^-1 (w x J w).  (w x Jw)_i = sum_jl B_i[j][l] w_j w_l
  // with B_i[j][l] = sum_m eps_ijm J_ml; the per-lane form over the products
  // p = (w0 w0, w1 w1, w2 w2, w0 w1, w0 w2, w1 w2) is G_t,p = -sum_i Jinv[t-9][i] coef_i,p
  T G[6];
  T Lm[4];   // J^-1 mixer: f_t's constant part is sum_m Lm[m] u_m
  {
    const int r = (t >= 9 && t < 12) ? t - 9 : -1;
    T coef[3][6];
    auto Jm = [&](int m, int l) { return M.J[m * 3 + l]; };
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;   // eps_{i,i1,i2} = +1, eps_{i,i2,i1} = -1
      auto B = [&](int j, int l) {
        return (j == i1 ? Jm(i2, l) : T(0)) - (j == i2 ? Jm(i1, l) : T(0));
      };
      coef[i][0] = B(0, 0); coef[i][1] = B(1, 1); coef[i][2] = B(2, 2);
      coef[i][3] = B(0, 1) + B(1, 0); coef[i][4] = B(0, 2) + B(2, 0); coef[i][5] = B(1, 2) + B(2, 1);
    }
    // mixer (blastermodel.py:95-101): M = [ly(u1+u3-u0-u2), lx(u1+u2-u0-u3), c(u2+u3-u0-u1)]
    const T mix[3][4] = {{-M.ly, M.ly, -M.ly, M.ly}, {-M.lx, M.lx, M.lx, -M.lx}, {-M.c, -M.c, M.c, M.c}};
#pragma unroll
    for (int p = 0; p < 6; ++p) {
      T g = T(0);
#pragma unroll
      for (int i = 0; i < 3; ++i) g += (r >= 0 ? M.Jinv[r * 3 + i] : T(0)) * coef[i][p];
      G[p] = -g;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      T l = T(0);
#pragma unroll
      for (int i = 0; i < 3; ++i) l += (r >= 0 ? M.Jinv[r * 3 + i] : T(0)) * mix[i][m];
      Lm[m] = l;
    }
  }
  // the lane's row of J (captured J w, mpcb_model.h f_nom_lin c[14..16]) on lanes 9..11
  const int jr = (t >= 9 && t < 12) ? t - 9 : 0;
  const T J0 = M.J[jr * 3], J1 = M.J[jr * 3 + 1], J2 = M.J[jr * 3 + 2];
  // constant part of f_t: the wind force / m and gravity (t = 6..8)
  T K0 = T(0);
  if (a.wind && t >= 6 && t < 9) K0 = a.wind[b * a.wind_sb + (t - 6)] * M.minv;
  if (t == 8) K0 -= M.g;
  const typename ScOf<T>::type kc;
  const typename ScOf<T>::sa sa;
  // the tangent's lane constants (TAN): direction e_t; its input part e_{t-12} on lanes 12..15
  TanConst<T> K{};
  T ev[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) ev[i] = T(t == i);
  if constexpr (TAN) {
    const int m = t >= NX ? t - NX : -1;
    K.dsl = m >= 0 ? M.minv : T(0);
    const T mixm[3] = {m < 0 ? T(0) : ((m == 1 || m == 3) ? M.ly : -M.ly),
                       m < 0 ? T(0) : ((m == 1 || m == 2) ? M.lx : -M.lx),
                       m < 0 ? T(0) : ((m == 2 || m == 3) ? M.c : -M.c)};
#pragma unroll
    for (int r = 0; r < 3; ++r)
      K.Ju[r] = fma(M.Jinv[r * 3], mixm[0], fma(M.Jinv[r * 3 + 1], mixm[1], M.Jinv[r * 3 + 2] * mixm[2]));
    K.kd[0] = -M.Jinv[0] * (M.J[8] - M.J[4]);
    K.kd[1] = -M.Jinv[4] * (M.J[0] - M.J[8]);
    K.kd[2] = -M.Jinv[8] * (M.J[4] - M.J[0]);
#pragma unroll
    for (int i = 0; i < 9; ++i) { K.J[i] = M.J[i]; K.Ji[i] = M.Jinv[i]; }
  }
  const int tv = var_index(t);             // the lane's variable column of [A|B] (-1: constant)
  const bool exp_lane = TAN && tv >= 0 && c_raw < nb;

  // ---- workspace addressing: the quad-blocked records of mpcb_split.h soa(), quad qd --------
  T* const xu0 = a.XU + qd * XU_REC * SS + q;
  T* const cc0 = TAN ? nullptr : a.CC + qd * CCS_REC * SS + q;
  T* const gp0 = ITER ? a.GP + qd * GP_REC * SS + q : nullptr;
  const int64_t xu_k = nq * XU_REC * SS, cc_k = nq * CCS_REC * SS, gp_k = nq * GP_REC * SS;

  // The wave's per-stage inputs (rollout: u_ref; iterate: xbar, ubar) staged in LDS once
  // (row_lds_elems): a per-interval global load here sat on the chain, and its vmcnt(0) wait
  // also drained the previous interval's stores -- 24 % of the wave's cycles parked (PMC).
  extern __shared__ __attribute__((aligned(16))) unsigned char row_dyn[];
  T* const lu = reinterpret_cast<T*>(row_dyn);          // [GROUPS][N][NU]: u of the stage
  T* const lx = lu + GROUPS * N * NU;                    // ITER: [GROUPS][N + 1][NX]: xbar
  // X: x_t (t < 12) / u_{t-12} (t >= 12) of the interval's start; x0's load is issued first
  T X = T(0);
  if (!ITER && t < NX) X = a.x0[b * a.x0_sb + t];
  {
    // eight loads in flight per lane before their LDS writes (one at a time, the staging was a
    // chain of global-load round trips: 2.5 us of the c2 wave's prologue), the group by compares
    auto stage_in = [&](T* dst, const int per, auto&& src) {
      const int total = GROUPS * per;
      for (int e0 = lane; e0 < total; e0 += 64 * 8) {
        T v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int e = e0 + 64 * u;
          const int g = (e >= per) + (e >= 2 * per) + (e >= 3 * per);
          const int64_t cg = qd * SS + g < nb ? qd * SS + g : nb - 1;
          v[u] = e < total ? src(a.b0 + cg, e - g * per) : T(0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (e0 + 64 * u < total) dst[e0 + 64 * u] = v[u];
      }
    };
    static_assert(GROUPS == 4, "stage_in's group compares");
    const int nu_e = N * NU, nx_e = (N + 1) * NX;
    if constexpr (ITER) {
      stage_in(lu, nu_e, [&](int64_t bb, int r) { return a.ubar[bb * (int64_t)nu_e + r]; });
      stage_in(lx, nx_e, [&](int64_t bb, int r) { return a.xbar[bb * (int64_t)nx_e + r]; });
    } else {
      stage_in(lu, nu_e, [&](int64_t bb, int r) { return a.uref[bb * a.uref_sb + r]; });
    }
    wave_lds_sync();
  }
  const T* const lxq = lx + q * (N + 1) * NX;
  const T* const luq = lu + q * N * NU;
  if (ITER && t < NX) X = lxq[t];

  WT(g_wt_p1, 1);
  for (int k = 0; k < N; ++k) {
    if (ITER && t < NX && k) X = lxq[k * NX + t];
    if (t >= NX) X = luq[k * NU + (t - NX)];
    xu0[k * xu_k + t * SS] = X;
    // per-interval constants: the inputs, the thrust scale and J^-1 M(u) + the constant forces
    const T u0 = rbc<12>(X), u1 = rbc<13>(X), u2 = rbc<14>(X), u3 = rbc<15>(X);
    const T s = ((u0 + u1) + (u2 + u3) + M.t_blast) * M.minv;
    const T Kt = fma(Lm[0], u0, fma(Lm[1], u1, fma(Lm[2], u2, fma(Lm[3], u3, K0))));
    T Xn = T(0);
    T dN[NX];   // TAN: the RK4 tangent accumulator
    // One interval.  SLOW = false: sin/cos without their range fallbacks (sc_core at stage 0,
    // angle addition at stages 1..3), so the four stages are one basic block in which the
    // scheduler interleaves the tangent of stage s with the sin/cos of stage s + 1 (a branch per
    // stage around the fallbacks kept them apart: P1 45 -> 39 us at c2).  It returns whether an
    // angle lane was outside those ranges; the instances (16-lane rows) with such a lane then
    // recompute the interval with SLOW = true (sc() and its fallback at every stage) before
    // anything of the interval but the CC record, which the second pass rewrites, is stored.  The
    // redo runs under an exec mask of those rows only, so the other instances of the wave keep the
    // fast pass's results bit for bit (a wave-wide redo made an instance's last bits depend on its
    // wave-mates: tests/test_gpu_edges.py).
    auto interval = [&](auto slow_tag) -> bool {
      constexpr bool SLOW = decltype(slow_tag)::value;
      bool bad = false;
      T Y = X, XN = T(0);
      T S0 = T(0), C0 = T(1);   // sin / cos of the interval start (MPCB_ROW_SC_ADD)
      T dS[NX];   // TAN: the stage's tangent input
#pragma unroll
      for (int i = 0; i < NX; ++i) dS[i] = ev[i];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        // sin/cos of the lane's own state (lanes 3..5: the Euler angles), 1/cos and tan on lane 4
        T S, C;
        const bool ang = t >= 3 && t < 6;   // the Euler-angle lanes: the only sin/cos used
        if constexpr (SLOW) {
          if constexpr (sizeof(T) == 8) sc(Y, &S, &C, kc);
          else sc(Y, &S, &C);
        } else if constexpr (sizeof(T) == 8 && MPCB_ROW_SC_ADD) {
          // stages 1..3 by angle addition from the interval start's sin/cos (Y = X + c h k): the
          // stage offset d = Y - X is small, so sin d and cos d - 1 are short Taylor series (|d| <=
          // 1/8: truncation below 2e-17 relative)
          if (st == 0) {
            sc_core(Y, &S, &C, kc);
            bad = bad || (ang && !(fabs(Y) < 524288.0));
            S0 = S; C0 = C;
          } else {
            const T d = Y - X;
            bad = bad || (ang && !(fabs(d) <= T(0.125)));
            const T d2 = d * d;
            T ps = hstep(sa.v[0], d2, sa.v[1]);
            ps = hstep(ps, d2, sa.v[2]);
            ps = hstep(ps, d2, sa.v[3]);
            const T sd = fma(d * d2, ps, d);                    // sin d
            T pc = hstep(sa.v[4], d2, sa.v[5]);
            pc = hstep(pc, d2, sa.v[6]);
            pc = hstep(pc, d2, sa.v[7]);
            pc = hstep(pc, d2, sa.v[8]);
            const T cm = d2 * pc;                               // cos d - 1
            S = S0 + fma(S0, cm, C0 * sd);
            C = C0 + fma(C0, cm, -(S0 * sd));
          }
        } else if constexpr (sizeof(T) == 8) {
          sc_core(Y, &S, &C, kc);
          bad = bad || (ang && !(fabs(Y) < 524288.0));
        } else {
          sc_core(Y, &S, &C);
          bad = bad || (ang && !(fabsf(Y) < 8192.0f));
        }
        const T R = recip(C);
        const T Tn = S * R;
        StageSc<T> c;
        c.sf = rbc<3>(S); c.cf = rbc<3>(C); c.st = rbc<4>(S); c.ct = rbc<4>(C);
        c.sp = rbc<5>(S); c.cp = rbc<5>(C); c.ict = rbc<4>(R); c.tt = rbc<4>(Tn);
        c.wx = rbc<9>(Y); c.wy = rbc<10>(Y); c.wz = rbc<11>(Y);
        c.a = c.sf * c.wy + c.cf * c.wz;
        c.b = c.cf * c.wy - c.sf * c.wz;
        c.cfst = c.cf * c.st;
        c.r0 = c.cp * c.cfst + c.sp * c.sf;
        c.r1 = c.sp * c.cfst - c.cp * c.sf;
        c.r2 = c.cf * c.ct;
        c.s = s;
        // lane t's row of f, as three independent partial sums
        T F0 = fma(kv, shl6(Y), Kt);
        T F1 = fma(k4, c.b, k1 * c.wx);
        T F2 = c.s * fma(kr0, c.r0, fma(kr1, c.r1, kr2 * c.r2));
        F0 = fma(c.a, fma(k2, c.tt, k3 * c.ict), F0);
        if constexpr (DJ) {
          F1 = fma(G[5], c.wy * c.wz, F1);
          F2 = fma(G[4], c.wx * c.wz, F2);
          F0 = fma(G[3], c.wx * c.wy, F0);
        } else {
          F1 = fma(G[0], c.wx * c.wx, F1);
          F2 = fma(G[1], c.wy * c.wy, F2);
          F0 = fma(G[2], c.wz * c.wz, F0);
          F1 = fma(G[3], c.wx * c.wy, F1);
          F2 = fma(G[4], c.wx * c.wz, F2);
          F0 = fma(G[5], c.wy * c.wz, F0);
        }
        const T F = F0 + (F1 + F2);
        const T JW = fma(J0, c.wx, fma(J1, c.wy, J2 * c.wz));
        if constexpr (TAN) {
          if constexpr (!DJ) { c.jw0 = rbc<9>(JW); c.jw1 = rbc<10>(JW); c.jw2 = rbc<11>(JW); }
          T dk[NX];
          tan_stage<T, DJ>(c, dS, K, dk);
          // RK4 tangent update (mpcb_model.h rk4_tan: same operations)
#pragma unroll
          for (int i = 0; i < NX; ++i) {
            if (st == 0) { dN[i] = dk[i]; dS[i] = fma(h2, dk[i], ev[i]); }
            else if (st == 1) { dN[i] = fma(T(2), dk[i], dN[i]); dS[i] = fma(h2, dk[i], ev[i]); }
            else if (st == 2) { dN[i] = fma(T(2), dk[i], dN[i]); dS[i] = fma(h, dk[i], ev[i]); }
            else dN[i] = fma(h6, dN[i] + dk[i], ev[i]);
          }
        } else {
          // captured scalars of this RK stage (f_nom_lin order), each from a lane that holds it
          T* const cs = cc0 + k * cc_k + st * LIN_N * SS;
          if (t >= 3 && t < 6) {
            cs[(2 * (t - 3)) * SS] = S;          // sf, st, sp
            cs[(2 * (t - 3) + 1) * SS] = C;      // cf, ct, cp
          }
          if (t == 4) {
            cs[6 * SS] = R;                      // ict
            cs[7 * SS] = Tn;                     // tt
          }
          if (t >= 9 && t < 12) {
            cs[(t + 5) * SS] = JW;               // jw0..2
            cs[(t + 8) * SS] = Y;                // wx, wy, wz
          }
          if (t == 0) {
            cs[8 * SS] = c.a;
            cs[9 * SS] = c.cfst;
            cs[10 * SS] = s;
            cs[11 * SS] = c.r0;
            cs[12 * SS] = c.r1;
            cs[13 * SS] = c.r2;
          }
        }
        // RK4 stage update (lane-local; f = 0 on the input lanes)
        if (st == 0) { XN = F; Y = fma(h2, F, X); }
        else if (st == 1) { XN = fma(T(2), F, XN); Y = fma(h2, F, X); }
        else if (st == 2) { XN = fma(T(2), F, XN); Y = fma(h, F, X); }
        else Xn = fma(h6, XN + F, X);
      }
      if constexpr (!SLOW) {
        // keep the fast pass's results ahead of the redo branch: left alone, the compiler sinks
        // the tangent (used only when no redo follows) below it, out of the nominal chain's block
        if constexpr (TAN) {
#pragma unroll
          for (int i = 0; i < NX; ++i) asm volatile("" ::"v"(dN[i]));
        }
        asm volatile("" ::"v"(Xn));
      }
      return bad;
    };
    {
      const uint64_t bad = __builtin_amdgcn_ballot_w64(interval(std::false_type{}));
      if ((bad >> (lane & 48)) & 0xFFFFull) (void)interval(std::true_type{});
    }
    if constexpr (TAN) {
      // column var_col(tv) of [A_k | B_k] into the ABT2 rows: entry (i, tv) at i * ABT2_W + tv.
      // (Staging the wave's four records in LDS and writing them as 16-B vectors measured the
      // same P1 time, 50.3 us at c2, with 75 more instructions per interval.)
      if (exp_lane) {
        T* const abt = rec2(a.ABT, k, ABT2_REC, nb, c, N, a.imajor) + tv;
#pragma unroll
        for (int i = 0; i < NX; ++i) abt[i * ABT2_W] = dN[i];
      }
    }
    if (ITER) {
      if (t < NX) gp0[k * gp_k + t * SS] = Xn - lxq[(k + 1) * NX + t];
    } else if (t < NX) {
      X = Xn;
    }
  }
  WT(g_wt_p1, 2);
  if (t < NX) {
    if (ITER) X = lxq[N * NX + t];
  } else {
    X = T(0);
  }
  xu0[N * xu_k + t * SS] = X;
  WT(g_wt_p1, 3);
}

// dynamic LDS of the row rollout: the wave's staged u (and, iterate mode, xbar) records
template <class T> static size_t row_lds_bytes(const SplitArgs<T>& a) {
  return (size_t)GROUPS * ((size_t)a.N * NU + (a.mode == MPCB_MODE_ITERATE ? (size_t)(a.N + 1) * NX : 0)) * sizeof(T);
}

// diagonal J (and J^-1): the gyroscopic products and their tangent shrink to one term per rate
template <class T> static bool row_dj(const SplitArgs<T>& a) {
  bool dj = true;
  for (int i = 0; i < 9; ++i)
    if (i % 4 != 0) dj = dj && a.M.J[i] == T(0) && a.M.Jinv[i] == T(0);
  return dj;
}

}  // namespace mpcb
