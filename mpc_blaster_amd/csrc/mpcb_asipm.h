// mpcb_asipm.h -- the 12/4 input box's interior-point fallback (oracle.ocp.pdas_solve: the
// instances whose active set has not converged after min(max_as_iter, AS_IPM_AFTER) passes are
// solved again by oracle.ocp.ipm_box_solve with the adaptive centring, input rows only).
//
// Why: the active set's least-index backup terminates finitely but can need thousands of passes
// (with a +-5 N wind and sine references, 262 of 3000 N = 18 instances took more than 60), while
// the interior point needs at most 24 iterations there.  On the c4 bench draws the active set needs
// at most 39 passes, so this kernel finds an empty list and its waves exit at once.
//
// Layout: the active-set kernel's 16 lanes per instance, 4 instances per wave; lane j owns
// direction j.  The fallback list (SplitArgs::as_fb: [0] count, [2 + t] chunk instance) is walked
// in rounds of one instance per group.  Per instance and stage the iterate lives in the instance's
// PS2 record (the active set's value-function snapshots are dead once it handed the instance
// over): lane j's six slots hold its component z of (dx, du), the Newton step dz of it and, on the
// input lanes, the slacks s_l, s_u and multipliers lambda_l, lambda_u of its row.  K and k go to
// the instance's KR2 record, read back by the forward sweep.  An iteration is
//   backward: the Riccati recursion of the Newton system linearised at the iterate (stage cost
//             gradient at ybar + z, zero gaps, Delta x_0 = 0) with D on the input diagonal and d
//             on the input gradient (the active-set kernel's products; D, d from the own row);
//   forward:  Delta du = K Delta dx + k, Delta dx' = [A|B] (Delta dx, Delta du), each input row's
//             largest step to the boundary of (s, lambda);
//   update:   the common step alpha = min(1, tau * that), then z, s, lambda move and mu = mean(lambda
//             s) and the residual are measured for the next iteration's test.
// Control flow is group-uniform (the DPP row broadcasts need whole rows).
#pragma once

#include "mpcb_as.h"

namespace mpcb {
namespace asq {

// (oracle.ocp.AS_IPM_ITERS and the IPM_* constants.)  fp32: the duality measure goes to 1e-8 (the
// 17/6 fp32 interior point stops at 1e-6, mpcb_full.h IPM17_TOL_F32, but here that left the
// weakly active rows 1.2e-3 off the solution; the oracle's interior point stopped at 1e-8 is
// 5.6e-6 off) with the residual bound and breakdown threshold of the 17/6 fp32 interior point
constexpr int AS_IPM_ITERS = 100;
template <class T> struct IpmTol;
template <> struct IpmTol<double> { static constexpr double TOL = 1e-12, BREAK = 1e-5, RES = 1e-9; };
template <> struct IpmTol<float> { static constexpr float TOL = 1e-8f, BREAK = 1e-3f, RES = 1e-5f; };
constexpr double ASI_SIG_MIN = 0.05, ASI_SIG_MAX = 0.9, ASI_TAU = 0.995, ASI_THETA = 0.1, ASI_STALL = 1e-6,
                 ASI_SHORT = 1e-2;
constexpr int ASI_SHORT_RUN = 10;
enum { IZ = 0, IDZ = 1, ISL = 2, ISU = 3, ILL = 4, ILU = 5, ISLOTS = 6 };
static_assert(16 * ISLOTS <= PS2_REC, "the iterate fits the instance's PS2 record");

// largest step t >= 0 with v + t dv >= 0 (inf when dv >= 0)
template <class T> __device__ __forceinline__ T maxstep(T v, T dv) { return dv < T(0) ? -v / dv : T(INFINITY); }

template <class T, bool ITER>
__device__ __forceinline__ void ipm_body(const SplitArgs<T>& args) {
  SplitArgs<T> a = args;
  a.XU = vglobal(a.XU); a.GP = vglobal(a.GP); a.ABT = vglobal(a.ABT); a.KR = vglobal(a.KR);
  a.PS = vglobal(a.PS); a.X = vglobal(a.X); a.U = vglobal(a.U); a.u0 = vglobal(a.u0);
  a.status = vglobal(a.status); a.qp_stats = vglobal(a.qp_stats);
  __shared__ T lds_px[GROUPS][NX * NX];
  __shared__ T SW[NZ * NZ];
  const int lane = threadIdx.x;
  const int q = lane >> 4;
  const int j = lane & 15;
  const int jx = j < NX ? j : 0;
  const int ju = j >= NX ? j - NX : 0;
  const bool stl = j < NX;
  const uint64_t mst = lane_mask(stl);
  T* const PX = lds_px[q];
  const int64_t nb = a.nb;
  const int N = a.N;
  const int64_t nq = (nb + SS - 1) / SS;
  const T h = (a.h / T(6)) * T(6);
  const Weights<T>& W = *a.W;
  const T lbm = W.lbu[ju], ubm = W.ubu[ju];
  const T wbox = ubm - lbm;
  using C = IpmTol<T>;
  for (int e = lane; e < NZ * NZ; e += 64) {
    const int r = e / NZ, cl = e % NZ;
    const T wq = (r < NX && cl < NX) ? W.Q[r * NX + cl] : T(0);
    const T wr = (r >= NX && cl >= NX) ? W.R[(r - NX) * NU + (cl - NX)] : T(0);
    SW[e] = a.s * (wq + wr);
  }
  wave_lds_sync();
  T swc[NZ];
#pragma unroll
  for (int i = 0; i < NZ; ++i) swc[i] = SW[i * NZ + j];
  T crow[6];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    crow[p] = (jx == p) ? T(1) : T(0);
    crow[3 + p] = ((jx == 6 + p) ? T(1) : T(0)) + ((jx == p) ? h : T(0));
  }
  T qn[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) qn[i] = stl ? W.QN[i * NX + jx] : T(0);
  const int tv = var_index(j);
  const int cslot = j < 3 ? j : j - 3;
  const int cnt = a.as_fb[0];
  const int64_t G = (int64_t)gridDim.x * GROUPS;
  for (int64_t t0 = (int64_t)blockIdx.x * GROUPS; t0 < cnt; t0 += G) {   // (wave-uniform)
    const int64_t t = t0 + q;
    const bool valid = t < cnt;
    const int64_t c = a.as_fb[2 + (valid ? t : t0)];   // an empty group shadows the round's first
    const int64_t b = a.b0 + c;
    const T* xr = a.xref + b * a.xref_sb;
    const T* ur = a.uref + b * a.uref_sb;
    const Arr<T> XU = arr(a.XU, XU_REC, nq, c);
    const Arr<T> GP = arr(ITER ? a.GP : (T*)nullptr, GP_REC, nq, c);
    const Arr<T> ABT = arr2(a.ABT, ABT2_REC, nq, c, N, a.imajor);
    const Arr<T> KR = arr2(a.KR, KR2_REC, nq, c, N, a.imajor);
    const Arr<T> PS = arr2(a.PS, PS2_REC, nq, c, N, a.imajor);
    const T* const cbase = tv >= 0 ? ABT.p0 + tv : W.ctab + cslot;
    const int64_t cstride = tv >= 0 ? ABT.stride : 0;
    const T* const refp = stl ? xr + jx : ur + ju;
    const int64_t refs = stl ? NX : NU;
    auto slot = [&](int k) { return PS.at(k) + j * ISLOTS; };
    // the lane's row of [A_k | B_k] (state lanes; the constant columns from crow)
    auto arow = [&](int k, T (&row)[NZ]) {
      T v[ABT2_W];
      ldv<T, ABT2_W, sizeof(T) == 8 ? 16 : 8>(ABT.at(k) + jx * ABT2_W, v);
#pragma unroll
      for (int s = 0; s < NVAR; ++s) row[var_col(s)] = v[s];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        row[p] = crow[p];
        row[6 + p] = crow[3 + p];
      }
    };
    // ---- start: du = clip(0, lb + theta w, ub - theta w), dx by the dynamics, s at the box, lambda = 1
    T z = (ITER && stl) ? a.x0[b * a.x0_sb + jx] - XU.at(0)[jx * SS] : T(0);
    T musum = T(0);
    for (int k = 0; k < N; ++k) {
      const T yb = XU.at(k)[j * SS];
      const T lo = lbm - yb, hi = ubm - yb;   // (input lanes) the box in du coordinates
      if (!stl) z = fmin(fmax(T(0), lo + T(ASI_THETA) * wbox), hi - T(ASI_THETA) * wbox);
      T* sp = slot(k);
      if (valid) sp[IZ] = z;
      if (!stl && valid) {
        sp[ISL] = z - lo;
        sp[ISU] = hi - z;
        sp[ILL] = T(1);
        sp[ILU] = T(1);
        musum += (z - lo) + (hi - z);
      }
      T row[NZ];
      arow(k, row);
      T acc[4] = {ITER ? GP.at(k)[jx * SS] : T(0), T(0), T(0), T(0)};
      dot16(acc, z, row);
      if (stl) z = sum4(acc);
    }
    T zN = z;   // (state lanes) dx_N
    const T rows2 = T(2 * N * NU);
    auto group_sum = [&](T v) { return (bc<NX>(v) + bc<NX + 1>(v)) + (bc<NX + 2>(v) + bc<NX + 3>(v)); };
    auto group_max = [&](T v) { return fmax(fmax(bc<NX>(v), bc<NX + 1>(v)), fmax(bc<NX + 2>(v), bc<NX + 3>(v))); };
    auto group_min = [&](T v) { return fmin(fmin(bc<NX>(v), bc<NX + 1>(v)), fmin(bc<NX + 2>(v), bc<NX + 3>(v))); };
    T mu = group_sum(stl ? T(0) : musum) / rows2, res = T(0);
    bool act = valid, conv = false, ok = true;
    T prev_alpha = T(1);
    int nshort = 0, its = 0;
    for (int it = 0; it < AS_IPM_ITERS; ++it) {
      act = act && (mu > T(C::TOL) || res > T(C::RES));
      if (!__any(act)) break;
      const T sig = fmin(fmax(T(1) - prev_alpha, T(ASI_SIG_MIN)), T(ASI_SIG_MAX));
      const T smu = sig * mu;
      // ---- backward: the Newton system's Riccati recursion
      T Pc[NX], pj;
      {
        const T vN = stl ? XU.at(N)[jx * SS] + zN - xr[(int64_t)N * NX + jx] : T(0);
        T acc[4] = {T(0), T(0), T(0), T(0)};
        dot12(acc, vN, qn);
        pj = stl ? sum4(acc) : T(0);
#pragma unroll
        for (int i = 0; i < NX; ++i) Pc[i] = qn[i];
      }
      bool qp_ok = true, fin = true;
      for (int k = N - 1; k >= 0; --k) {
        T col[NX];
        {
          const T* rows = cbase + (int64_t)k * cstride;
#pragma unroll
          for (int i = 0; i < NX; ++i) col[i] = rows[i * ABT2_W];
        }
        const T yb = XU.at(k)[j * SS];
        const T* sp = slot(k);
        const T zk = sp[IZ];
        const T e = yb + zk - refp[(int64_t)k * refs];
        // the own input row's barrier terms D, d (oracle.ocp.ipm_box_solve newton)
        T Dm = T(0), dm = T(0);
        if (!stl) {
          const T sl = sp[ISL], su = sp[ISU], ll = sp[ILL], lu = sp[ILU];
          const T rl = zk - (lbm - yb) - sl, ru = (ubm - yb) - zk - su;
          Dm = ll / sl + lu / su;
          dm = -smu * (T(1) / sl - T(1) / su) + (ll / sl) * rl - (lu / su) * ru;
        }
        fin = fin && isfin(Dm) && isfin(dm) && isfin(zk);
        const T pt = pj;
        T hj;
        T G[NZ];
        if constexpr (sizeof(T) == 4) {
          T acc[4] = {T(0), T(0), T(0), T(0)};
          dot12(acc, pt, col);
          hj = sum4(acc);
          float y[16], g[16];
          to_columns(outer12(Pc, col), y);
          to_columns(outer12(col, y), g);
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
        {
          T acc[4] = {hj, T(0), T(0), T(0)};
          dot16(acc, e, swc);
          hj = sum4(acc);
#pragma unroll
          for (int i = 0; i < NZ; ++i) G[i] += swc[i];
        }
        T Ht[NU * NU], ht[NU], Hux_t[NU];
        static_for<NU>([&](auto mm) {
          constexpr int m = decltype(mm)::value;
          Ht[m * NU + 0] = bc<NX + 0>(G[NX + m]);
          Ht[m * NU + 1] = bc<NX + 1>(G[NX + m]);
          Ht[m * NU + 2] = bc<NX + 2>(G[NX + m]);
          Ht[m * NU + 3] = bc<NX + 3>(G[NX + m]);
          ht[m] = bc<NX + m>(hj) + bc<NX + m>(dm);
          Ht[m * NU + m] += bc<NX + m>(Dm);
          Hux_t[m] = G[NX + m];
        });
        T Lc[10];
        chol4(Ht, Lc);
#pragma unroll
        for (int i = 0; i < 10; ++i) qp_ok = qp_ok && (Lc[i] == Lc[i]);
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
        T Pn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) Pn[i] = G[i];
#pragma unroll
        for (int m = 0; m < NU; ++m) diag12(Pn, G[NX + m], Kj[m]);
        if (valid) {
          T* kr = KR.at(k);
          if (stl) {
#pragma unroll
            for (int m = 0; m < NU; ++m) kr[m * KR2_W + j] = Kj[m];
          } else {
            kr[ju * KR2_W + 12] = sel<NU>(kff, ju);
          }
        }
        if (stl) {
#pragma unroll
          for (int i = 0; i < NX; ++i) PX[j * NX + i] = Pn[i];
        }
        wave_lds_sync();
        static_for<NX>([&](auto ii) {
          constexpr int i = decltype(ii)::value;
          Pc[i] = sel_le<i>(jx, Pn[i], PX[i * NX + jx]);
        });
        pj = pn;
        wave_lds_sync();
      }
      // group verdicts (every lane of the group holds them)
      {
        const uint64_t bad_fin = lane_mask(!fin), bad_qp = lane_mask(!qp_ok);
        fin = ((bad_fin >> (16 * q)) & 0xFFFFu) == 0;
        qp_ok = ((bad_qp >> (16 * q)) & 0xFFFFu) == 0;
      }
      ok = ok && (fin || !valid || !act);   // (a finished group's recomputed pass is not its verdict)
      act = act && fin;
      const bool brk = !qp_ok && act && mu <= T(C::BREAK) && res <= T(C::RES);
      conv = conv || brk;
      act = act && !brk;
      ok = ok && (qp_ok || !act);
      // ---- forward: the Newton step and each input row's largest step
      T amax = T(INFINITY);
      z = T(0);   // Delta dx_0 = 0
      for (int k = 0; k < N; ++k) {
        T row[NZ];
        arow(k, row);
        T kr[KR2_W];
        ldv<T, KR2_W, sizeof(T) == 8 ? 16 : 8>(KR.at(k) + ju * KR2_W, kr);
        {
          T acc[4] = {kr[NX], T(0), T(0), T(0)};
          T krow[NX];
#pragma unroll
          for (int i = 0; i < NX; ++i) krow[i] = kr[i];
          dot12(acc, z, krow);
          z = csel(mst, z, sum4(acc));   // input lanes: Delta du
        }
        T* sp = slot(k);
        if (valid) sp[IDZ] = z;
        if (!stl) {
          const T yb = XU.at(k)[j * SS];
          const T zk = sp[IZ], sl = sp[ISL], su = sp[ISU], ll = sp[ILL], lu = sp[ILU];
          const T rl = zk - (lbm - yb) - sl, ru = (ubm - yb) - zk - su;
          const T dsl = z + rl, dsu = ru - z;
          const T dll = (smu - ll * sl - ll * dsl) / sl, dlu = (smu - lu * su - lu * dsu) / su;
          amax = fmin(amax, fmin(fmin(maxstep(sl, dsl), maxstep(su, dsu)), fmin(maxstep(ll, dll), maxstep(lu, dlu))));
        }
        T acc[4] = {T(0), T(0), T(0), T(0)};
        dot16(acc, z, row);
        if (stl) z = sum4(acc);   // Delta dx_{k+1}
      }
      const T dzN = z;
      T alpha = fmin(T(1), T(ASI_TAU) * group_min(stl ? T(INFINITY) : amax));
      prev_alpha = alpha;
      nshort = alpha < T(ASI_SHORT) ? nshort + 1 : 0;
      const bool stall = act && (alpha < T(ASI_STALL) || nshort >= ASI_SHORT_RUN);
      const bool near = mu <= T(C::BREAK) && res <= T(C::RES);
      conv = conv || (stall && near);
      ok = ok && !(stall && !near);
      act = act && !stall;
      if (!act) alpha = T(0);
      its += act ? 1 : 0;
      // ---- update: the common step, then mu and the residual at the new iterate
      if (__any(act)) {
        T ms = T(0), rs = T(0);
        for (int k = 0; k < N; ++k) {
          T* sp = slot(k);
          const T zk = sp[IZ], dz = sp[IDZ];
          if (act) sp[IZ] = zk + alpha * dz;
          if (!stl) {
            const T yb = XU.at(k)[j * SS];
            const T lo = lbm - yb, hi = ubm - yb;
            T sl = sp[ISL], su = sp[ISU], ll = sp[ILL], lu = sp[ILU];
            const T rl = zk - lo - sl, ru = hi - zk - su;
            const T dsl = dz + rl, dsu = ru - dz;
            const T dll = (smu - ll * sl - ll * dsl) / sl, dlu = (smu - lu * su - lu * dsu) / su;
            if (act) {
              sl += alpha * dsl; su += alpha * dsu; ll += alpha * dll; lu += alpha * dlu;
              sp[ISL] = sl; sp[ISU] = su; sp[ILL] = ll; sp[ILU] = lu;
            }
            const T zn = act ? zk + alpha * dz : zk;
            ms += ll * sl + lu * su;
            rs = fmax(rs, fmax(fabs(zn - lo - sl), fabs(hi - zn - su)));
          }
        }
        if (act) zN = zN + alpha * dzN;
        const T mu_n = group_sum(stl ? T(0) : ms) / rows2, res_n = group_max(stl ? T(0) : rs);
        if (act) {
          mu = mu_n;
          res = res_n;
        }
      }
    }
    // ---- outputs: X = xbar + dx, U = ubar + du; status (P2's QP verdict carries over, as in the
    // active-set kernel's finish)
    int32_t st = (conv || (mu <= T(C::TOL) && res <= T(C::RES))) ? MPCB_STATUS_OK : MPCB_STATUS_MAXITER;
    if (!ok) st = MPCB_STATUS_QP_FAIL;
    if (st == MPCB_STATUS_OK && !(mu <= T(C::TOL) && res <= T(C::RES))) st = MPCB_STATUS_MINSTEP;
    bool ofin = true;
    uint64_t alo = 0, ahi = 0;   // (fp32, input lanes) the components at their bounds
    const T dact = T(1e-4) * wbox;
    for (int k = 0; k <= N; ++k) {
      const T y = XU.at(k)[j * SS] + (k < N ? slot(k)[IZ] : zN);
      if (!stl && k < N) {
        alo |= (uint64_t)(y <= lbm + dact) << k;
        ahi |= (uint64_t)(y >= ubm - dact) << k;
      }
      if (valid) {
        if (stl) {
          if (a.X) a.X[(b * (N + 1) + k) * NX + jx] = y;
        } else if (k < N) {
          if (a.U) a.U[(b * N + k) * NU + ju] = y;
          if (k == 0) {
            a.u0[b * NU + ju] = y;
            ofin = ofin && isfin(y);
          }
        }
      }
    }
    const uint64_t bad = lane_mask(!ofin);
    ofin = ((bad >> (16 * q)) & 0xFFFFu) == 0;
    if constexpr (sizeof(T) == 4) {
      // crossover: the interior point's active set (components within 1e-4 of the box width of a
      // bound) goes to the refinement kernel like an active-set instance, which refactors it in
      // full (kc = N - 1), refines in fp64 residuals and corrects the set (the fp32 interior
      // point alone stops ~1e-4 off the minimiser)
      if (valid && a.as_ref && st == MPCB_STATUS_OK && ofin) {   // (group-uniform)
        int tk = 0;
        if (j == 0) tk = atomicAdd(a.as_ref, 1);
        tk = bc<0>(tk);
        if (tk < a.as_ref_cap) {
          int* e = a.as_ref + AS_REF_HDR + (int64_t)tk * AS_REF_W;
          const int32_t q0 = a.qp_stats ? a.qp_stats[2 * b] : 0, q1 = a.qp_stats ? a.qp_stats[2 * b + 1] : 0;
          as_ref_put<false>(e, j, (int)c, 1, q0 + its, q1 + its * N, alo, ahi);
          if (j == 0) e[AS_REF_KC] = N - 1;
        }
      }
    }
    if (valid && j == NX) {
      const int32_t st0 = a.status[b];
      a.status[b] = !ofin ? MPCB_STATUS_NAN : (st0 != MPCB_STATUS_OK ? st0 : st);
      if (a.qp_stats) {
        a.qp_stats[2 * b] += its;
        a.qp_stats[2 * b + 1] += its * N;
      }
    }
  }
}

}  // namespace asq
}  // namespace mpcb
