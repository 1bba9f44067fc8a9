// mpcb_box.hip — the input-box QP of the SQP_RTI step (thrust box lbu <= u <= ubu on stages
// 0..N-1, blastermodel.py:259-270 / idxbu, JSON :11,86,148; BASELINE config c4).
//
// acados solves this QP with HPIPM's interior point.  Here it is solved exactly by the primal-dual
// active set with the Kim-Park block-principal-pivoting safeguard, exactly as the oracle does
// (oracle.ocp.pdas_solve): every iteration solves the equality-constrained LQ problem for the
// current sets by a masked Riccati recursion, then collects the infeasible set
//   V = {free u < lb} U {free u > ub} U {u at lb, mu < 0} U {u at ub, mu > 0}
// and exchanges it (all of V while |V| keeps dropping or for pbar = 3 tries, else only its
// largest-index element).  |V| = 0 is the KKT point of the strictly convex QP.
//
// Work split: the first iteration IS the unconstrained P2 Riccati pass, which (with a.AB/a.GH set)
// also exports column j of [A_k | B_k] and the input rows of the stage Hessian.  This kernel then
// iterates over that cached linearisation — a masked backward pass costs the Riccati algebra
// only (no RK4 tangent) — with the same 16-lanes-per-instance layout as P2 (lane j owns direction
// j, 4 instances per wavefront).  The forward pass exchanges (dx, du) through LDS: the input lanes
// form du_k = K_k dx_k + k_k (or the fixed value) and the multipliers, the state lanes form
// dx_{k+1} = [A_k | B_k] (dx_k, du_k) + gap_k from row j of the cached [A|B].
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/mpcb.h"
#include "mpcb_kernels.h"
#include "mpcb_split.h"

namespace mpcb {

#ifdef MPCB_STAMPS
// Diagnostic build only: per-region cycles of the 16-lane forward pass (PASS_FWD) of workgroup 0
// (PASS_BOX: [0..4] forward-stage regions over all passes, [5] masked backward passes, [6] the
// forward tail, [7] active-set updates; [8] iterations, [9] backward stages run by the wave)
__device__ unsigned long long g_bstamps[12];
#define BSTAMP(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); bst_acc[i] += t_ - bst_prev; bst_prev = t_; }
#else
#define BSTAMP(i)
#endif

#ifndef MPCB_BOX_WAVES
#define MPCB_BOX_WAVES 2
#endif
// 1: a masked pass restarts at the highest changed stage from a stored value-function snapshot
// (P_k, p_k written by every pass); 0: every masked pass runs the full recursion, no snapshots
#ifndef MPCB_BOX_RESTART
#define MPCB_BOX_RESTART 1
#endif
#ifndef MPCB_BOX_FWD_DEPTH   // forward-pass prefetch depth (stages) in the active-set kernel
#define MPCB_BOX_FWD_DEPTH 1
#endif

// MODE (the same passes serve three uses):
//   PASS_BOX   input boxes: active-set iterations (the first backward pass is P2's)
//   PASS_SMALL unconstrained, [A|B] cached by lin_kernel: one backward and one forward pass
//   PASS_FWD   unconstrained, P2 already made the backward pass (and cached [A|B]^T): forward only
enum { PASS_BOX = 1, PASS_SMALL = 0, PASS_FWD = 2 };
template <class T, int MODE>
__device__ __forceinline__ void box_body(const SplitArgs<T>& a) {
  constexpr bool BOX = MODE == PASS_BOX;
  __shared__ GroupLds<T> lds_all[GROUPS];
  const int lane = threadIdx.x;
  const int q = lane >> 4;
  const int j = lane & 15;
  const int jx = j < NX ? j : 0;
  const int ju = j >= NX ? j - NX : 0;
  GroupLds<T>& L = lds_all[q];
  const int64_t c_raw = (int64_t)blockIdx.x * GROUPS + q;
  const bool valid = c_raw < a.nb;
  const int64_t c = valid ? c_raw : a.nb - 1;   // inactive groups shadow the last instance
  const int64_t nb = a.nb;
  const int64_t b = a.b0 + c;
  const int N = a.N;
  const T s = a.s;
  const Weights<T>& W = *a.W;
  const bool iterate = a.mode == MPCB_MODE_ITERATE;
  const T* xr = a.xref + b * a.xref_sb;
  const T* ur = a.uref + b * a.uref_sb;
  const T lbm = W.lbu[ju], ubm = W.ubu[ju];
  constexpr T eps = sizeof(T) == 8 ? T(2.220446049250313e-16) : T(1.1920929e-7);
  const T tol_u = T(16) * eps * (fabs(lbm) + fabs(ubm) + T(1));

  uint64_t low[NU], up[NU];   // active sets per input component, bit k = stage k (group-uniform)
#pragma unroll
  for (int m = 0; m < NU; ++m) { low[m] = 0; up[m] = 0; }
  bool done = false;
  int32_t st = MPCB_STATUS_OK;
  int best = 0x7fffffff, pcount = 3;
  int n_fwd = 0, n_bst = 0;   // this instance's forward passes / masked backward stages (qp_stats)

  // Stages above the highest stage whose active set changed keep their gains: each backward
  // pass restarts at kc (group-uniform; N - 1 on the first masked pass) from the value function
  // snapshot P_{kc+1}, p_{kc+1} the previous pass stored (a.PS), and idles where k > kc.
  int kc = N - 1;
#ifdef MPCB_STAMPS
  unsigned long long bst_prev = __builtin_amdgcn_s_memtime(), bst_acc[12] = {};
#endif
  for (int it = 0;; ++it) {
    BSTAMP(7);
    // ------------------------------------------------ masked Riccati over the cached [A|B]
    // (iteration 0 is the unconstrained pass P2 already made: its gains are in KR)
    int kmax = kc;
#pragma unroll
    for (int g = 0; g < GROUPS; ++g) {
      const int o = __shfl(kc, g * 16);
      kmax = o > kmax ? o : kmax;
    }
    if (BOX && it > 0 && !done && kc >= 0) n_bst += kc + 1;
    if (BOX && !done) ++n_fwd;
#ifdef MPCB_STAMPS
    bst_acc[8] += 1;
    if (BOX && it > 0 && kmax >= 0) bst_acc[9] += kmax + 1;
#endif
    if ((BOX ? it > 0 : MODE == PASS_SMALL) && kmax >= 0) {
      T pj = T(0);
      T Pc[NX];
      {
        const T xN = soa(a.XU, N, XU_REC, nb, c)[jx * SS];
        L.v[j] = (j < NX) ? xN - xr[(int64_t)N * NX + jx] : T(0);
        wave_lds_sync();
        if (kc == N - 1) {
          T acc = T(0);
#pragma unroll
          for (int i = 0; i < NX; ++i) acc += W.QN[jx * NX + i] * L.v[i];
          pj = acc;
#pragma unroll
          for (int i = 0; i < NX; ++i) Pc[i] = (j < NX) ? W.QN[i * NX + jx] : T(0);
        } else if (kc >= 0) {
          const T* ps = soa(a.PS, kc + 1, PS_REC, nb, c) + jx * SS;
#pragma unroll
          for (int i = 0; i < NX; ++i) Pc[i] = (j < NX) ? ps[i * NX * SS] : T(0);
          pj = (j < NX) ? ps[NX * NX * SS] : T(0);
        }
        if (kc >= 0 && j < NX) {
#pragma unroll
          for (int i = 0; i < NX; ++i) L.P[j * NX + i] = Pc[i];
        }
        wave_lds_sync();
      }
      bool qp_ok = true;
      // stage data prefetched one stage ahead: column j of [A|B], own (ybar - yref) component,
      // the input part of ubar (masking), the gap (iterate mode)
      T pcol[NX], pe, pub[NU], pgp[NX];
      auto bload = [&](int k) {
        const int tv = var_index(j);
        if (tv >= 0) {
          const T* ab = soa(a.AB, k, AB_REC, nb, c) + tv * SS;
#pragma unroll
          for (int i = 0; i < NX; ++i) pcol[i] = ab[i * NVAR * SS];
        } else {   // position / velocity directions: e_j, e_j + h e_{j-6}
#pragma unroll
          for (int i = 0; i < NX; ++i) pcol[i] = (i == j ? T(1) : T(0)) + ((j >= 6 && i == j - 6) ? a.h : T(0));
        }
        const T* xu = soa(a.XU, k, XU_REC, nb, c);
        pe = xu[j * SS] - ((j < NX) ? xr[(int64_t)k * NX + jx] : ur[(int64_t)k * NU + ju]);
#pragma unroll
        for (int m = 0; m < NU; ++m) pub[m] = xu[(NX + m) * SS];
        if (iterate) {
          const T* gp = soa(a.GP, k, GP_REC, nb, c);
#pragma unroll
          for (int i = 0; i < NX; ++i) pgp[i] = gp[i * SS];
        }
      };
      bload(kmax);
      for (int k = kmax; k >= 0; --k) {
        const bool act = k <= kc;   // this group's stage is recomputed
        T col[NX], ubk[NU], gpk[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) { col[i] = pcol[i]; gpk[i] = pgp[i]; }
#pragma unroll
        for (int m = 0; m < NU; ++m) ubk[m] = pub[m];
        L.v[j] = pe;
        if (k > 0) bload(k - 1);
        T pt = pj;
        if (iterate) {
#pragma unroll
          for (int i = 0; i < NX; ++i) pt += Pc[i] * gpk[i];
        }
        L.hv[j] = pt;
        if constexpr (sizeof(T) == 8) {
#pragma unroll
          for (int i = 0; i < NX; ++i) L.X[j * NX + i] = col[i];
        }
        wave_lds_sync();
        T hj = T(0);
#pragma unroll
        for (int l = 0; l < NX; ++l) hj += col[l] * L.hv[l];
        T G[NZ];
        if constexpr (sizeof(T) == 4) {
          float y[16], g[16];
          to_columns(outer12(Pc, col), y);
          to_columns(outer12(col, y), g);
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
        if (BOX && act && valid && j >= NX) {   // unmasked input rows: the forward's multipliers
          T* gh = soa(a.GH, k, GH_REC, nb, c) + ju * SS;
#pragma unroll
          for (int i = 0; i < NZ; ++i) gh[i * NU * SS] = G[i];
          gh[NZ * NU * SS] = hj;
        }
#pragma unroll
        for (int m = 0; m < NU; ++m) L.Hu[j * NU + m] = G[NX + m];
        wave_lds_sync();
        L.hv[j] = hj;
        wave_lds_sync();
        T Ht[NU * NU], ht[NU], Hux_t[NU];
#pragma unroll
        for (int m = 0; m < NU; ++m) {
#pragma unroll
          for (int n = 0; n < NU; ++n) Ht[m * NU + n] = L.Hu[(NX + n) * NU + m];
          ht[m] = L.hv[NX + m];
          Hux_t[m] = G[NX + m];
        }
        if constexpr (BOX) {
          // fixed components: du_m = delta_m (bound - ubar), row/column m of H_uu -> identity
          const T* ub = ubk;
          bool fixed[NU];
          T delta[NU];
#pragma unroll
          for (int m = 0; m < NU; ++m) {
            const bool lo = (low[m] >> k) & 1ull, hi = (up[m] >> k) & 1ull;
            fixed[m] = lo || hi;
            delta[m] = lo ? (W.lbu[m] - ub[m]) : (hi ? (W.ubu[m] - ub[m]) : T(0));
          }
          T hn[NU];
#pragma unroll
          for (int m = 0; m < NU; ++m) {
            T acc = ht[m];
#pragma unroll
            for (int n = 0; n < NU; ++n) acc += fixed[n] ? Ht[m * NU + n] * delta[n] : T(0);
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
        T Pn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          T acc = G[i];
#pragma unroll
          for (int m = 0; m < NU; ++m) acc += L.Hu[i * NU + m] * Kj[m];
          Pn[i] = acc;
        }
        if (act && valid) {
          T* kr = soa(a.KR, k, KR_REC, nb, c);
          if (j < NX) {
#pragma unroll
            for (int m = 0; m < NU; ++m) kr[(4 * j + m) * SS] = Kj[m];
          } else {
            kr[(4 * NX + ju) * SS] = sel<NU>(kff, ju);
          }
        }
        wave_lds_sync();
        if (act && j < NX) {   // symmetric by construction (see riccati_body)
#pragma unroll
          for (int i = 0; i < NX; ++i) {
            if (i <= j) L.P[j * NX + i] = Pn[i];
            if (i < j) L.P[i * NX + j] = Pn[i];
          }
        }
        if (act) pj = pn;
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < NX; ++i) Pc[i] = (j < NX) ? L.P[jx * NX + i] : T(0);
        if (MPCB_BOX_RESTART && BOX && act && valid && j < NX && k > 0) {   // snapshot P_k, p_k for a later restart
          T* ps = soa(a.PS, k, PS_REC, nb, c) + j * SS;
#pragma unroll
          for (int i = 0; i < NX; ++i) ps[i * NX * SS] = Pc[i];
          ps[NX * NX * SS] = pj;
        }
      }
      if (!qp_ok) st = MPCB_STATUS_QP_FAIL;
    }

    BSTAMP(5);
    // ------------------------------------------------ forward pass, multipliers, violations
    uint64_t vlo = 0, vhi = 0, vfl = 0, vfu = 0;   // input lanes: violation sets of component ju
    const bool write = valid && !done;
    T dxj = T(0);   // state lanes: component jx of dx_k
    if (iterate && j < NX) dxj = a.x0[b * a.x0_sb + jx] - soa(a.XU, 0, XU_REC, nb, c)[jx * SS];
    // prefetched DEPTH stages ahead (two register sets, slots fixed by unrolling by two; one
    // stage in the register-heavy active-set kernel): own ybar component; input lanes: row ju of
    // the gains (K | k) and of the stage Hessian (+ h_u); state lanes: row jx of [A|B], the gap
    constexpr int DEPTH = BOX ? MPCB_BOX_FWD_DEPTH : 2;
    T fyb[2], fa[2][NZ + 1], fb[2][NX + 1];
    auto fload = [&](int k, auto sl_tag) {
      constexpr int sl = decltype(sl_tag)::value;
      fyb[sl] = soa(a.XU, k, XU_REC, nb, c)[j * SS];
      if (j >= NX) {
        if constexpr (BOX) {
          const T* gh = soa(a.GH, k, GH_REC, nb, c) + ju * SS;
#pragma unroll
          for (int i = 0; i <= NZ; ++i) fa[sl][i] = gh[i * NU * SS];
        }
        const T* kr = soa(a.KR, k, KR_REC, nb, c);
#pragma unroll
        for (int i = 0; i < NX; ++i) fb[sl][i] = kr[(4 * i + ju) * SS];
        fb[sl][NX] = kr[(4 * NX + ju) * SS];
      } else {
        const T* ab = soa(a.ABT, k, AB_REC, nb, c) + jx * SS;
#pragma unroll
        for (int t = 0; t < NVAR; ++t) fa[sl][t] = ab[t * NX * SS];
        fa[sl][NZ] = iterate ? soa(a.GP, k, GP_REC, nb, c)[jx * SS] : T(0);
      }
    };
    auto stage = [&](int k, auto sl_tag) {
      constexpr int sl = decltype(sl_tag)::value;
      BSTAMP(0);
      T ra[NZ + 1], rb[NX + 1];
#pragma unroll
      for (int i = 0; i <= NZ; ++i) ra[i] = fa[sl][i];
#pragma unroll
      for (int i = 0; i <= NX; ++i) rb[i] = fb[sl][i];
      const T yb = fyb[sl];
      if (k + DEPTH < N) fload(k + DEPTH, sl_tag);
      BSTAMP(1);
      L.v[j] = dxj;   // input lanes overwrite their slot with du below
      wave_lds_sync();
      const bool lo = (sel<NU>(low, ju) >> k) & 1ull, hi = (sel<NU>(up, ju) >> k) & 1ull;
      if (j >= NX) {
        // four partial sums: the stage's serial chain is these dot products, not their flops
        T d4[4] = {rb[NX], T(0), T(0), T(0)};
#pragma unroll
        for (int i = 0; i < NX; ++i) d4[i & 3] += rb[i] * L.v[i];
        const T du = (d4[0] + d4[1]) + (d4[2] + d4[3]);
        // fixed components: the masked recursion set kff = delta and a zero gain row
        dxj = du;
      }
      wave_lds_sync();
      BSTAMP(2);
      if (j >= NX) L.v[j] = dxj;
      wave_lds_sync();
      T z[NZ];
#pragma unroll
      for (int i = 0; i < NZ; ++i) z[i] = L.v[i];
      BSTAMP(3);
      if (j >= NX) {
        const T du = dxj;
        const T uk = yb + du;
        if (write && a.U) a.U[(b * N + k) * NU + ju] = uk;
        if (write && k == 0) a.u0[b * NU + ju] = uk;
        if constexpr (BOX) {
        T mu = ra[NZ], mabs = fabs(ra[NZ]);
#pragma unroll
        for (int i = 0; i < NZ; ++i) {
          mu += ra[i] * z[i];
          mabs += fabs(ra[i] * z[i]);
        }
        // violations beyond the rounding noise of u and mu: in fp32 a degenerate component
        // (at its bound with mu ~ 0) would otherwise flip sides from one pass to the next
        const T tol_mu = T(64) * eps * mabs;
        const bool fr = !(lo || hi);
        vlo |= (uint64_t)(fr && uk < lbm - tol_u) << k;
        vhi |= (uint64_t)(fr && uk > ubm + tol_u) << k;
        vfl |= (uint64_t)(lo && mu < -tol_mu) << k;
        vfu |= (uint64_t)(hi && mu > tol_mu) << k;
        }
      } else {
        if (write && a.X) a.X[(b * (N + 1) + k) * NX + jx] = yb + dxj;
        // constant columns: position (identity) and velocity (identity + h into position)
        const T zc = (jx < 3) ? L.v[jx] + a.h * L.v[jx + 6] : ((jx >= 6 && jx < 9) ? L.v[jx] : T(0));
        T a4[4] = {ra[NZ], zc, T(0), T(0)};
#pragma unroll
        for (int t = 0; t < NVAR; ++t) a4[(t + 2) & 3] += ra[t] * z[var_col(t)];
        dxj = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      }
      wave_lds_sync();
      BSTAMP(4);
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    fload(0, S0());
    if (DEPTH == 2 && N > 1) fload(1, S1());
    for (int k = 0; k < N; k += DEPTH) {
      stage(k, S0());
      if (DEPTH == 2 && k + 1 < N) stage(k + 1, S1());
    }
    if (write && a.X && j < NX) a.X[(b * (N + 1) + N) * NX + jx] = soa(a.XU, N, XU_REC, nb, c)[jx * SS] + dxj;
    BSTAMP(6);

    if constexpr (!BOX) break;
    // ------------------------------------------------ active-set update (Kim-Park)
    const uint64_t V = vlo | vhi | vfl | vfu;
    const int cnt = (j >= NX) ? __popcll(V) : 0;
    const int firstk = (j >= NX && V) ? __ffsll((long long)V) - 1 : 64;
    int nV = 0, first = 64 * NU;
#pragma unroll
    for (int m = 0; m < NU; ++m) {
      nV += __shfl(cnt, q * 16 + NX + m);
      const int fm = __shfl(firstk, q * 16 + NX + m) * NU + m;
      first = fm < first ? fm : first;
    }
    const bool gconv = nV == 0;
    const bool full = (nV < best) || (pcount > 0);
    pcount = (nV < best) ? 3 : (full ? pcount - 1 : pcount);
    best = nV < best ? nV : best;
    const uint64_t selm =
        full ? V : ((first < 64 * NU && (first % NU) == ju && j >= NX) ? (1ull << (first / NU)) : 0ull);
    const uint64_t nlow = (sel<NU>(low, ju) | (selm & vlo)) & ~(selm & vfl);
    const uint64_t nup = (sel<NU>(up, ju) | (selm & vhi)) & ~(selm & vfu);
    uint64_t changed = 0;
#pragma unroll
    for (int m = 0; m < NU; ++m) {
      const int src = q * 16 + NX + m;
      const uint64_t nl = __shfl(nlow, src);
      const uint64_t nu_ = __shfl(nup, src);
      if (!done && !gconv) {
        changed |= (nl ^ low[m]) | (nu_ ^ up[m]);
        low[m] = nl;
        up[m] = nu_;
      }
    }
    // (the first masked pass is complete: P2 stored no snapshots)
    kc = changed ? ((it == 0 || !MPCB_BOX_RESTART) ? N - 1 : 63 - __clzll(changed)) : -1;
    if (!done && gconv) done = true;
    if (__all(done || !valid)) break;
    if (it + 1 >= a.max_as_iter) {
      if (!done) st = (st == MPCB_STATUS_OK) ? MPCB_STATUS_MAXITER : st;
      break;
    }
  }
#ifdef MPCB_STAMPS
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int i_ = 0; i_ < 12; ++i_) g_bstamps[i_] = bst_acc[i_];
#endif
  if (valid && j == NX) {
    T u0c[NU];
    load_vec<NU>(a.u0 + b * NU, u0c);
    bool fin = true;
#pragma unroll
    for (int m = 0; m < NU; ++m) fin = fin && isfin(u0c[m]);
    // the QP status of the unconstrained pass (P2 wrote it) carries over
    const int32_t st0 = MODE != PASS_SMALL ? a.status[b] : MPCB_STATUS_OK;
    a.status[b] = !fin ? MPCB_STATUS_NAN : (st0 != MPCB_STATUS_OK ? st0 : st);
    if (BOX && a.qp_stats) {
      a.qp_stats[2 * b] = n_fwd;
      a.qp_stats[2 * b + 1] = n_bst;
    }
  }
}

// fp32 register budget: MPCB_BOX_WAVES waves per SIMD (latency-bound: the iterations of one
// wave are serial, so co-resident waves are what hides the barrier / LDS / MFMA latencies)
template <int MODE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MPCB_BOX_WAVES, 8)))
box_kernel_f32(SplitArgs<float> a) { box_body<float, MODE>(a); }
template <int MODE>
__global__ void __launch_bounds__(64) box_kernel_f64(SplitArgs<double> a) { box_body<double, MODE>(a); }

// ---- small unconstrained batches -------------------------------------------------------------
// The Riccati pass of the split path integrates 16 RK4 tangents per stage inside its serial
// backward recursion; at a few thousand instances (c2: 4096, one wavefront per SIMD) that
// recursion is latency-bound.  Here the tangents move to a fully parallel kernel over
// (instance quad, stage) that caches [A_k | B_k] (AB and ABT orders), and the serial passes run
// the Riccati algebra only (box_body<T, false>).
template <class T>
__global__ void __launch_bounds__(64) lin_kernel(SplitArgs<T> a) {
  __shared__ T cc[CCS_REC * SS];
  const int lane = threadIdx.x;
  const int q = lane >> 4;
  const int j = lane & 15;
  const int k = blockIdx.y;
  const int64_t nb = a.nb;
  const int64_t q0 = blockIdx.x;                 // instance quad
  const int64_t nq = (nb + SS - 1) / SS;
  if (q0 >= nq) return;
  // the quad's stage-k capture is contiguous: 80 x 4 elements
  const T* src = soa(a.CC, k, CCS_REC, nb, q0 * SS);
  for (int e = lane; e < CCS_REC * SS; e += 64) cc[e] = src[e];
  __syncthreads();
  T dx[NX], du[NU], col[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) dx[i] = (j == i) ? T(1) : T(0);
#pragma unroll
  for (int m = 0; m < NU; ++m) du[m] = (j == NX + m) ? T(1) : T(0);
  rk4_tan_g<T, false>([&](int i) { return cc[i * SS + q]; }, dx, du, a.h, a.M, col);
  const int64_t c = q0 * SS + q;
  const int tv = var_index(j);
  if (tv >= 0) {
    T* ab = soa(a.AB, k, AB_REC, nb, c);
    T* abt = soa(a.ABT, k, AB_REC, nb, c);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      ab[(i * NVAR + tv) * SS] = col[i];
      abt[(tv * NX + i) * SS] = col[i];
    }
  }
}

template <class T> hipError_t launch_small(const SplitArgs<T>& a, hipStream_t st) {
  const unsigned g = (unsigned)((a.nb + GROUPS - 1) / GROUPS);
  MPCB_LAUNCH(PH_LIN, (lin_kernel<T>), dim3(g, a.N), dim3(64), 0, st, a);
  if constexpr (sizeof(T) == 4)
    MPCB_LAUNCH(PH_RICCATI, (box_kernel_f32<PASS_SMALL>), dim3(g), dim3(64), 0, st, a);
  else
    MPCB_LAUNCH(PH_RICCATI, (box_kernel_f64<PASS_SMALL>), dim3(g), dim3(64), 0, st, a);
  return dry_run() ? hipSuccess : hipGetLastError();
}

template hipError_t launch_small<double>(const SplitArgs<double>&, hipStream_t);
template hipError_t launch_small<float>(const SplitArgs<float>&, hipStream_t);

}  // namespace mpcb

#ifdef MPCB_STAMPS
extern "C" int mpcb_debug_stamps_box(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::g_bstamps), sizeof(unsigned long long) * 12) == hipSuccess ? 0 : -2;
}
#endif
