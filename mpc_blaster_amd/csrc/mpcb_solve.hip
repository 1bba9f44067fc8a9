// mpcb_solve.hip — fused batched SQP_RTI step for the BLASTER MPC (gfx950 / MI355X).
//
// Replaces, per instance, one acados ``ocp_solver.solve()`` (src/scripts/simulation_blaster.py:80)
// of the OCP built by blastermodel.py:214-292: ERK4 + forward sensitivities (sim_erk), the
// Gauss-Newton LINEAR_LS QP, the Riccati-structured QP solve (HPIPM's role), full step.
//
// Layout: one wavefront = GROUPS (4) independent instances; an instance owns a 16-lane group and
// lane j of the group owns DIRECTION j of the 16-dim (x, u) space (j < 12: state, j >= 12: input).
//  * Pass 1 (forward): nominal RK4 rollout (or copy of the given iterate); every lane of the group
//    computes the same trajectory, lane j stores component j to the slot workspace.
//  * Pass 2 (backward Riccati): at stage k lane j integrates RK4 with a forward tangent seeded
//    by e_j -> column j of [A_k | B_k] lands in lane j without forming any Jacobian.  The value
//    function P (12x12) and the stage Hessian columns are exchanged through LDS; lane j builds
//    column j of G = [A|B]^T P [A|B], the 4x4 input block is factorised (Cholesky) redundantly
//    in every lane, lane j < 12 produces column j of the gain K and of the next P.  Gains go to
//    the workspace.
//  * Pass 3 (forward): dx_{k+1} = JVP of RK4 along (dx_k, du_k) (+ gap), du_k = K_k dx_k + kff_k;
//    writes X = xbar + dx, U = ubar + du.  With input boxes, pass 3 also evaluates the multipliers
//    and the primal-dual active-set update; passes 2-3 repeat until the active set repeats.
//
// HBM traffic per instance is compulsory I/O (x0, refs, u0, X, U) plus the workspace, which is
// indexed by launch slot (not by instance), so its footprint stays bounded by the resident grid.
#include <hip/hip_runtime.h>

#include "../../include/mpcb.h"
#include "mpcb_common.h"

#ifndef MPCB_WAVES
#define MPCB_WAVES
#endif

namespace mpcb {

template <class T, int BOX>
__global__ void __launch_bounds__(64) MPCB_WAVES solve_kernel(SolveArgs<T> a) {
  __shared__ GroupLds<T> lds_all[GROUPS];
  const int lane = threadIdx.x;
  const int q = lane >> 4;
  const int j = lane & 15;
  const int jx = j < NX ? j : 0;       // clamped state index
  const int ju = j >= NX ? j - NX : 0; // clamped input index
  GroupLds<T>& L = lds_all[q];
  const int N = a.N;
  constexpr int RN = Rec<BOX>::n;
  const T s = a.s;
  const Weights<T>& W = *a.W;
  const bool iterate = a.mode == MPCB_MODE_ITERATE;
  T* slot = a.scratch + (int64_t)blockIdx.x * a.slot_elems;
  T* XU = slot;                                        // [(N+1)][64]       xbar | ubar
  T* CC = XU + (int64_t)(N + 1) * 64;                  // [N][GROUPS][CC_REC] lin. scalars | gap
  T* KR = CC + (int64_t)N * GROUPS * CC_REC;           // [N][64][RN]       gains (+box extras)

  for (int64_t wave = blockIdx.x; wave * GROUPS < a.B; wave += gridDim.x) {
    const int64_t b_raw = wave * GROUPS + q;
    const bool valid = b_raw < a.B;
    const int64_t b = valid ? b_raw : a.B - 1;   // inactive groups recompute the last instance
    T w[3] = {T(0), T(0), T(0)};
    if (a.wind) {
      w[0] = a.wind[b * a.wind_sb + 0];
      w[1] = a.wind[b * a.wind_sb + 1];
      w[2] = a.wind[b * a.wind_sb + 2];
    }
    const T* xr = a.xref + b * a.xref_sb;
    const T* ur = a.uref + b * a.uref_sb;
    const T* x0p = a.x0 + b * a.x0_sb;

    // ------------------------------------------------------------------ pass 1: nominal
    // Every lane of the group integrates the same nominal trajectory; lane 0 of the group
    // publishes xbar/ubar (XU), the 80 captured linearisation scalars per interval and the gap
    // (CC).  ROLLOUT: xbar = RK4 rollout of u_ref from x0 (gap 0).  ITERATE: the given iterate.
    {
      const T* xbp = a.xbar + b * (int64_t)(N + 1) * NX;
      const T* ubp = a.ubar + b * (int64_t)N * NU;
      T xb[NX], ub[NU];
      load_vec<NX>(iterate ? xbp : x0p, xb);
      for (int k = 0; k < N; ++k) {
        if (iterate) load_vec<NX>(xbp + (int64_t)k * NX, xb);
        load_vec<NU>(iterate ? ubp + (int64_t)k * NU : ur + (int64_t)k * NU, ub);
        T* cc = CC + ((int64_t)k * GROUPS + q) * CC_REC;
        if (j == 0) {
          store_vec<NX>(XU + (int64_t)k * 64 + q * 16, xb);
          store_vec<NU>(XU + (int64_t)k * 64 + q * 16 + NX, ub);
        }
        T xn[NX];
        rk4_nom<T>(xb, ub, a.h, a.M, w, xn, [&](int stage, const T* c) {
          if (j == 0) store_vec<LIN_N>(cc + stage * LIN_N, c);
        });
        if (iterate) {
          T gp[NX];
          const T* nx = xbp + (int64_t)(k + 1) * NX;
#pragma unroll
          for (int i = 0; i < NX; ++i) gp[i] = xn[i] - nx[i];
          if (j == 0) store_vec<NX>(cc + LIN_STAGE, gp);
        } else {
#pragma unroll
          for (int i = 0; i < NX; ++i) xb[i] = xn[i];
        }
      }
      if (iterate) load_vec<NX>(xbp + (int64_t)N * NX, xb);
      if (j == 0) {
        store_vec<NX>(XU + (int64_t)N * 64 + q * 16, xb);
#pragma unroll
        for (int m = 0; m < NU; ++m) XU[(int64_t)N * 64 + q * 16 + NX + m] = T(0);
      }
    }
    __syncthreads();

    uint64_t low[NU], up[NU];
#pragma unroll
    for (int m = 0; m < NU; ++m) { low[m] = 0; up[m] = 0; }
    bool done = false;
    int32_t st = MPCB_STATUS_OK;
    int best = 0x7fffffff, pcount = 3;   // Kim-Park safeguard state (uniform per group)

    for (int it = 0;; ++it) {
      // ------------------------------------------------------------------ pass 2: Riccati
      T pj;       // p_{k+1}[j]
      {
        const T xN = XU[(int64_t)N * 64 + q * 16 + jx];
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
        __syncthreads();
      }
      T kff_out[NU];
      bool qp_ok = true;
      for (int k = N - 1; k >= 0; --k) {
        T col[NX];
        {
          const T* cc = CC + ((int64_t)k * GROUPS + q) * CC_REC;
          // e = ybar - yref (component j), exchanged through LDS for block-diagonal W
          const T ybar = XU[(int64_t)k * 64 + lane];
          L.v[j] = ybar - ((j < NX) ? xr[(int64_t)k * NX + jx] : ur[(int64_t)k * NU + ju]);
          // tangent RK4 seeded with e_j: column j of [A|B]
          T dx[NX], du[NU];
#pragma unroll
          for (int i = 0; i < NX; ++i) dx[i] = (j == i) ? T(1) : T(0);
#pragma unroll
          for (int m = 0; m < NU; ++m) du[m] = (j == NX + m) ? T(1) : T(0);
          rk4_tan<T>(cc, dx, du, a.h, a.M, col);
          // gap b = Phi(xbar_k, ubar_k) - xbar_{k+1};  pt = p + P b  (P symmetric: row j = col j)
          T pt = pj;
          if (iterate) {
#pragma unroll
            for (int i = 0; i < NX; ++i) pt += L.P[jx * NX + i] * cc[LIN_STAGE + i];
          }
          L.hv[j] = pt;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) L.X[j * NX + i] = col[i];
        __syncthreads();
        // h_j = col_j . pt
        T hj = T(0);
#pragma unroll
        for (int l = 0; l < NX; ++l) hj += col[l] * L.hv[l];
        // y = P col_j
        T y[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) y[i] = T(0);
#pragma unroll
        for (int l = 0; l < NX; ++l) {
          const T cl = col[l];
#pragma unroll
          for (int i = 0; i < NX; ++i) y[i] += L.P[l * NX + i] * cl;
        }
        // G[:, j] = [A|B]^T y  + s * blkdiag(Q, R)[:, j]
        T G[NZ];
#pragma unroll
        for (int i = 0; i < NZ; ++i) {
          T acc = T(0);
#pragma unroll
          for (int l = 0; l < NX; ++l) acc += L.X[i * NX + l] * y[l];
          G[i] = acc;
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
        __syncthreads();   // all reads of L.v / L.hv / L.X done; Hu visible
        L.hv[j] = hj;
        __syncthreads();
        T Ht[NU * NU], ht[NU], Hux_t[NU];
#pragma unroll
        for (int m = 0; m < NU; ++m) {
#pragma unroll
          for (int n = 0; n < NU; ++n) Ht[m * NU + n] = L.Hu[(NX + n) * NU + m];
          ht[m] = L.hv[NX + m];
          Hux_t[m] = G[NX + m];
        }
        // ---- input-box masking (fixed components: du_m = delta_m)
        if constexpr (BOX) {
          T ub[NU];
          load_vec<NU>(XU + (int64_t)k * 64 + q * 16 + NX, ub);
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
        qp_ok = qp_ok && ok;
        T kff[NU], Kj[NU], nh[NU];
#pragma unroll
        for (int m = 0; m < NU; ++m) nh[m] = -ht[m];
        chol4_solve(Lc, nh, kff);
#pragma unroll
        for (int m = 0; m < NU; ++m) nh[m] = -Hux_t[m];
        chol4_solve(Lc, nh, Kj);
        // p_new = h_x + H_ux^T kff (unmasked H_ux);  P_new col j = G[0:12] + H_ux^T K[:, j]
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
        // ---- store gains (and box extras)
        T* rec = KR + ((int64_t)k * 64 + lane) * RN;
        if (j < NX) {
#pragma unroll
          for (int m = 0; m < NU; ++m) rec[m] = Kj[m];
        } else {
          rec[0] = sel<NU>(kff, ju);
          if constexpr (BOX) {
            // row NX+m of the stage Hessian (== this lane's column by symmetry) and h_u[m]
#pragma unroll
            for (int i = 0; i < NZ; ++i) rec[4 + i] = G[i];
            rec[4 + NZ] = hj;
          }
        }
#pragma unroll
        for (int m = 0; m < NU; ++m) kff_out[m] = kff[m];
        __syncthreads();   // everyone finished reading L.P / L.Hu
        // Store P_{k} symmetric by construction: entry (r, c) comes from lane max(r, c).  The
        // plain column-wise update drifts antisymmetric and that drift is amplified stage to
        // stage (fp32 u0 error 2e-1 -> 2e-6 with this, fp64 1e-7 -> 1e-15).
        if (j < NX) {
#pragma unroll
          for (int i = 0; i < NX; ++i) {
            if (i <= j) L.P[j * NX + i] = Pn[i];
            if (i < j) L.P[i * NX + j] = Pn[i];
          }
        }
        pj = pn;
        __syncthreads();
      }
      if (!qp_ok) st = MPCB_STATUS_QP_FAIL;

      // ------------------------------------------------------------------ pass 3: forward
      const bool need_fwd = BOX || a.X != nullptr || a.U != nullptr || iterate;
      // lanes NX+m: infeasibility sets of component m (bit k = stage k)
      uint64_t vlo = 0, vhi = 0, vfl = 0, vfu = 0;
      T u0v[NU];
      if (need_fwd) {
        T dxk[NX];
        {
          const T* p = XU + q * 16;
#pragma unroll
          for (int i = 0; i < NX; ++i) dxk[i] = iterate ? x0p[i] - p[i] : T(0);
        }
        const bool write = valid && !done;
        for (int k = 0; k < N; ++k) {
          T duk[NU];
#pragma unroll
          for (int m = 0; m < NU; ++m) duk[m] = KR[((int64_t)k * 64 + q * 16 + NX + m) * RN];
#pragma unroll
          for (int l = 0; l < NX; ++l) {
            const T* r = KR + ((int64_t)k * 64 + q * 16 + l) * RN;
#pragma unroll
            for (int m = 0; m < NU; ++m) duk[m] += r[m] * dxk[l];
          }
          T ub[NU];
          load_vec<NU>(XU + (int64_t)k * 64 + q * 16 + NX, ub);
          if (k == 0) {
#pragma unroll
            for (int m = 0; m < NU; ++m) u0v[m] = ub[m] + duk[m];
          }
          if constexpr (BOX) {
            if (j >= NX) {
              const int m = ju;
              const T* r = KR + ((int64_t)k * 64 + lane) * RN;
              const bool lo = (sel<NU>(low, m) >> k) & 1ull, hi = (sel<NU>(up, m) >> k) & 1ull;
              T mu = r[4 + NZ];
#pragma unroll
              for (int i = 0; i < NX; ++i) mu += r[4 + i] * dxk[i];
#pragma unroll
              for (int n = 0; n < NU; ++n) mu += r[4 + NX + n] * duk[n];
              const T uk = sel<NU>(ub, m) + sel<NU>(duk, m);
              const bool fr = !(lo || hi);
              vlo |= (uint64_t)(fr && uk < W.lbu[m]) << k;
              vhi |= (uint64_t)(fr && uk > W.ubu[m]) << k;
              vfl |= (uint64_t)(lo && mu < T(0)) << k;
              vfu |= (uint64_t)(hi && mu > T(0)) << k;
            }
          }
          if (write) {
            const T ybar = XU[(int64_t)k * 64 + lane];
            if (a.X && j < NX) a.X[(b * (N + 1) + k) * NX + j] = ybar + sel<NX>(dxk, j);
            if (a.U && j >= NX) a.U[(b * N + k) * NU + ju] = ybar + sel<NU>(duk, ju);
          }
          const T* cc = CC + ((int64_t)k * GROUPS + q) * CC_REC;
          T dphi[NX];
          rk4_tan<T>(cc, dxk, duk, a.h, a.M, dphi);
          if (iterate) {
#pragma unroll
            for (int i = 0; i < NX; ++i) dxk[i] = dphi[i] + cc[LIN_STAGE + i];
          } else {
#pragma unroll
            for (int i = 0; i < NX; ++i) dxk[i] = dphi[i];
          }
        }
        if (write && a.X && j < NX) {
          const T xN = XU[(int64_t)N * 64 + q * 16 + jx];
          a.X[(b * (N + 1) + N) * NX + j] = xN + sel<NX>(dxk, j);
        }
      } else {
        T ub[NU];
        load_vec<NU>(XU + q * 16 + NX, ub);
#pragma unroll
        for (int m = 0; m < NU; ++m) u0v[m] = ub[m] + kff_out[m];
      }
      if (valid && !done && j >= NX) a.u0[b * NU + ju] = sel<NU>(u0v, ju);

      if constexpr (!BOX) {
        break;
      } else {
        // active-set update (Kim-Park block principal pivoting, mirrors oracle.ocp.pdas_solve):
        // V = {free u<lb} U {free u>ub} U {at lb, mu<0} U {at ub, mu>0}; |V| = 0 <=> KKT.
        const uint64_t V = vlo | vhi | vfl | vfu;
        int cnt = (j >= NX) ? __popcll(V) : 0;
        int firstk = (j >= NX && V) ? __ffsll((long long)V) - 1 : 64;
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
        uint64_t selm = full ? V : ((first < 64 * NU && (first % NU) == ju && j >= NX) ? (1ull << (first / NU)) : 0ull);
        const uint64_t nlow = (sel<NU>(low, ju) | (selm & vlo)) & ~(selm & vfl);
        const uint64_t nup = (sel<NU>(up, ju) | (selm & vhi)) & ~(selm & vfu);
        const bool gchanged = !gconv;
#pragma unroll
        for (int m = 0; m < NU; ++m) {
          const int src = q * 16 + NX + m;
          const uint64_t nl = __shfl(nlow, src);
          const uint64_t nu_ = __shfl(nup, src);
          if (!done && !gconv) { low[m] = nl; up[m] = nu_; }
        }
        if (!done && !gchanged) done = true;
        const bool all_done = __all(done || !valid);
        if (all_done) break;
        if (it + 1 >= a.max_as_iter) {
          if (!done) st = (st == MPCB_STATUS_OK) ? MPCB_STATUS_MAXITER : st;
          break;
        }
      }
    }
    __syncthreads();
    // status: acados-style codes; NaN guard on u0
    if (valid && j == NX) {
      T u0c[NU];
      load_vec<NU>(a.u0 + b * NU, u0c);
      bool fin = true;
#pragma unroll
      for (int m = 0; m < NU; ++m) fin = fin && isfin(u0c[m]);
      a.status[b] = fin ? st : MPCB_STATUS_NAN;
    }
    __syncthreads();
  }
}

template <class T> int64_t solve_slot_elems(int N, int box) {
  const int RN = box ? Rec<1>::n : Rec<0>::n;
  return (int64_t)(N + 1) * 64 + (int64_t)N * GROUPS * CC_REC + (int64_t)N * 64 * RN;
}

template <class T> hipError_t launch_solve(const SolveArgs<T>& a, int grid, hipStream_t st) {
  if (a.box)
    MPCB_LAUNCH(PH_RICCATI, (solve_kernel<T, 1>), dim3(grid), dim3(64), 0, st, a);
  else
    MPCB_LAUNCH(PH_RICCATI, (solve_kernel<T, 0>), dim3(grid), dim3(64), 0, st, a);
  return dry_run() ? hipSuccess : hipGetLastError();
}

template hipError_t launch_solve<double>(const SolveArgs<double>&, int, hipStream_t);
template hipError_t launch_solve<float>(const SolveArgs<float>&, int, hipStream_t);
template int64_t solve_slot_elems<double>(int, int);
template int64_t solve_slot_elems<float>(int, int);

}  // namespace mpcb
