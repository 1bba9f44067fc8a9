// mpcb_full.hip — one SQP_RTI step of the reference's full 17-state / 6-input OCP
// (blastermodel.py:70-292, acados_ocp_blasterModel.json: N = 60, Tf = 2,
// W = diag(Q17, R6), W_e = 10 Q17, 25 parameters).
//
// Three launches per chunk:
//   nominal17q 16 lanes per instance (lanes 0-4 evaluate the five sin/cos of each f17 and
//              broadcast them by DPP): the RK4 rollout of u_ref from x0 (or a copy of the
//              persistent iterate) into the workspace;
//   lin17ws    stage-parallel linearisation, 16 lanes per (instance, stage): lanes 0..13
//              integrate the RK4 tangents seeded with e_j of the 14 dense directions, so column j of
//              [A_k | B_k] lands in a lane (what acados' forward VDE computes); lanes 14 / 15 write
//              the 9 structural columns; gaps in iterate mode (lin17_packed, also behind
//              mpcb_linearize);
//   riccati    the Riccati pass, its forward pass and the interior point of the boxes:
//              riccati17q_kernel (mpcb_r17.hip, 16 lanes per instance), ending with the forward
//              pass (du = K dx + k, dx' = [A|B] (dx, du) + gap) that writes u0, X = xbar + dx,
//              U = ubar + du, status.  (Round 1's 32-lane riccati17_kernel, behind MPCB_R17=0 until
//              round 2, is gone: it had no polish and no test, so nothing pinned it.)
// The 12/4 slice has its own MI355X-tuned kernels (mpcb_split.hip); this path carries the full
// model at the reference's own dimensions and is not on the BASELINE benchmark configs.
#include <hip/hip_runtime.h>

#include "../../include/mpcb.h"
#include "mpcb_common.h"
#include "mpcb_full.h"

namespace mpcb {


// The RK4 rollout with 16 lanes per instance (4 instances per wavefront): the serial chain's
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
  MPCB_LAUNCH(PH_NOMINAL, (nominal17q_kernel<T>), dim3((unsigned)((a.nb + 3) / 4)), dim3(64), 0, st, a);
  if (ev) (void)hipEventRecord(ev[1], st);
  MPCB_LAUNCH(PH_LIN17, (lin17ws_kernel<T>), dim3((unsigned)((a.nb * a.N + GQ17 - 1) / GQ17)), dim3(64), 0, st, a);
  if (ev) (void)hipEventRecord(ev[2], st);
  const hipError_t e = launch_riccati17q<T>(a, st);
  if (e != hipSuccess) return e;
  if (ev) (void)hipEventRecord(ev[3], st);
  return dry_run() ? hipSuccess : hipGetLastError();
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
