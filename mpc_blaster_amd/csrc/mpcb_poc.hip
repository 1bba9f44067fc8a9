// mpcb_poc.hip — batched point-of-contact (POC) Jacobians of the blaster stream.
//
// Restates Jacobian_POC_Solver.solveJacobians (src/scripts/Jacobian_POC_Solver.py:222-296) for
// B independent vehicle poses at once.  Per pose: the stream leaves the nozzle at
// p0 = (T_w_b T_b_s2)[:3, 3] with v0 = (T_w_b T_b_s2)[:3, :3] (0, 0, -V) (htm.py:7-36,
// :153-163); p_dot = v, v_dot = -M_c v + g is integrated by RK4 with 10 steps (:62-92); the
// ground-hit time solves z(T) = 0 by Newton with a forward-difference slope (dT = 1e-5, from
// T = 0.1, until |z| <= 1e-3, negative iterates reflected; :116-151); POC = p(T); the Jacobians
// are forward differences (eps = 1e-6) w.r.t. the Euler angles, the nozzle angles and the
// position, one root solve per perturbation.
//
// Layout: one 16-lane row per pose (4 poses per wavefront).  Lane 0 solves the nominal pose,
// lanes 1..8 the eight perturbed ones (Euler 3, nozzle 2, position 3), lanes 9..15 shadow lane 0;
// the nominal POC reaches the perturbed lanes by DPP row broadcast.  The Newton iteration counts
// differ per lane (divergence is bounded by max_iter).  fp64: the forward differences amplify
// rounding by 1/eps = 1e6.
#include <hip/hip_runtime.h>

#include "../../include/mpcb.h"
#include "mpcb_kernels.h"

namespace mpcb {

struct PocArgs {
  int64_t B;
  const double* pose;   // [B, 8]: phi, theta, psi, alpha1, alpha2, x, y, z
  double V;             // stream velocity
  double Mc[9];         // drag matrix (row-major; a scalar M_c is M_c I)
  int max_iter;
  double t_blast;
  double* poc;          // [B, 3]
  double* J_eul;        // [B, 3, 3]
  double* J_mot;        // [B, 3, 2]
  double* J_pos;        // [B, 3, 3]
  double* p25;          // [B, 25] or nullptr
  int32_t* status;      // [B]
};

constexpr double POC_EPS = 1e-6, POC_DT = 1e-5, POC_TOL = 1e-3, POC_T0 = 0.1;
constexpr int POC_STEPS = 10;

__device__ __forceinline__ void poc_f(const double* s, const double* Mc, double* d) {
  d[0] = s[3];
  d[1] = s[4];
  d[2] = s[5];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    d[3 + i] = -(Mc[i * 3] * s[3] + Mc[i * 3 + 1] * s[4] + Mc[i * 3 + 2] * s[5]) + (i == 2 ? -9.81 : 0.0);
}

// ERK4, 10 equal steps over [0, T]
__device__ __forceinline__ void poc_integrate(const double* x0, double T, const double* Mc, double* x) {
  const double h = T / POC_STEPS;
#pragma unroll
  for (int i = 0; i < 6; ++i) x[i] = x0[i];
  for (int st = 0; st < POC_STEPS; ++st) {
    double k1[6], k2[6], k3[6], k4[6], s[6];
    poc_f(x, Mc, k1);
#pragma unroll
    for (int i = 0; i < 6; ++i) s[i] = x[i] + 0.5 * h * k1[i];
    poc_f(s, Mc, k2);
#pragma unroll
    for (int i = 0; i < 6; ++i) s[i] = x[i] + 0.5 * h * k2[i];
    poc_f(s, Mc, k3);
#pragma unroll
    for (int i = 0; i < 6; ++i) s[i] = x[i] + h * k3[i];
    poc_f(s, Mc, k4);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = x[i] + (h / 6.0) * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
  }
}

__device__ __forceinline__ void mat4(const double* A, const double* B, double* C) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += A[i * 4 + k] * B[k * 4 + j];
      C[i * 4 + j] = acc;
    }
}

__device__ __forceinline__ double row_bcast0(double v) {
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150, 0xF, 0xF, false);   // row_newbcast:0
}

__global__ void __launch_bounds__(64) poc_kernel(PocArgs a) {
  const int lane = threadIdx.x;
  const int g = lane & 15;                              // 0 nominal, 1..8 perturbed
  const int64_t b_raw = (int64_t)blockIdx.x * 4 + (lane >> 4);
  const bool valid = b_raw < a.B;
  const int64_t b = valid ? b_raw : a.B - 1;
  double pose[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) pose[i] = a.pose[b * 8 + i];
  // coordinate perturbed by this lane: 1..3 Euler, 4..5 nozzle, 6..8 position
#pragma unroll
  for (int i = 0; i < 8; ++i) pose[i] = (g == i + 1) ? pose[i] + POC_EPS : pose[i];
  double x0[6];
  {
    double sf, cf, st, ct, sp, cp, s1, c1, s2, c2;
    sincos(pose[0], &sf, &cf);
    sincos(pose[1], &st, &ct);
    sincos(pose[2], &sp, &cp);
    sincos(pose[3], &s1, &c1);
    sincos(pose[4], &s2, &c2);
    // T_w_b (htm.py:30-36): Rotation.from_euler('zyx', [psi, theta, phi]) = Rx(phi) Ry(theta) Rz(psi)
    const double Tw[16] = {ct * cp, -ct * sp, st, pose[5],
                           sf * st * cp + cf * sp, -sf * st * sp + cf * cp, -sf * ct, pose[6],
                           -cf * st * cp + sf * sp, cf * st * sp + sf * cp, cf * ct, pose[7],
                           0.0, 0.0, 0.0, 1.0};
    // T_b_s2 = hbs1 @ hs1s2 @ hs2n (htm.py:7-28)
    const double h1[16] = {1, 0, 0, 0.01672, 0, 1, 0, 0, 0, 0, 1, -0.22937, 0, 0, 0, 1};
    const double h2[16] = {c1, 0, s1, 0.0425, 0, 1, 0, 0, -s1, 0, c1, 0, 0, 0, 0, 1};
    const double h3[16] = {1, 0, 0, -0.05322, 0, c2, s2, 0, 0, -s2, c2, -0.15946, 0, 0, 0, 1};
    double t12[16], tbs[16], T[16];
    mat4(h1, h2, t12);
    mat4(t12, h3, tbs);
    mat4(Tw, tbs, T);
    x0[0] = T[3];
    x0[1] = T[7];
    x0[2] = T[11];
#pragma unroll
    for (int i = 0; i < 3; ++i) x0[3 + i] = T[i * 4 + 2] * (-a.V);
  }
  // ground-hit time (Jacobian_POC_Solver.py:116-151)
  double TN = POC_T0, err = 100.0, x[6];
  int it = 0;
  while (fabs(err) > POC_TOL && it < a.max_iter) {
    poc_integrate(x0, TN, a.Mc, x);
    const double f = x[2];
    poc_integrate(x0, TN + POC_DT, a.Mc, x);
    const double fp = (x[2] - f) / POC_DT;
    double T1 = TN - f / fp;
    if (T1 < 0) T1 = -T1;
    poc_integrate(x0, T1, a.Mc, x);
    err = x[2];
    TN = T1;
    ++it;
  }
  const bool ok = fabs(err) <= POC_TOL;
  poc_integrate(x0, TN, a.Mc, x);
  const double P0[3] = {row_bcast0(x[0]), row_bcast0(x[1]), row_bcast0(x[2])};
  const uint64_t bad = __ballot(!ok);
  if (!valid) return;
  const int64_t o = b;
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) a.poc[o * 3 + i] = x[i];
    const uint64_t mine = (bad >> (lane & 48)) & 0x1FF;   // lanes 0..8 of this row
    a.status[o] = mine ? MPCB_STATUS_MAXITER : MPCB_STATUS_OK;
    if (a.p25) a.p25[o * 25 + 24] = a.t_blast;
  } else if (g <= 8) {
    double J[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) J[i] = (x[i] - P0[i]) / POC_EPS;
    // J_eul[:, g-1], J_mot[:, g-4], J_pos[:, g-6]; p25 = vec(J_mot) | vec(J_eul) | vec(J_pos) | T_blast
    if (g <= 3) {
#pragma unroll
      for (int i = 0; i < 3; ++i) a.J_eul[o * 9 + i * 3 + (g - 1)] = J[i];
      if (a.p25)
#pragma unroll
        for (int i = 0; i < 3; ++i) a.p25[o * 25 + 6 + (g - 1) * 3 + i] = J[i];
    } else if (g <= 5) {
#pragma unroll
      for (int i = 0; i < 3; ++i) a.J_mot[o * 6 + i * 2 + (g - 4)] = J[i];
      if (a.p25)
#pragma unroll
        for (int i = 0; i < 3; ++i) a.p25[o * 25 + (g - 4) * 3 + i] = J[i];
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) a.J_pos[o * 9 + i * 3 + (g - 6)] = J[i];
      if (a.p25)
#pragma unroll
        for (int i = 0; i < 3; ++i) a.p25[o * 25 + 15 + (g - 6) * 3 + i] = J[i];
    }
  }
}

hipError_t launch_poc(const PocArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(poc_kernel, dim3((unsigned)((a.B + 3) / 4)), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace mpcb

extern "C" int mpcb_poc_jacobians(int64_t B, const double* pose, double stream_velocity, const double* Mc,
                                  int max_iter, double t_blast, double* poc, double* J_eul, double* J_mot,
                                  double* J_pos, double* p25, int32_t* status, void* stream) {
  if (B < 0 || max_iter < 1 || !Mc) return -1;
  if (B == 0) return 0;
  if (!pose || !poc || !J_eul || !J_mot || !J_pos || !status) return -1;
  mpcb::PocArgs a;
  a.B = B;
  a.pose = pose;
  a.V = stream_velocity;
  for (int i = 0; i < 9; ++i) a.Mc[i] = Mc[i];
  a.max_iter = max_iter;
  a.t_blast = t_blast;
  a.poc = poc;
  a.J_eul = J_eul;
  a.J_mot = J_mot;
  a.J_pos = J_pos;
  a.p25 = p25;
  a.status = status;
  return mpcb::launch_poc(a, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}
