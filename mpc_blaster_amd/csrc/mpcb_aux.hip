// mpcb_aux.hip — linearisation (debug/parity), plant step, synthetic inputs, u0 histogram.
#include <hip/hip_runtime.h>

#include "../../include/mpcb.h"
#include "mpcb_kernels.h"

namespace mpcb {

// ------------------------------------------------------------------------ linearisation
// Same lane mapping as the solve kernel: 4 instances per wave, lane j = direction j.
template <class T>
__global__ void __launch_bounds__(64) linearize_kernel(int64_t B, int N, T h, Model<T> M,
                                                       const T* __restrict__ xbar,
                                                       const T* __restrict__ ubar,
                                                       const T* __restrict__ wind, int64_t wind_sb,
                                                       T* __restrict__ A, T* __restrict__ Bm,
                                                       T* __restrict__ xnext) {
  const int lane = threadIdx.x, q = lane >> 4, j = lane & 15;
  const int64_t b = (int64_t)blockIdx.x * GROUPS + q;
  if (b >= B) return;
  T w[3] = {T(0), T(0), T(0)};
  if (wind) { w[0] = wind[b * wind_sb]; w[1] = wind[b * wind_sb + 1]; w[2] = wind[b * wind_sb + 2]; }
  T dx[NX], du[NU];
#pragma unroll
  for (int i = 0; i < NX; ++i) dx[i] = (j == i) ? T(1) : T(0);
#pragma unroll
  for (int m = 0; m < NU; ++m) du[m] = (j == NX + m) ? T(1) : T(0);
  for (int k = 0; k < N; ++k) {
    T x[NX], u[NU], phi[NX], col[NX];
    const T* xp = xbar + (b * (N + 1) + k) * NX;
    const T* up = ubar + (b * N + k) * NU;
#pragma unroll
    for (int i = 0; i < NX; ++i) x[i] = xp[i];
#pragma unroll
    for (int m = 0; m < NU; ++m) u[m] = up[m];
    rk4<T, true>(x, dx, u, du, h, M, w, phi, col);
    const int64_t base = b * N + k;
    if (j < NX) {
#pragma unroll
      for (int i = 0; i < NX; ++i) A[(base * NX + i) * NX + j] = col[i];
      T mine = phi[0];
#pragma unroll
      for (int i = 1; i < NX; ++i) mine = (j == i) ? phi[i] : mine;
      xnext[base * NX + j] = mine;
    } else {
#pragma unroll
      for (int i = 0; i < NX; ++i) Bm[(base * NX + i) * NU + (j - NX)] = col[i];
    }
  }
}

template <class T>
hipError_t launch_linearize(int64_t B, int N, T h, const Model<T>& M, const T* xbar, const T* ubar,
                            const T* wind, int64_t wind_sb, T* A, T* Bm, T* xnext, hipStream_t st) {
  const int64_t grid = (B + GROUPS - 1) / GROUPS;
  hipLaunchKernelGGL((linearize_kernel<T>), dim3((unsigned)grid), dim3(64), 0, st, B, N, h, M, xbar,
                     ubar, wind, wind_sb, A, Bm, xnext);
  return hipGetLastError();
}

// ------------------------------------------------------------------------ plant step
template <class T>
__global__ void __launch_bounds__(256) sim_step_kernel(int64_t B, T h, Model<T> M,
                                                       const T* __restrict__ x,
                                                       const T* __restrict__ u,
                                                       const T* __restrict__ wind, int64_t wind_sb,
                                                       T* __restrict__ xo) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  T w[3] = {T(0), T(0), T(0)};
  if (wind) { w[0] = wind[b * wind_sb]; w[1] = wind[b * wind_sb + 1]; w[2] = wind[b * wind_sb + 2]; }
  T xv[NX], uv[NU], xn[NX], dd[1];
#pragma unroll
  for (int i = 0; i < NX; ++i) xv[i] = x[b * NX + i];
#pragma unroll
  for (int m = 0; m < NU; ++m) uv[m] = u[b * NU + m];
  rk4<T, false>(xv, nullptr, uv, nullptr, h, M, w, xn, dd);
#pragma unroll
  for (int i = 0; i < NX; ++i) xo[b * NX + i] = xn[i];
}

template <class T>
hipError_t launch_sim_step(int64_t B, T h, const Model<T>& M, const T* x, const T* u, const T* wind,
                           int64_t wind_sb, T* xo, hipStream_t st) {
  const int64_t grid = (B + 255) / 256;
  hipLaunchKernelGGL((sim_step_kernel<T>), dim3((unsigned)grid), dim3(256), 0, st, B, h, M, x, u,
                     wind, wind_sb, xo);
  return hipGetLastError();
}

// ------------------------------------------------------------------------ Philox inputs
// Philox4x32-10 (Salmon et al. SC'11); bit-identical to oracle/philox.py.
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    const uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

#pragma clang fp contract(off)
template <class T>
__global__ void __launch_bounds__(256) gen_inputs_kernel(int64_t B, int N, double dt, uint64_t seed,
                                                         uint64_t id_offset, int ref_kind,
                                                         T* __restrict__ x0, T* __restrict__ xref,
                                                         int64_t xref_sb, T* __restrict__ uref,
                                                         int64_t uref_sb, T* __restrict__ wind) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t id = id_offset + (uint64_t)b;
  double U[18];
#pragma unroll
  for (int d = 0; d < 9; ++d) {
    uint32_t c[4] = {(uint32_t)id, (uint32_t)(id >> 32), (uint32_t)d, 0u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    U[2 * d] = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) * 1.1102230246251565e-16;
    U[2 * d + 1] = ((double)(c[2] >> 5) * 67108864.0 + (double)(c[3] >> 6)) * 1.1102230246251565e-16;
  }
  const double half[NX] = {1.0, 1.0, 1.0, 0.17, 0.17, 0.35, 0.5, 0.5, 0.5, 0.087, 0.087, 0.087};
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const double t = 2.0 * U[i] - 1.0;
    const double hv = (i == 2) ? 3.5 : 0.0;
    x0[b * NX + i] = (T)(hv + half[i] * t);
  }
  if (wind) {
#pragma unroll
    for (int i = 0; i < 3; ++i) wind[b * 3 + i] = (T)(5.0 * (2.0 * U[12 + i] - 1.0));
  }
  if (ref_kind == 1) {
    const double amp = 0.2 + 0.8 * U[15];
    const double om = 0.5 + 1.5 * U[16];
    const double ph = 6.283185307179586 * U[17];
    T* xr = xref + b * xref_sb;
    for (int k = 0; k <= N; ++k) {
      const double t = (double)k * dt;
      const double ang = om * t + ph;
      const double wt = om * t;
      const double sa = sin(ang), ca = cos(ang), sw = sin(wt), cw = cos(wt);
      T* r = xr + (int64_t)k * NX;
      for (int i = 0; i < NX; ++i) r[i] = T(0);
      r[0] = (T)(amp * sa);
      r[1] = (T)(amp * ca);
      r[2] = (T)(3.5 + 0.2 * sw);
      r[6] = (T)(amp * om * ca);
      r[7] = (T)(-amp * om * sa);
      r[8] = (T)(0.2 * om * cw);
    }
  } else if (xref_sb != 0 || b == 0) {
    T* xr = xref + b * xref_sb;
    for (int k = 0; k <= N; ++k)
      for (int i = 0; i < NX; ++i) xr[(int64_t)k * NX + i] = (i == 2) ? T(3.5) : T(0);
  }
  if (uref_sb != 0 || b == 0) {
    T* ur = uref + b * uref_sb;
    for (int k = 0; k < N * NU; ++k) ur[k] = T(22.0725);
  }
}
#pragma clang fp contract(on)

template <class T>
hipError_t launch_gen_inputs(int64_t B, int N, T dt, uint64_t seed, uint64_t id_offset, int ref_kind,
                             T* x0, T* xref, int64_t xref_sb, T* uref, int64_t uref_sb, T* wind,
                             hipStream_t st) {
  const int64_t grid = (B + 255) / 256;
  hipLaunchKernelGGL((gen_inputs_kernel<T>), dim3((unsigned)grid), dim3(256), 0, st, B, N, (double)dt,
                     seed, id_offset, ref_kind, x0, xref, xref_sb, uref, uref_sb, wind);
  return hipGetLastError();
}

// ------------------------------------------------------------------------ histogram
template <class T>
__global__ void __launch_bounds__(256) histogram_kernel(int64_t B, int nu, const T* __restrict__ u0,
                                                        double lo, double hi, int nbins,
                                                        unsigned long long* __restrict__ counts) {
  extern __shared__ unsigned int hist[];
  for (int i = threadIdx.x; i < nu * nbins; i += blockDim.x) hist[i] = 0u;
  __syncthreads();
  const double scale = (double)nbins / (hi - lo);
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    for (int m = 0; m < nu; ++m) {
      const double v = (double)u0[b * nu + m];
      int bin = (int)floor((v - lo) * scale);
      bin = bin < 0 ? 0 : (bin >= nbins ? nbins - 1 : bin);
      if (v != v) bin = nbins - 1;
      atomicAdd(&hist[m * nbins + bin], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nu * nbins; i += blockDim.x)
    if (hist[i]) atomicAdd(&counts[i], (unsigned long long)hist[i]);
}

template <class T>
hipError_t launch_histogram(int64_t B, int nu, const T* u0, double lo, double hi, int nbins,
                            unsigned long long* counts, hipStream_t st) {
  int64_t grid = (B + 255) / 256;
  if (grid > 1024) grid = 1024;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((histogram_kernel<T>), dim3((unsigned)grid), dim3(256),
                     (size_t)nu * nbins * sizeof(unsigned int), st, B, nu, u0, lo, hi, nbins, counts);
  return hipGetLastError();
}

// ------------------------------------------------------------------------ quaternion helpers
// utils/MathUtils.py: quatMultiplication (:5-23), unitQuatInversion (:25-39), quat2Rot (:41-54);
// one thread per pair, fp64, same operation order as the reference's expressions
__global__ void __launch_bounds__(256) quat_ops_kernel(int64_t B, const double* __restrict__ q1,
                                                       const double* __restrict__ q2,
                                                       double* __restrict__ prod, double* __restrict__ inv,
                                                       double* __restrict__ rot) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double w1 = q1[4 * b], x1 = q1[4 * b + 1], y1 = q1[4 * b + 2], z1 = q1[4 * b + 3];
  if (prod) {
    const double w2 = q2[4 * b], x2 = q2[4 * b + 1], y2 = q2[4 * b + 2], z2 = q2[4 * b + 3];
    prod[4 * b] = w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2;
    prod[4 * b + 1] = w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2;
    prod[4 * b + 2] = w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2;
    prod[4 * b + 3] = w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2;
  }
  if (inv) {
    inv[4 * b] = w1;
    inv[4 * b + 1] = -x1;
    inv[4 * b + 2] = -y1;
    inv[4 * b + 3] = -z1;
  }
  if (rot) {
    double* R = rot + 9 * b;
    R[0] = 2.0 * (w1 * w1 + x1 * x1) - 1.0;
    R[1] = 2.0 * (x1 * y1 - w1 * z1);
    R[2] = 2.0 * (x1 * z1 + w1 * y1);
    R[3] = 2.0 * (x1 * y1 + w1 * z1);
    R[4] = 2.0 * (w1 * w1 + y1 * y1) - 1.0;
    R[5] = 2.0 * (y1 * z1 - w1 * x1);
    R[6] = 2.0 * (x1 * z1 - w1 * y1);
    R[7] = 2.0 * (y1 * z1 + w1 * x1);
    R[8] = 2.0 * (w1 * w1 + z1 * z1) - 1.0;
  }
}

hipError_t launch_quat_ops(int64_t B, const double* q1, const double* q2, double* prod, double* inv,
                           double* rot, hipStream_t st) {
  const int64_t grid = (B + 255) / 256;
  hipLaunchKernelGGL(quat_ops_kernel, dim3((unsigned)grid), dim3(256), 0, st, B, q1, q2, prod, inv, rot);
  return hipGetLastError();
}

#define MPCB_INST(T)                                                                              \
  template hipError_t launch_linearize<T>(int64_t, int, T, const Model<T>&, const T*, const T*,  \
                                          const T*, int64_t, T*, T*, T*, hipStream_t);           \
  template hipError_t launch_sim_step<T>(int64_t, T, const Model<T>&, const T*, const T*,        \
                                         const T*, int64_t, T*, hipStream_t);                    \
  template hipError_t launch_gen_inputs<T>(int64_t, int, T, uint64_t, uint64_t, int, T*, T*,     \
                                           int64_t, T*, int64_t, T*, hipStream_t);               \
  template hipError_t launch_histogram<T>(int64_t, int, const T*, double, double, int,           \
                                          unsigned long long*, hipStream_t);
MPCB_INST(double)
MPCB_INST(float)

}  // namespace mpcb
