// mpcb_as.hip — the input-box QP of the SQP_RTI step (thrust box lbu <= u <= ubu on stages
// 0..N-1, blastermodel.py:259-270 / idxbu, JSON :11,86,148; BASELINE config c4), second design.
//
// Algorithm and iterates are those of the first active-set kernel (mpcb_box.hip PASS_BOX) and
// of the oracle (oracle.ocp.pdas_solve): primal-dual active set with the Kim-Park block-principal
// pivoting safeguard over P2's exported linearisation; the masked Riccati backward pass restarts
// at the highest stage whose active set changed, from the value function P2 / the previous pass
// stored there.  16 lanes per instance, lane j owning direction j, 4 instances per wavefront.
//
// What is new is how the 16 lanes of an instance exchange values.  The first kernel made every
// exchange through LDS (write, read back: a ~100-cycle round trip on the serial chain of each
// stage, three per forward stage) and measured ~7k cycles per forward stage and ~19k per
// backward stage at c4 (tools/stamps.py c4).  Here each exchange is a DPP row broadcast inside
// the FMA that consumes it (v_fmac_{f32,f64}_dpp ... row_newbcast:L reads lane L's operand):
//   forward, per stage, no LDS at all:
//     du_m  = kff_m + sum_{i<12} K[m][i] dx_i        input lanes, dx_i broadcast from state lane i
//     acc_j = r0_j + sum_{l<16} row_j[l] z_l         every lane, z_l broadcast from lane l
//   where a state lane's row is row i of [A|B] (r0 = gap: acc = dx'_i) and an input lane's row is
//   row m of the stage Hessian [G_ux G_uu] (r0 = h_u: acc = the box multiplier mu_m), so one
//   instruction stream serves both kinds of lane;
//   backward, per stage: h = [A|B]^T (p + P gap), the stage cost, the 4x4 input block and the
//   P update by broadcasts; only the transpose that keeps P symmetric goes through LDS.
// Workspace pointers are formed once per lane (the stage-k record is base + k * stride), and the
// active-set masks are kept per component by the input lanes (broadcast when the backward pass
// needs all four) instead of in every lane.
#define MPCB_AS_OWNER
#include "mpcb_as.h"
#include "mpcb_asipm.h"

namespace mpcb {

template <bool W32, bool ITER = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MPCB_AS_WAVES, 8)))
as_kernel_f32(SplitArgs<float> a) { asq::as_body<float, true, W32, ITER>(a); }
template <bool W32, bool ITER = false>
__global__ void __launch_bounds__(64) as_kernel_f64(SplitArgs<double> a) { asq::as_body<double, true, W32, ITER>(a); }
// the fp32 refinement of the listed instances (mpcb_as.h as_body REF)
template <bool W32, bool ITER = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MPCB_AS_WAVES, 8)))
as_ref_kernel_f32(SplitArgs<float> a) { asq::as_body<float, true, W32, ITER, true>(a); }
template <class T, bool ITER = false>
__global__ void __launch_bounds__(64) fwd_rm_kernel(SplitArgs<T> a) { asq::as_body<T, false, false, ITER>(a); }
template <class T, bool ITER = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? 2 : 1, 8)))
as_ipm_kernel(SplitArgs<T> a) {
  asq::ipm_body<T, ITER>(a);
}

template <class T> hipError_t launch_as(const SplitArgs<T>& a, hipStream_t st) {
  unsigned g = (unsigned)((a.nb + GROUPS - 1) / GROUPS);
  const size_t lds = a.N <= asq::OUT_NMAX ? (size_t)GROUPS * asq::out_elems<T>(a.N) * sizeof(T) : 0;
  if (a.as_queue && !dry_run()) {   // as many waves as stay resident; the rest of the chunk comes off the counter
    static const unsigned resident = [] {
      int dev = 0, cus = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
      return (unsigned)cus * 4u * (sizeof(T) == 4 ? (unsigned)MPCB_AS_WAVES : 1u);
    }();
    if (g > resident) g = resident;
    const hipError_t e = hipMemsetAsync(a.as_queue, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
  }
  if (a.as_fb && !dry_run()) {   // the interior-point fallback's list starts empty
    const hipError_t e = hipMemsetAsync(a.as_fb, 0, 2 * sizeof(int), st);
    if (e != hipSuccess) return e;
  }
  if (a.as_ref && !dry_run()) {   // the refinement list starts empty
    const hipError_t e = hipMemsetAsync(a.as_ref, 0, AS_REF_HDR * sizeof(int), st);
    if (e != hipSuccess) return e;
  }
  const bool w32 = a.N <= 32;   // (the stage masks fit 32 bits)
  const bool it = MPCB_AS_ITER_T && a.mode == MPCB_MODE_ITERATE;
  if constexpr (sizeof(T) == 4) {
    if (it) {
      if (w32) MPCB_LAUNCH(PH_FORWARD, (as_kernel_f32<true, true>), dim3(g), dim3(64), lds, st, a);
      else MPCB_LAUNCH(PH_FORWARD, (as_kernel_f32<false, true>), dim3(g), dim3(64), lds, st, a);
    } else {
      if (w32) MPCB_LAUNCH(PH_FORWARD, (as_kernel_f32<true>), dim3(g), dim3(64), lds, st, a);
      else MPCB_LAUNCH(PH_FORWARD, (as_kernel_f32<false>), dim3(g), dim3(64), lds, st, a);
    }
  } else {
    if (it) {
      if (w32) MPCB_LAUNCH(PH_FORWARD, (as_kernel_f64<true, true>), dim3(g), dim3(64), lds, st, a);
      else MPCB_LAUNCH(PH_FORWARD, (as_kernel_f64<false, true>), dim3(g), dim3(64), lds, st, a);
    } else {
      if (w32) MPCB_LAUNCH(PH_FORWARD, (as_kernel_f64<true>), dim3(g), dim3(64), lds, st, a);
      else MPCB_LAUNCH(PH_FORWARD, (as_kernel_f64<false>), dim3(g), dim3(64), lds, st, a);
    }
  }
  // the instances the active set handed over (usually none: the waves read an empty list and
  // exit).  Not in the launch log, which keeps the active-set kernel as the phase's kernel.
  if (a.as_fb && !dry_run()) {
    static const unsigned resident_ipm = [] {
      int dev = 0, cus = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
      return (unsigned)cus * 4u * (sizeof(T) == 4 ? 2u : 1u);
    }();
    unsigned gi = (unsigned)((a.nb + GROUPS - 1) / GROUPS);
    if (gi > resident_ipm) gi = resident_ipm;
    if (a.mode == MPCB_MODE_ITERATE) hipLaunchKernelGGL((as_ipm_kernel<T, true>), dim3(gi), dim3(64), 0, st, a);
    else hipLaunchKernelGGL((as_ipm_kernel<T, false>), dim3(gi), dim3(64), 0, st, a);
  }
  // the listed fp32 instances' refinement (a few hundred of c4's 65,536), after the fallback, whose
  // results it refines too.  Not in the launch log either (above).
  if constexpr (sizeof(T) == 4) {
    if (a.as_ref && !dry_run()) {
      static const unsigned resident_ref = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
          cus = 256;
        return (unsigned)cus * 4u * (unsigned)MPCB_AS_WAVES;
      }();
      unsigned gr = (unsigned)((a.nb + GROUPS - 1) / GROUPS);
      const size_t lds_ref = (size_t)GROUPS * asq::ref_elems<float>(a.N) * sizeof(float);
      if (gr > resident_ref) gr = resident_ref;
      if (it) {
        if (w32) hipLaunchKernelGGL((as_ref_kernel_f32<true, true>), dim3(gr), dim3(64), lds_ref, st, a);
        else hipLaunchKernelGGL((as_ref_kernel_f32<false, true>), dim3(gr), dim3(64), lds_ref, st, a);
      } else {
        if (w32) hipLaunchKernelGGL((as_ref_kernel_f32<true>), dim3(gr), dim3(64), lds_ref, st, a);
        else hipLaunchKernelGGL((as_ref_kernel_f32<false>), dim3(gr), dim3(64), lds_ref, st, a);
      }
    }
  }
  return dry_run() ? hipSuccess : hipGetLastError();
}
// forward pass of the unconstrained small-chunk path from P2's row-major exports (ABT2, KR2)
template <class T> hipError_t launch_fwd_rm(const SplitArgs<T>& a, hipStream_t st) {
  const unsigned g = (unsigned)((a.nb + GROUPS - 1) / GROUPS);
  const size_t lds = a.N <= asq::OUT_NMAX ? (size_t)GROUPS * asq::out_elems<T>(a.N) * sizeof(T) : 0;
  if (MPCB_AS_ITER_T && a.mode == MPCB_MODE_ITERATE)
    MPCB_LAUNCH(PH_FORWARD, (fwd_rm_kernel<T, true>), dim3(g), dim3(64), lds, st, a);
  else
    MPCB_LAUNCH(PH_FORWARD, (fwd_rm_kernel<T>), dim3(g), dim3(64), lds, st, a);
  return dry_run() ? hipSuccess : hipGetLastError();
}
template hipError_t launch_fwd_rm<double>(const SplitArgs<double>&, hipStream_t);
template hipError_t launch_fwd_rm<float>(const SplitArgs<float>&, hipStream_t);
template hipError_t launch_as<double>(const SplitArgs<double>&, hipStream_t);
template hipError_t launch_as<float>(const SplitArgs<float>&, hipStream_t);

}  // namespace mpcb

#ifdef MPCB_REF_STAMPS
extern "C" int mpcb_debug_ref_stamps(unsigned long long* out, int reset) {
  if (reset) {
    const unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(mpcb::asq::g_refst), z, sizeof(z)) == hipSuccess ? 0 : -2;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::asq::g_refst), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -2;
}
#endif
#ifdef MPCB_REF_TRACE
extern "C" int mpcb_debug_ref_trace(int* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::asq::g_ref_trace), sizeof(int) * 128 * 20) == hipSuccess ? 0 : -2;
}
#endif
#ifdef MPCB_STAMPS
extern "C" int mpcb_debug_wt_p3(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::asq::g_wt_p3), sizeof(unsigned long long) * MPCB_WT_MAX * 7) == hipSuccess ? 0 : -2;
}
extern "C" int mpcb_debug_stamps_as(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::asq::g_astamps), sizeof(unsigned long long) * 12) == hipSuccess ? 0 : -2;
}
#endif
