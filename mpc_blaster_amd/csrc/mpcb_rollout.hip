// mpcb_rollout.hip — P1 of the split path with a 16-lane row per instance (small chunks: c2):
// the kernel around mpcb_row.h's row_body and its launcher.
#include "mpcb_common.h"

namespace mpcb {
WT_TABLE(g_wt_p1)
}  // namespace mpcb

#include "mpcb_row.h"

namespace mpcb {

template <class T, bool ITER, bool DJ, bool TAN>
__global__ void __launch_bounds__(64) nominal_row_kernel(SplitArgs<T> a) {
  row_body<T, ITER, DJ, TAN>(a);
}

template <class T, bool TAN>
static void launch_row_m(const SplitArgs<T>& a, hipStream_t st) {
  const dim3 grid((unsigned)((a.nb + SS - 1) / SS));
  const size_t lds = row_lds_bytes(a);   // (<= 33 KiB at N = 64, fp64, iterate)
  const bool dj = row_dj(a);
  const bool it = a.mode == MPCB_MODE_ITERATE;
  if (dj) {
    if (it) MPCB_LAUNCH(PH_NOMINAL, (nominal_row_kernel<T, true, true, TAN>), grid, dim3(64), lds, st, a);
    else MPCB_LAUNCH(PH_NOMINAL, (nominal_row_kernel<T, false, true, TAN>), grid, dim3(64), lds, st, a);
  } else {
    if (it) MPCB_LAUNCH(PH_NOMINAL, (nominal_row_kernel<T, true, false, TAN>), grid, dim3(64), lds, st, a);
    else MPCB_LAUNCH(PH_NOMINAL, (nominal_row_kernel<T, false, false, TAN>), grid, dim3(64), lds, st, a);
  }
}

template <class T> hipError_t launch_nominal_row(const SplitArgs<T>& a, hipStream_t st) {
  // (the tangent export is built for fp64 only: mpcb_create sets tin there)
  if (sizeof(T) == 8 && a.tin) launch_row_m<T, sizeof(T) == 8>(a, st);
  else launch_row_m<T, false>(a, st);
  return dry_run() ? hipSuccess : hipGetLastError();
}

template hipError_t launch_nominal_row<double>(const SplitArgs<double>&, hipStream_t);
#ifdef MPCB_STAMPS
extern "C" int mpcb_debug_wt_p1(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcb::g_wt_p1), sizeof(unsigned long long) * MPCB_WT_MAX * 7) == hipSuccess ? 0 : -2;
}
#endif
template hipError_t launch_nominal_row<float>(const SplitArgs<float>&, hipStream_t);

}  // namespace mpcb
