// fp64 matrix-core microbenchmark, one wave alone on its SIMD (gfx950), for the question whether
// the c2 Riccati contractions (Y = P [A|B], G = [A|B]^T Y; round-4 verdict item 4) could move
// from row-broadcast VALU FMAs to v_mfma_f64_16x16x4_f64.  Cycles (s_memtime) per instruction of
//   0  8 independent v_mfma_f64_16x16x4_f64 accumulators, back to back (issue / throughput)
//   1  one dependent accumulator chain (latency)
//   2  8 independent MFMAs, each followed by 8 independent v_fma_f64 (co-execution: ~max of the two
//      streams if the VALU issues under the matrix core, their sum if not)
//   3  the 64 v_fma_f64 of case 2 alone
//   4  8 independent v_fmac_f64_dpp row_newbcast (the current contraction instruction)
// Build: hipcc --offload-arch=gfx950 -O2 tools/micro/mfma64_check.hip -o tools/micro/mfma64_check
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
#define R8(x) x x x x x x x x

template <int K>
__global__ void kern(double* o, unsigned long long* t) {
  const double x = o[threadIdx.x];
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = d4{x + i, x - i, x * i, x};
  double f[8];
  for (int i = 0; i < 8; ++i) f[i] = x + 0.5 * i;
  const double b = 1.0000001, c = 1e-9;
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 16; ++it) {
    if constexpr (K == 0) {
      R8({ for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc[i], 0, 0, 0); })
    } else if constexpr (K == 1) {
      R8({ for (int i = 0; i < 8; ++i) acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc[0], 0, 0, 0); })
    } else if constexpr (K == 2) {
      R8({ for (int i = 0; i < 8; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc[i], 0, 0, 0);
        asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\t"
                     "v_fma_f64 %3, %3, %8, %9\n\tv_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\t"
                     "v_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9\n\t"
                     : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7])
                     : "v"(b), "v"(c));
      } })
    } else if constexpr (K == 3) {
      R8({ for (int i = 0; i < 8; ++i) {
        asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\t"
                     "v_fma_f64 %3, %3, %8, %9\n\tv_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\t"
                     "v_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9\n\t"
                     : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7])
                     : "v"(b), "v"(c));
      } })
    } else {
      R8({ asm volatile("s_nop 4\n\t"
                     "v_fmac_f64_dpp %0, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %2, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %3, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %4, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %5, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %6, %8, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %7, %8, %9 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
                     : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7])
                     : "v"(b), "v"(c)); })
    }
  }
  asm volatile("s_nop 0" ::: "memory");
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3] + f[i];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = s;
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}

template <int K> static double run(double* o, unsigned long long* t, int n_instr) {
  hipLaunchKernelGGL(kern<K>, dim3(1), dim3(64), 0, 0, o, t);   // warm
  hipLaunchKernelGGL(kern<K>, dim3(1), dim3(64), 0, 0, o, t);
  unsigned long long h = 0;
  (void)hipMemcpy(&h, t, sizeof(h), hipMemcpyDeviceToHost);
  return (double)h / n_instr;
}

int main() {
  double* o;
  unsigned long long* t;
  (void)hipMalloc(&o, 64 * sizeof(double));
  (void)hipMemset(o, 0, 64 * sizeof(double));
  (void)hipMalloc(&t, sizeof(unsigned long long));
  const int n = 16 * 8 * 8;   // instructions of the measured kind per case
  printf("mfma_f64_16x16x4 independent x8   %.1f cycles per MFMA\n", run<0>(o, t, n));
  printf("mfma_f64_16x16x4 dependent chain  %.1f cycles per MFMA\n", run<1>(o, t, n));
  printf("mfma + 8 v_fma_f64 (co-exec)      %.1f cycles per (MFMA + 8 FMA)\n", run<2>(o, t, n));
  printf("8 v_fma_f64 alone                 %.1f cycles per 8 FMA\n", run<3>(o, t, n));
  printf("v_fmac_f64_dpp independent x8     %.1f cycles per instruction\n", run<4>(o, t, n * 8 / 8));
  return 0;
}
