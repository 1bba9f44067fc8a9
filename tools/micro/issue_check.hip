// Issue-rate microbenchmark of one wave alone on its SIMD (gfx950), the situation of the c2
// kernels: cycles (s_memtime) per instruction of 8 interleaved independent chains of
//   fma64:    v_fma_f64 (distinct registers per chain)
//   fmadpp:   v_fmac_f64_dpp row_newbcast (the P2 products)
//   movdpp:   v_mov_b64_dpp row_newbcast (the rollout's broadcasts)
//   mul64 / add64: v_mul_f64 / v_add_f64
//   fma32:    v_fma_f32
//   cnd32:    v_cndmask_b32 (the quadrant selects of sin/cos)
//   rcp64:    v_rcp_f64
// and, for the DPP forms, a dependent chain (latency).  Build: hipcc --offload-arch=gfx950 -O2
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))
#define CH8(op)                                                                                   \
  asm volatile(R64(op " %0, %0, %8, %9\n\t" op " %1, %1, %8, %9\n\t" op " %2, %2, %8, %9\n\t"          \
                   op " %3, %3, %8, %9\n\t" op " %4, %4, %8, %9\n\t" op " %5, %5, %8, %9\n\t"          \
                   op " %6, %6, %8, %9\n\t" op " %7, %7, %8, %9\n\t")                                   \
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
               : "v"(b), "v"(c))
#define CH8B(op)                                                                                  \
  asm volatile(R64(op " %0, %0, %8\n\t" op " %1, %1, %8\n\t" op " %2, %2, %8\n\t"                      \
                   op " %3, %3, %8\n\t" op " %4, %4, %9\n\t" op " %5, %5, %9\n\t"                      \
                   op " %6, %6, %9\n\t" op " %7, %7, %9\n\t")                                           \
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
               : "v"(b), "v"(c))

template <int K>
__global__ void kern(double* o, unsigned long long* t) {
  double a[8];
  for (int i = 0; i < 8; ++i) a[i] = o[threadIdx.x] + i;
  double b = 1.0000001, c = 1e-9;
  float af[8];
  for (int i = 0; i < 8; ++i) af[i] = (float)a[i];
  float bf = 1.0000001f, cf = 1e-9f;
  unsigned long long t0 = 0, t1 = 0;
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
  if constexpr (K == 0) {
    CH8("v_fma_f64");
  } else if constexpr (K == 1) {
    asm volatile(R64("v_fmac_f64_dpp %0, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %2, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %3, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %4, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %5, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %6, %8, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %7, %8, %9 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t")
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
                 : "v"(b), "v"(c));
  } else if constexpr (K == 2) {
    asm volatile(R64("v_mov_b64_dpp %0, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %1, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %2, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %3, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %4, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %5, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %6, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
                     "v_mov_b64_dpp %7, %9 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t")
                 : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), "=&v"(a[6]), "=&v"(a[7])
                 : "v"(b), "v"(c));
  } else if constexpr (K == 3) {
    CH8B("v_mul_f64");
  } else if constexpr (K == 4) {
    CH8B("v_add_f64");
  } else if constexpr (K == 5) {
    asm volatile(R64("v_fma_f32 %0, %0, %8, %9\n\tv_fma_f32 %1, %1, %8, %9\n\tv_fma_f32 %2, %2, %8, %9\n\t"
                     "v_fma_f32 %3, %3, %8, %9\n\tv_fma_f32 %4, %4, %8, %9\n\tv_fma_f32 %5, %5, %8, %9\n\t"
                     "v_fma_f32 %6, %6, %8, %9\n\tv_fma_f32 %7, %7, %8, %9\n\t")
                 : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3]), "+v"(af[4]), "+v"(af[5]), "+v"(af[6]), "+v"(af[7])
                 : "v"(bf), "v"(cf));
  } else if constexpr (K == 6) {
    asm volatile(R64("v_cndmask_b32 %0, %0, %8, vcc\n\tv_cndmask_b32 %1, %1, %8, vcc\n\tv_cndmask_b32 %2, %2, %8, vcc\n\t"
                     "v_cndmask_b32 %3, %3, %8, vcc\n\tv_cndmask_b32 %4, %4, %9, vcc\n\tv_cndmask_b32 %5, %5, %9, vcc\n\t"
                     "v_cndmask_b32 %6, %6, %9, vcc\n\tv_cndmask_b32 %7, %7, %9, vcc\n\t")
                 : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3]), "+v"(af[4]), "+v"(af[5]), "+v"(af[6]), "+v"(af[7])
                 : "v"(bf), "v"(cf) : "vcc");
  } else if constexpr (K == 7) {
    asm volatile(R64("v_rcp_f64 %0, %8\n\tv_rcp_f64 %1, %8\n\tv_rcp_f64 %2, %8\n\tv_rcp_f64 %3, %8\n\t"
                     "v_rcp_f64 %4, %9\n\tv_rcp_f64 %5, %9\n\tv_rcp_f64 %6, %9\n\tv_rcp_f64 %7, %9\n\t")
                 : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), "=&v"(a[6]), "=&v"(a[7])
                 : "v"(b), "v"(c));
  } else if constexpr (K == 9) {   // s_memtime rate: a long dependent chain also timed by events
    for (int r = 0; r < 200; ++r) asm volatile(R64("v_fma_f64 %0, %0, %1, %2\n\t") : "+v"(a[0]) : "v"(b), "v"(c));
  } else if constexpr (K == 8) {   // dependent DPP fmac chain (latency), no s_nop
    asm volatile(R64("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t")
                 : "+v"(a[0]) : "v"(b), "v"(c));
  }
  t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 8; ++i) a[0] += a[i] + af[i];
  o[threadIdx.x] = a[0];
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

int main() {
  double* o;
  unsigned long long* t;
  hipMalloc(&o, 64 * 8);
  hipMalloc(&t, 8);
  hipMemset(o, 0, 64 * 8);
  struct { const char* n; void (*k)(double*, unsigned long long*); int per; } ks[] = {
      {"fma64 x8", kern<0>, 512}, {"fmac64_dpp x8", kern<1>, 512}, {"mov_b64_dpp x8", kern<2>, 512},
      {"mul64 x8", kern<3>, 512}, {"add64 x8", kern<4>, 512}, {"fma32 x8", kern<5>, 512},
      {"cndmask32 x8", kern<6>, 512}, {"rcp64 x8", kern<7>, 512}, {"fmac64_dpp dep", kern<8>, 64}};
  for (auto& k : ks) {
    unsigned long long best = ~0ull;
    for (int r = 0; r < 5; ++r) {
      hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, o, t);
      unsigned long long h;
      hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
      if (h < best) best = h;
    }
    printf("%-16s %.2f cycles per instruction\n", k.n, (double)best / k.per);
  }
  // s_memtime rate vs wall clock: a long dependent chain timed both ways
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern<9>, dim3(1), dim3(64), 0, 0, o, t);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern<9>, dim3(1), dim3(64), 0, 0, o, t);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h;
  hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
  printf("s_memtime %llu ticks in %.3f ms (event): %.3f GHz; %.2f ticks per dependent fma64\n", h, ms,
         h / (ms * 1e6), (double)h / (200 * 64));
  return 0;
}
