// Latency / issue microbenchmark of one wave per SIMD (gfx950): cycles per instruction of
//   dep:   a dependent v_fma_f64 chain
//   ind2/ind4: 2 / 4 interleaved independent chains
//   dppdep: dependent (v_mov_b64_dpp row_newbcast -> v_fma_f64) pairs
//   fmacdpp: dependent v_fmac_f64_dpp row_newbcast chain
//   f32dep: dependent v_fma_f32 chain
// Output: cycles (s_memtime) per instruction, averaged over the 64 lanes' identical work.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP16(x) x x x x x x x x x x x x x x x x
__global__ void dep(double* o, unsigned long long* t) {
  double a = o[threadIdx.x], b = 1.0000001, c = 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) { REP16(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));) }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = a; if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void ind2(double* o, unsigned long long* t) {
  double a = o[threadIdx.x], a2 = a + 1, b = 1.0000001, c = 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) { REP16(asm volatile("v_fma_f64 %0, %0, %2, %3\n\tv_fma_f64 %1, %1, %2, %3" : "+v"(a), "+v"(a2) : "v"(b), "v"(c));) }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = a + a2; if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void ind4(double* o, unsigned long long* t) {
  double a = o[threadIdx.x], a2 = a + 1, a3 = a + 2, a4 = a + 3, b = 1.0000001, c = 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) { REP16(asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_fma_f64 %1, %1, %4, %5\n\tv_fma_f64 %2, %2, %4, %5\n\tv_fma_f64 %3, %3, %4, %5" : "+v"(a), "+v"(a2), "+v"(a3), "+v"(a4) : "v"(b), "v"(c));) }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = a + a2 + a3 + a4; if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void dppdep(double* o, unsigned long long* t) {
  double a = o[threadIdx.x], b = 1.0000001, c = 1e-9, d;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) { REP16(asm volatile("s_nop 1\n\tv_mov_b64_dpp %1, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fma_f64 %0, %1, %2, %3" : "+v"(a), "=&v"(d) : "v"(b), "v"(c));) }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = a; if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void fmacdpp(double* o, unsigned long long* t) {
  double a = o[threadIdx.x], b = 1.0000001, acc = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) { REP16(asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(a), "v"(b));) }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = acc; if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void f32dep(double* o, unsigned long long* t) {
  float a = (float)o[threadIdx.x], b = 1.0000001f, c = 1e-9f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) { REP16(asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));) }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = a; if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void rcpdep(double* o, unsigned long long* t) {
  double a = o[threadIdx.x] + 2.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) { REP16(asm volatile("v_rcp_f64 %0, %0" : "+v"(a));) }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = a; if (threadIdx.x == 0) t[0] = t1 - t0;
}
int main() {
  double* o; unsigned long long* t;
  hipMalloc(&o, 64 * 8); hipMalloc(&t, 8); hipMemset(o, 0, 64 * 8);
  struct { const char* n; void (*k)(double*, unsigned long long*); int per; } ks[] = {
      {"dep fma_f64", dep, 1}, {"ind2 fma_f64", ind2, 2}, {"ind4 fma_f64", ind4, 4},
      {"dpp mov+fma", dppdep, 2}, {"fmac_dpp dep", fmacdpp, 1}, {"dep fma_f32", f32dep, 1},
      {"dep rcp_f64", rcpdep, 1}};
  for (auto& k : ks) {
    unsigned long long best = ~0ull;
    for (int r = 0; r < 5; ++r) {
      hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, o, t);
      unsigned long long h; hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
      if (h < best) best = h;
    }
    // s_memtime counts at the shader clock on gfx9 (cycles)
    printf("%-14s %.2f cycles per instruction\n", k.n, (double)best / (64.0 * 16 * k.per));
  }
  return 0;
}
