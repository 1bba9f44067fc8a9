// check: v_fmac_f32_dpp / v_fmac_f64_dpp with row_newbcast:L broadcast lane L of each 16-lane row
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k32(float* o) {
  const int l = threadIdx.x;
  float acc = 0.f, a = (float)(l + 1), b = 1.0f;
  asm volatile("s_nop 4\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(a), "v"(b));
  o[l] = acc;
}
__global__ void k64(double* o) {
  const int l = threadIdx.x;
  double acc = 0.0, a = (double)(l + 1), b = 1.0;
  asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(a), "v"(b));
  o[l] = acc;
}
int main() {
  float* f; double* d;
  hipMalloc(&f, 256); hipMalloc(&d, 512);
  k32<<<1, 64>>>(f); k64<<<1, 64>>>(d);
  float hf[64]; double hd[64];
  hipMemcpy(hf, f, 256, hipMemcpyDeviceToHost); hipMemcpy(hd, d, 512, hipMemcpyDeviceToHost);
  int bad32 = 0, bad64 = 0;
  for (int l = 0; l < 64; ++l) {
    const float want = (float)((l / 16) * 16 + 5 + 1);
    if (hf[l] != want) ++bad32;
    if (hd[l] != (double)want) ++bad64;
  }
  printf("f32 lanes 0,17,40: %g %g %g  bad32=%d\n", hf[0], hf[17], hf[40], bad32);
  printf("f64 lanes 0,17,40: %g %g %g  bad64=%d\n", hd[0], hd[17], hd[40], bad64);
  return 0;
}
