// VALU issue rate of v_fmac_f32 vs its DPP row_newbcast form vs an SGPR operand.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, float x, float y, int iters) {
  float a[12], t[12];
  for (int m = 0; m < 12; ++m) { a[m] = x + m + threadIdx.x; t[m] = 0.f; }
  float w = y * threadIdx.x;
  float s = __builtin_amdgcn_readfirstlane(__float_as_int(x)) ;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 12; ++m) {
      if constexpr (MODE == 0) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(t[m]) : "v"(a[m]), "v"(w));
      if constexpr (MODE == 1) asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(t[m]) : "v"(a[m]), "v"(w));
      if constexpr (MODE == 2) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(t[m]) : "s"(s), "v"(w));
      if constexpr (MODE == 3) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*(double*)&t[m & ~1]) : "v"(*(double*)&a[m & ~1]), "v"(*(double*)&a[0]));
    }
  }
  float r = 0; for (int m = 0; m < 12; ++m) r += t[m];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}
int main() {
  float* out; CK(hipMalloc(&out, 4096 * 256 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 2000;
  const char* names[] = {"v_fmac_f32", "v_fmac_f32_dpp row_newbcast", "v_fmac_f32 sgpr", "v_pk_fma_f32"};
  for (int blocks : {256 * 2, 256 * 8}) {
    for (int mode = 0; mode < 4; ++mode) {
      auto launch = [&] {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 1.f, 2.f, iters);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 1.f, 2.f, iters);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 1.f, 2.f, iters);
        if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 1.f, 2.f, iters);
      };
      launch(); CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      const double instr_per_simd = double(blocks) * 4 * iters * 12 / 1024.0;  // wave-instructions per SIMD
      printf("%-30s waves/SIMD=%d  %.3f ms  %.2f ns/instr/SIMD (%.2f cyc @2.4GHz)\n", names[mode],
             blocks * 4 / 1024, ms, ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
    }
  }
  return 0;
}
