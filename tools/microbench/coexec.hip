// Can an f32 MFMA wave and a VALU wave on the same SIMD run concurrently?
// Block = 8 waves (2 per SIMD): waves 0-3 run MFMA chains, waves 4-7 run VALU FMAs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
template <int MFMA_KIND, bool DO_M, bool DO_V>
__global__ __launch_bounds__(512) void k(float* out, float x, int iters_m, int iters_v) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float r = 0.f;
  if (wave < 4) {
    if (DO_M) {
      f32x16 acc0 = {}, acc1 = {};
      float a = x * threadIdx.x, b = x + threadIdx.x;
      bf16x8 ab = {1, 2, 3, 4, 5, 6, 7, 8};
      for (int i = 0; i < iters_m; ++i) {
        if (MFMA_KIND == 0) {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, acc1, 0, 0, 0);
        } else {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, ab, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, ab, acc1, 0, 0, 0);
        }
      }
      for (int j = 0; j < 16; ++j) r += acc0[j] + acc1[j];
    }
  } else if (DO_V) {
    float t[12], a[12];
    for (int m = 0; m < 12; ++m) { a[m] = x + m; t[m] = 0.f; }
    float w = x * threadIdx.x;
    for (int i = 0; i < iters_v; ++i) {
#pragma unroll
      for (int m = 0; m < 12; ++m) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(t[m]) : "v"(a[m]), "v"(w));
    }
    for (int m = 0; m < 12; ++m) r += t[m];
  }
  out[blockIdx.x * 512 + threadIdx.x] = r;
}
int main() {
  float* out; CK(hipMalloc(&out, 256 * 512 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int im = 4000, iv = 2700;  // roughly equal alone-times
  auto run = [&](const char* name, auto kern) {
    hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, out, 1.0f, im, iv);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, out, 1.0f, im, iv);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %.3f ms\n", name, ms);
  };
  run("f32 mfma only", k<0, true, false>);
  run("valu only", k<0, false, true>);
  run("f32 mfma + valu", k<0, true, true>);
  run("bf16 mfma only", k<1, true, false>);
  run("bf16 mfma + valu", k<1, true, true>);
  return 0;
}
