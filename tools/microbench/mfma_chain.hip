// Microbenchmark: how close do blend_skin16-shaped MFMA chains get to the
// fp32 MFMA peak?  Each wave runs tiles of 37 dependent
// v_mfma_f32_16x16x4_f32 (one accumulator chain, A in 37 VGPRs), W blocks of
// 4 waves per CU (W waves per SIMD).  B operand:
//   MODE 0: registers (no LDS),
//   MODE 1: ds_read_b128 one 4-MFMA group ahead (blend_skin16's mfma16_tile),
//   MODE 2: MODE 1 + a workgroup barrier after every tile,
//   MODE 3: ds_read_b128 two groups ahead.
// Question: what does the chain structure itself cost, before DMA, LBS and
// stores?  Build: hipcc --offload-arch=gfx950 -O3 -o mfma_chain mfma_chain.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kSteps = 37, kGroups = 10;

template <int MODE, int W>
__global__ __launch_bounds__(256, W) void chains(const float* __restrict__ in, float* __restrict__ out, int tiles) {
  __shared__ f32x4 lds[kGroups * 64];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < kGroups * 64; i += 256) lds[i] = f32x4{in[i & 255], in[(i + 1) & 255], in[(i + 2) & 255], in[(i + 3) & 255]};
  __syncthreads();
  float a[kGroups * 4];
#pragma unroll
  for (int k = 0; k < kGroups * 4; ++k) a[k] = in[(blockIdx.x * 7 + k * 13 + lane) & 255];
  f32x4 breg[kGroups];
#pragma unroll
  for (int g = 0; g < kGroups; ++g) breg[g] = lds[g * 64 + lane];
  f32x4 sum = {};
  for (int t = 0; t < tiles; ++t) {
    f32x4 acc = {};
    if constexpr (MODE == 0) {
#pragma unroll
      for (int g = 0; g < kGroups; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (4 * g + q < kSteps) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * g + q], breg[g][q], acc, 0, 0, 0);
    } else if constexpr (MODE == 1 || MODE == 2) {
      f32x4 bn = lds[lane];
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        const f32x4 bv = bn;
        if (g + 1 < kGroups) bn = lds[(g + 1) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (4 * g + q < kSteps) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * g + q], bv[q], acc, 0, 0, 0);
      }
      if constexpr (MODE == 2) __syncthreads();
    } else {
      f32x4 b0 = lds[lane], b1 = lds[64 + lane];
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        const f32x4 bv = b0;
        b0 = b1;
        if (g + 2 < kGroups) b1 = lds[(g + 2) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (4 * g + q < kSteps) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * g + q], bv[q], acc, 0, 0, 0);
      }
    }
    sum += acc;
  }
  out[blockIdx.x * 256 + threadIdx.x] = sum[0] + sum[1] + sum[2] + sum[3];
}

template <int MODE, int W>
void run(const float* in, float* out, int n_cu) {
  const int tiles = 2000;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((chains<MODE, W>), dim3(n_cu * W), dim3(256), 0, 0, in, out, tiles);
  CK(hipEventRecord(e0));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((chains<MODE, W>), dim3(n_cu * W), dim3(256), 0, 0, in, out, tiles);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 20;
  const double flop = double(n_cu) * W * 4 * tiles * kSteps * 2048.0;
  printf("mode %d  waves/SIMD %d  %.3f ms  %.1f TF/s  (%.1f %% of 157.3)\n", MODE, W, ms, flop / ms * 1e-9,
         flop / ms * 1e-9 / 157.3 * 100);
}

int main() {
  float *in, *out;
  CK(hipMalloc(&in, 256 * 4));
  CK(hipMalloc(&out, 256 * 256 * 8 * 4));
  CK(hipMemset(in, 0, 256 * 4));
  int n_cu = 0;
  CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 1>(in, out, n_cu);
    run<0, 2>(in, out, n_cu);
    run<0, 3>(in, out, n_cu);
    run<1, 1>(in, out, n_cu);
    run<1, 2>(in, out, n_cu);
    run<1, 3>(in, out, n_cu);
    run<2, 3>(in, out, n_cu);
    run<3, 3>(in, out, n_cu);
  }
  return 0;
}
