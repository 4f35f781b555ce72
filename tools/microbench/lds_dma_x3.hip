// lds_dma_x3.hip -- LDS-DMA layout and alignment facts used by skin_ring:
//  (1) where global_load_lds_dwordx3 puts lane l's 12 bytes (base + 12 l, or
//      base + 16 l like dwordx4?);
//  (2) whether global_load_lds_dwordx4 reads correctly from a source that is
//      only 8-byte aligned (odd hand rows of the [n][778][3] v_posed are).
// Each lane l sources floats {off + 4l .. off + 4l + 3} (x4) or {3l .. 3l+2} (x3).
//   hipcc --offload-arch=gfx950 -O3 -o lds_dma_x3 lds_dma_x3.hip && ./lds_dma_x3
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error line %d\n", __LINE__); return 1; } } while (0)

template <int SIZE>
__global__ void probe(const float* __restrict__ src, float* __restrict__ out, int off) {
  __shared__ float lds[512];
  for (int i = threadIdx.x; i < 512; i += 64) lds[i] = -1.f;
  __syncthreads();
  const float* g = src + off + (SIZE / 4) * threadIdx.x;
  if constexpr (SIZE == 12)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)(lds + 8), 12, 0, 0);
  else
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)(lds + 8), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}

int main() {
  float h[512], *ds, *dout, o[512];
  for (int i = 0; i < 512; ++i) h[i] = float(i);
  CK(hipMalloc(&ds, sizeof(h)));
  CK(hipMalloc(&dout, sizeof(o)));
  CK(hipMemcpy(ds, h, sizeof(h), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(probe<12>, dim3(1), dim3(64), 0, 0, ds, dout, 0);
  CK(hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost));
  int dense = 0, strided = 0;
  for (int l = 0; l < 64; ++l)
    for (int c = 0; c < 3; ++c) {
      dense += o[8 + 3 * l + c] == float(3 * l + c);
      strided += o[8 + 4 * l + c] == float(3 * l + c);
    }
  printf("dwordx3: lane l at base + 12 l: %d/192 floats, at base + 16 l: %d/192\n", dense, strided);
  for (int off : {0, 1, 2, 3}) {
    hipLaunchKernelGGL(probe<16>, dim3(1), dim3(64), 0, 0, ds, dout, off);
    CK(hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost));
    int ok = 0;
    for (int i = 0; i < 256; ++i) ok += o[8 + i] == float(off + i);
    printf("dwordx4 from a source %2d B past 16-B alignment: %d/256 floats correct\n", 4 * off, ok);
  }
  return 0;
}
