// Microbenchmark: HBM copy bandwidth of the skin_span access patterns over
// the MANO vertex layout ([n][778][3] f32, 65,536 hands), no arithmetic.
// Build: hipcc --offload-arch=gfx950 -O3 -o span_patterns span_patterns.hip
// A unit is 16 hand rows x 64 vertices (16 x 768 B, rows 9,336 B apart), moved
// as 12 float4 per lane (flat row-major sweep); units differ only in which
// wave takes which unit when:
//   ranges     each wave a contiguous range of units (tile-major)
//   stride     unit u on wave u mod n_waves (the chip sweeps memory in order)
//   tileblock  a block's 4 waves share one tile (spans w, w + 4, ...), blocks
//              stride over tiles
//   copy16     flat float4 copy of the whole buffer (the ceiling)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
constexpr int NV = 778, VS = 3 * NV, SPANS = 12;  // 12 full spans (tail ignored here)

__device__ __forceinline__ void copy_unit(const float* __restrict__ in, float* __restrict__ out, long tile,
                                          int s, int lane) {
  const long base = tile * 16 * VS + 192 * s;
  f32x4u v[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int idx = 64 * i + lane, row = idx / 48, c4 = idx - 48 * row;
    v[i] = *reinterpret_cast<const f32x4u*>(in + base + row * VS + 4 * c4);
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int idx = 64 * i + lane, row = idx / 48, c4 = idx - 48 * row;
    *reinterpret_cast<f32x4u*>(out + base + row * VS + 4 * c4) = v[i] * 2.f;
  }
}

__global__ __launch_bounds__(256) void ranges(const float* in, float* out, long tiles) {
  const long w = blockIdx.x * 4L + (threadIdx.x >> 6), nw = gridDim.x * 4L, units = tiles * SPANS;
  for (long u = w * units / nw; u < (w + 1) * units / nw; ++u) copy_unit(in, out, u / SPANS, int(u % SPANS), threadIdx.x & 63);
}

__global__ __launch_bounds__(256) void stride(const float* in, float* out, long tiles) {
  const long w = blockIdx.x * 4L + (threadIdx.x >> 6), nw = gridDim.x * 4L, units = tiles * SPANS;
  for (long u = w; u < units; u += nw) copy_unit(in, out, u / SPANS, int(u % SPANS), threadIdx.x & 63);
}

__global__ __launch_bounds__(256) void tileblock(const float* in, float* out, long tiles) {
  const int wave = threadIdx.x >> 6;
  for (long t = blockIdx.x; t < tiles; t += gridDim.x)
    for (int s = wave; s < SPANS; s += 4) copy_unit(in, out, t, s, threadIdx.x & 63);
}

__global__ __launch_bounds__(256) void copy16(const f32x4* __restrict__ in, f32x4* __restrict__ out, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += gridDim.x * 256L) out[i] = in[i] * 2.f;
}

int main() {
  const long n = 65536, tiles = n / 16;
  const size_t nf = size_t(n) * VS;
  float *a, *b;
  CK(hipMalloc(&a, nf * 4)); CK(hipMalloc(&b, nf * 4));
  CK(hipMemset(a, 0, nf * 4)); CK(hipMemset(b, 0, nf * 4));
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 100; ++i) launch();
    CK(hipDeviceSynchronize());
    const int it = 100;
    CK(hipEventRecord(e0));
    for (int i = 0; i < it; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
    printf("%-28s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  };
  const double span_bytes = 2.0 * tiles * SPANS * 16 * 768;
  for (int bpc : {1, 2, 4, 8}) {
    const unsigned g = unsigned(ncu * bpc);
    char nm[64];
    snprintf(nm, 64, "ranges (%d blk/CU)", bpc);
    timeit(nm, span_bytes, [&] { hipLaunchKernelGGL(ranges, dim3(g), dim3(256), 0, 0, a, b, tiles); });
    snprintf(nm, 64, "stride (%d blk/CU)", bpc);
    timeit(nm, span_bytes, [&] { hipLaunchKernelGGL(stride, dim3(g), dim3(256), 0, 0, a, b, tiles); });
    snprintf(nm, 64, "tileblock (%d blk/CU)", bpc);
    timeit(nm, span_bytes, [&] { hipLaunchKernelGGL(tileblock, dim3(g), dim3(256), 0, 0, a, b, tiles); });
  }
  timeit("copy16", 2.0 * nf * 4, [&] { hipLaunchKernelGGL(copy16, dim3(ncu * 8), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, long(nf / 4)); });
  return 0;
}
