// Microbenchmark: the standalone LBS's memory stream without the LBS.
// skin_pair's unit (4 hand rows x 64 vertices of the [n][778][3] f32 layout,
// 3 float4 per lane) in grid-stride order over 65,536 hands, one wave per
// SIMD, loads issued D units ahead (register sets), optionally with each
// unit's 4 hands' transforms (3 KB from a [n][16][12] array, as skin_pair
// re-reads them per unit) and optionally through an LDS stage.
// Question: what do the per-unit transforms reads and the LDS round trip
// cost against the bare row copy?
// Build: hipcc --offload-arch=gfx950 -O3 -o unit_stream unit_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
constexpr int NV = 778, VS = 3 * NV, SPANS = 12;  // full spans only

template <int TR, int LDS, int D>
__global__ __launch_bounds__(256, 1) void unit_stream(const float* __restrict__ in, const f32x4* __restrict__ tr,
                                                      float* __restrict__ out, float* __restrict__ sink, long n) {
  __shared__ f32x4 stage[4][2][3 * 64 + 3 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long b = blockIdx.x, nb = gridDim.x;
  const long w = ((nb % 8) ? b : (b % 8) * (nb / 8) + b / 8) * 4 + wave, nw = nb * 4;
  const long units = n / 4 * SPANS;
  int off[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int idx = 64 * i + lane, row = idx / 48, c4 = idx % 48;
    off[i] = row * VS + 4 * c4;
  }
  f32x4 v[D][3], t[D][3];
  auto load = [&](long u, int set) {
    const long q = u / SPANS;
    const int s = int(u - q * SPANS);
    const float* src = in + q * 4 * VS + 3 * 64 * s;
#pragma unroll
    for (int i = 0; i < 3; ++i) v[set][i] = *reinterpret_cast<const f32x4u*>(src + off[i]);
    if (TR) {
#pragma unroll
      for (int i = 0; i < 3; ++i) t[set][i] = tr[q * 192 + 64 * i + lane];
    }
  };
  float acc = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (w + d * nw < units) load(w + d * nw, d);
  long u = w;
  int k = 0;
  for (; u < units; u += nw, ++k) {
    const int set = k % D;
    f32x4 c[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) c[i] = v[set][i];
    if (TR) {
#pragma unroll
      for (int i = 0; i < 3; ++i) acc += t[set][i][0];
    }
    if (LDS) {
      f32x4* st = stage[wave][k & 1];
#pragma unroll
      for (int i = 0; i < 3; ++i) st[64 * i + lane] = c[i];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < 3; ++i) c[i] = st[64 * i + ((lane + 1) & 63)];
    }
    if (u + D * nw < units) load(u + D * nw, set);
    const long q = u / SPANS;
    const int s = int(u - q * SPANS);
    float* dst = out + q * 4 * VS + 3 * 64 * s;
#pragma unroll
    for (int i = 0; i < 3; ++i) *reinterpret_cast<f32x4u*>(dst + off[i]) = c[i] * 2.f;
  }
  if (acc == 1234.5f) sink[0] = acc;
}

template <int TR, int LDS, int D>
void run(const float* a, const f32x4* tr, float* o, float* sink, long n, int n_cu) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL((unit_stream<TR, LDS, D>), dim3(n_cu), dim3(256), 0, 0, a, tr, o, sink, n);
  CK(hipEventRecord(e0));
  const int reps = 100;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((unit_stream<TR, LDS, D>), dim3(n_cu), dim3(256), 0, 0, a, tr, o, sink, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double rows = 2.0 * double(n) * SPANS * 64 * 12;
  printf("transforms=%d lds=%d depth=%d  %.4f ms  rows %.0f GB/s  (x %.4f = 778-vertex ms)\n", TR, LDS, D, ms,
         rows / ms * 1e-6, ms * NV / (SPANS * 64.0));
}

int main() {
  const long n = 65536;
  float *a, *o, *sink;
  f32x4* tr;
  CK(hipMalloc(&a, size_t(n) * VS * 4));
  CK(hipMalloc(&o, size_t(n) * VS * 4));
  CK(hipMalloc(&tr, size_t(n) * 192 * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0x3c, size_t(n) * VS * 4));
  CK(hipMemset(tr, 0x3c, size_t(n) * 192 * 4));
  int n_cu = 0;
  CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 0, 1>(a, tr, o, sink, n, n_cu);
    run<0, 0, 2>(a, tr, o, sink, n, n_cu);
    run<0, 0, 3>(a, tr, o, sink, n, n_cu);
    run<1, 0, 1>(a, tr, o, sink, n, n_cu);
    run<1, 0, 2>(a, tr, o, sink, n, n_cu);
    run<1, 0, 3>(a, tr, o, sink, n, n_cu);
    run<0, 1, 2>(a, tr, o, sink, n, n_cu);
    run<1, 1, 2>(a, tr, o, sink, n, n_cu);
    run<1, 1, 3>(a, tr, o, sink, n, n_cu);
  }
  return 0;
}
