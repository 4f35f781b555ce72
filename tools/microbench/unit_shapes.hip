// Microbenchmark: does the standalone LBS's unit SHAPE set its stream rate?
// skin_pair streams units of 4 hand rows x 64 vertices (four 768-B segments
// 9,336 B apart).  Here the same bytes per unit (3 KB in, 3 KB out, 3 float4
// per lane, one wave per SIMD, grid-stride order with XCD-aware worker ids,
// D units in flight in register sets) in other shapes over the
// [65,536][778][3] f32 layout (full 64-vertex spans only, 768 of 778
// vertices, as unit_stream.hip):
//   R = 4: 4 rows x 64 vertices (skin_pair's unit)
//   R = 2: 2 rows x 128 vertices
//   R = 1: 1 row x 256 vertices (one contiguous 3-KB segment)
//   R = 0: flat 3-KB chunks of the whole array (no row structure)
// with optionally the unit's transforms re-read (768 B per hand: 3 KB for 4
// rows, as skin_pair does; 768 B for one row).
// Build: hipcc --offload-arch=gfx950 -O3 -o unit_shapes unit_shapes.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
constexpr int NV = 778, VS = 3 * NV;

template <int R, int TR, int D>
__global__ __launch_bounds__(256, 1) void unit_shapes(const float* __restrict__ in, const f32x4* __restrict__ tr,
                                                      float* __restrict__ out, float* __restrict__ sink, long n) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long b = blockIdx.x, nb = gridDim.x;
  const long w = ((nb % 8) ? b : (b % 8) * (nb / 8) + b / 8) * 4 + wave, nw = nb * 4;
  // units: R rows x (256 / R) vertices; per group of R hands 768 / (256 / R) = 3 R units
  constexpr int RR = R == 0 ? 1 : R;
  constexpr int SEG = 3 * 256 / RR;                 // floats per row segment
  constexpr int UPG = 3 * RR;                       // units per group of RR hands (full spans)
  const long units = R == 0 ? n * VS / 768 : n / RR * UPG;
  int off[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int idx = 4 * (64 * i + lane);            // float index within the unit's 768 floats
    off[i] = R == 0 ? idx : (idx / SEG) * VS + idx % SEG;
  }
  auto base = [&](long u) -> long {
    if (R == 0) return u * 768;
    const long g = u / UPG;
    const int s = int(u - g * UPG);
    return g * RR * VS + long(s) * SEG;
  };
  f32x4 v[D][3], t[D][3];
  auto load = [&](long u, int set) {
    const float* src = in + base(u);
#pragma unroll
    for (int i = 0; i < 3; ++i) v[set][i] = *reinterpret_cast<const f32x4u*>(src + off[i]);
    if (TR) {
      const long h = R == 0 ? (u * 768) / VS : (u / UPG) * RR;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (64 * i + lane < 48 * RR) t[set][i] = tr[h * 48 + 64 * i + lane];
    }
  };
  float acc = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (w + d * nw < units) load(w + d * nw, d);
  int k = 0;
  for (long u = w; u < units; u += nw, ++k) {
    const int set = k % D;
    f32x4 c[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) c[i] = v[set][i];
    if (TR) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (64 * i + lane < 48 * RR) acc += t[set][i][0];
    }
    if (u + D * nw < units) load(u + D * nw, set);
    float* dst = out + base(u);
#pragma unroll
    for (int i = 0; i < 3; ++i) *reinterpret_cast<f32x4u*>(dst + off[i]) = c[i] * 2.f;
  }
  if (acc == 1234.5f) sink[0] = acc;
}

template <int R, int TR, int D>
void run(const float* a, const f32x4* tr, float* o, float* sink, long n, int n_cu) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL((unit_shapes<R, TR, D>), dim3(n_cu), dim3(256), 0, 0, a, tr, o, sink, n);
  CK(hipEventRecord(e0));
  const int reps = 200;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((unit_shapes<R, TR, D>), dim3(n_cu), dim3(256), 0, 0, a, tr, o, sink, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipGetLastError());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = 2.0 * double(n) * 768 * 12;  // 768 of 778 vertices in and out
  printf("{\"rows\": %d, \"transforms\": %d, \"depth\": %d, \"ms\": %.4f, \"GBs\": %.0f, \"ms_778\": %.4f}\n", R, TR, D,
         ms, bytes / ms * 1e-6, ms * NV / 768.0);
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
    run<4, 1, 2>(a, tr, o, sink, n, n_cu);
    run<2, 1, 2>(a, tr, o, sink, n, n_cu);
    run<1, 1, 2>(a, tr, o, sink, n, n_cu);
    run<0, 1, 2>(a, tr, o, sink, n, n_cu);
    run<4, 0, 2>(a, tr, o, sink, n, n_cu);
    run<1, 0, 2>(a, tr, o, sink, n, n_cu);
    run<0, 0, 2>(a, tr, o, sink, n, n_cu);
    run<4, 1, 3>(a, tr, o, sink, n, n_cu);
    run<1, 1, 3>(a, tr, o, sink, n, n_cu);
  }
  return 0;
}
