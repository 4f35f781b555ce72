// Microbenchmark: HBM copy bandwidth of (R hand rows x V vertices) units over
// the MANO vertex layout ([n][778][3] f32, 65,536 hands, rows 9,336 B apart),
// grid-stride unit order, the next unit's rows loaded before the current one
// is stored (skin_span's register prefetch), B blocks of 4 waves per CU.
// Question: does a unit of fewer rows (a more compact chip-wide window) or
// fewer waves stream closer to the flat-copy ceiling?
// Build: hipcc --offload-arch=gfx950 -O3 -o span_rows span_rows.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
constexpr int NV = 778, VS = 3 * NV;

template <int R, int V>
struct Unit {
  static constexpr int kRowF4 = 3 * V / 4;           // float4 per row segment
  static constexpr int kF4 = R * kRowF4 / 64;        // float4 per lane
  static constexpr int kSpans = NV / V;              // full spans per row (tail not copied)
  static_assert(R * kRowF4 % 64 == 0, "unit must be whole wave sweeps");
};

// ORDER 0: grid-stride over (tile, span) units; 1: a wave takes tiles
// w, w + nw, ... and sweeps all spans of each (tile-major per wave).
template <int R, int V, int B, int ORDER = 0>
__global__ __launch_bounds__(256, B) void span_rows(const float* __restrict__ in, float* __restrict__ out,
                                                    long n) {
  using U = Unit<R, V>;
  const int lane = threadIdx.x & 63;
  // XCD-aware worker id (consecutive ids on one XCD), as skin_span
  const long b = blockIdx.x, nb = gridDim.x;
  const long w = ((b % 8) * (nb / 8) + b / 8) * 4 + (threadIdx.x >> 6), nw = nb * 4;
  const long units = n / R * U::kSpans;
  f32x4u v[U::kF4];
  auto load = [&](long u) {
    const long t = u / U::kSpans;
    const int s = int(u - t * U::kSpans);
    const float* src = in + t * R * VS + 3 * V * s;
#pragma unroll
    for (int i = 0; i < U::kF4; ++i) {
      const int idx = 64 * i + lane, row = idx / U::kRowF4, c4 = idx - U::kRowF4 * row;
      v[i] = *reinterpret_cast<const f32x4u*>(src + row * VS + 4 * c4);
    }
  };
  auto next = [&](long u) {
    if (ORDER == 0) return u + nw;
    const long t = u / U::kSpans;
    const int s = int(u - t * U::kSpans);
    return s + 1 < U::kSpans ? u + 1 : (t + nw) * U::kSpans;
  };
  const long u0 = ORDER == 0 ? w : w * U::kSpans;
  if (u0 < units) load(u0);
  for (long u = u0; u < units; u = next(u)) {
    f32x4u c[U::kF4];
#pragma unroll
    for (int i = 0; i < U::kF4; ++i) c[i] = v[i];
    if (next(u) < units) load(next(u));
    const long t = u / U::kSpans;
    const int s = int(u - t * U::kSpans);
    float* dst = out + t * R * VS + 3 * V * s;
#pragma unroll
    for (int i = 0; i < U::kF4; ++i) {
      const int idx = 64 * i + lane, row = idx / U::kRowF4, c4 = idx - U::kRowF4 * row;
      *reinterpret_cast<f32x4u*>(dst + row * VS + 4 * c4) = c[i] * 2.f;
    }
  }
}

__global__ __launch_bounds__(256) void copy16(const f32x4* __restrict__ in, f32x4* __restrict__ out, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += gridDim.x * 256L) out[i] = in[i] * 2.f;
}

template <int R, int V, int B, int ORDER = 0>
void run(const float* a, float* o, long n, int n_cu) {
  using U = Unit<R, V>;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL((span_rows<R, V, B, ORDER>), dim3(n_cu * B), dim3(256), 0, 0, a, o, n);
  CK(hipEventRecord(e0));
  const int reps = 100;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((span_rows<R, V, B, ORDER>), dim3(n_cu * B), dim3(256), 0, 0, a, o, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = 2.0 * double(n) * U::kSpans * V * 12;
  printf("%s R=%2d V=%3d blocks/CU=%d  f4/lane=%2d  %.4f ms  %.0f GB/s  (x %.4f = full-row ms)\n", ORDER ? "tile-major " : "grid-stride", R, V, B, U::kF4, ms,
         bytes / ms * 1e-6, ms * NV / (U::kSpans * V));
}

int main() {
  const long n = 65536;
  const size_t nf = size_t(n) * VS;
  float *a, *o;
  CK(hipMalloc(&a, nf * 4));
  CK(hipMalloc(&o, nf * 4));
  CK(hipMemset(a, 0, nf * 4));
  int n_cu = 0;
  CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  for (int rep = 0; rep < 2; ++rep) {
    {
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      const long n4 = long(nf / 4);
      for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(copy16, dim3(n_cu * 8), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)o, n4);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(copy16, dim3(n_cu * 8), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)o, n4);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("flat float4 copy           %.4f ms  %.0f GB/s\n", ms / 100, 2.0 * nf * 4 / (ms / 100) * 1e-6);
    }
    run<16, 64, 1>(a, o, n, n_cu);
    run<16, 64, 2>(a, o, n, n_cu);
    run<8, 64, 1>(a, o, n, n_cu);
    run<8, 64, 2>(a, o, n, n_cu);
    run<4, 64, 1>(a, o, n, n_cu);
    run<4, 64, 2>(a, o, n, n_cu);
    run<4, 256, 1>(a, o, n, n_cu);
    run<4, 256, 2>(a, o, n, n_cu);
    run<4, 128, 1>(a, o, n, n_cu);
    run<4, 128, 2>(a, o, n, n_cu);
    run<2, 256, 1>(a, o, n, n_cu);
    run<2, 256, 2>(a, o, n, n_cu);
    run<1, 256, 1>(a, o, n, n_cu);
    run<1, 256, 2>(a, o, n, n_cu);
    run<16, 16, 1>(a, o, n, n_cu);
    run<16, 16, 2>(a, o, n, n_cu);
    run<4, 64, 1, 1>(a, o, n, n_cu);
    run<4, 64, 2, 1>(a, o, n, n_cu);
    run<16, 64, 1, 1>(a, o, n, n_cu);
    run<8, 64, 1, 1>(a, o, n, n_cu);
  }
  return 0;
}
