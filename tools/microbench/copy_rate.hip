// Microbenchmark: the HBM copy ceiling for the standalone LBS's byte stream
// (612 MB in, 612 MB out: 65,536 hands x 9,336 B), as a function of the
// bytes each wave keeps in flight and of the waves per CU.
// Kernel: every wave takes chunks of 64 x U float4 in grid-stride order
// (XCD-aware wave ids), issues the U loads of chunk i + 1 before the U stores
// of chunk i (a register double buffer), NT = nontemporal loads and stores.
// Question: how far below a well-fed copy is skin_pair's 0.27 ms?
// Build: hipcc --offload-arch=gfx950 -O3 -o copy_rate copy_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U, int NT>
__device__ __forceinline__ void ld(f32x4 (&v)[U], const f32x4* p, int lane) {
#pragma unroll
  for (int i = 0; i < U; ++i) {
    if (NT) v[i] = __builtin_nontemporal_load(p + 64 * i + lane);
    else v[i] = p[64 * i + lane];
  }
}
template <int U, int NT>
__device__ __forceinline__ void st(const f32x4 (&v)[U], f32x4* p, int lane) {
#pragma unroll
  for (int i = 0; i < U; ++i) {
    if (NT) __builtin_nontemporal_store(v[i] * 2.f, p + 64 * i + lane);
    else p[64 * i + lane] = v[i] * 2.f;
  }
}

template <int U, int B, int NT>
__global__ __launch_bounds__(256, B) void copy_chunks(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                                       long chunks) {
  const int lane = threadIdx.x & 63;
  const long b = blockIdx.x, nb = gridDim.x;
  const long w = ((nb % 8) ? b : (b % 8) * (nb / 8) + b / 8) * 4 + (threadIdx.x >> 6), nw = nb * 4;
  f32x4 v[U], c[U];
  long u = w;
  if (u < chunks) ld<U, NT>(v, in + u * 64 * U, lane);
  for (; u < chunks; u += nw) {
#pragma unroll
    for (int i = 0; i < U; ++i) c[i] = v[i];
    if (u + nw < chunks) ld<U, NT>(v, in + (u + nw) * 64 * U, lane);
    st<U, NT>(c, out + u * 64 * U, lane);
  }
}

template <int U, int B, int NT>
void run(const f32x4* a, f32x4* o, long n4, int n_cu) {
  const long chunks = n4 / (64 * U);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(n_cu * B);
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL((copy_chunks<U, B, NT>), grid, dim3(256), 0, 0, a, o, chunks);
  CK(hipEventRecord(e0));
  const int reps = 100;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((copy_chunks<U, B, NT>), grid, dim3(256), 0, 0, a, o, chunks);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = 2.0 * double(chunks) * 64 * U * 16;
  printf("U=%2d (%2d KB/wave in flight)  waves/SIMD=%d  nt=%d  %.4f ms  %.0f GB/s  (%.4f ms per 1.274 GB)\n", U,
         U * 64 * 16 * 2 / 1024, B, NT, ms, bytes / ms * 1e-6, 1.274e9 / (bytes / ms * 1e-3) );
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const long n4 = 65536L * 9336 / 16;  // 612 MB each way
  f32x4 *a, *o;
  CK(hipMalloc(&a, n4 * 16));
  CK(hipMalloc(&o, n4 * 16));
  CK(hipMemset(a, 0x3c, n4 * 16));
  int n_cu = 0;
  CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  for (int rep = 0; rep < 2; ++rep) {
    run<1, 1, 0>(a, o, n4, n_cu);
    run<1, 2, 0>(a, o, n4, n_cu);
    run<1, 4, 0>(a, o, n4, n_cu);
    run<1, 8, 0>(a, o, n4, n_cu);
    run<2, 1, 0>(a, o, n4, n_cu);
    run<2, 2, 0>(a, o, n4, n_cu);
    run<2, 4, 0>(a, o, n4, n_cu);
    run<3, 1, 0>(a, o, n4, n_cu);
    run<3, 2, 0>(a, o, n4, n_cu);
    run<4, 1, 0>(a, o, n4, n_cu);
    run<4, 2, 0>(a, o, n4, n_cu);
    run<4, 4, 0>(a, o, n4, n_cu);
    run<8, 1, 0>(a, o, n4, n_cu);
    run<8, 2, 0>(a, o, n4, n_cu);
    run<2, 2, 1>(a, o, n4, n_cu);
    run<4, 1, 1>(a, o, n4, n_cu);
    run<4, 2, 1>(a, o, n4, n_cu);
    run<8, 1, 1>(a, o, n4, n_cu);
  }
  return 0;
}
