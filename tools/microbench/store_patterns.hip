// Microbenchmark: HBM store / copy patterns of the MANO output ([n][778][3] f32).
// Build: hipcc --offload-arch=gfx950 -O3 -o store_patterns store_patterns.hip
// Every variant writes (or copies) the same 65,536 x 9,336 B; no arithmetic, so
// the time is the memory path's for that access pattern.
//   rows12    the kernels' pattern: a wave owns 16 hands x 16-vertex groups;
//             lane (q, col) stores 12 B (dwordx3) for hands 4q + r, r = 0..3
//   rows12nt  same with nontemporal stores
//   lds16     the wave stages its 16 x 192 B tile in LDS, then stores each
//             hand row with 16-B lanes (12 lanes per 192-B row)
//   lds16x4   the same over 4 consecutive groups (768 B per hand row)
//   win32     rows12's units, but each hand row's 48 floats leave as 12 dwordx4
//             from the 32-B-aligned position at or below the segment start
//             (the sector-aligned window a carry of <= 6 floats per hand row
//             from the previous group would give; same bytes, aligned)
//   flat16    contiguous float4 stream (the write ceiling)
//   copy12    rows12 read + rows12 write (skin's pattern), copy16 float4 copy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NV = 778, VS = 3 * NV, NG = 49;

__device__ __forceinline__ void range(long units, long w, long nw, long& b, long& e) {
  b = w * units / nw; e = (w + 1) * units / nw;
}

template <bool kNT>
__global__ __launch_bounds__(256) void rows12(float* __restrict__ out, long n) {
  const int lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  long u, ue;
  range((n / 16) * NG, blockIdx.x * 4L + (threadIdx.x >> 6), gridDim.x * 4L, u, ue);
  for (; u < ue; ++u) {
    const long tile = u / NG; const int g = int(u - tile * NG);
    const int vb = min(16 * g, NV - 16);
    float* base = out + tile * 16 * VS + 3 * (vb + col);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      f32x3 v = {float(u), float(r), float(lane)};
      f32x3* p = reinterpret_cast<f32x3*>(base + (4 * q + r) * VS);
      if (kNT) __builtin_nontemporal_store(v, p); else *p = v;
    }
  }
}

template <int kG>
__global__ __launch_bounds__(256) void lds16(float* __restrict__ out, long n) {
  __shared__ float tile_s[4][16 * 48 * kG + 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  float* s = tile_s[wave];
  long u, ue;
  const int ngk = (NG + kG - 1) / kG;
  range((n / 16) * ngk, blockIdx.x * 4L + wave, gridDim.x * 4L, u, ue);
  for (; u < ue; ++u) {
    const long tile = u / ngk; const int gk = int(u - tile * ngk);
    int vb = 16 * kG * gk; if (vb > NV - 16 * kG) vb = NV - 16 * kG;
    // stage: lane (q, col) of sub-group i writes hand 4q + r, vertex 16 i + col
#pragma unroll
    for (int i = 0; i < kG; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* d = s + (4 * q + r) * (48 * kG) + 3 * (16 * i + col);
        d[0] = float(u); d[1] = float(r); d[2] = float(lane);
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    // store: a hand row is 48 kG floats = 12 kG float4
    float* base = out + tile * 16 * VS + 3 * vb;
    constexpr int per_row = 12 * kG;
    for (int i = lane; i < 16 * per_row; i += 64) {
      const int h = i / per_row, c = i - h * per_row;
      const float* sp = s + h * (48 * kG) + 4 * c;
      f32x4 v = {sp[0], sp[1], sp[2], sp[3]};
      float* dp = base + h * VS + 4 * c;
      dp[0] = v[0]; dp[1] = v[1]; dp[2] = v[2]; dp[3] = v[3];
    }
  }
}

__global__ __launch_bounds__(256) void win32(float* __restrict__ out, long n) {
  const int lane = threadIdx.x & 63;
  long u, ue;
  range((n / 16) * NG, blockIdx.x * 4L + (threadIdx.x >> 6), gridDim.x * 4L, u, ue);
  for (; u < ue; ++u) {
    const long tile = u / NG; const int g = int(u - tile * NG);
    const int vb = min(16 * g, NV - 16);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int idx = lane + 64 * i, h = idx / 12, c = idx - 12 * h;
      long start = (tile * 16 + h) * VS + 3 * vb;
      start -= start & 7;  // 32-B aligned window start
      *reinterpret_cast<f32x4*>(out + start + 4 * c) = f32x4{float(u), float(h), float(c), 1.f};
    }
  }
}

// rows12set: blend_skin_h3's order -- a block of 8 waves holds 8 16-hand
// tiles (128 consecutive hands) and walks the 49 groups; at a time its waves
// write the same 192-B column span of 128 rows.
__global__ __launch_bounds__(512) void rows12set(float* __restrict__ out, long n) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  long u, ue;
  range((n / 128) * NG, blockIdx.x, gridDim.x, u, ue);
  for (; u < ue; ++u) {
    const long set = u / NG; const int g = int(u - set * NG);
    const int vb = min(16 * g, NV - 16);
    float* base = out + (set * 128 + wave * 16) * VS + 3 * (vb + col);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<f32x3*>(base + (4 * q + r) * VS) = f32x3{float(u), float(r), float(lane)};
  }
}

// rows12vs: the vertex-stationary order -- a block of 7 waves owns 7
// consecutive groups (set b % 7 of the 49) and walks a range of 16-hand
// tiles; at a time its waves write one 1,344-B span of each of 16 rows.
__global__ __launch_bounds__(448) void rows12vs(float* __restrict__ out, long n) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  const int gset = blockIdx.x % 7;
  const long nr = gridDim.x / 7;
  long t, te;
  range(n / 16, blockIdx.x / 7, nr, t, te);
  const int vb = min(16 * (7 * gset + wave), NV - 16);
  for (; t < te; ++t) {
    float* base = out + t * 16 * VS + 3 * (vb + col);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<f32x3*>(base + (4 * q + r) * VS) = f32x3{float(t), float(r), float(lane)};
  }
}

__global__ __launch_bounds__(256) void flat16(f32x4* __restrict__ out, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += gridDim.x * 256L) out[i] = f32x4{1, 2, 3, float(i)};
}

__global__ __launch_bounds__(256) void copy12(const float* __restrict__ in, float* __restrict__ out, long n) {
  const int lane = threadIdx.x & 63, q = lane >> 4, col = lane & 15;
  long u, ue;
  range((n / 16) * NG, blockIdx.x * 4L + (threadIdx.x >> 6), gridDim.x * 4L, u, ue);
  for (; u < ue; ++u) {
    const long tile = u / NG; const int g = int(u - tile * NG);
    const int vb = min(16 * g, NV - 16);
    const long off = tile * 16 * VS + 3 * (vb + col);
    f32x3 v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = *reinterpret_cast<const f32x3*>(in + off + (4 * q + r) * VS);
#pragma unroll
    for (int r = 0; r < 4; ++r) *reinterpret_cast<f32x3*>(out + off + (4 * q + r) * VS) = v[r] * 2.f;
  }
}

__global__ __launch_bounds__(256) void copy16(const f32x4* __restrict__ in, f32x4* __restrict__ out, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += gridDim.x * 256L) out[i] = in[i] * 2.f;
}

int main() {
  const long n = 65536;
  const size_t nf = size_t(n) * VS;
  float *a, *b;
  CK(hipMalloc(&a, nf * 4)); CK(hipMalloc(&b, nf * 4));
  CK(hipMemset(a, 0, nf * 4)); CK(hipMemset(b, 0, nf * 4));
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 20; ++i) launch();
    CK(hipDeviceSynchronize());
    const int it = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < it; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
    printf("%-34s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  };
  const double W = double(nf) * 4;
  for (int bpc : {2, 4, 8}) {
    const unsigned g = unsigned(ncu * bpc);
    char nm[64];
    snprintf(nm, 64, "rows12 (%d blk/CU)", bpc);
    timeit(nm, W, [&] { hipLaunchKernelGGL(rows12<false>, dim3(g), dim3(256), 0, 0, b, n); });
    snprintf(nm, 64, "rows12nt (%d blk/CU)", bpc);
    timeit(nm, W, [&] { hipLaunchKernelGGL(rows12<true>, dim3(g), dim3(256), 0, 0, b, n); });
    snprintf(nm, 64, "lds16 (%d blk/CU)", bpc);
    timeit(nm, W, [&] { hipLaunchKernelGGL(lds16<1>, dim3(g), dim3(256), 0, 0, b, n); });
    snprintf(nm, 64, "lds16x4 (%d blk/CU)", bpc);
    timeit(nm, W, [&] { hipLaunchKernelGGL(lds16<4>, dim3(g), dim3(256), 0, 0, b, n); });
    snprintf(nm, 64, "win32 (%d blk/CU)", bpc);
    timeit(nm, W, [&] { hipLaunchKernelGGL(win32, dim3(g), dim3(256), 0, 0, b, n); });
    snprintf(nm, 64, "copy12 (%d blk/CU)", bpc);
    timeit(nm, 2 * W, [&] { hipLaunchKernelGGL(copy12, dim3(g), dim3(256), 0, 0, a, b, n); });
  }
  for (int bpc : {1, 2}) {
    char nm[64];
    snprintf(nm, 64, "rows12set (%d blk/CU, 8 waves)", bpc);
    timeit(nm, W, [&] { hipLaunchKernelGGL(rows12set, dim3(ncu * bpc), dim3(512), 0, 0, b, n); });
    const unsigned gvs = unsigned((ncu * bpc) / 7 * 7);
    snprintf(nm, 64, "rows12vs (%u blk, 7 waves)", gvs);
    timeit(nm, W, [&] { hipLaunchKernelGGL(rows12vs, dim3(gvs), dim3(448), 0, 0, b, n); });
  }
  timeit("flat16", W, [&] { hipLaunchKernelGGL(flat16, dim3(ncu * 8), dim3(256), 0, 0, (f32x4*)b, long(nf / 4)); });
  timeit("copy16", 2 * W, [&] { hipLaunchKernelGGL(copy16, dim3(ncu * 8), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, long(nf / 4)); });
  return 0;
}
