// store_war.hip -- can a VGPR that an in-flight VMEM store still has to read
// be overwritten by a later instruction on gfx950?  (the f16x3 fault)
//
// The round-1 failing blend_skin_h3 build ended each vertex group with 8
// global_store_dwordx3 whose data registers the NEXT group's ds_read_b128
// (LDS -> VGPR) overwrote right after a `s_waitcnt vmcnt(8) lgkmcnt(0)`
// barrier, i.e. with those stores possibly still queued.  This kernel
// reproduces that shape: each wave first queues kFill dwordx4 stores (memory
// back-pressure), then
//
//     global_store_dwordx3 v[addr], v[40:42], off      (the checked store)
//     <overwrite of v[40:43]>                           (no wait in between)
//
// with the overwrite by MODE: 0 v_mov_b32 (VALU), 1 ds_read_b128 (LDS load),
// 2 v_mfma_f32_16x16x32_f16 (MFMA result), 3 global_load_dwordx4 (VMEM load).
// The host checks every stored dword per 16-lane quarter.
//
//   hipcc --offload-arch=gfx950 -O3 -o store_war store_war.hip && ./store_war
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 64;
constexpr int kBlocks = 1024;
constexpr int kFill = 16;            // back-pressure stores per iteration
constexpr int kFillFloats = 1 << 26;  // 256 MB fill region

template <int MODE>
__global__ __launch_bounds__(256) void store_war_kernel(float* __restrict__ out, f32x4* __restrict__ fill,
                                                        const f32x4* __restrict__ src) {
  __shared__ f32x4 lds[256];
  const int lane = threadIdx.x & 63;
  lds[threadIdx.x] = f32x4{-1.f, -2.f, -3.f, -4.f};
  __syncthreads();
  const unsigned lds_addr = unsigned(threadIdx.x) * 16u;
  const int64_t gid = int64_t(blockIdx.x) * 256 + threadIdx.x;
  for (int it = 0; it < kIters; ++it) {
    // queue stores to spread-out lines of a large buffer
#pragma unroll
    for (int f = 0; f < kFill; ++f) {
      const int64_t idx = ((gid * kFill + f) * 977 + it * 131) & (kFillFloats / 4 - 1);
      fill[idx] = f32x4{float(f), 0.f, 0.f, 0.f};
    }
    float* dst = out + (int64_t(it) * kBlocks * 256 + gid) * 3;
    const float v0 = float(gid) + 0.25f, v1 = float(it) + 0.5f, v2 = float(lane) + 0.75f;
    if constexpr (MODE == 0) {
      asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v42, %3\n\ts_nop 4\n\t"
                   "global_store_dwordx3 %0, v[40:42], off\n\t"
                   "v_mov_b32 v40, -1.0\n\tv_mov_b32 v41, -1.0\n\tv_mov_b32 v42, -1.0\n\t"
                   :: "v"(dst), "v"(v0), "v"(v1), "v"(v2) : "v40", "v41", "v42", "v43", "memory");
    } else if constexpr (MODE == 1) {
      asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v42, %3\n\ts_nop 4\n\t"
                   "global_store_dwordx3 %0, v[40:42], off\n\t"
                   "ds_read_b128 v[40:43], %4\n\ts_waitcnt lgkmcnt(0)\n\t"
                   :: "v"(dst), "v"(v0), "v"(v1), "v"(v2), "v"(lds_addr) : "v40", "v41", "v42", "v43", "memory");
    } else if constexpr (MODE == 2) {
      asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v42, %3\n\t"
                   "v_mov_b32 v44, 0x3c003c00\n\tv_mov_b32 v45, 0x3c003c00\n\tv_mov_b32 v46, 0x3c003c00\n\t"
                   "v_mov_b32 v47, 0x3c003c00\n\ts_nop 4\n\t"
                   "global_store_dwordx3 %0, v[40:42], off\n\t"
                   "v_mfma_f32_16x16x32_f16 v[40:43], v[44:47], v[44:47], 0\n\ts_nop 7\n\ts_nop 7\n\t"
                   :: "v"(dst), "v"(v0), "v"(v1), "v"(v2) : "v40", "v41", "v42", "v43", "v44", "v45",
                      "v46", "v47", "memory");
    } else {
      const f32x4* s = src + (threadIdx.x & 255);
      asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v42, %3\n\ts_nop 4\n\t"
                   "global_store_dwordx3 %0, v[40:42], off\n\t"
                   "global_load_dwordx4 v[40:43], %4, off\n\ts_waitcnt vmcnt(0)\n\t"
                   :: "v"(dst), "v"(v0), "v"(v1), "v"(v2), "v"(s) : "v40", "v41", "v42", "v43", "memory");
    }
  }
}

template <int MODE>
int run(float* d_out, f32x4* d_fill, const f32x4* d_src, const char* name) {
  const size_t n = size_t(kIters) * kBlocks * 256 * 3;
  CHECK(hipMemset(d_out, 0, n * sizeof(float)));
  hipLaunchKernelGGL(store_war_kernel<MODE>, dim3(kBlocks), dim3(256), 0, 0, d_out, d_fill, d_src);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::vector<float> h(n);
  CHECK(hipMemcpy(h.data(), d_out, n * sizeof(float), hipMemcpyDeviceToHost));
  unsigned long bad[4][3] = {};
  for (int it = 0; it < kIters; ++it)
    for (int64_t gid = 0; gid < int64_t(kBlocks) * 256; ++gid) {
      const int lane = int(gid & 63);
      const float want[3] = {float(gid) + 0.25f, float(it) + 0.5f, float(lane) + 0.75f};
      const float* got = &h[(size_t(it) * kBlocks * 256 + gid) * 3];
      for (int c = 0; c < 3; ++c) bad[lane >> 4][c] += got[c] != want[c];
    }
  printf("%-26s wrong dwords (x,y,z) lanes 0-15 %lu,%lu,%lu  16-31 %lu,%lu,%lu  32-47 %lu,%lu,%lu  48-63 %lu,%lu,%lu  (of %lu each)\n",
         name, bad[0][0], bad[0][1], bad[0][2], bad[1][0], bad[1][1], bad[1][2], bad[2][0], bad[2][1], bad[2][2],
         bad[3][0], bad[3][1], bad[3][2], (unsigned long)kIters * kBlocks * 256 / 4);
  return 0;
}

int main() {
  float* d_out;
  f32x4 *d_fill, *d_src;
  CHECK(hipMalloc(&d_out, size_t(kIters) * kBlocks * 256 * 3 * sizeof(float)));
  CHECK(hipMalloc(&d_fill, size_t(kFillFloats) * sizeof(float)));
  CHECK(hipMalloc(&d_src, 256 * sizeof(f32x4)));
  CHECK(hipMemset(d_src, 0xff, 256 * sizeof(f32x4)));
  int rc = 0;
  for (int rep = 0; rep < 2; ++rep) {
    rc |= run<0>(d_out, d_fill, d_src, "v_mov_b32 overwrite");
    rc |= run<1>(d_out, d_fill, d_src, "ds_read_b128 overwrite");
    rc |= run<2>(d_out, d_fill, d_src, "v_mfma overwrite");
    rc |= run<3>(d_out, d_fill, d_src, "global_load_dwordx4 overwrite");
  }
  return rc;
}
