// pk_load.hip -- the round-1 f16x3 fault shape (pk_shape.hip) under memory
// load from the same wave (DESIGN.md section 4, f16x3 lanes-48..63 fault).
//
// pk_shape.hip runs the failing instruction sequence in isolation:
//   P  v_pk_fma_f32 v[52:53], ...                      (C's source)
//   M1 v_mfma_f32_16x16x32_f16 ...
//   F  two v_fma_f32
//   C  v_pk_fma_f32 v[76:77], v[52:53], s[20:21], 0 op_sel_hi:[1,1,0]   (checked)
//   C2 v_pk_fma_f32 ...
//   M2 v_mfma_f32_16x16x32_f16 ...
//   M3 v_mfma_f32_16x16x32_f16 v[52:55], ...           (overwrites C's source)
// and finds no wrong value.  In the failing kernel the wave had up to 8
// global_store_dwordx3 of the previous rows queued (the failures only in the
// instantiations that store rest_verts too, at a rate that follows memory
// load).  Here each iteration first queues S point stores (dwordx3, like the
// kernel's) and/or L dwordx4 loads that land during the shape, then runs it.
// MODE bits: 1 = stores before, 2 = loads in flight, 4 = without M3 (control),
// 8 = C with a VGPR multiplier instead of the SGPR pair (control).
//
//   hipcc --offload-arch=gfx950 -O3 -o pk_load pk_load.hip && ./pk_load
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int kIters = 128;
constexpr long kBufF4 = 1L << 25;  // 512 MB store / load region (float4s)

#define SETUP                                                                                   \
  "v_mov_b32 v40, %2\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, 0.5\n\tv_mov_b32 v43, 0.5\n\t"        \
  "v_mov_b32 v44, %4\n\tv_mov_b32 v45, %5\n\tv_mov_b32 v52, 0x49742400\n\tv_mov_b32 v53, 0x49742400\n\t" \
  "v_mov_b32 v46, 2.0\n\tv_mov_b32 v47, 2.0\n\ts_mov_b32 s20, 2.0\n\ts_mov_b32 s21, 2.0\n\t"       \
  "v_mov_b32 v60, 0x3c003c00\n\tv_mov_b32 v61, 0x3c003c00\n\tv_mov_b32 v62, 0x3c003c00\n\t"       \
  "v_mov_b32 v63, 0x3c003c00\n\tv_mov_b32 v64, 1.0\n\tv_mov_b32 v65, 1.0\n\tv_mov_b32 v66, 1.0\n\t" \
  "v_mov_b32 v67, 1.0\n\tv_mov_b32 v48, 0\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\tv_mov_b32 v51, 0\n\ts_nop 7\n\t"
#define STORES                                                                                   \
  "global_store_dwordx3 %8, v[80:82], off\n\tglobal_store_dwordx3 %8, v[84:86], off offset:256\n\t" \
  "global_store_dwordx3 %8, v[88:90], off offset:512\n\tglobal_store_dwordx3 %8, v[92:94], off offset:768\n\t" \
  "global_store_dwordx3 %8, v[96:98], off offset:1024\n\tglobal_store_dwordx3 %8, v[100:102], off offset:1280\n\t" \
  "global_store_dwordx3 %8, v[104:106], off offset:1536\n\tglobal_store_dwordx3 %8, v[108:110], off offset:1792\n\t"
#define LOADS                                                                                    \
  "global_load_dwordx4 v[112:115], %9, off\n\tglobal_load_dwordx4 v[116:119], %9, off offset:1024\n\t" \
  "global_load_dwordx4 v[120:123], %9, off offset:2048\n\tglobal_load_dwordx4 v[124:127], %9, off offset:3072\n\t"
#define P_ "v_pk_fma_f32 v[52:53], v[40:41], v[42:43], v[44:45] op_sel_hi:[1,0,1]\n\t"
#define M1 "v_mfma_f32_16x16x32_f16 v[56:59], v[60:63], v[60:63], v[64:67]\n\t"
#define F_ "v_fma_f32 v68, v40, v42, v44\n\tv_fma_f32 v69, v41, v42, v45\n\t"
#define C_S "v_pk_fma_f32 v[76:77], v[52:53], s[20:21], 0 op_sel_hi:[1,1,0]\n\t"
#define C_V "v_pk_fma_f32 v[76:77], v[52:53], v[46:47], 0 op_sel_hi:[1,1,0]\n\t"
#define C2 "v_pk_fma_f32 v[70:71], v[68:69], s[20:21], 0 op_sel_hi:[1,1,0]\n\t"
#define M2 "v_mfma_f32_16x16x32_f16 v[72:75], v[60:63], v[60:63], v[64:67]\n\t"
#define M3 "v_mfma_f32_16x16x32_f16 v[52:55], v[60:63], v[60:63], v[48:51]\n\t"
#define TAIL "s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t" \
             "v_mov_b32 %0, v76\n\tv_mov_b32 %1, v77\n\tv_mov_b32 %6, v70\n\tv_mov_b32 %7, v71\n\t"
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", \
             "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65",  \
             "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v112", \
             "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123",     \
             "v124", "v125", "v126", "v127", "s20", "s21", "memory"

template <int MODE>
__device__ __forceinline__ void shape(float a0, float a1, float c0, float c1, float& x, float& y, float& x2,
                                      float& y2, float* st, const float* ld) {
#define RUN(body)                                                                                 \
  asm volatile(SETUP body TAIL                                                                     \
               : "=v"(x), "=v"(y), "+v"(a0), "+v"(a1), "+v"(c0), "+v"(c1), "=v"(x2), "=v"(y2)     \
               : "v"(st), "v"(ld)                                                                  \
               : CLOB)
#define SEQ(pre, c, m3) RUN(pre P_ M1 F_ c C2 M2 m3)
  constexpr bool kS = MODE & 1, kL = MODE & 2, kNoM3 = MODE & 4, kVgpr = MODE & 8;
  if constexpr (kS && kL) {
    if constexpr (kVgpr) SEQ(STORES LOADS, C_V, M3);
    else if constexpr (kNoM3) SEQ(STORES LOADS, C_S, "");
    else SEQ(STORES LOADS, C_S, M3);
  } else if constexpr (kS) {
    if constexpr (kVgpr) SEQ(STORES, C_V, M3);
    else if constexpr (kNoM3) SEQ(STORES, C_S, "");
    else SEQ(STORES, C_S, M3);
  } else if constexpr (kL) {
    SEQ(LOADS, C_S, M3);
  } else {
    SEQ("", C_S, M3);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void pk_kernel(unsigned* __restrict__ bad, float* __restrict__ sbuf,
                                                 const float* __restrict__ lbuf) {
  const int lane = threadIdx.x & 63;
  const long wave = (long(blockIdx.x) * 256 + threadIdx.x) >> 6;
  unsigned nb[4] = {0, 0, 0, 0};
  for (int it = 0; it < kIters; ++it) {
    const float a0 = float(lane + it), a1 = float(lane - it), c0 = 0.25f * float(it), c1 = -0.5f * float(lane);
    // each (wave, iteration) writes / reads its own 2-KB / 4-KB region, spread over 512 MB
    const long region = (wave * kIters + it) * 2654435761L & (kBufF4 / 512 - 1);
    float* st = sbuf + region * 2048 + lane * 4;
    const float* ld = lbuf + region * 2048 + lane * 4;
    float x, y, x2, y2;
    shape<MODE>(a0, a1, c0, c1, x, y, x2, y2, st, ld);
    const float px = fmaf(a0, 0.5f, c0), py = fmaf(a1, 0.5f, c1);
    nb[0] += x != px * 2.0f;
    nb[1] += y != py * 2.0f;
    nb[2] += x2 != px * 2.0f;
    nb[3] += y2 != py * 2.0f;
  }
  for (int k = 0; k < 4; ++k) atomicAdd(&bad[4 * (lane >> 4) + k], nb[k]);
}

template <int MODE>
int run(unsigned* d, float* sbuf, const float* lbuf, const char* name, int blocks) {
  CHECK(hipMemset(d, 0, 16 * sizeof(unsigned)));
  for (int r = 0; r < 4; ++r) hipLaunchKernelGGL(pk_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, d, sbuf, lbuf);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  unsigned h[16];
  CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  printf("%-36s blocks %5d: C lo/hi, C2 lo/hi wrong per quarter:", name, blocks);
  for (int q = 0; q < 4; ++q) printf("  q%d %u/%u %u/%u", q, h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]);
  printf("  (of %ld)\n", 4L * blocks * 4 * 16 * kIters);
  return 0;
}

int main() {
  unsigned* d;
  float *sbuf, *lbuf;
  CHECK(hipMalloc(&d, 16 * sizeof(unsigned)));
  CHECK(hipMalloc(&sbuf, kBufF4 * 16));
  CHECK(hipMalloc(&lbuf, kBufF4 * 16));
  CHECK(hipMemset(lbuf, 0, kBufF4 * 16));
  int rc = 0;
  for (int blocks : {1024, 4096}) {
    rc |= run<0>(d, sbuf, lbuf, "shape alone", blocks);
    rc |= run<1>(d, sbuf, lbuf, "8 point stores before", blocks);
    rc |= run<2>(d, sbuf, lbuf, "4 loads in flight", blocks);
    rc |= run<3>(d, sbuf, lbuf, "stores + loads", blocks);
    rc |= run<1 | 4>(d, sbuf, lbuf, "stores, no M3 (control)", blocks);
    rc |= run<1 | 8>(d, sbuf, lbuf, "stores, VGPR multiplier (control)", blocks);
    rc |= run<3 | 4>(d, sbuf, lbuf, "stores + loads, no M3 (control)", blocks);
    rc |= run<3 | 8>(d, sbuf, lbuf, "stores + loads, VGPR mult (control)", blocks);
  }
  return rc;
}
