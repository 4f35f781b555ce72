// pk_shape.hip -- the exact instruction shape of the round-1 f16x3 fault, with
// ablations.  The failing blend_skin_h3 build computed the
// x coordinate of hand rows 14-15 as the LOW half of
//
//   v_pk_fma_f32 v[100:101], v[104:105], v[172:173], v[100:101] op_sel_hi:[1,0,1]   (P)
//   v_mfma_f32_16x16x32_f16 v[104:107], ..., v[160:163]                           (M1)
//   v_fma_f32 v130, ... ; v_fma_f32 v131, ...                                      (F)
//   v_pk_fma_f32 v[132:133], v[100:101], s[4:5], 0 op_sel_hi:[1,1,0]              (C)
//   v_pk_fma_f32 v[136:137], v[130:131], s[4:5], 0 op_sel_hi:[1,1,0]
//   v_mfma_f32_16x16x32_f16 v[120:123], ...                                        (M2)
//   v_mfma_f32_16x16x32_f16 v[100:103], ..., v[152:155]   <- writes C's source     (M3)
//
// and lanes 48-63 of the low half came out wrong.  This kernel runs that shape
// (registers renamed) and variants, and counts wrong x / y per lane quarter:
//   0 full shape            1 without M3 (no MFMA write of C's source)
//   2 C with a VGPR pair instead of s[4:5]      3 full shape, s_nop 1 after C
//   4 M3 in place (SrcC = D = C's source)       5 without M1
//
//   hipcc --offload-arch=gfx950 -O3 -o pk_shape pk_shape.hip && ./pk_shape
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

constexpr int kIters = 256;
constexpr int kBlocks = 512;

// v40:41 = (a0, a1); v42:43 = (b, -) (P: v[52:53] = v[40:41] * v42 + v[44:45]);
// v44:45 = (c0, c1); s[20:21] = (2, 2); C: v[54:55] = v[52:53] * 2 + 0.
#define SETUP                                                                                   \
  "v_mov_b32 v40, %2\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, 0.5\n\tv_mov_b32 v43, 0.5\n\t"        \
  "v_mov_b32 v44, %4\n\tv_mov_b32 v45, %5\n\tv_mov_b32 v52, 0x49742400\n\tv_mov_b32 v53, 0x49742400\n\t" \
  "v_mov_b32 v46, 2.0\n\tv_mov_b32 v47, 2.0\n\ts_mov_b32 s20, 2.0\n\ts_mov_b32 s21, 2.0\n\t"       \
  "v_mov_b32 v60, 0x3c003c00\n\tv_mov_b32 v61, 0x3c003c00\n\tv_mov_b32 v62, 0x3c003c00\n\t"       \
  "v_mov_b32 v63, 0x3c003c00\n\tv_mov_b32 v64, 1.0\n\tv_mov_b32 v65, 1.0\n\tv_mov_b32 v66, 1.0\n\t" \
  "v_mov_b32 v67, 1.0\n\tv_mov_b32 v48, 0\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\tv_mov_b32 v51, 0\n\ts_nop 7\n\t"
#define P_ "v_pk_fma_f32 v[52:53], v[40:41], v[42:43], v[44:45] op_sel_hi:[1,0,1]\n\t"
#define M1 "v_mfma_f32_16x16x32_f16 v[56:59], v[60:63], v[60:63], v[64:67]\n\t"
#define F_ "v_fma_f32 v68, v40, v42, v44\n\tv_fma_f32 v69, v41, v42, v45\n\t"
#define C_S "v_pk_fma_f32 v[76:77], v[52:53], s[20:21], 0 op_sel_hi:[1,1,0]\n\t"
#define C_V "v_pk_fma_f32 v[76:77], v[52:53], v[46:47], 0 op_sel_hi:[1,1,0]\n\t"
#define C2 "v_pk_fma_f32 v[70:71], v[68:69], s[20:21], 0 op_sel_hi:[1,1,0]\n\t"
#define M2 "v_mfma_f32_16x16x32_f16 v[72:75], v[60:63], v[60:63], v[64:67]\n\t"
#define M3 "v_mfma_f32_16x16x32_f16 v[52:55], v[60:63], v[60:63], v[48:51]\n\t"
#define M3I "v_mfma_f32_16x16x32_f16 v[52:55], v[60:63], v[60:63], v[52:55]\n\t"
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", \
             "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65",  \
             "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "s20", "s21"

template <int MODE>
__device__ __forceinline__ void shape(float a0, float a1, float c0, float c1, float& x, float& y, float& x2,
                                      float& y2) {
  // x, y: C's result (the checked low / high halves); x2, y2: C2's
#define RUN(body)                                                                                    \
  asm volatile(SETUP body "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"                            \
               "v_mov_b32 %0, v76\n\tv_mov_b32 %1, v77\n\tv_mov_b32 %6, v70\n\tv_mov_b32 %7, v71\n\t" \
               : "=v"(x), "=v"(y), "+v"(a0), "+v"(a1), "+v"(c0), "+v"(c1), "=v"(x2), "=v"(y2)        \
               :                                                                                     \
               : CLOB)
  if constexpr (MODE == 0) RUN(P_ M1 F_ C_S C2 M2 M3);
  else if constexpr (MODE == 1) RUN(P_ M1 F_ C_S C2 M2);
  else if constexpr (MODE == 2) RUN(P_ M1 F_ C_V C2 M2 M3);
  else if constexpr (MODE == 3) RUN(P_ M1 F_ C_S C2 "s_nop 1\n\t" M2 M3);
  else if constexpr (MODE == 4) RUN(P_ M1 F_ C_S C2 M2 M3I);
  else RUN(P_ F_ C_S C2 M2 M3);
}

template <int MODE>
__global__ __launch_bounds__(256) void shape_kernel(unsigned* __restrict__ bad) {
  const int lane = threadIdx.x & 63;
  unsigned nb[4] = {0, 0, 0, 0};
  for (int it = 0; it < kIters; ++it) {
    const float a0 = float(lane + it), a1 = float(lane - it), c0 = 0.25f * float(it), c1 = -0.5f * float(lane);
    float x, y, x2, y2;
    shape<MODE>(a0, a1, c0, c1, x, y, x2, y2);
    const float px = fmaf(a0, 0.5f, c0), py = fmaf(a1, 0.5f, c1);  // P
    nb[0] += x != px * 2.0f;                                        // C low
    nb[1] += y != py * 2.0f;                                        // C high
    nb[2] += x2 != px * 2.0f;                                       // C2 low (F = P)
    nb[3] += y2 != py * 2.0f;
  }
  for (int k = 0; k < 4; ++k) atomicAdd(&bad[4 * (lane >> 4) + k], nb[k]);
}

template <int MODE>
int run(unsigned* d, const char* name, int waves_per_simd) {
  CHECK(hipMemset(d, 0, 16 * sizeof(unsigned)));
  hipLaunchKernelGGL(shape_kernel<MODE>, dim3(kBlocks * waves_per_simd), dim3(256), 0, 0, d);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  unsigned h[16];
  CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  printf("%-34s x%d: C lo/hi, C2 lo/hi wrong per quarter:", name, waves_per_simd);
  for (int q = 0; q < 4; ++q) printf("  q%d %u/%u %u/%u", q, h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]);
  printf("  (of %u)\n", unsigned(kBlocks * waves_per_simd * 4 * 16 * kIters / 4));
  return 0;
}

int main() {
  unsigned* d;
  CHECK(hipMalloc(&d, 16 * sizeof(unsigned)));
  int rc = 0;
  for (int w : {1, 4}) {
    rc |= run<0>(d, "0 full shape", w);
    rc |= run<1>(d, "1 no M3", w);
    rc |= run<2>(d, "2 VGPR pair in C", w);
    rc |= run<3>(d, "3 s_nop 1 after C2", w);
    rc |= run<4>(d, "4 M3 in place", w);
    rc |= run<5>(d, "5 no M1", w);
  }
  return rc;
}
