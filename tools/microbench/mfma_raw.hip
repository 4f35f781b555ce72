// mfma_raw.hip -- how many wait states must separate v_mfma_f32_16x16x32_f16
// from a VALU read of its result on gfx950 (the f16x3 lanes-48..63 fault).
//
// The MFMA-to-VALU dependency is not interlocked by the hardware: the compiler
// pads it with independent instructions or s_nop.  This kernel issues, with
// hard-wired registers in inline asm (no compiler padding),
//
//     v_mfma_f32_16x16x32_f16 v[40:43], v[44:47], v[48:51], v[40:43]
//     s_nop 0  x PAD                      (PAD wait states)
//     <VALU access>                       (mfma_access MODE: read D, read D with
//                                          v_pk_fma_f32, write SrcC, write D)
//
// with A = B = 1.0 (so D = C + 32 in every lane) and a lane-specific C, and
// counts per 16-lane quarter how many results show the hazard's signature
// (a stale D, a corrupted SrcC, a late MFMA write over the VALU's).  One block of 4 waves per CU (a 96 KB LDS
// reservation), so each SIMD runs one wave and nothing else fills the gap.
// `+mfma` variants put a second, MFMA-only wave on each SIMD (2 blocks per CU,
// the LDS reservation halved), which delays the dependent read.
//
//   hipcc --offload-arch=gfx950 -O3 -o mfma_raw mfma_raw.hip && ./mfma_raw
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
constexpr int kBlocks = 256;  // one per CU

// The MFMA's operands: A = B = eight f16 ones per lane (0x3c00 pairs), so D = C + 32.
#define MFMA_SETUP                                                                            \
  "v_mov_b32 v40, %4\n\tv_mov_b32 v41, %5\n\tv_mov_b32 v42, %6\n\tv_mov_b32 v43, %7\n\t"     \
  "v_mov_b32 v44, 0x3c003c00\n\tv_mov_b32 v45, 0x3c003c00\n\tv_mov_b32 v46, 0x3c003c00\n\t"  \
  "v_mov_b32 v47, 0x3c003c00\n\tv_mov_b32 v48, 0x3c003c00\n\tv_mov_b32 v49, 0x3c003c00\n\t"  \
  "v_mov_b32 v50, 0x3c003c00\n\tv_mov_b32 v51, 0x3c003c00\n\t"                               \
  "v_mov_b32 v56, 1.0\n\tv_mov_b32 v57, 1.0\n\tv_mov_b32 v58, 0\n\tv_mov_b32 v59, 0\n\ts_nop 7\n\t"
#define DRAIN "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
#define OUT4(a, b, c, d) "v_mov_b32 %0, " a "\n\tv_mov_b32 %1, " b "\n\tv_mov_b32 %2, " c "\n\tv_mov_b32 %3, " d
#define CLOBBERS "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", \
                 "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
#define PADDING ".rept %8\n\ts_nop 0\n\t.endr\n\t"

// Modes (PAD wait states after the MFMA, then the VALU access):
//   0 RAW   v_mov_b32 reads of D          -> expect C + 32   (stale: C)
//   1 RAWPK v_pk_fma_f32 (x 1 + 0) of D   -> expect C + 32   (stale: C)
//   2 WARC  v_mov_b32 writes SrcC (D elsewhere, v[60:63]) -> expect C + 32 (corrupt: 1e6 + 32)
//   3 WAW   v_mov_b32 writes D (1e6)      -> expect 1e6      (late MFMA write: C + 32)
//   4 WARPK v_pk_fma_f32 reads v[40:43], PAD, then an MFMA WRITES v[40:43]
//           (SrcC elsewhere) -> expect C      (clobbered read: anything else)
//   5 WARV  the same with four v_fma_f32 reads (control)
template <int PAD, int MODE>
__device__ __forceinline__ void mfma_access(float c0, float c1, float c2, float c3, float& o0,
                                            float& o1, float& o2, float& o3) {
  if constexpr (MODE == 0) {
    asm volatile(MFMA_SETUP "v_mfma_f32_16x16x32_f16 v[40:43], v[44:47], v[48:51], v[40:43]\n\t" PADDING
                 "v_mov_b32 v52, v40\n\tv_mov_b32 v53, v41\n\tv_mov_b32 v54, v42\n\tv_mov_b32 v55, v43\n\t"
                 DRAIN OUT4("v52", "v53", "v54", "v55")
                 : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)
                 : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "n"(PAD) : CLOBBERS);
  } else if constexpr (MODE == 1) {
    asm volatile(MFMA_SETUP "v_mfma_f32_16x16x32_f16 v[40:43], v[44:47], v[48:51], v[40:43]\n\t" PADDING
                 "v_pk_fma_f32 v[52:53], v[40:41], v[56:57], v[58:59]\n\t"
                 "v_pk_fma_f32 v[54:55], v[42:43], v[56:57], v[58:59]\n\t"
                 DRAIN OUT4("v52", "v53", "v54", "v55")
                 : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)
                 : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "n"(PAD) : CLOBBERS);
  } else if constexpr (MODE == 2) {
    asm volatile(MFMA_SETUP "v_mfma_f32_16x16x32_f16 v[60:63], v[44:47], v[48:51], v[40:43]\n\t" PADDING
                 "v_mov_b32 v40, 0x49742400\n\tv_mov_b32 v41, 0x49742400\n\t"
                 "v_mov_b32 v42, 0x49742400\n\tv_mov_b32 v43, 0x49742400\n\t"
                 DRAIN OUT4("v60", "v61", "v62", "v63")
                 : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)
                 : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "n"(PAD) : CLOBBERS);
  } else if constexpr (MODE == 3) {
    asm volatile(MFMA_SETUP "v_mfma_f32_16x16x32_f16 v[40:43], v[44:47], v[48:51], v[40:43]\n\t" PADDING
                 "v_mov_b32 v40, 0x49742400\n\tv_mov_b32 v41, 0x49742400\n\t"
                 "v_mov_b32 v42, 0x49742400\n\tv_mov_b32 v43, 0x49742400\n\t"
                 DRAIN OUT4("v40", "v41", "v42", "v43")
                 : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)
                 : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "n"(PAD) : CLOBBERS);
  } else if constexpr (MODE == 4 || MODE == 5) {
    // A VALU read of v[40:43] (packed: two v_pk_fma_f32; scalar: four
    // v_fma_f32), PAD, then an MFMA that WRITES v[40:43] (its SrcC is
    // v[60:63] = 1e6, so its result is 1e6 + 32): the VALU must see C.
#define READ_PK "v_pk_fma_f32 v[52:53], v[40:41], v[56:57], v[58:59]\n\tv_pk_fma_f32 v[54:55], v[42:43], v[56:57], v[58:59]\n\t"
#define READ_V "v_fma_f32 v52, v40, v56, v58\n\tv_fma_f32 v53, v41, v56, v58\n\tv_fma_f32 v54, v42, v56, v58\n\tv_fma_f32 v55, v43, v56, v58\n\t"
#define WAR_BODY(read)                                                                               \
  asm volatile(MFMA_SETUP "v_mov_b32 v60, 0x49742400\n\tv_mov_b32 v61, 0x49742400\n\t"              \
               "v_mov_b32 v62, 0x49742400\n\tv_mov_b32 v63, 0x49742400\n\ts_nop 7\n\t" read PADDING \
               "v_mfma_f32_16x16x32_f16 v[40:43], v[44:47], v[48:51], v[60:63]\n\t"                   \
               DRAIN OUT4("v52", "v53", "v54", "v55")                                               \
               : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)                                             \
               : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "n"(PAD) : CLOBBERS)
    if constexpr (MODE == 4) WAR_BODY(READ_PK);
    else WAR_BODY(READ_V);
  } else {
    // VALU producer -> (independent MFMA) -> PAD -> v_pk_fma_f32 consumer, the
    // shape of the round-1 failing sequence: v52/v53 hold 1e6 until the
    // producer writes c0/c1 (6: scalar v_fma_f32 x2; 7: v_pk_fma_f32; 8:
    // scalar producer, no MFMA in between); the consumer computes x * 1 + 0.
#define PROD_S "v_fma_f32 v52, v40, v56, v58\n\tv_fma_f32 v53, v41, v56, v58\n\t"
#define PROD_P "v_pk_fma_f32 v[52:53], v[40:41], v[56:57], v[58:59]\n\t"
#define MFMA_MID "v_mfma_f32_16x16x32_f16 v[60:63], v[44:47], v[48:51], v[60:63]\n\t"
#define RAW_BODY(prod, mid)                                                                          \
  asm volatile(MFMA_SETUP "v_mov_b32 v52, 0x49742400\n\tv_mov_b32 v53, 0x49742400\n\t"              \
               "v_mov_b32 v60, 0\n\tv_mov_b32 v61, 0\n\tv_mov_b32 v62, 0\n\tv_mov_b32 v63, 0\n\ts_nop 7\n\t" \
               prod mid PADDING "v_pk_fma_f32 v[54:55], v[52:53], v[56:57], v[58:59]\n\t"            \
               DRAIN OUT4("v54", "v55", "v52", "v53")                                               \
               : "=v"(o0), "=v"(o1), "=v"(o2), "=v"(o3)                                             \
               : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "n"(PAD) : CLOBBERS)
    if constexpr (MODE == 6) RAW_BODY(PROD_S, MFMA_MID);
    else if constexpr (MODE == 7) RAW_BODY(PROD_P, MFMA_MID);
    else RAW_BODY(PROD_S, "");
  }
}

template <int PAD, int MODE, bool kMfmaSibling>
__global__ __launch_bounds__(256) void raw_kernel(unsigned* __restrict__ stale, unsigned* __restrict__ other,
                                                  float* __restrict__ sink) {
  extern __shared__ float reserve[];
  const int lane = threadIdx.x & 63;
  if (kMfmaSibling && (blockIdx.x & 1)) {
    // odd blocks: MFMA-only waves sharing the SIMDs with the even blocks' test waves
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
    f16x8 a = {}, b = {};
    a[0] = _Float16(float(lane));
    b[0] = _Float16(1.0f);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < 4 * kIters; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
    sink[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3] + reserve[0] * 0.f;
    return;
  }
  unsigned n_stale = 0, n_other = 0;
  for (int it = 0; it < kIters; ++it) {
    const float c = float(lane * 4 + it % 7);
    float o[4];
    mfma_access<PAD, MODE>(c, c + 1.f, c + 2.f, c + 3.f, o[0], o[1], o[2], o[3]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // want: the architecturally correct value; bad: the hazard's signature.
      const float cr = c + float(r);
      // modes 6-8 return (x, y, x, y) of the consumer / producer: c0, c1, c0, c1
      const float cv = MODE >= 6 ? c + float(r & 1) : cr;
      const float want = MODE == 3 ? 1.0e6f : MODE >= 4 ? cv : cr + 32.f;
      const float bad = MODE == 2 ? 1.0e6f + 32.f : MODE == 3 ? cr + 32.f : MODE >= 6 ? 1.0e6f
                        : MODE >= 4 ? 1.0e6f + 32.f : cr;
      n_stale += o[r] == bad;
      n_other += o[r] != bad && o[r] != want;
    }
  }
  atomicAdd(&stale[lane >> 4], n_stale);
  atomicAdd(&other[lane >> 4], n_other);
}

template <int PAD, int MODE, bool kSib>
int run(unsigned* d_stale, unsigned* d_other, float* d_sink) {
  CHECK(hipMemset(d_stale, 0, 4 * sizeof(unsigned)));
  CHECK(hipMemset(d_other, 0, 4 * sizeof(unsigned)));
  const size_t lds = kSib ? 48 * 1024 : 96 * 1024;  // 1 block per CU, or 2 (test + MFMA sibling)
  auto k = raw_kernel<PAD, MODE, kSib>;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  hipLaunchKernelGGL(k, dim3(kSib ? 2 * kBlocks : kBlocks), dim3(256), lds, 0, d_stale, d_other, d_sink);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  unsigned s[4], o[4];
  CHECK(hipMemcpy(s, d_stale, sizeof(s), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(o, d_other, sizeof(o), hipMemcpyDeviceToHost));
  const unsigned long per_q = (unsigned long)kBlocks * 4 * 16 * kIters * 4;
  static const char* names[] = {"RAW", "RAW_pk", "WAR_C", "WAW", "WAR_pk", "WAR_v", "RAWs_m", "RAWp_m", "RAWs"};
  printf("%-7s pad %2d %-6s hazard: lanes 0-15 %8u 16-31 %8u 32-47 %8u 48-63 %8u | other %u %u %u %u (of %lu per quarter)\n",
         names[MODE], PAD, kSib ? "+mfma" : "", s[0], s[1], s[2], s[3], o[0], o[1], o[2], o[3], per_q);
  return 0;
}

template <int PAD>
int run_valu(unsigned* s, unsigned* o, float* k) {
  int rc = 0;
  for (int rep = 0; rep < 2; ++rep) {
    rc |= run<PAD, 6, false>(s, o, k);
    rc |= run<PAD, 7, false>(s, o, k);
    rc |= run<PAD, 8, false>(s, o, k);
    rc |= run<PAD, 6, true>(s, o, k);
    rc |= run<PAD, 7, true>(s, o, k);
    rc |= run<PAD, 8, true>(s, o, k);
  }
  return rc;
}

template <int PAD>
int run_war(unsigned* s, unsigned* o, float* k) {
  int rc = 0;
  rc |= run<PAD, 4, false>(s, o, k);
  rc |= run<PAD, 5, false>(s, o, k);
  rc |= run<PAD, 4, true>(s, o, k);
  rc |= run<PAD, 5, true>(s, o, k);
  return rc;
}

template <int PAD>
int run_pad(unsigned* s, unsigned* o, float* k) {
  int rc = 0;
  rc |= run<PAD, 0, false>(s, o, k);
  rc |= run<PAD, 1, false>(s, o, k);
  rc |= run<PAD, 2, false>(s, o, k);
  rc |= run<PAD, 3, false>(s, o, k);
  rc |= run<PAD, 0, true>(s, o, k);
  rc |= run<PAD, 1, true>(s, o, k);
  rc |= run<PAD, 2, true>(s, o, k);
  rc |= run<PAD, 3, true>(s, o, k);
  return rc;
}

int main(int argc, char** argv) {
  unsigned *d_stale, *d_other;
  float* d_sink;
  CHECK(hipMalloc(&d_stale, 4 * sizeof(unsigned)));
  CHECK(hipMalloc(&d_other, 4 * sizeof(unsigned)));
  CHECK(hipMalloc(&d_sink, 2 * kBlocks * 256 * sizeof(float)));
  int rc = 0;
  if (argc > 1 && argv[1][0] == 'v') {  // ./mfma_raw valu: VALU -> v_pk_fma_f32 RAW across an MFMA
    rc |= run_valu<0>(d_stale, d_other, d_sink);
    rc |= run_valu<1>(d_stale, d_other, d_sink);
    rc |= run_valu<2>(d_stale, d_other, d_sink);
    rc |= run_valu<4>(d_stale, d_other, d_sink);
    return rc;
  }
  if (argc > 1 && argv[1][0] == 'w') {  // ./mfma_raw war: the VALU-read -> MFMA-write pairs only
    rc |= run_war<0>(d_stale, d_other, d_sink);
    rc |= run_war<1>(d_stale, d_other, d_sink);
    rc |= run_war<2>(d_stale, d_other, d_sink);
    rc |= run_war<3>(d_stale, d_other, d_sink);
    rc |= run_war<4>(d_stale, d_other, d_sink);
    rc |= run_war<6>(d_stale, d_other, d_sink);
    rc |= run_war<8>(d_stale, d_other, d_sink);
    return rc;
  }
  rc |= run_pad<0>(d_stale, d_other, d_sink);
  rc |= run_pad<1>(d_stale, d_other, d_sink);
  rc |= run_pad<2>(d_stale, d_other, d_sink);
  rc |= run_pad<3>(d_stale, d_other, d_sink);
  rc |= run_pad<4>(d_stale, d_other, d_sink);
  rc |= run_pad<5>(d_stale, d_other, d_sink);
  rc |= run_pad<6>(d_stale, d_other, d_sink);
  rc |= run_pad<7>(d_stale, d_other, d_sink);
  rc |= run_pad<8>(d_stale, d_other, d_sink);
  rc |= run_pad<9>(d_stale, d_other, d_sink);
  rc |= run_pad<10>(d_stale, d_other, d_sink);
  rc |= run_pad<11>(d_stale, d_other, d_sink);
  rc |= run_pad<12>(d_stale, d_other, d_sink);
  return rc;
}
