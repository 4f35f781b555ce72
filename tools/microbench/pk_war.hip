// pk_war.hip -- isolates the f16x3 lanes-48..63 fault of round 1.
//
// Round 1 saw blend_skin_h3 return wrong coordinate-0 vertices in lanes 48-63
// of some tiles when hipcc SLP-packed the LBS apply into v_pk_fma_f32; the
// failing disassembly had a v_pk_fma_f32 immediately followed by a VALU write
// of one of its SOURCE registers.  This kernel runs exactly that pair with
// hard-wired registers (inline asm, so no compiler hazard padding):
//
//     v_pk_fma_f32 v[46:47], v[40:41], v[42:43], v[44:45]
//     <pad>
//     v_mov_b32    v<src>, <new value>        (write-after-read of a source)
//
// and checks, per lane, whether the packed FMA consumed the old or the new
// source value.  Variants: which source register is overwritten (a.lo, a.hi,
// b.lo, c.lo), the pad (none / s_nop 0 / 1 / 3), a scalar v_fma_f32 pair
// instead of the packed op (control), and whether two sibling waves of the
// block run an f32 MFMA chain at the same time (the fault was seen beside
// MFMAs).  Output: mismatches per 16-lane quarter of the wave.
//
//   hipcc --offload-arch=gfx950 -O3 -o pk_war pk_war.hip && ./pk_war
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 64;
constexpr int kBlocks = 2048;

// SRC: 0 a.lo (v40), 1 a.hi (v41), 2 b.lo (v42), 3 c.lo (v44); PAD: -1 none, else s_nop PAD;
// PACKED: v_pk_fma_f32 or two v_fma_f32.
#define STR2(x) #x
#define STR(x) STR2(x)

template <int SRC, int PAD, bool PACKED>
__device__ __forceinline__ void war_pair(float a0, float a1, float b0, float b1, float c0, float c1,
                                         float nv, float& o0, float& o1) {
  // clang-format off
#define LOAD "v_mov_b32 v40, %2\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, %4\n\tv_mov_b32 v43, %5\n\t" \
             "v_mov_b32 v44, %6\n\tv_mov_b32 v45, %7\n\ts_nop 4\n\t"
#define FMA_P "v_pk_fma_f32 v[46:47], v[40:41], v[42:43], v[44:45]\n\t"
#define FMA_S "v_fma_f32 v46, v40, v42, v44\n\tv_fma_f32 v47, v41, v43, v45\n\t"
#define TAIL "s_nop 4\n\tv_mov_b32 %0, v46\n\tv_mov_b32 %1, v47\n\t"
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47"
#define W(reg) "v_mov_b32 " reg ", %8\n\t"
  // clang-format on
  constexpr const char* dummy = "";
  (void)dummy;
#define EMIT(fma, pad, reg)                                                            \
  asm volatile(LOAD fma pad W(reg) TAIL                                               \
               : "=v"(o0), "=v"(o1)                                                   \
               : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "v"(c0), "v"(c1), "v"(nv)        \
               : CLOB)
#define EMIT_PAD(fma, reg)                                  \
  if constexpr (PAD < 0) EMIT(fma, "", reg);                \
  else if constexpr (PAD == 0) EMIT(fma, "s_nop 0\n\t", reg); \
  else if constexpr (PAD == 1) EMIT(fma, "s_nop 1\n\t", reg); \
  else EMIT(fma, "s_nop 3\n\t", reg);
#define EMIT_SRC(fma)                 \
  if constexpr (SRC == 0) { EMIT_PAD(fma, "v40") } \
  else if constexpr (SRC == 1) { EMIT_PAD(fma, "v41") } \
  else if constexpr (SRC == 2) { EMIT_PAD(fma, "v42") } \
  else { EMIT_PAD(fma, "v44") }
  if constexpr (PACKED) {
    EMIT_SRC(FMA_P)
  } else {
    EMIT_SRC(FMA_S)
  }
}

// Waves 0-1 (when kMfma) run a dependent f32 MFMA chain for the duration; the
// other waves (all four otherwise) run the WAR pair kIters times.
template <int SRC, int PAD, bool PACKED, bool kMfma>
__global__ __launch_bounds__(256) void war_kernel(const float* __restrict__ in, unsigned* __restrict__ bad,
                                                  float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  if (kMfma && wave < 2) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float x = in[lane], y = in[64 + lane];
    for (int i = 0; i < 8 * kIters; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc, 0, 0, 0);
    sink[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
    return;
  }
  unsigned miss = 0;
  for (int it = 0; it < kIters; ++it) {
    const float* p = in + ((it * 7 + lane) & 127);
    const float a0 = p[0], a1 = p[1], b0 = p[2], b1 = p[3], c0 = p[4], c1 = p[5];
    const float nv = 1000.0f + float(it);
    float o0, o1;
    war_pair<SRC, PAD, PACKED>(a0, a1, b0, b1, c0, c1, nv, o0, o1);
    const float e0 = fmaf(a0, b0, c0), e1 = fmaf(a1, b1, c1);
    miss += (o0 != e0) + (o1 != e1);
  }
  atomicAdd(&bad[lane >> 4], miss);
}

template <int SRC, int PAD, bool PACKED, bool kMfma>
int run(const float* d_in, unsigned* d_bad, float* d_sink, const char* name) {
  CHECK(hipMemset(d_bad, 0, 4 * sizeof(unsigned)));
  hipLaunchKernelGGL((war_kernel<SRC, PAD, PACKED, kMfma>), dim3(kBlocks), dim3(256), 0, 0, d_in, d_bad, d_sink);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  unsigned h[4];
  CHECK(hipMemcpy(h, d_bad, sizeof(h), hipMemcpyDeviceToHost));
  const unsigned long total = (unsigned long)kBlocks * (kMfma ? 2 : 4) * 16 * kIters * 2;
  printf("%-44s lanes 0-15: %8u  16-31: %8u  32-47: %8u  48-63: %8u   (of %lu results per quarter)\n", name,
         h[0], h[1], h[2], h[3], total);
  return 0;
}

int main() {
  std::vector<float> in(256);
  for (int i = 0; i < 256; ++i) in[i] = 1.0f + 0.01f * float(i % 97) - 0.3f * float(i % 5);
  float *d_in, *d_sink;
  unsigned* d_bad;
  CHECK(hipMalloc(&d_in, 256 * sizeof(float)));
  CHECK(hipMalloc(&d_sink, kBlocks * 256 * sizeof(float)));
  CHECK(hipMalloc(&d_bad, 4 * sizeof(unsigned)));
  CHECK(hipMemcpy(d_in, in.data(), 256 * sizeof(float), hipMemcpyHostToDevice));
  int rc = 0;
  rc |= run<0, -1, false, false>(d_in, d_bad, d_sink, "scalar fma x2, write a.lo, no pad");
  rc |= run<0, -1, false, true>(d_in, d_bad, d_sink, "scalar fma x2, write a.lo, no pad, +MFMA");
  rc |= run<0, -1, true, false>(d_in, d_bad, d_sink, "pk_fma, write a.lo, no pad");
  rc |= run<1, -1, true, false>(d_in, d_bad, d_sink, "pk_fma, write a.hi, no pad");
  rc |= run<2, -1, true, false>(d_in, d_bad, d_sink, "pk_fma, write b.lo, no pad");
  rc |= run<3, -1, true, false>(d_in, d_bad, d_sink, "pk_fma, write c.lo, no pad");
  rc |= run<0, -1, true, true>(d_in, d_bad, d_sink, "pk_fma, write a.lo, no pad, +MFMA");
  rc |= run<1, -1, true, true>(d_in, d_bad, d_sink, "pk_fma, write a.hi, no pad, +MFMA");
  rc |= run<2, -1, true, true>(d_in, d_bad, d_sink, "pk_fma, write b.lo, no pad, +MFMA");
  rc |= run<3, -1, true, true>(d_in, d_bad, d_sink, "pk_fma, write c.lo, no pad, +MFMA");
  rc |= run<0, 0, true, false>(d_in, d_bad, d_sink, "pk_fma, write a.lo, s_nop 0");
  rc |= run<0, 0, true, true>(d_in, d_bad, d_sink, "pk_fma, write a.lo, s_nop 0, +MFMA");
  rc |= run<0, 1, true, false>(d_in, d_bad, d_sink, "pk_fma, write a.lo, s_nop 1");
  rc |= run<0, 1, true, true>(d_in, d_bad, d_sink, "pk_fma, write a.lo, s_nop 1, +MFMA");
  rc |= run<0, 3, true, true>(d_in, d_bad, d_sink, "pk_fma, write a.lo, s_nop 3, +MFMA");
  rc |= run<3, 1, true, true>(d_in, d_bad, d_sink, "pk_fma, write c.lo, s_nop 1, +MFMA");
  return rc;
}
