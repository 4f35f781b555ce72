// lbs_dpp.h -- per-vertex blend of 16 joint transforms with DPP row broadcasts.
//
// The blended skinning transform of vertex v for hand h (mano_np.py:112) is
//   T_v = sum_j W[v][j] A_j(h),  A_j the 3x4 world transform of joint j.
// A wavefront holds 64 (hand, vertex) pairs, one per lane, but a 16-lane DPP
// row always works on ONE hand.  Lane k of a row loads the 12 floats of joint k
// of that row's hand (3 x dwordx4); `v_fmac_f32_dpp ... row_newbcast:j` then
// feeds A_j[m] of lane j to every lane of its row as the FMA's first operand,
// so the 192 multiply-adds per vertex read the transforms straight from VGPRs:
// no scalar loads (and their per-chunk waits), no LDS broadcast reads.
#pragma once

#include <hip/hip_runtime.h>

// T[0..11] += a(lane j of the row)[0..11] * w[J].  The leading s_nop 1 gives
// the two wait states a DPP source needs after a VALU write (hipcc inserts no
// hazard padding inside inline asm).
#define MANO_FMA_DPP(T, a, wj, J)                                                                 \
  asm volatile("s_nop 1\n\t"                                                                      \
               "v_fmac_f32_dpp %0, %12, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %1, %13, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %2, %14, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %3, %15, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %4, %16, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %5, %17, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %6, %18, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %7, %19, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %8, %20, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %9, %21, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %10, %22, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t" \
               "v_fmac_f32_dpp %11, %23, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"     \
               : "+v"(T[0]), "+v"(T[1]), "+v"(T[2]), "+v"(T[3]), "+v"(T[4]), "+v"(T[5]),        \
                 "+v"(T[6]), "+v"(T[7]), "+v"(T[8]), "+v"(T[9]), "+v"(T[10]), "+v"(T[11])       \
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),   \
                 "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(wj))

namespace mano {

typedef float lbs_f32x4 __attribute__((ext_vector_type(4)));

// Lane k of each 16-lane row loads joint k's 3x4 transform of hand `Ah`.
__device__ __forceinline__ void lbs_load_joint_row(const float* __restrict__ Ah, int lane,
                                                   float a[12]) {
  const lbs_f32x4* p = reinterpret_cast<const lbs_f32x4*>(Ah + (lane & 15) * 12);
  const lbs_f32x4 x = p[0], y = p[1], z = p[2];
  a[0] = x[0]; a[1] = x[1]; a[2] = x[2]; a[3] = x[3];
  a[4] = y[0]; a[5] = y[1]; a[6] = y[2]; a[7] = y[3];
  a[8] = z[0]; a[9] = z[1]; a[10] = z[2]; a[11] = z[3];
}

// T = sum_j w[j] A_j (A from the row broadcasts of `a`).
__device__ __forceinline__ void lbs_blend16(float T[12], const float a[12], const float w[16]) {
#pragma unroll
  for (int m = 0; m < 12; ++m) T[m] = 0.f;
  MANO_FMA_DPP(T, a, w[0], 0);
  MANO_FMA_DPP(T, a, w[1], 1);
  MANO_FMA_DPP(T, a, w[2], 2);
  MANO_FMA_DPP(T, a, w[3], 3);
  MANO_FMA_DPP(T, a, w[4], 4);
  MANO_FMA_DPP(T, a, w[5], 5);
  MANO_FMA_DPP(T, a, w[6], 6);
  MANO_FMA_DPP(T, a, w[7], 7);
  MANO_FMA_DPP(T, a, w[8], 8);
  MANO_FMA_DPP(T, a, w[9], 9);
  MANO_FMA_DPP(T, a, w[10], 10);
  MANO_FMA_DPP(T, a, w[11], 11);
  MANO_FMA_DPP(T, a, w[12], 12);
  MANO_FMA_DPP(T, a, w[13], 13);
  MANO_FMA_DPP(T, a, w[14], 14);
  MANO_FMA_DPP(T, a, w[15], 15);
}

}  // namespace mano
