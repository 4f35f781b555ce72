// mano_joint.h -- one (hand, joint) lane of the MANO articulation, shared by
// articulate_kernel (mano_articulate.hip) and the fused forward kernel
// (mano_kernels.hip, blend_skin16 with kArt): Rodrigues (mano_np.py:117-148),
// the folded joint regression (:83), the kinematic chain (:96-104) by
// wavefront shuffles and the rest-pose removal (:106-110).  Contraction is off
// and every fma is spelled out, so both call sites (built with different
// machine schedulers) produce the same bits.  Not installed.
#pragma once

#include "mano_internal.h"

namespace mano {
namespace {

// R - I for one axis-angle vector r = (x, y, z).
// mano_np.py:130-147 computes R = cos I + (1 - cos) r^ r^T + sin [r^]x with
// theta clamped to float64 eps.  With K = [r]x this equals
//   R - I = a K + b K^2,  K^2 = r r^T - theta^2 I,
//   a = sin(theta)/theta, b = (1 - cos theta)/theta^2 = 2 sin^2(theta/2)/theta^2,
// which has no 0/0 and no 1 - cos cancellation in float32.  Below theta = 1e-2
// the Taylor series to theta^4 is exact in float32.  Returning R - I (not R)
// keeps the small pose features of :91 free of the cancellation too.
//
// Contraction is off in the articulation helpers and fmaf is spelled out, so
// their rounding does not depend on how the compiler contracts the inlined
// code (results are reproducible across builds and call sites).
__device__ __forceinline__ void rodrigues_minus_eye(float x, float y, float z, float rm[9]) {
#pragma clang fp contract(off)
  const float th2 = x * x + y * y + z * z;
  float a, b;
  if (th2 < 1e-4f) {
    a = 1.0f - th2 * (1.0f / 6.0f) + th2 * th2 * (1.0f / 120.0f);
    b = 0.5f - th2 * (1.0f / 24.0f) + th2 * th2 * (1.0f / 720.0f);
  } else {
    // One sincos of the half angle: sin(theta) = 2 sin(theta/2) cos(theta/2).
    const float th = sqrtf(th2);
    const float inv = 1.0f / th;
    float sh, ch;
    sincosf(0.5f * th, &sh, &ch);
    a = 2.0f * sh * ch * inv;
    const float shr = sh * inv;
    b = 2.0f * shr * shr;
  }
  rm[0] = b * (x * x - th2);
  rm[1] = fmaf(b, x * y, -a * z);
  rm[2] = fmaf(b, x * z, a * y);
  rm[3] = fmaf(b, y * x, a * z);
  rm[4] = b * (y * y - th2);
  rm[5] = fmaf(b, y * z, -a * x);
  rm[6] = fmaf(b, z * x, -a * y);
  rm[7] = fmaf(b, z * y, a * x);
  rm[8] = b * (z * z - th2);
}

// ---------------------------------------------------------------------------
// One (hand, joint) lane of the articulation, shared by articulate_kernel and
// the fused forward kernel.  The 16 lanes of a hand are consecutive
// (lane & 15 == joint), so the chain's parent transform arrives by shuffle.
// Out: rm = R_j - I (the pose feature, :91), J = rest joint (:83), t = posed
// joint = G_j[:3, 3] (:96-104), A = G_j with the rest pose removed (:106-110),
// row-major 3x4.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void articulate_joint(float x, float y, float z,
                                                 const float (&beta)[kShape], int j, int src,
                                                 int dep, int max_depth,
                                                 const float* __restrict__ joint_template,
                                                 const float* __restrict__ joint_shape,
                                                 float (&rm)[9], float (&J)[3], float (&t)[3],
                                                 float (&A)[12]) {
#pragma clang fp contract(off)
  rodrigues_minus_eye(x, y, z, rm);
  // Rest joint of joint j (mano_np.py:83, folded: Jreg.(T + S.beta)).
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float acc = joint_template[j * 3 + c];
#pragma unroll
    for (int s = 0; s < kShape; ++s) acc = fmaf(joint_shape[(j * 3 + c) * kShape + s], beta[s], acc);
    J[c] = acc;
  }
  // World rotation / translation, initialised to the root form G_0 = [R_0 | J_0] (:97).
  float Rl[9], Rw[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rl[i] = Rw[i] = rm[i] + ((i % 4 == 0) ? 1.f : 0.f);
  t[0] = J[0];
  t[1] = J[1];
  t[2] = J[2];
  // Chain (:98-104): G_j = G_parent . [R_j | J_j - J_parent], one tree level per
  // iteration; the parent's finished transform arrives by a wavefront shuffle.
  for (int d = 1; d <= max_depth; ++d) {
    float pR[9], pt[3], pJ[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) pR[i] = __shfl(Rw[i], src);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      pt[c] = __shfl(t[c], src);
      pJ[c] = __shfl(J[c], src);
    }
    if (dep == d) {
      const float d0 = J[0] - pJ[0], d1 = J[1] - pJ[1], d2 = J[2] - pJ[2];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
          Rw[r * 3 + c] = pR[r * 3 + 0] * Rl[0 * 3 + c] + pR[r * 3 + 1] * Rl[1 * 3 + c] +
                          pR[r * 3 + 2] * Rl[2 * 3 + c];
        t[r] = pR[r * 3 + 0] * d0 + pR[r * 3 + 1] * d1 + pR[r * 3 + 2] * d2 + pt[r];
      }
    }
  }
  // Skinning transform A_j = [Rw | t - Rw J] (rest-pose removal, :106-110).
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    A[r * 4 + 0] = Rw[r * 3 + 0];
    A[r * 4 + 1] = Rw[r * 3 + 1];
    A[r * 4 + 2] = Rw[r * 3 + 2];
    A[r * 4 + 3] = t[r] - (Rw[r * 3 + 0] * J[0] + Rw[r * 3 + 1] * J[1] + Rw[r * 3 + 2] * J[2]);
  }
}

}  // namespace
}  // namespace mano
