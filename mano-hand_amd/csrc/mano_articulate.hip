// mano_articulate.hip -- gfx950 (MI355X) articulation kernels of the MANO
// forward pass: the first of mano_forward's two launches, and the standalone
// PCA-pose and Rodrigues kernels.
//
//   articulate    one lane per (hand, joint), 16 hands per 256-thread block
//                 (optionally the PCA pose map of set_params, mano_np.py:66-72,
//                 first): Rodrigues (:117-148) in sinc / half-angle form, rest
//                 joints J = Jreg.T + (Jreg.S).beta (:83, folded in float64 at
//                 model load), the 16-joint chain (:96-104) as 3 dependent
//                 levels of wavefront shuffles (5 fingers x depth 3), the
//                 rest-pose removal (:106-110) -> 3x4 transforms, and the 135
//                 pose features (R_j - I, :87-91) written into the X rows the
//                 blend GEMM reads as MFMA A fragments.
//
// A source of its own: mano_kernels.hip (the MFMA kernels) is compiled with
// the max-ILP scheduler, which made this latency-bound kernel slower.
#include "mano_internal.h"

namespace mano {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
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

// Optional per-joint outputs of a valid lane: posed joints (+ trans), rest
// joints, local rotations R_j = I + rm.
__device__ __forceinline__ void store_joint_outputs(int64_t h, int j, const float* __restrict__ trans,
                                                    const float (&rm)[9], const float (&J)[3],
                                                    const float (&t)[3], float* __restrict__ joints,
                                                    float* __restrict__ rest_joints,
                                                    float* __restrict__ rot_mats) {
  if (joints) {
    float* o = joints + h * (kJoints * 3) + 3 * j;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = t[c] + (trans ? trans[h * 3 + c] : 0.f);
  }
  if (rest_joints) {
    float* o = rest_joints + h * (kJoints * 3) + 3 * j;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = J[c];
  }
  if (rot_mats) {
    float* o = rot_mats + h * (kJoints * 9) + 9 * j;
#pragma unroll
    for (int i = 0; i < 9; ++i) o[i] = rm[i] + ((i % 4 == 0) ? 1.f : 0.f);
  }
}

// ---------------------------------------------------------------------------
// articulate: one lane per (hand, joint), 16 hands per 256-thread block.  The
// X rows (kXStride floats, k-permuted, mano_internal.h) are assembled in LDS
// -- each lane drops its 9 features in place -- and leave as one contiguous
// 10-KB dwordx4 stream; transforms and joints are stored straight from the
// lanes (48 and 12 contiguous bytes each).
// ---------------------------------------------------------------------------
// PCA pose of one (hand, joint) lane (set_params' PCA branch, mano_np.py:66-72):
// joint 0 takes the global rotation, joint j >= 1 the three entries
// 3 (j - 1) + c of c . basis[:N] + mean.  Same operation order as
// pose_from_pca_kernel (fmaf chain over i, then + mean), so the fused and the
// standalone PCA maps agree bit for bit.
__device__ __forceinline__ void pca_joint_pose(const PcaInput& in, const float* __restrict__ basis,
                                               const float* __restrict__ mean, int64_t h, int j,
                                               float (&aa)[3]) {
  if (j == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) aa[c] = in.rot ? in.rot[h * in.rot_stride + c] : 0.f;
    return;
  }
  const float* coef = in.pca + h * in.pca_stride;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int mm = 3 * (j - 1) + c;
    float v = 0.f;
    for (int i = 0; i < in.n_comps; ++i) v = fmaf(coef[i], basis[i * kPca + mm], v);
    aa[c] = v + mean[mm];
  }
}

// kFromPca: the pose comes from PCA coefficients (pca_joint_pose prologue, the
// basis rows in use staged in LDS) instead of the axis-angle `pose` input.
template <bool kFromPca>
__global__ __launch_bounds__(256) void articulate_kernel(
    const float* __restrict__ betas, int64_t betas_stride, const float* __restrict__ pose,
    const float* __restrict__ trans, const float* __restrict__ joint_template,
    const float* __restrict__ joint_shape, const int32_t* __restrict__ parents,
    const int32_t* __restrict__ depth, int max_depth, int64_t n,
    float* __restrict__ features, float* __restrict__ transforms, float* __restrict__ joints,
    float* __restrict__ rest_joints, float* __restrict__ rot_mats, PcaInput pca,
    const float* __restrict__ pca_basis, const float* __restrict__ pca_mean) {
  __shared__ f32x4 xs4[16 * kXStride / 4];
  // The block's 16 rows of posed joints (48 floats each), staged so they
  // leave as one contiguous dwordx4 stream like the X rows (three 4-B
  // stores per lane at a 12-B stride cost the in-path step ~7 us).
  __shared__ f32x4 jo4[16 * kJoints * 3 / 4];
  // The folded joint regressor (J = Jt + Js . beta, 528 floats), staged once
  // per block: each lane reads its joint's 33 values from LDS, not HBM/L2.
  __shared__ float jt_s[kJoints * 3];
  __shared__ float js_s[kJoints * 3 * kShape];
  float* xs = reinterpret_cast<float*>(xs4);
  const int tid = threadIdx.x;
  const int j = tid & (kJoints - 1);
  const int hl = tid >> 4;
  const int64_t h0 = int64_t(blockIdx.x) * 16;
  const int64_t h = min(h0 + hl, n - 1);  // tail lanes repeat the last hand
  const bool valid = h0 + hl < n;
  // a caller's joints buffer that is not 16-B aligned takes the per-lane stores
  const bool joints_direct = (reinterpret_cast<uintptr_t>(joints) & 15) != 0;

  // Every global load of the prologue is issued before the first LDS write
  // (the lane's pose and betas, then the block's regressor fold): written as
  // load-then-store loops, hipcc waited for each load before its ds_write --
  // three serial round trips before any arithmetic.
  float aa[3] = {0.f, 0.f, 0.f};
  if constexpr (!kFromPca) {
    const float* p = pose + h * (kJoints * 3) + 3 * j;
    aa[0] = p[0];
    aa[1] = p[1];
    aa[2] = p[2];
  }
  float beta[kShape];
#pragma unroll
  for (int s = 0; s < kShape; ++s) beta[s] = betas[h * betas_stride + s];
  constexpr int kJs = kJoints * 3 * kShape;  // 480 = 256 + 224
  const float js0 = joint_shape[tid];
  const float js1 = tid + 256 < kJs ? joint_shape[tid + 256] : 0.f;
  const float jt0 = tid < kJoints * 3 ? joint_template[tid] : 0.f;
  js_s[tid] = js0;
  if (tid + 256 < kJs) js_s[tid + 256] = js1;
  if (tid < kJoints * 3) jt_s[tid] = jt0;
  const float* basis_s = nullptr;
  const float* mean_s = nullptr;
  if constexpr (kFromPca) {
    __shared__ float pb_s[kPca * kPca + kPca];
    for (int i = tid; i < pca.n_comps * kPca; i += 256) pb_s[i] = pca_basis[i];
    if (tid < kPca) pb_s[kPca * kPca + tid] = pca_mean[tid];
    basis_s = pb_s;
    mean_s = pb_s + kPca * kPca;
  }
  __syncthreads();

  if constexpr (kFromPca) {
    pca_joint_pose(pca, basis_s, mean_s, h, j, aa);
    if (valid && pca.pose_out) {
#pragma unroll
      for (int c = 0; c < 3; ++c) pca.pose_out[h * (kJoints * 3) + 3 * j + c] = aa[c];
    }
  }
  const int par = parents[j];
  const int src = ((tid & 63) & ~(kJoints - 1)) + (par < 0 ? 0 : par);
  float rm[9], J[3], t[3], Aj[12];
  articulate_joint(aa[0], aa[1], aa[2], beta, j, src, depth[j], max_depth, jt_s, js_s, rm, J, t, Aj);
  if (valid) {
    f32x4* A = reinterpret_cast<f32x4*>(transforms + h * kTransformFloats + j * 12);
    A[0] = f32x4{Aj[0], Aj[1], Aj[2], Aj[3]};
    A[1] = f32x4{Aj[4], Aj[5], Aj[6], Aj[7]};
    A[2] = f32x4{Aj[8], Aj[9], Aj[10], Aj[11]};
    store_joint_outputs(h, j, trans, rm, J, t, joints_direct ? joints : nullptr, rest_joints, rot_mats);
  }
  if (joints && !joints_direct) {
    float* o = reinterpret_cast<float*>(jo4) + hl * (kJoints * 3) + 3 * j;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = t[c] + (trans ? trans[h * 3 + c] : 0.f);
  }

  // Row of X: k < 10 beta, 10 <= k < 145 features (k = 10 + 9(j-1) + 3 row +
  // col, the ravel order of :91), X[h][145] = 1, zeros up to kXStride.
  float* x = xs + hl * kXStride;
  if (j == 0) {
#pragma unroll
    for (int s = 0; s < kShape; ++s) x[x_pos(s)] = beta[s];
    x[x_pos(kK)] = 1.f;
#pragma unroll
    for (int k = kK + 1; k < kXStride; ++k) x[x_pos(k)] = 0.f;
  } else {
#pragma unroll
    for (int m = 0; m < 9; ++m) x[x_pos(kShape + 9 * (j - 1) + m)] = rm[m];
  }
  __syncthreads();
  const int n_rows = int(n - h0 < 16 ? n - h0 : 16);
  if (joints && !joints_direct) {
    f32x4* jd = reinterpret_cast<f32x4*>(joints + h0 * (kJoints * 3));
    for (int i = tid; i < n_rows * (kJoints * 3 / 4); i += 256) jd[i] = jo4[i];
  }
  f32x4* dst = reinterpret_cast<f32x4*>(features + h0 * kXStride);
  for (int i = tid; i < n_rows * (kXStride / 4); i += 256) dst[i] = xs4[i];
}

// ---------------------------------------------------------------------------
// PCA pose (mano_np.py:66-72) and standalone Rodrigues (:117-148).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pose_from_pca_kernel(
    const float* __restrict__ pca, int n_comps, int64_t pca_stride, const float* __restrict__ rot,
    int64_t rot_stride, const float* __restrict__ basis, const float* __restrict__ mean,
    float* __restrict__ pose, int64_t n) {
  const int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x;
  const int64_t h = idx / (kJoints * 3);
  const int m = int(idx - h * (kJoints * 3));
  if (h >= n) return;
  float v;
  if (m < 3) {
    v = rot ? rot[h * rot_stride + m] : 0.f;
  } else {
    const int mm = m - 3;
    v = 0.f;
    const float* c = pca + h * pca_stride;
    for (int i = 0; i < n_comps; ++i) v = fmaf(c[i], basis[i * kPca + mm], v);
    v += mean[mm];
  }
  pose[h * (kJoints * 3) + m] = v;
}

__global__ __launch_bounds__(256) void rodrigues_kernel(const float* __restrict__ aa,
                                                        float* __restrict__ rot, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  float rm[9];
  rodrigues_minus_eye(aa[3 * i], aa[3 * i + 1], aa[3 * i + 2], rm);
#pragma unroll
  for (int k = 0; k < 9; ++k) rot[9 * i + k] = rm[k] + ((k % 4 == 0) ? 1.f : 0.f);
}

}  // namespace

hipError_t launch_articulate(const DeviceModel& m, int64_t n, const float* betas,
                             int64_t betas_stride, const float* pose, const float* trans,
                             float* features, float* transforms, float* joints,
                             float* rest_joints, float* rot_mats, hipStream_t stream,
                             const PcaInput* pca) {
  const int64_t blocks = (n + 15) / 16;
  auto launch = [&](auto kernel, const PcaInput& in) {
    hipLaunchKernelGGL(kernel, dim3(unsigned(blocks)), dim3(256), 0, stream, betas, betas_stride,
                       pose, trans, m.joint_template, m.joint_shape, m.parents, m.depth,
                       m.max_depth, n, features, transforms, joints, rest_joints, rot_mats, in,
                       m.pca_basis, m.pca_mean);
  };
  if (pca) launch(articulate_kernel<true>, *pca);
  else launch(articulate_kernel<false>, PcaInput{});
  return hipGetLastError();
}

hipError_t launch_pose_from_pca(const DeviceModel& m, int64_t n, const float* pca, int n_comps,
                                int64_t pca_stride, const float* rot, int64_t rot_stride,
                                float* pose, hipStream_t stream) {
  const int64_t threads = n * kJoints * 3;
  hipLaunchKernelGGL(pose_from_pca_kernel, dim3(unsigned((threads + 255) / 256)), dim3(256), 0,
                     stream, pca, n_comps, pca_stride, rot, rot_stride, m.pca_basis, m.pca_mean,
                     pose, n);
  return hipGetLastError();
}

hipError_t launch_rodrigues(int64_t n, const float* aa, float* rot, hipStream_t stream) {
  hipLaunchKernelGGL(rodrigues_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, stream, aa,
                     rot, n);
  return hipGetLastError();
}


}  // namespace mano
