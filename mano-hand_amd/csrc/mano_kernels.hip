// mano_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the MANO forward pass.
//
// Reference hot path: MANOModel.update() in /root/reference/mano_np.py:79-115.
// It is split into three launches, all on the caller's stream:
//
//   articulate  one lane per (hand, joint), 32 hands per 512-thread block:
//               Rodrigues (mano_np.py:117-148) in sinc / half-angle form,
//               rest joints J = Jreg.T + (Jreg.S).beta (:83, folded in float64
//               at model load), the 16-joint chain (:96-104) as 3 dependent
//               levels of wavefront shuffles (5 fingers x depth 3), the
//               rest-pose removal (:106-110) and the 135 pose features
//               (R_j - I, :87-91) written straight into MFMA A-fragment tiles.
//   blend       v_posed = T + [beta | features] . [S ; P]   (:81 and :87-93)
//               as one K = 145 GEMM on v_mfma_f32_32x32x2_f32.  Each wave keeps
//               its 32 hands' A fragments in VGPRs for the whole launch; the
//               4 waves of a block share the basis column tile, staged in LDS by
//               global_load_lds (LDS-DMA), double-buffered.
//   skin        LBS (:112-115): one lane per vertex keeps its 16 skinning
//               weights in VGPRs; the hand's 16 3x4 transforms are wave-uniform
//               (scalar loads); v_posed streams in and verts stream out.
#include "mano_internal.h"

namespace mano {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// R - I for one axis-angle vector r = (x, y, z).
// mano_np.py:130-147 computes R = cos I + (1 - cos) r^ r^T + sin [r^]x with
// theta clamped to float64 eps.  With K = [r]x this equals
//   R - I = a K + b K^2,  K^2 = r r^T - theta^2 I,
//   a = sin(theta)/theta, b = (1 - cos theta)/theta^2 = 2 sin^2(theta/2)/theta^2,
// which has no 0/0 and no 1 - cos cancellation in float32.  Below theta = 1e-2
// the Taylor series to theta^4 is exact in float32.  Returning R - I (not R)
// keeps the small pose features of :91 free of the cancellation too.
__device__ __forceinline__ void rodrigues_minus_eye(float x, float y, float z, float rm[9]) {
  const float th2 = x * x + y * y + z * z;
  float a, b;
  if (th2 < 1e-4f) {
    a = 1.0f - th2 * (1.0f / 6.0f) + th2 * th2 * (1.0f / 120.0f);
    b = 0.5f - th2 * (1.0f / 24.0f) + th2 * th2 * (1.0f / 720.0f);
  } else {
    const float th = sqrtf(th2);
    a = sinf(th) / th;
    const float sh = sinf(0.5f * th) / th;
    b = 2.0f * sh * sh;
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
// articulate: 512 threads = 32 hands x 16 joints = exactly one MFMA hand tile.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(512) void articulate_kernel(
    const float* __restrict__ betas, int64_t betas_stride, const float* __restrict__ pose,
    const float* __restrict__ trans, const float* __restrict__ joint_template,
    const float* __restrict__ joint_shape, const int32_t* __restrict__ parents,
    const int32_t* __restrict__ depth, int max_depth, int64_t n,
    float* __restrict__ features, float* __restrict__ transforms, float* __restrict__ joints,
    float* __restrict__ rest_joints, float* __restrict__ rot_mats) {
  __shared__ f32x4 tile[kKGroups * 64];
  float* tilef = reinterpret_cast<float*>(tile);

  const int tid = threadIdx.x;
  const int j = tid & (kJoints - 1);
  const int hl = tid >> 4;  // hand within the tile
  const int64_t h = int64_t(blockIdx.x) * kHandTile + hl;
  const bool valid = h < n;

  float x = 0.f, y = 0.f, z = 0.f;
  if (valid) {
    const float* p = pose + h * (kJoints * 3) + 3 * j;
    x = p[0];
    y = p[1];
    z = p[2];
  }
  float rm[9];
  rodrigues_minus_eye(x, y, z, rm);

  float beta[kShape];
#pragma unroll
  for (int s = 0; s < kShape; ++s) beta[s] = valid ? betas[h * betas_stride + s] : 0.f;

  // Rest joint of joint j (mano_np.py:83, folded: Jreg.(T + S.beta)).
  float J[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float acc = joint_template[j * 3 + c];
#pragma unroll
    for (int s = 0; s < kShape; ++s) acc = fmaf(joint_shape[(j * 3 + c) * kShape + s], beta[s], acc);
    J[c] = acc;
  }

  // World rotation / translation, initialised to the root form G_0 = [R_0 | J_0] (:97).
  float Rw[9], t[3];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rw[i] = rm[i] + ((i % 4 == 0) ? 1.f : 0.f);
  t[0] = J[0];
  t[1] = J[1];
  t[2] = J[2];
  float Rl[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rl[i] = Rw[i];

  // Chain (:98-104): G_j = G_parent . [R_j | J_j - J_parent], one tree level per
  // iteration; the parent's finished transform arrives by a wavefront shuffle.
  const int par = parents[j];
  const int dep = depth[j];
  const int src = ((tid & 63) & ~(kJoints - 1)) + (par < 0 ? 0 : par);
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

  if (valid) {
    // Skinning transform A_j = [Rw | t - Rw J] (rest-pose removal, :106-110).
    float* A = transforms + h * kTransformFloats + j * 12;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      A[r * 4 + 0] = Rw[r * 3 + 0];
      A[r * 4 + 1] = Rw[r * 3 + 1];
      A[r * 4 + 2] = Rw[r * 3 + 2];
      A[r * 4 + 3] = t[r] - (Rw[r * 3 + 0] * J[0] + Rw[r * 3 + 1] * J[1] + Rw[r * 3 + 2] * J[2]);
    }
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
      for (int i = 0; i < 9; ++i) o[i] = Rl[i];
    }
  }

  // Blend-GEMM A operand: X[h][k], k < 10 beta, 10 <= k < 145 features
  // (k = 10 + 9(j-1) + 3 row + col, the ravel order of :91), zeros up to 152.
  // Fragment layout for v_mfma_f32_32x32x2_f32: step s = k/2 holds
  // X[hand = lane & 31][k = 2s + (lane >> 5)]; 4 steps packed per float4.
  auto put = [&](int k, float v) {
    const int s = k >> 1;
    const int ln = hl + 32 * (k & 1);
    tilef[(((s >> 2) * 64) + ln) * 4 + (s & 3)] = v;
  };
  if (j == 0) {
#pragma unroll
    for (int s = 0; s < kShape; ++s) put(s, beta[s]);
#pragma unroll
    for (int k = kK; k < kKGroups * 8; ++k) put(k, 0.f);
  } else {
#pragma unroll
    for (int m = 0; m < 9; ++m) put(kShape + 9 * (j - 1) + m, rm[m]);
  }
  __syncthreads();
  f32x4* dst = reinterpret_cast<f32x4*>(features + int64_t(blockIdx.x) * kTileFloats);
  for (int i = tid; i < kKGroups * 64; i += 512) dst[i] = tile[i];
}

// ---------------------------------------------------------------------------
// blend: 256 threads = 4 waves x 32 hands; loop over all 32-column tiles.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void stage_basis_tile(const float* __restrict__ basis_tiles, int t,
                                                 f32x4* buf, int wave, int lane) {
  const float* src = basis_tiles + int64_t(t) * kTileFloats + lane * 4;
  for (int g = wave; g < kKGroups; g += 4) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + g * 256),
        (__attribute__((address_space(3))) void*)(buf + g * 64), 16, 0, 0);
  }
}

__global__ __launch_bounds__(256, 2) void blend_kernel(
    const float* __restrict__ features, const float* __restrict__ basis_tiles,
    const float* __restrict__ template_cols, float* __restrict__ vposed, int64_t n,
    int n_cols, int n_col_tiles) {
  __shared__ f32x4 bs[2][kKGroups * 64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t ht = int64_t(blockIdx.x) * 4 + wave;
  const int64_t n_ht = (n + kHandTile - 1) / kHandTile;
  const bool active = ht < n_ht;

  float a[kKGroups * 4];
  {
    const f32x4* src = reinterpret_cast<const f32x4*>(features + (active ? ht : 0) * kTileFloats) + lane;
#pragma unroll
    for (int g = 0; g < kKGroups; ++g) {
      const f32x4 v = active ? src[g * 64] : f32x4{0.f, 0.f, 0.f, 0.f};
      a[4 * g + 0] = v[0];
      a[4 * g + 1] = v[1];
      a[4 * g + 2] = v[2];
      a[4 * g + 3] = v[3];
    }
  }

  stage_basis_tile(basis_tiles, 0, bs[0], wave, lane);
  __syncthreads();

  const int hi = lane >> 5;
  const int col_in_tile = lane & 31;
  for (int t = 0; t < n_col_tiles; ++t) {
    if (t + 1 < n_col_tiles) stage_basis_tile(basis_tiles, t + 1, bs[(t + 1) & 1], wave, lane);
    const f32x4* b = bs[t & 1];
    f32x16 acc = {};
#pragma unroll
    for (int g = 0; g < kKGroups; ++g) {
      const f32x4 bv = b[g * 64 + lane];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (4 * g + q < kKSteps) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * g + q], bv[q], acc, 0, 0, 0);
      }
    }
    // D[hand][col]: col = lane & 31, hand = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
    const int col = t * kColTile + col_in_tile;
    if (active && col < n_cols) {
      const float tv = template_cols[col];
      const int64_t h0 = ht * kHandTile;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t h = h0 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (h < n) vposed[h * n_cols + col] = acc[r] + tv;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// skin: lane = vertex, wave = run of kSkinHands hands; grid (hand runs, vertex groups).
// ---------------------------------------------------------------------------
constexpr int kSkinHands = 16;

__global__ __launch_bounds__(256) void skin_kernel(
    const float* __restrict__ weights, const float* __restrict__ transforms,
    const float* __restrict__ vposed, const float* __restrict__ trans, float* __restrict__ verts,
    int64_t n, int n_verts) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int v = blockIdx.y * 64 + lane;
  const bool vvalid = v < n_verts;
  float w[kJoints];
  {
    const f32x4* wp = reinterpret_cast<const f32x4*>(weights + int64_t(vvalid ? v : 0) * kJoints);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 q = vvalid ? wp[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      w[4 * i + 0] = q[0];
      w[4 * i + 1] = q[1];
      w[4 * i + 2] = q[2];
      w[4 * i + 3] = q[3];
    }
  }
  const int64_t h0 = (int64_t(blockIdx.x) * 4 + wave) * kSkinHands;
  const int64_t h1 = h0 + kSkinHands < n ? h0 + kSkinHands : n;
  const int64_t stride = int64_t(n_verts) * 3;
  for (int64_t h = h0; h < h1; ++h) {
    const float* Ah = transforms + h * kTransformFloats;  // wave-uniform -> scalar loads
    float T[12];
#pragma unroll
    for (int m = 0; m < 12; ++m) T[m] = w[0] * Ah[m];
#pragma unroll
    for (int jj = 1; jj < kJoints; ++jj) {
#pragma unroll
      for (int m = 0; m < 12; ++m) T[m] = fmaf(w[jj], Ah[jj * 12 + m], T[m]);
    }
    float t0 = 0.f, t1 = 0.f, t2 = 0.f;
    if (trans) {
      t0 = trans[h * 3 + 0];
      t1 = trans[h * 3 + 1];
      t2 = trans[h * 3 + 2];
    }
    if (vvalid) {
      const float* p = vposed + h * stride + 3 * v;
      const float p0 = p[0], p1 = p[1], p2 = p[2];
      float* o = verts + h * stride + 3 * v;
      o[0] = fmaf(T[0], p0, fmaf(T[1], p1, fmaf(T[2], p2, T[3]))) + t0;
      o[1] = fmaf(T[4], p0, fmaf(T[5], p1, fmaf(T[6], p2, T[7]))) + t1;
      o[2] = fmaf(T[8], p0, fmaf(T[9], p1, fmaf(T[10], p2, T[11]))) + t2;
    }
  }
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
                             float* rest_joints, float* rot_mats, hipStream_t stream) {
  const int64_t blocks = (n + kHandTile - 1) / kHandTile;
  hipLaunchKernelGGL(articulate_kernel, dim3(unsigned(blocks)), dim3(512), 0, stream, betas,
                     betas_stride, pose, trans, m.joint_template, m.joint_shape, m.parents,
                     m.depth, m.max_depth, n, features, transforms, joints, rest_joints, rot_mats);
  return hipGetLastError();
}

hipError_t launch_blend(const DeviceModel& m, int64_t n, const float* features, float* vposed,
                        hipStream_t stream) {
  const int64_t n_ht = (n + kHandTile - 1) / kHandTile;
  const int64_t blocks = (n_ht + 3) / 4;
  hipLaunchKernelGGL(blend_kernel, dim3(unsigned(blocks)), dim3(256), 0, stream, features,
                     m.basis_tiles, m.template_cols, vposed, n, m.n_cols, m.n_col_tiles);
  return hipGetLastError();
}

hipError_t launch_skin(const DeviceModel& m, int64_t n, const float* transforms,
                       const float* vposed, const float* trans, float* verts,
                       hipStream_t stream) {
  const int64_t runs = (n + 4 * kSkinHands - 1) / (4 * kSkinHands);
  const unsigned vgroups = unsigned((m.n_verts + 63) / 64);
  hipLaunchKernelGGL(skin_kernel, dim3(unsigned(runs), vgroups), dim3(256), 0, stream, m.weights,
                     transforms, vposed, trans, verts, n, m.n_verts);
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
