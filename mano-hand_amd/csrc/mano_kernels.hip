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
//               weights in VGPRs; the hand's 16 3x4 transforms reach every
//               lane by DPP row broadcasts (lbs_dpp.h); v_posed streams in and
//               verts stream out.
#include "lbs_dpp.h"
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
    float* __restrict__ features, float* __restrict__ transforms,
    float* __restrict__ features16, float* __restrict__ tfrag16, float* __restrict__ joints,
    float* __restrict__ rest_joints, float* __restrict__ rot_mats) {
  __shared__ f32x4 tile[kKGroups * 64];
  __shared__ f32x4 tile16[2 * kTile16Floats / 4];
  __shared__ f32x4 ttile16[2 * kTFrag16Floats / 4];
  float* tilef = reinterpret_cast<float*>(tile);
  float* tile16f = reinterpret_cast<float*>(tile16);
  float* ttile16f = reinterpret_cast<float*>(ttile16);

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

  // Skinning transform A_j = [Rw | t - Rw J] (rest-pose removal, :106-110).
  float Aj[12];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    Aj[r * 4 + 0] = Rw[r * 3 + 0];
    Aj[r * 4 + 1] = Rw[r * 3 + 1];
    Aj[r * 4 + 2] = Rw[r * 3 + 2];
    Aj[r * 4 + 3] = t[r] - (Rw[r * 3 + 0] * J[0] + Rw[r * 3 + 1] * J[1] + Rw[r * 3 + 2] * J[2]);
  }
  // ... and in the fused kernel's MFMA A-fragment layout (mano_internal.h):
  // hand (hl & 15) of 16-hand tile (hl >> 4), joint j = 4 s + (lane >> 4).
  {
    const int ln16 = (hl & 15) + 16 * (j & 3);
    float* t16 = ttile16f + (hl >> 4) * kTFrag16Floats;
#pragma unroll
    for (int ck = 0; ck < 12; ++ck) t16[(ck * 64 + ln16) * 4 + (j >> 2)] = Aj[ck];
  }
  if (valid) {
    float* A = transforms + h * kTransformFloats + j * 12;
#pragma unroll
    for (int m = 0; m < 12; ++m) A[m] = Aj[m];
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
  // (k = 10 + 9(j-1) + 3 row + col, the ravel order of :91), X[h][145] = 1
  // (selects the template row of the basis), zeros up to 152.
  // Fragment layout for v_mfma_f32_32x32x2_f32: step s = k/2 holds
  // X[hand = lane & 31][k = 2s + (lane >> 5)]; 4 steps packed per float4.
  float* t16 = tile16f + (hl >> 4) * kTile16Floats;
  auto put = [&](int k, float v) {
    const int s = k >> 1;
    const int ln = hl + 32 * (k & 1);
    if (k < kKGroups * 8) tilef[(((s >> 2) * 64) + ln) * 4 + (s & 3)] = v;
    if (k < kGroups16 * 16) {  // 16x16x4 fragments: step s16 = k / 4, lane (hl & 15) + 16 (k & 3)
      const int s16 = k >> 2;
      t16[(((s16 >> 2) * 64) + (hl & 15) + 16 * (k & 3)) * 4 + (s16 & 3)] = v;
    }
  };
  if (j == 0) {
#pragma unroll
    for (int s = 0; s < kShape; ++s) put(s, beta[s]);
    put(kK, 1.f);  // X[:, 145] = 1 multiplies the template row of the basis
#pragma unroll
    for (int k = kK + 1; k < kGroups16 * 16; ++k) put(k, 0.f);
  } else {
#pragma unroll
    for (int m = 0; m < 9; ++m) put(kShape + 9 * (j - 1) + m, rm[m]);
  }
  __syncthreads();
  f32x4* dst = reinterpret_cast<f32x4*>(features + int64_t(blockIdx.x) * kTileFloats);
  for (int i = tid; i < kKGroups * 64; i += 512) dst[i] = tile[i];
  f32x4* d16 = reinterpret_cast<f32x4*>(features16 + int64_t(blockIdx.x) * 2 * kTile16Floats);
  for (int i = tid; i < 2 * kTile16Floats / 4; i += 512) d16[i] = tile16[i];
  f32x4* t16d = reinterpret_cast<f32x4*>(tfrag16 + int64_t(blockIdx.x) * 2 * kTFrag16Floats);
  for (int i = tid; i < 2 * kTFrag16Floats / 4; i += 512) t16d[i] = ttile16[i];
}

// ---------------------------------------------------------------------------
// blend: 256 threads = 4 waves x 32 hands; loop over all 32-column tiles.
// ---------------------------------------------------------------------------
template <int kWaves = 4>
__device__ __forceinline__ void stage_basis_tile(const float* __restrict__ basis_tiles, int t,
                                                 f32x4* buf, int wave, int lane) {
  const float* src = basis_tiles + int64_t(t) * kTileFloats + lane * 4;
  for (int g = wave; g < kKGroups; g += kWaves) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + g * 256),
        (__attribute__((address_space(3))) void*)(buf + g * 64), 16, 0, 0);
  }
}

__device__ __forceinline__ f32x16 mfma_tile(const float (&a)[kKGroups * 4], const f32x4* __restrict__ b,
                                            int lane) {
  // 73 dependent MFMAs (one accumulator; the 64-cycle dependent latency equals
  // the issue interval).  The LDS read of K-group g+1 is issued before the
  // four MFMAs of group g and pinned there with a scheduling barrier, so its
  // latency hides under them (hipcc otherwise sinks it to a wait per group).
  f32x16 acc = {};
  f32x4 bn = b[lane];
#pragma unroll
  for (int g = 0; g < kKGroups; ++g) {
    const f32x4 bv = bn;
    if (g + 1 < kKGroups) bn = b[(g + 1) * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * g + q < kKSteps) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * g + q], bv[q], acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ void store_vposed_tile(float* __restrict__ vposed, const f32x16& acc,
                                                  int64_t h0, int col, int64_t n, int n_cols,
                                                  int hi) {
  // D[hand][col]: col = lane & 31, hand = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
  if (col < n_cols) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t h = h0 + (r & 3) + 8 * (r >> 2) + 4 * hi;
      if (h < n) vposed[h * n_cols + col] = acc[r];
    }
  }
}

__device__ __forceinline__ void stage_basis_tile16(const float* __restrict__ basis16, int t,
                                                   f32x4* buf, int wave, int lane) {
  const float* src = basis16 + int64_t(t) * kTile16Floats + lane * 4;
  for (int g = wave; g < kGroups16; g += 4) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + g * 256),
        (__attribute__((address_space(3))) void*)(buf + g * 64), 16, 0, 0);
  }
}

__global__ __launch_bounds__(256, 2) void blend_kernel(
    const float* __restrict__ features, const float* __restrict__ basis_tiles,
    float* __restrict__ vposed, int64_t n, int n_cols, int n_col_tiles) {
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
      const f32x4 v = src[g * 64];
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
  const int64_t h0 = ht * kHandTile;
  // The template is row k = 145 of the basis (X[:, 145] = 1), so the MFMA chain
  // yields v_posed directly.  Tile t's stores are issued one iteration late,
  // before tile t+2's LDS-DMA, so the barrier's vmcnt(0) only waits on old
  // stores and the DMA the MFMA chain has already hidden.
  f32x16 prev = {};
  for (int t = 0; t < n_col_tiles; ++t) {
    if (active && t > 0) store_vposed_tile(vposed, prev, h0, (t - 1) * kColTile + col_in_tile, n, n_cols, hi);
    if (t + 1 < n_col_tiles) stage_basis_tile(basis_tiles, t + 1, bs[(t + 1) & 1], wave, lane);
    prev = mfma_tile(a, bs[t & 1], lane);
    __syncthreads();
  }
  if (active) store_vposed_tile(vposed, prev, h0, (n_col_tiles - 1) * kColTile + col_in_tile, n, n_cols, hi);
}

// ---------------------------------------------------------------------------
// blend_skin16: the fused kernel on v_mfma_f32_16x16x4_f32 (16-hand tiles,
// 16-vertex groups).  Same algorithm as blend_skin (GEMM tiles x, y, z of a
// vertex group + 12 LBS transform tiles, register-local apply), but a wave
// needs ~half the registers (37 A-fragment VGPRs, 4-register accumulators),
// so the transform fragments stay resident and 3 waves share each SIMD --
// enough to cover the 40-cycle dependent latency of the 16x16x4 chains and
// each other's barrier / LDS / store stalls.
// ---------------------------------------------------------------------------
typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16_tile(const float (&a)[kGroups16 * 4],
                                             const f32x4* __restrict__ b, int lane) {
  f32x4 acc = {};
  f32x4 bn = b[lane];
#pragma unroll
  for (int g = 0; g < kGroups16; ++g) {
    const f32x4 bv = bn;
    if (g + 1 < kGroups16) bn = b[(g + 1) * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * g + q < kSteps16) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * g + q], bv[q], acc, 0, 0, 0);
  }
  return acc;
}

template <bool kTrans>
__global__ __launch_bounds__(256, 3) void blend_skin16_kernel(
    const float* __restrict__ features16, const float* __restrict__ basis16,
    const float* __restrict__ wfrag16, const float* __restrict__ tfrag16,
    const float* __restrict__ trans, float* __restrict__ verts, float* __restrict__ vposed,
    int64_t n, int n_verts, int n_groups) {
  __shared__ f32x4 bs[2][kGroups16 * 64];  // basis tile ring 2 x 10 KB
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nt16 = (n + 15) / 16;
  const int64_t t16 = int64_t(blockIdx.x) * 4 + wave;
  const bool active = t16 < nt16;
  const int64_t tc = active ? t16 : nt16 - 1;
  const int64_t h0 = tc * 16;
  const int row0 = 4 * (lane >> 4);  // D rows (hands) of this lane: row0 + r
  const int col = lane & 15;         // D column (vertex of the group)

  float a[kGroups16 * 4];
  {
    const f32x4* src = reinterpret_cast<const f32x4*>(features16 + tc * kTile16Floats) + lane;
#pragma unroll
    for (int g = 0; g < kGroups16; ++g) {
      const f32x4 v = src[g * 64];
      a[4 * g + 0] = v[0];
      a[4 * g + 1] = v[1];
      a[4 * g + 2] = v[2];
      a[4 * g + 3] = v[3];
    }
  }
  f32x4 F[12];  // LBS A fragments, tile (c, k) = c * 4 + k, resident for all groups
  {
    const f32x4* src = reinterpret_cast<const f32x4*>(tfrag16 + tc * kTFrag16Floats) + lane;
#pragma unroll
    for (int i = 0; i < 12; ++i) F[i] = src[i * 64];
  }
  __shared__ float trs[4][16 * 3];  // the wave's 16 translations, read back at the stores
  if constexpr (kTrans) {
    if (lane < 48) {
      const int64_t h = h0 + lane / 3;
      trs[wave][lane] = trans[(h < n ? h : n - 1) * 3 + lane % 3];
    }
  }
  const int vstride32 = 3 * n_verts;
  const int64_t n_left = n - h0;
  const int n_valid = active ? (n_left < 16 ? int(n_left) : 16) : 0;
  float* vtile = verts + h0 * int64_t(vstride32);
  float* ptile = vposed ? vposed + h0 * int64_t(vstride32) : nullptr;
  const int n_tiles = 3 * n_groups;

  stage_basis_tile16(basis16, 0, bs[0], wave, lane);
  __syncthreads();

  for (int grp = 0; grp < n_groups; ++grp) {
    const f32x4 wf = reinterpret_cast<const f32x4*>(wfrag16 + int64_t(grp) * kWFrag16Floats)[lane];
    f32x4 p[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int t = 3 * grp + q;
      if (t + 1 < n_tiles) stage_basis_tile16(basis16, t + 1, bs[(t + 1) & 1], wave, lane);
      p[q] = mfma16_tile(a, bs[t & 1], lane);
      __syncthreads();
    }
    int vb = grp * 16;
    if (vb > n_verts - 16) vb = n_verts - 16;
    const int voff = 3 * (vb + col);
    f32x4 out[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = 3 - kk;  // translation column first, as in the skin kernel
        const f32x4 f = F[c * 4 + k];
        f32x4 T = {};
        T = __builtin_amdgcn_mfma_f32_16x16x4f32(f[0], wf[0], T, 0, 0, 0);
        T = __builtin_amdgcn_mfma_f32_16x16x4f32(f[1], wf[1], T, 0, 0, 0);
        T = __builtin_amdgcn_mfma_f32_16x16x4f32(f[2], wf[2], T, 0, 0, 0);
        T = __builtin_amdgcn_mfma_f32_16x16x4f32(f[3], wf[3], T, 0, 0, 0);
        if (k == 3) {
          out[c] = T;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) out[c][r] = fmaf(T[r], p[k][r], out[c][r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hr = row0 + r;
      if (hr < n_valid) {
        float o0 = out[0][r], o1 = out[1][r], o2 = out[2][r];
        if constexpr (kTrans) {
          o0 += trs[wave][hr * 3 + 0];
          o1 += trs[wave][hr * 3 + 1];
          o2 += trs[wave][hr * 3 + 2];
        }
        float* o = vtile + unsigned(hr * vstride32 + voff);
        o[0] = o0;
        o[1] = o1;
        o[2] = o2;
        if (ptile) {
          float* pv = ptile + unsigned(hr * vstride32 + voff);
          pv[0] = p[0][r];
          pv[1] = p[1][r];
          pv[2] = p[2][r];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// skin: lane = vertex, wave = run of kSkinHands hands; grid (hand runs, vertex groups).
// ---------------------------------------------------------------------------
constexpr int kSkinHands = 16;

__global__ __launch_bounds__(256) void skin_kernel(
    const float* __restrict__ weights, const float* __restrict__ transforms,
    const float* __restrict__ vposed, const float* __restrict__ trans, int trans_stride,
    float* __restrict__ verts, int64_t n, int n_verts) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // No lane is ever masked: the last vertex group is shifted back to end at
  // vertex V-1 (it re-computes, and re-writes with identical values, a few
  // vertices of the previous group), and an odd tail hand is processed twice.
  // Branch-free bodies keep hipcc from sinking the blend into a store branch
  // or waiting vmcnt(0) at control-flow joins.
  int vbase = int(blockIdx.y) * 64;
  if (vbase > n_verts - 64) vbase = n_verts - 64;
  if (vbase < 0) vbase = 0;
  const int v = min(vbase + lane, n_verts - 1);
  float w[kJoints];
  {
    const f32x4* wp = reinterpret_cast<const f32x4*>(weights + int64_t(v) * kJoints);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 q = wp[i];
      w[4 * i + 0] = q[0];
      w[4 * i + 1] = q[1];
      w[4 * i + 2] = q[2];
      w[4 * i + 3] = q[3];
    }
  }
  const int64_t h0 = (int64_t(blockIdx.x) * 4 + wave) * kSkinHands;
  if (h0 >= n) return;
  const int cnt = int(n - h0 < kSkinHands ? n - h0 : kSkinHands);  // hands of this wave
  const int64_t stride = int64_t(n_verts) * 3;
  const float* vrow = vposed + h0 * stride + 3 * v;
  float* orow = verts + h0 * stride + 3 * v;
  const float* Abase = transforms + h0 * kTransformFloats;
  // v_posed rows and transforms ping-pong: each buffer is re-loaded (two
  // hands ahead) right after it is consumed, so no register rotation waits on
  // a fresh load and ~2 hands of loads stay in flight per wave.
  float P[2][3], AJ[2][12];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int k = min(u, cnt - 1);
    const float* q = vrow + int64_t(k) * stride;
    P[u][0] = q[0];
    P[u][1] = q[1];
    P[u][2] = q[2];
    lbs_load_joint_row(Abase + k * kTransformFloats, lane, AJ[u]);
  }
  for (int i = 0; i < cnt; i += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = min(i + u, cnt - 1);
      float T[12];
      lbs_blend16(T, AJ[u], w);
      const float* tp = trans + (h0 + k) * trans_stride;  // stride 0: a zero vector
      const float t0 = tp[0], t1 = tp[1], t2 = tp[2];
      const float p0 = P[u][0], p1 = P[u][1], p2 = P[u][2];
      const int kn = min(i + u + 2, cnt - 1);
      const float* q = vrow + int64_t(kn) * stride;
      P[u][0] = q[0];
      P[u][1] = q[1];
      P[u][2] = q[2];
      lbs_load_joint_row(Abase + kn * kTransformFloats, lane, AJ[u]);
      float* o = orow + int64_t(k) * stride;
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
                             float* features, float* transforms, float* features16,
                             float* tfrag16, float* joints,
                             float* rest_joints, float* rot_mats, hipStream_t stream) {
  const int64_t blocks = (n + kHandTile - 1) / kHandTile;
  hipLaunchKernelGGL(articulate_kernel, dim3(unsigned(blocks)), dim3(512), 0, stream, betas,
                     betas_stride, pose, trans, m.joint_template, m.joint_shape, m.parents,
                     m.depth, m.max_depth, n, features, transforms, features16, tfrag16, joints,
                     rest_joints, rot_mats);
  return hipGetLastError();
}

hipError_t launch_blend(const DeviceModel& m, int64_t n, const float* features, float* vposed,
                        hipStream_t stream) {
  const int64_t n_ht = (n + kHandTile - 1) / kHandTile;
  const int64_t blocks = (n_ht + 3) / 4;
  hipLaunchKernelGGL(blend_kernel, dim3(unsigned(blocks)), dim3(256), 0, stream, features,
                     m.basis_tiles, vposed, n, m.n_cols, m.n_col_tiles);
  return hipGetLastError();
}

hipError_t launch_blend_skin(const DeviceModel& m, int64_t n, const float* features16,
                             const float* tfrag16, const float* trans, float* verts,
                             float* vposed, hipStream_t stream) {
  const int64_t nt16 = (n + 15) / 16;
  const dim3 grid{unsigned((nt16 + 3) / 4)}, block{256u};
  if (trans)
    hipLaunchKernelGGL(blend_skin16_kernel<true>, grid, block, 0, stream, features16, m.basis16,
                       m.wfrag16, tfrag16, trans, verts, vposed, n, m.n_verts, m.n_groups16);
  else
    hipLaunchKernelGGL(blend_skin16_kernel<false>, grid, block, 0, stream, features16, m.basis16,
                       m.wfrag16, tfrag16, trans, verts, vposed, n, m.n_verts, m.n_groups16);
  return hipGetLastError();
}

hipError_t launch_skin(const DeviceModel& m, int64_t n, const float* transforms,
                       const float* vposed, const float* trans, float* verts,
                       hipStream_t stream) {
  const int64_t runs = (n + 4 * kSkinHands - 1) / (4 * kSkinHands);
  const unsigned vgroups = unsigned((m.n_verts + 63) / 64);
  hipLaunchKernelGGL(skin_kernel, dim3(unsigned(runs), vgroups), dim3(256), 0, stream, m.weights,
                     transforms, vposed, trans ? trans : m.zeros, trans ? 3 : 0, verts, n,
                     m.n_verts);
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
