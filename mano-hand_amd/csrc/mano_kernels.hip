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
// blend_skin: the blend GEMM with LBS fused behind it.
//
// One 768-thread block = 4 "M" waves + 8 "S" waves (one M and two S per SIMD),
// 128 hands.  M wave w keeps its 32 hands' A fragments in VGPRs and runs the
// MFMA chains; the block's four M waves share each basis tile, staged in LDS by
// LDS-DMA (double-buffered, one barrier per tile).  Vertices come in groups of
// 32 whose basis columns are packed as three tiles (x, y, z of the same 32
// vertices), so after a group's three tiles lane l of M wave w holds the full
// v_posed point of vertex (l & 31) for 16 hands.  It hands those 48 values to
// its two S waves through LDS; they blend the skinning transforms (DPP row
// broadcasts, lbs_dpp.h) and write verts while the M wave already runs the
// next group's MFMAs -- the MFMA pipe and the VALU of every SIMD stay busy at
// once and v_posed never touches HBM.
//
// Barrier-delimited iteration t:  M waves compute tile t (group t/3);  S waves
// skin group t/3 - 1, in three chunks (one per tile of the current group).
// ---------------------------------------------------------------------------
constexpr int kGroupVerts = 32;
constexpr int kFusedM = 4;                   // M waves per block
constexpr int kFusedThreads = kFusedM * 3 * 64;
constexpr int kVpFloats = 3 * 16 * 64;       // one M wave's v_posed hand-off: [q][r/4][lane][4]

__device__ __forceinline__ f32x16 mfma_tile(const float (&a)[kKGroups * 4], const f32x4* __restrict__ b,
                                            int lane) {
  f32x16 acc = {};
  f32x4 bn = b[lane];
#pragma unroll
  for (int g = 0; g < kKGroups; ++g) {
    const f32x4 bv = bn;
    if (g + 1 < kKGroups) bn = b[(g + 1) * 64 + lane];  // next group's fragments in flight
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * g + q < kKSteps) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * g + q], bv[q], acc, 0, 0, 0);
  }
  return acc;
}

// Block barriers of the fused kernel.  __syncthreads() would also drain every
// outstanding global store and load (vmcnt(0)) of the S waves at each of the
// ~78 barriers; only LDS traffic is handed across them.  M waves wait for their
// LDS-DMA basis staging (vmcnt) and v_posed LDS writes (lgkmcnt); S waves only
// for their LDS reads.  The "memory" clobber keeps the compiler from moving
// LDS accesses across.
__device__ __forceinline__ void barrier_m() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void barrier_s() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void put_acc(f32x4* __restrict__ dst, const f32x16& acc, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) dst[j * 64 + lane] = f32x4{acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]};
}

template <bool kTrans>
__global__ __launch_bounds__(kFusedThreads, 1) void blend_skin_kernel(
    const float* __restrict__ features, const float* __restrict__ basis_groups,
    const float* __restrict__ template_groups, const float* __restrict__ weights,
    const float* __restrict__ transforms, const float* __restrict__ trans,
    float* __restrict__ verts, float* __restrict__ vposed, int64_t n, int n_verts,
    int n_groups) {
  __shared__ f32x4 bs[2][kKGroups * 64];              // basis tile ring      38,912 B
  __shared__ f32x4 vps[2][kFusedM][kVpFloats / 4];    // v_posed hand-off     98,304 B
  __shared__ float trs[kFusedM][kHandTile][4];         // translations          2,048 B
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool is_m = wave < kFusedM;
  const int mw = is_m ? wave : (wave - kFusedM) >> 1;  // M wave (hand tile) this wave serves
  const int sh = (wave - kFusedM) & 1;                 // S waves: which half of the 16 rows
  const int64_t n_ht = (n + kHandTile - 1) / kHandTile;
  const int64_t ht = int64_t(blockIdx.x) * kFusedM + mw;
  const int64_t h0 = ht * kHandTile;
  const int n_tiles = 3 * n_groups;
  const int hi = lane >> 5;
  const int col = lane & 31;

  // The two roles run separate loops with the same barrier count (n_tiles + 4
  // s_barrier each), so neither role's registers are live in the other's code.
  if (is_m) {
    float a[kKGroups * 4];
    const int64_t htc = ht < n_ht ? ht : n_ht - 1;
    const f32x4* src = reinterpret_cast<const f32x4*>(features + htc * kTileFloats) + lane;
#pragma unroll
    for (int g = 0; g < kKGroups; ++g) {
      const f32x4 v = src[g * 64];
      a[4 * g + 0] = v[0];
      a[4 * g + 1] = v[1];
      a[4 * g + 2] = v[2];
      a[4 * g + 3] = v[3];
    }
    stage_basis_tile(basis_groups, 0, bs[0], wave, lane);
    barrier_m();
    f32x16 acc0 = {}, acc1 = {};
    for (int t = 0; t < n_tiles + 3; ++t) {
      if (t < n_tiles) {
        if (t + 1 < n_tiles) stage_basis_tile(basis_groups, t + 1, bs[(t + 1) & 1], wave, lane);
        const f32x4* b = bs[t & 1];
        const int q = t % 3;
#ifdef MANO_ABLATE_NO_M  // diagnostic builds only (tools/microbench)
        if (q == 0) {
          acc0 = f32x16{};
        } else if (q == 1) {
          acc1 = f32x16{};
        } else {
          f32x4* dst = vps[(t / 3) & 1][mw];
          put_acc(dst, acc0, lane);
          put_acc(dst + 256, acc1, lane);
          put_acc(dst + 512, acc0, lane);
        }
        (void)b;
#else
        if (q == 0) {
          acc0 = mfma_tile(a, b, lane);
        } else if (q == 1) {
          acc1 = mfma_tile(a, b, lane);
        } else {
          const f32x16 acc2 = mfma_tile(a, b, lane);
          f32x4* dst = vps[(t / 3) & 1][mw];
          put_acc(dst, acc0, lane);
          put_acc(dst + 256, acc1, lane);
          put_acc(dst + 512, acc2, lane);
        }
#endif
      }
      barrier_m();
    }
    return;
  }

  // ---- S waves ----
  // S wave `sh` owns MFMA rows r = 8 sh + i (i = 0..7) of its M wave's tile:
  // row r of lane l is hand h0 + (r & 3) + 8 (r >> 2) + 4 (l >> 5).  The 8 rows'
  // hands never change, so their 16 joint transforms are loaded ONCE into 96
  // VGPRs and reused for all vertex groups; per group an S wave only reads the
  // 24 v_posed values it needs from LDS and streams verts out.
  const int64_t hmax = n - 1;
  const int64_t vstride = int64_t(n_verts) * 3;
  const int64_t hbase = h0 + 16 * sh + 4 * hi;  // row i -> hand hbase + (i & 3) + 8 (i >> 2)
  float AJ[8][12];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t h = hbase + (i & 3) + 8 * (i >> 2);
    lbs_load_joint_row(transforms + (h < hmax ? h : hmax) * kTransformFloats, lane, AJ[i]);
  }
  if constexpr (kTrans) {  // the tile's 32 translations go to LDS (no VGPRs held)
    if (sh == 0 && lane < kHandTile) {
      const int64_t h = h0 + lane;
      const float* tp = trans + (h < hmax ? h : hmax) * 3;
      trs[mw][lane][0] = tp[0];
      trs[mw][lane][1] = tp[1];
      trs[mw][lane][2] = tp[2];
    }
  }
  barrier_s();
  // Pass grp = -1 only keeps the barrier count equal to the M waves' (n_tiles + 3).
  for (int grp = -1; grp < n_groups; ++grp) {
    int vb = grp * kGroupVerts;
    if (vb > n_verts - kGroupVerts) vb = n_verts - kGroupVerts;
    const int v = vb + col;
    float w[kJoints];
    float tx = 0.f, ty = 0.f, tz = 0.f;
    if (grp >= 0) {
      const f32x4* wp = reinterpret_cast<const f32x4*>(weights + int64_t(v) * kJoints);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 qv = wp[i];
        w[4 * i + 0] = qv[0];
        w[4 * i + 1] = qv[1];
        w[4 * i + 2] = qv[2];
        w[4 * i + 3] = qv[3];
      }
      tx = template_groups[(grp * 3 + 0) * kColTile + col];
      ty = template_groups[(grp * 3 + 1) * kColTile + col];
      tz = template_groups[(grp * 3 + 2) * kColTile + col];
    }
    const float* vsrc = reinterpret_cast<const float*>(vps[(grp < 0 ? 0 : grp) & 1][mw]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (grp >= 0) {
        const int li = ((2 * sh + (i >> 2)) * 64 + lane) * 4 + (i & 3);
        const float p0 = vsrc[li] + tx, p1 = vsrc[1024 + li] + ty, p2 = vsrc[2048 + li] + tz;
        float T[12];
        lbs_blend16(T, AJ[i], w);
        float o0 = fmaf(T[0], p0, fmaf(T[1], p1, fmaf(T[2], p2, T[3])));
        float o1 = fmaf(T[4], p0, fmaf(T[5], p1, fmaf(T[6], p2, T[7])));
        float o2 = fmaf(T[8], p0, fmaf(T[9], p1, fmaf(T[10], p2, T[11])));
        if constexpr (kTrans) {
          const int hl = 16 * sh + 4 * hi + (i & 3) + 8 * (i >> 2);
          o0 += trs[mw][hl][0];
          o1 += trs[mw][hl][1];
          o2 += trs[mw][hl][2];
        }
        const int64_t h = hbase + (i & 3) + 8 * (i >> 2);
        if (h < n) {
          float* o = verts + h * vstride + 3 * v;
          o[0] = o0;
          o[1] = o1;
          o[2] = o2;
          if (vposed) {
            float* pv = vposed + h * vstride + 3 * v;
            pv[0] = p0;
            pv[1] = p1;
            pv[2] = p2;
          }
        }
      }
      // three barriers per group, after rows 2, 5 and 7 (one per M-wave tile)
      if (i == 2 || i == 5 || i == 7) barrier_s();
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

hipError_t launch_blend_skin(const DeviceModel& m, int64_t n, const float* features,
                             const float* transforms, const float* trans, float* verts,
                             float* vposed, hipStream_t stream) {
  const int64_t n_ht = (n + kHandTile - 1) / kHandTile;
  const int64_t blocks = (n_ht + kFusedM - 1) / kFusedM;
  if (trans)
    hipLaunchKernelGGL(blend_skin_kernel<true>, dim3(unsigned(blocks)), dim3(kFusedThreads), 0,
                       stream, features, m.basis_groups, m.template_groups, m.weights, transforms,
                       trans, verts, vposed, n, m.n_verts, m.n_groups);
  else
    hipLaunchKernelGGL(blend_skin_kernel<false>, dim3(unsigned(blocks)), dim3(kFusedThreads), 0,
                       stream, features, m.basis_groups, m.template_groups, m.weights, transforms,
                       trans, verts, vposed, n, m.n_verts, m.n_groups);
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
