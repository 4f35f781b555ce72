// mano_internal.h -- device-buffer layout shared by the C-ABI host code
// (mano_abi.hip) and the gfx950 kernels (mano_kernels.hip).  Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mano {

constexpr int kJoints = 16;                    // mano_np.py:35
constexpr int kShape = 10;                     // mano_np.py:36
constexpr int kPoseFeats = 9 * (kJoints - 1);  // 135, mano_np.py:87-91
constexpr int kPca = 45;                       // dump_model.py:8

// Blend GEMM operand geometry (v_mfma_f32_32x32x2_f32: one K-pair per step).
// Row k of the combined basis: k < 10 shape direction k, 10 <= k < 145 pose
// direction k - 10, k = 145 zero pad.
constexpr int kK = kShape + kPoseFeats;        // 145
constexpr int kKSteps = (kK + 1) / 2;          // 73 MFMA steps (K padded to 146)
constexpr int kKGroups = (kKSteps + 3) / 4;    // 19 float4 groups per lane
constexpr int kTileFloats = kKGroups * 64 * 4; // 4864 floats = 19,456 B per tile
constexpr int kHandTile = 32;                  // hands per MFMA row tile
constexpr int kColTile = 32;                   // basis columns per MFMA col tile
constexpr int kTransformFloats = kJoints * 12; // 3x4 skinning transform per joint
// Blend GEMM A operand X (the per-hand row [beta | features | 1 | 0 ...]) in
// the workspace: one row of kXStride floats per hand, k-permuted within each
// block of 16 so that a v_mfma_f32_16x16x4_f32 A-fragment lane reads its four
// consecutive steps with one dwordx4: row position 16 g + 4 r + q holds
//   k = 16 g + 4 q + r        (r = lane >> 4 of the reading lane, q = step % 4)
// i.e. x_pos(k) = 16 (k >> 4) + 4 (k & 3) + ((k >> 2) & 3).  K is padded to
// 160 with zeros (X[:, 145] = 1 multiplies the template row of the basis).
constexpr int kXStride = 160;
__host__ __device__ constexpr int x_pos(int k) { return 16 * (k >> 4) + 4 * (k & 3) + ((k >> 2) & 3); }
// Fused blend_skin kernel operands (v_mfma_f32_16x16x4_f32, 16-hand tiles,
// 16-vertex groups; the LBS transforms T_{c,k}[hand][v] = sum_j A_j[c][k] W[v][j]
// are one 16x16 tile per (c, k) over K = 16 joints):
//   A fragments (from X) per 16 hands, lane l, step s = 4g + q:
//       X[16 t + (l & 15)][k = 4 s + (l >> 4)]            (K padded to 160)
//   basis16 per vertex group (3 tiles x, y, z): [10][64][4]:
//       B[k = 4 s + (l >> 4)][3 (vb + (l & 15)) + coord]
//   LBS A fragments per 16 hands (read from the [n][16][3][4] transforms):
//       F_{c,k}[q] = A_{4 q + (l >> 4)}(16 t + (l & 15))[c][k]
//   wfrag16 per vertex group: [64][4]: W[vb + (l & 15)][4 s + (l >> 4)]
constexpr int kSteps16 = (kK + 1 + 3) / 4;     // 37 MFMA steps (K = 146 -> 148)
constexpr int kGroups16 = (kSteps16 + 3) / 4;  // 10 float4 groups per lane
constexpr int kTile16Floats = kGroups16 * 64 * 4;   // 2560 floats = 10 KB
constexpr int kWFrag16Floats = 64 * 4;         // 256 floats per 16-vertex group

// f16x3 precision mode (mano_kernels_h3.hip): every fp32 operand x is carried
// as an unevaluated pair of halves x = hi + lo (hi = f16(x), lo = f16(x - hi),
// 22 significant bits) and each product as hi.hi + hi.lo + lo.hi on
// v_mfma_f32_16x16x32_f16: the three partial products are exact in the fp32
// accumulator, only lo.lo (< 2^-22 relative) is dropped.  Operands are scaled
// by powers of two so their lo halves stay normal (scaling is exact).
//   A operand of the blend GEMM: the X rows (unscaled), read from the same
//     k-permuted fp32 rows the fp32 path uses and split in registers.
//   B operand: the basis x 2^basis_exp, pre-split at model load into
//     basis_h3[group][piece][64 lanes][8 halves], one 1-KB piece per
//     (coord c, part hi/lo, K-step s of 32) = (2c + part) * 5 + s, pieces 30/31
//     the LBS weight fragments [Wh ; Wh] and [Wl ; 0] (x 2^kH3WeightExp).
//     Lane l of a K-step-s piece holds B[k = 32 s + 8 (l >> 4) + j][vertex
//     vb + (l & 15)], j = 0..7 (the 16x16x32 operand map).
//   LBS A operand: transforms x 2^kH3FrameExp, split per lane at load:
//     lane l holds [Fh | Fl](hand l & 15)[k = 8 (l >> 4) + j] with k < 16 the
//     hi halves of joints 0..15 and k >= 16 the lo halves, so
//     [Fh | Fl] . [Wh ; Wh] + [Fh | Fl] . [Wl ; 0] = Fh Wh + Fl Wh + Fh Wl.
constexpr int kH3Steps = 5;                          // K = 160 = 5 x 32
constexpr int kH3PieceHalves = 64 * 8;               // one 1-KB fragment piece
constexpr int kH3WPiece = 6 * kH3Steps;              // 30: [Wh ; Wh], 31: [Wl ; 0]
constexpr int kH3GroupPieces = kH3WPiece + 2;        // 32 KB per 16-vertex group
constexpr int kH3GroupHalves = kH3GroupPieces * kH3PieceHalves;
constexpr int kH3FrameExp = 6;                       // transforms x 64 (|A| < 1000)
constexpr int kH3WeightExp = 14;                     // weights x 16384 (|W| <= 1)

// Device-resident model buffer (float32, layouts chosen for the kernels).
struct DeviceModel {
  float* basis_tiles;   // [n_col_tiles][kKGroups][64][4] MFMA B fragments
  float* weights;       // [V][16] skinning weights
  float* joint_template;// [16][3]   J_regressor . mesh_template       (float64 fold)
  float* joint_shape;   // [16][3][10] J_regressor . mesh_shape_basis (float64 fold)
  int32_t* parents;     // [16], -1 at the root
  int32_t* depth;       // [16] depth in the kinematic tree (root 0)
  float* pca_basis;     // [45][45]
  float* pca_mean;      // [45]
  float* zeros;         // [64] zero vector (stand-in operand for an absent trans)
  float* basis16;       // [n_groups16][3][kTile16Floats]
  float* wfrag16;       // [n_groups16][kWFrag16Floats]
  uint16_t* basis_h3;   // [n_groups16][kH3GroupHalves] f16 bits (f16x3 mode)
  float h3_vposed_unscale;  // 2^-basis_exp: GEMM accumulator -> v_posed
  float h3_lbs_unscale;     // 2^-(kH3FrameExp + kH3WeightExp): LBS sum -> verts
  int32_t precision;    // MANO_PRECISION_* of mano_forward / blend_skin / skin
  int32_t has_pca;      // created with pose_pca_basis / pose_pca_mean
  int32_t max_depth;
  int32_t n_verts;
  int32_t n_cols;       // 3V
  int32_t n_col_tiles;  // ceil(3V / 32)
  int32_t n_groups16;   // ceil(V / 16) groups of the 16x16 fused kernel (last one shifted)
  int32_t n_cu;         // compute units of the device (sizes the persistent grids)
};

// Workspace carving (all offsets 256-B aligned).
struct Workspace {
  size_t features_off, transforms_off, vposed_off, total;
};

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

inline Workspace workspace_layout(const DeviceModel& m, int64_t n) {
  Workspace w;
  w.features_off = 0;
  w.transforms_off = align256(w.features_off + size_t(n) * kXStride * sizeof(float));
  w.vposed_off = align256(w.transforms_off + size_t(n) * kTransformFloats * sizeof(float));
  w.total = align256(w.vposed_off + size_t(n) * m.n_cols * sizeof(float));
  return w;
}

// PCA pose input of the articulation (mano_forward_pca): pose = [rot |
// pca[:n_comps] . pose_pca_basis[:n_comps] + mean] (mano_np.py:66-72).
struct PcaInput {
  const float* pca;
  int32_t n_comps;
  int64_t pca_stride;
  const float* rot;      // nullable: zero root rotation
  int64_t rot_stride;
  float* pose_out;       // nullable: the [n][16][3] pose used
};

// Kernel launchers (mano_kernels.hip).  All asynchronous on `stream`.
// `pca` non-NULL: the pose comes from PCA coefficients (`pose` unused).
hipError_t launch_articulate(const DeviceModel& m, int64_t n, const float* betas,
                             int64_t betas_stride, const float* pose, const float* trans,
                             float* features, float* transforms, float* joints,
                             float* rest_joints, float* rot_mats, hipStream_t stream,
                             const PcaInput* pca = nullptr);
hipError_t launch_blend(const DeviceModel& m, int64_t n, const float* features,
                        float* vposed, hipStream_t stream);
hipError_t launch_blend_skin(const DeviceModel& m, int64_t n, const float* features,
                             const float* transforms, const float* trans, float* verts,
                             float* vposed, hipStream_t stream);
hipError_t launch_skin(const DeviceModel& m, int64_t n, const float* transforms,
                       const float* vposed, const float* trans, float* verts,
                       hipStream_t stream);
// f16x3 mode (mano_kernels_h3.hip): same operands and outputs as
// launch_blend_skin / launch_skin.
hipError_t launch_blend_skin_h3(const DeviceModel& m, int64_t n, const float* features,
                                const float* transforms, const float* trans, float* verts,
                                float* vposed, hipStream_t stream);
hipError_t launch_skin_h3(const DeviceModel& m, int64_t n, const float* transforms,
                          const float* vposed, const float* trans, float* verts,
                          hipStream_t stream);
hipError_t launch_pose_from_pca(const DeviceModel& m, int64_t n, const float* pca,
                                int n_comps, int64_t pca_stride, const float* rot,
                                int64_t rot_stride, float* pose, hipStream_t stream);
hipError_t launch_rodrigues(int64_t n, const float* aa, float* rot, hipStream_t stream);
hipError_t launch_synthetic_inputs(uint64_t seed, int64_t first, int64_t n, float beta_sigma,
                                   float pose_sigma, float trans_range, float* betas, float* pose,
                                   float* trans, hipStream_t stream);

}  // namespace mano
