// mano_internal.h -- the device model buffer, workspace carving and kernel
// launchers shared by the C-ABI host code (mano_abi.hip) and the gfx950
// kernels (mano_kernels*.hip).  Layout constants: mano_layout.h.  Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "mano_layout.h"

namespace mano {

// Device-resident model buffer (float32, layouts chosen for the kernels).
struct DeviceModel {
  float* basis_tiles;   // [n_col_tiles][kKGroups][64][4] MFMA B fragments
  float* basis_tiles_v; // [kAlignVariants][n_col_tiles][...] sector-aligned variants (NULL: none, mano_layout.h)
  float* weights;       // [V][16] skinning weights
  float* joint_template;// [16][3]   J_regressor . mesh_template       (float64 fold)
  float* joint_shape;   // [16][3][10] J_regressor . mesh_shape_basis (float64 fold)
  int32_t* parents;     // [16], -1 at the root
  int32_t* depth;       // [16] depth in the kinematic tree (root 0)
  float* pca_basis;     // [45][45]
  float* pca_mean;      // [45]
  float* zeros;         // [64] zero vector (stand-in operand for an absent trans)
  int32_t* status;      // status flags [kStatusFlags] (device address of pinned host memory):
                        // flag b is set to 1 by a kernel raising MANO_DEVICE_* bit 1 << b
  float* basis16;       // [n_groups16][3][kTile16Floats]
  float* wfrag16;       // [n_groups16][kWFrag16Floats]
  float* basis16v;      // [kAlignVariants][n_groups16][3][kTile16Floats] sector-aligned variants,
  float* wfrag16v;      // [kAlignVariants][n_groups16][kWFrag16Floats]   NULL when V has none (mano_layout.h)
  uint16_t* basis_h3;   // [n_groups16][kH3GroupHalves] f16 bits (f16x3 mode)
  uint16_t* basis_h3v;  // [kAlignVariants][n_groups16][kH3GroupHalves] sector-aligned variants (or NULL)
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

constexpr int kStatusFlags = 16;  // one int32 per MANO_DEVICE_* bit (64 B)

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
// The 4-hand-unit fp32 LBS (mano_skin_quad.hip); launch_skin uses it when
// skin_quad_supported(m) (16 <= V <= 832: W of every group resident in LDS).
bool skin_quad_supported(const DeviceModel& m);
// `in_place` (verts == vposed): skin_pair's in-place fp32 units, when
// skin_in_place_supported(m, n); otherwise hipErrorNotSupported (the caller
// then stages the rows elsewhere first).
bool skin_in_place_supported(const DeviceModel& m, int64_t n);
hipError_t launch_skin_quad(const DeviceModel& m, int64_t n, const float* transforms,
                            const float* vposed, const float* trans, float* verts,
                            hipStream_t stream, bool h3 = false, bool in_place = false);
// f16x3 mode (mano_kernels_h3.hip): same operands and outputs as
// launch_blend_skin (verts only: no v_posed output) / launch_skin.
hipError_t launch_blend_skin_h3(const DeviceModel& m, int64_t n, const float* features,
                                const float* transforms, const float* trans, float* verts,
                                hipStream_t stream);
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
