// mano_abi.hip -- the extern "C" boundary declared in include/mano_hip.h.
//
// Host side of the device-resident model buffer: validates arguments, folds the
// joint regression in float64, packs the blend basis into MFMA B-fragment
// tiles, carves the workspace and launches the kernels of mano_kernels.hip.
// No C++ exception crosses the ABI; errors are status codes + a thread-local
// message.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "../../include/mano_hip.h"
#include "mano_internal.h"

struct mano_model {
  uint32_t magic;
  int device;
  mano::DeviceModel dm;
  void* block;  // single device allocation holding every array of dm
};

namespace {

constexpr uint32_t kMagic = 0x4d414e4fu;  // "MANO"
thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(MANO_EHIP, "%s: %s (%d)", what, hipGetErrorString(e), int(e));
}

// Switch to the model's device for the duration of a call, restore after.
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int check_model(const mano_model* m) {
  if (!m) return fail(MANO_EINVAL, "model handle is NULL");
  if (m->magic != kMagic) return fail(MANO_ESTATE, "model handle is invalid or destroyed");
  return MANO_OK;
}

// `full`: the unfused stages need the v_posed region too; the fused forward
// only the feature tiles and skinning transforms.
int check_workspace(const mano_model* m, int64_t n, const void* ws, size_t ws_bytes,
                    bool full = true) {
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  const size_t need = full ? w.total : w.vposed_off;
  if (!ws) return fail(MANO_EINVAL, "workspace is NULL");
  if (ws_bytes < need)
    return fail(MANO_ESMALL, "workspace has %zu bytes, %zu needed for %lld hands", ws_bytes,
                need, (long long)n);
  if (reinterpret_cast<uintptr_t>(ws) % 256 != 0)
    return fail(MANO_EINVAL, "workspace must be 256-byte aligned");
  return MANO_OK;
}

constexpr int64_t kMaxHands = int64_t(1) << 30;

// IEEE binary16 bits of a float, round to nearest even (host side of the
// f16x3 operand split; overflow saturates to infinity, tiny values go
// subnormal).
uint16_t f16_bits(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) return uint16_t(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0u));
  if (absx >= 0x477ff000u) return uint16_t(sign | 0x7c00u);  // rounds past 65504
  if (absx < 0x38800000u) {  // below the smallest normal half (2^-14): subnormal or zero
    const float a = std::fabs(f) * 16777216.0f;  // units of 2^-24, exact scaling
    const float r = std::nearbyint(a);           // default rounding mode: to nearest even
    return uint16_t(sign | uint32_t(r));
  }
  const uint32_t mant = absx & 0x7fffffu;
  uint32_t h = ((absx >> 23) - 112u) << 10 | (mant >> 13);
  const uint32_t rest = mant & 0x1fffu;
  if (rest > 0x1000u || (rest == 0x1000u && (h & 1u))) ++h;
  return uint16_t(sign | h);
}

float f16_value(uint16_t h) {
  const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  float v = e == 0 ? std::ldexp(float(m), -24) : std::ldexp(float(m | 0x400u), int(e) - 25);
  if (e == 31) v = m ? NAN : INFINITY;
  return (h & 0x8000u) ? -v : v;
}

void split_f16(double x, uint16_t& hi, uint16_t& lo) {
  const float xf = float(x);
  hi = f16_bits(xf);
  lo = f16_bits(xf - f16_value(hi));
}

}  // namespace

namespace mano {
// The thread-local message of mano_last_error(), for the other ABI files.
int set_error(int code, const char* msg) {
  g_last_error = msg;
  return code;
}
}  // namespace mano

extern "C" {

int mano_abi_version(void) { return 2; }

const char* mano_last_error(void) { return g_last_error.c_str(); }

int mano_model_create(int device, int32_t n_verts, const double* mesh_template,
                      const double* mesh_shape_basis, const double* mesh_pose_basis,
                      const double* j_regressor, const double* skinning_weights,
                      const int32_t* parents, const double* pose_pca_basis,
                      const double* pose_pca_mean, mano_model** out) {
  using namespace mano;
  g_last_error.clear();
  if (!out) return fail(MANO_EINVAL, "out is NULL");
  *out = nullptr;
  if (device < 0) return fail(MANO_EINVAL, "device %d is negative", device);
  if (n_verts < 32 || n_verts > (1 << 24))
    return fail(MANO_EINVAL, "n_verts %d out of range [32, 2^24]", n_verts);
  if (!mesh_template || !mesh_shape_basis || !mesh_pose_basis || !j_regressor ||
      !skinning_weights || !parents)
    return fail(MANO_EINVAL, "a required model array is NULL");
  if ((pose_pca_basis == nullptr) != (pose_pca_mean == nullptr))
    return fail(MANO_EINVAL, "pose_pca_basis and pose_pca_mean must both be given or both NULL");
  if (parents[0] != -1) return fail(MANO_EINVAL, "parents[0] must be -1 (root)");
  std::vector<int32_t> depth(kJoints, 0);
  int max_depth = 0;
  for (int i = 1; i < kJoints; ++i) {
    if (parents[i] < 0 || parents[i] >= i)
      return fail(MANO_EINVAL, "parents[%d] = %d must satisfy 0 <= p < %d", i, parents[i], i);
    depth[i] = depth[parents[i]] + 1;
    if (depth[i] > max_depth) max_depth = depth[i];
  }

  int n_dev = 0;
  hipError_t e = hipGetDeviceCount(&n_dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  if (device >= n_dev) return fail(MANO_EINVAL, "device %d >= device count %d", device, n_dev);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  int n_cu = 0;
  e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return hip_fail(e, "hipDeviceGetAttribute(multiprocessor count)");

  const int V = n_verts;
  const int n_cols = 3 * V;
  const int n_col_tiles = (n_cols + kColTile - 1) / kColTile;

  // ---- host float64 folds (J regression into beta space, mano_np.py:83) ----
  std::vector<float> jt(kJoints * 3), js(kJoints * 3 * kShape);
  for (int j = 0; j < kJoints; ++j) {
    for (int c = 0; c < 3; ++c) {
      double acc = 0.0;
      for (int v = 0; v < V; ++v) acc += j_regressor[size_t(j) * V + v] * mesh_template[size_t(v) * 3 + c];
      jt[j * 3 + c] = float(acc);
      for (int s = 0; s < kShape; ++s) {
        double a2 = 0.0;
        for (int v = 0; v < V; ++v)
          a2 += j_regressor[size_t(j) * V + v] * mesh_shape_basis[(size_t(v) * 3 + c) * kShape + s];
        js[(j * 3 + c) * kShape + s] = float(a2);
      }
    }
  }

  // ---- blend basis as MFMA B-fragment tiles ----
  // tile t, group g, lane l, slot q  <-  Basis[k = 2(4g+q) + (l>>5)][col = 32t + (l&31)]
  std::vector<float> tiles(size_t(n_col_tiles) * kTileFloats, 0.f);
  for (int t = 0; t < n_col_tiles; ++t)
    for (int g = 0; g < kKGroups; ++g)
      for (int l = 0; l < 64; ++l)
        for (int q = 0; q < 4; ++q) {
          const int k = 2 * (4 * g + q) + (l >> 5);
          const int col = t * kColTile + (l & 31);
          float v = 0.f;
          if (col < n_cols) {
            if (k < kShape)
              v = float(mesh_shape_basis[size_t(col) * kShape + k]);
            else if (k < kK)
              v = float(mesh_pose_basis[size_t(col) * kPoseFeats + (k - kShape)]);
            else if (k == kK)
              v = float(mesh_template[col]);  // multiplied by X[:, 145] = 1
          }
          tiles[((size_t(t) * kKGroups + g) * 64 + l) * 4 + q] = v;
        }
  // 16x16x4 fused layout: group g = 16 vertices from min(16g, V-16).
  const int n_groups16 = (V + 15) / 16;
  std::vector<float> b16(size_t(n_groups16) * 3 * kTile16Floats, 0.f);
  std::vector<float> w16(size_t(n_groups16) * kWFrag16Floats, 0.f);
  for (int g = 0; g < n_groups16; ++g) {
    const int vb = std::max(0, std::min(16 * g, V - 16));
    for (int l = 0; l < 64; ++l) {
      const int v = vb + (l & 15);
      for (int st = 0; st < 4; ++st)
        if (v < V)
          w16[size_t(g) * kWFrag16Floats + l * 4 + st] =
              float(skinning_weights[size_t(v) * kJoints + 4 * st + (l >> 4)]);
      for (int q = 0; q < 3; ++q)
        for (int gg = 0; gg < kGroups16; ++gg)
          for (int qq = 0; qq < 4; ++qq) {
            const int k = 4 * (4 * gg + qq) + (l >> 4);
            float val = 0.f;
            if (k <= kK && v < V) {
              const size_t colv = size_t(v) * 3 + q;
              val = k < kShape ? float(mesh_shape_basis[colv * kShape + k])
                    : k < kK   ? float(mesh_pose_basis[colv * kPoseFeats + (k - kShape)])
                               : float(mesh_template[colv]);
            }
            b16[((size_t(g) * 3 + q) * kGroups16 + gg) * 256 + l * 4 + qq] = val;
          }
    }
  }
  // f16x3 pieces (mano_internal.h): basis x 2^basis_exp with the largest
  // entry at most 2^14, split hi/lo; weights x 2^kH3WeightExp.
  double bmax = 0.0;
  for (size_t i = 0; i < size_t(V) * 3 * kShape; ++i) bmax = std::max(bmax, std::fabs(mesh_shape_basis[i]));
  for (size_t i = 0; i < size_t(V) * 3 * kPoseFeats; ++i) bmax = std::max(bmax, std::fabs(mesh_pose_basis[i]));
  for (size_t i = 0; i < size_t(V) * 3; ++i) bmax = std::max(bmax, std::fabs(mesh_template[i]));
  const int basis_exp = bmax > 0.0 ? 14 - int(std::ceil(std::log2(bmax))) : 0;
  const double bscale = std::ldexp(1.0, basis_exp), wscale = std::ldexp(1.0, kH3WeightExp);
  std::vector<uint16_t> bh3(size_t(n_groups16) * kH3GroupHalves, 0);
  for (int g = 0; g < n_groups16; ++g) {
    const int vb = std::max(0, std::min(16 * g, V - 16));
    uint16_t* G = bh3.data() + size_t(g) * kH3GroupHalves;
    for (int l = 0; l < 64; ++l) {
      const int v = vb + (l & 15);
      for (int j = 0; j < 8; ++j) {
        const int kq = 8 * (l >> 4) + j;  // K index inside a 32-step
        for (int c = 0; c < 3; ++c)
          for (int s = 0; s < kH3Steps; ++s) {
            const int k = 32 * s + kq;
            double val = 0.0;
            if (k <= kK && v < V) {
              const size_t colv = size_t(v) * 3 + c;
              val = k < kShape ? mesh_shape_basis[colv * kShape + k]
                    : k < kK   ? mesh_pose_basis[colv * kPoseFeats + (k - kShape)]
                               : mesh_template[colv];
            }
            uint16_t hi, lo;
            split_f16(val * bscale, hi, lo);
            G[(size_t((2 * c) * kH3Steps + s) * 64 + l) * 8 + j] = hi;
            G[(size_t((2 * c + 1) * kH3Steps + s) * 64 + l) * 8 + j] = lo;
          }
        uint16_t hi, lo;
        split_f16(skinning_weights[size_t(v) * kJoints + (kq & 15)] * wscale, hi, lo);
        G[(size_t(kH3WPiece) * 64 + l) * 8 + j] = hi;                       // [Wh ; Wh]
        G[(size_t(kH3WPiece + 1) * 64 + l) * 8 + j] = kq < 16 ? lo : 0;     // [Wl ; 0]
      }
    }
  }
  std::vector<float> wts(size_t(V) * kJoints);
  for (size_t i = 0; i < wts.size(); ++i) wts[i] = float(skinning_weights[i]);
  std::vector<float> pca(kPca * kPca, 0.f), pmean(kPca, 0.f), zeros(64, 0.f);
  if (pose_pca_basis) {
    for (int i = 0; i < kPca * kPca; ++i) pca[i] = float(pose_pca_basis[i]);
    for (int i = 0; i < kPca; ++i) pmean[i] = float(pose_pca_mean[i]);
  }

  // ---- one device block, 256-B aligned sub-arrays ----
  struct Part { const void* src; size_t bytes; size_t off; };
  enum { kBasis, kWeights, kJt, kJs, kParents, kDepth, kPcaB, kPcaM, kZeros, kBasis16, kW16, kBasisH3, kNParts };
  std::vector<Part> parts(kNParts);
  parts[kBasis] = {tiles.data(), tiles.size() * 4, 0};
  parts[kWeights] = {wts.data(), wts.size() * 4, 0};
  parts[kJt] = {jt.data(), jt.size() * 4, 0};
  parts[kJs] = {js.data(), js.size() * 4, 0};
  parts[kParents] = {parents, kJoints * 4, 0};
  parts[kDepth] = {depth.data(), kJoints * 4, 0};
  parts[kPcaB] = {pca.data(), pca.size() * 4, 0};
  parts[kPcaM] = {pmean.data(), pmean.size() * 4, 0};
  parts[kZeros] = {zeros.data(), zeros.size() * 4, 0};
  parts[kBasis16] = {b16.data(), b16.size() * 4, 0};
  parts[kW16] = {w16.data(), w16.size() * 4, 0};
  parts[kBasisH3] = {bh3.data(), bh3.size() * 2, 0};
  size_t total = 0;
  for (auto& p : parts) {
    p.off = total;
    total = align256(total + p.bytes);
  }
  void* block = nullptr;
  e = hipMalloc(&block, total);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(model buffer)");
  for (auto& p : parts) {
    e = hipMemcpy(static_cast<char*>(block) + p.off, p.src, p.bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(block);
      return hip_fail(e, "hipMemcpy(model buffer)");
    }
  }
  mano_model* m = new (std::nothrow) mano_model();
  if (!m) {
    (void)hipFree(block);
    return fail(MANO_EINVAL, "out of host memory");
  }
  char* b = static_cast<char*>(block);
  m->magic = kMagic;
  m->device = device;
  m->block = block;
  auto at = [&](int i) { return reinterpret_cast<float*>(b + parts[i].off); };
  m->dm.basis_tiles = at(kBasis);
  m->dm.weights = at(kWeights);
  m->dm.joint_template = at(kJt);
  m->dm.joint_shape = at(kJs);
  m->dm.parents = reinterpret_cast<int32_t*>(at(kParents));
  m->dm.depth = reinterpret_cast<int32_t*>(at(kDepth));
  m->dm.pca_basis = at(kPcaB);
  m->dm.pca_mean = at(kPcaM);
  m->dm.zeros = at(kZeros);
  m->dm.basis16 = at(kBasis16);
  m->dm.wfrag16 = at(kW16);
  m->dm.basis_h3 = reinterpret_cast<uint16_t*>(at(kBasisH3));
  m->dm.h3_vposed_unscale = float(std::ldexp(1.0, -basis_exp));
  m->dm.h3_lbs_unscale = float(std::ldexp(1.0, -(kH3FrameExp + kH3WeightExp)));
  m->dm.precision = MANO_PRECISION_FP32;
  m->dm.has_pca = pose_pca_basis != nullptr;
  m->dm.n_groups16 = n_groups16;
  m->dm.max_depth = max_depth;
  m->dm.n_verts = V;
  m->dm.n_cols = n_cols;
  m->dm.n_col_tiles = n_col_tiles;
  m->dm.n_cu = n_cu;
  *out = m;
  return MANO_OK;
}

int mano_model_destroy(mano_model* m) {
  g_last_error.clear();
  if (!m) return MANO_OK;
  if (m->magic != kMagic) return fail(MANO_ESTATE, "model handle is invalid or destroyed");
  DeviceGuard guard(m->device);
  m->magic = 0;
  hipError_t e = hipFree(m->block);
  delete m;
  if (e != hipSuccess) return hip_fail(e, "hipFree(model buffer)");
  return MANO_OK;
}

int mano_model_info(const mano_model* m, int32_t* n_verts, int32_t* device) {
  if (int rc = check_model(m)) return rc;
  if (n_verts) *n_verts = m->dm.n_verts;
  if (device) *device = m->device;
  return MANO_OK;
}

int mano_model_set_precision(mano_model* m, int32_t precision) {
  g_last_error.clear();
  if (int rc = check_model(m)) return rc;
  if (precision != MANO_PRECISION_FP32 && precision != MANO_PRECISION_F16X3)
    return fail(MANO_EINVAL, "precision %d is not MANO_PRECISION_FP32 (0) or _F16X3 (1)", precision);
  m->dm.precision = precision;
  return MANO_OK;
}

int mano_model_get_precision(const mano_model* m, int32_t* precision) {
  if (int rc = check_model(m)) return rc;
  if (!precision) return fail(MANO_EINVAL, "precision is NULL");
  *precision = m->dm.precision;
  return MANO_OK;
}

size_t mano_workspace_bytes(const mano_model* m, int64_t n) {
  if (check_model(m) || n < 0) return 0;
  return mano::workspace_layout(m->dm, n).total;
}

size_t mano_forward_workspace_bytes(const mano_model* m, int64_t n) {
  if (check_model(m) || n < 0) return 0;
  return mano::workspace_layout(m->dm, n).vposed_off;  // X rows + transforms
}

int mano_workspace_offsets(const mano_model* m, int64_t n, size_t* features_off,
                           size_t* transforms_off, size_t* vposed_off) {
  if (int rc = check_model(m)) return rc;
  if (n < 0) return fail(MANO_EINVAL, "n_hands %lld < 0", (long long)n);
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  if (features_off) *features_off = w.features_off;
  if (transforms_off) *transforms_off = w.transforms_off;
  if (vposed_off) *vposed_off = w.vposed_off;
  return MANO_OK;
}

int mano_stage_articulate(const mano_model* m, int64_t n, const float* betas,
                          int64_t betas_stride, const float* pose, const float* trans,
                          float* joints, float* rest_joints, float* rot_mats, void* ws,
                          size_t ws_bytes, void* stream) {
  if (int rc = check_model(m)) return rc;
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (n == 0) return MANO_OK;
  if (!betas || !pose) return fail(MANO_EINVAL, "betas and pose are required");
  if (betas_stride != 0 && betas_stride < mano::kShape)
    return fail(MANO_EINVAL, "betas_stride %lld must be 0 or >= 10", (long long)betas_stride);
  if (int rc = check_workspace(m, n, ws, ws_bytes, false)) return rc;
  DeviceGuard guard(m->device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  char* base = static_cast<char*>(ws);
  hipError_t e = mano::launch_articulate(
      m->dm, n, betas, betas_stride, pose, trans, reinterpret_cast<float*>(base + w.features_off),
      reinterpret_cast<float*>(base + w.transforms_off), joints, rest_joints, rot_mats,
      static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "articulate launch");
  return MANO_OK;
}

int mano_stage_blend(const mano_model* m, int64_t n, float* rest_verts, void* ws, size_t ws_bytes,
                     void* stream) {
  if (int rc = check_model(m)) return rc;
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (n == 0) return MANO_OK;
  if (int rc = check_workspace(m, n, ws, ws_bytes)) return rc;
  DeviceGuard guard(m->device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  char* base = static_cast<char*>(ws);
  float* vp = rest_verts ? rest_verts : reinterpret_cast<float*>(base + w.vposed_off);
  hipError_t e = mano::launch_blend(m->dm, n, reinterpret_cast<const float*>(base + w.features_off),
                                    vp, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "blend launch");
  return MANO_OK;
}

int mano_stage_skin(const mano_model* m, int64_t n, const float* rest_verts, const float* trans,
                    float* verts, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = check_model(m)) return rc;
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (n == 0) return MANO_OK;
  if (!verts) return fail(MANO_EINVAL, "verts is required");
  if (int rc = check_workspace(m, n, ws, ws_bytes)) return rc;
  DeviceGuard guard(m->device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  char* base = static_cast<char*>(ws);
  const float* vp = rest_verts ? rest_verts : reinterpret_cast<const float*>(base + w.vposed_off);
  auto launch = m->dm.precision == MANO_PRECISION_F16X3 ? mano::launch_skin_h3 : mano::launch_skin;
  hipError_t e =
      launch(m->dm, n, reinterpret_cast<const float*>(base + w.transforms_off), vp,
                        trans, verts, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "skin launch");
  return MANO_OK;
}

int mano_stage_blend_skin(const mano_model* m, int64_t n, float* rest_verts, const float* trans,
                          float* verts, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = check_model(m)) return rc;
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (n == 0) return MANO_OK;
  if (!verts) return fail(MANO_EINVAL, "verts is required");
  if (int rc = check_workspace(m, n, ws, ws_bytes, false)) return rc;
  DeviceGuard guard(m->device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  char* base = static_cast<char*>(ws);
  auto launch = m->dm.precision == MANO_PRECISION_F16X3 ? mano::launch_blend_skin_h3
                                                          : mano::launch_blend_skin;
  hipError_t e = launch(
      m->dm, n, reinterpret_cast<const float*>(base + w.features_off),
      reinterpret_cast<const float*>(base + w.transforms_off), trans, verts, rest_verts,
      static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "blend_skin launch");
  return MANO_OK;
}

int mano_forward(const mano_model* m, int64_t n, const float* betas, int64_t betas_stride,
                 const float* pose, const float* trans, float* verts, float* joints,
                 float* rest_verts, float* rest_joints, float* rot_mats, void* ws,
                 size_t ws_bytes, void* stream) {
  g_last_error.clear();
  if (int rc = check_model(m)) return rc;
  if (n > 0 && !verts) return fail(MANO_EINVAL, "verts is required");
  if (int rc = mano_stage_articulate(m, n, betas, betas_stride, pose, trans, joints, rest_joints,
                                     rot_mats, ws, ws_bytes, stream))
    return rc;
  return mano_stage_blend_skin(m, n, rest_verts, trans, verts, ws, ws_bytes, stream);
}

int mano_pose_from_pca(const mano_model* m, int64_t n, const float* pca, int32_t n_comps,
                       int64_t pca_stride, const float* rot, int64_t rot_stride, float* pose,
                       void* stream) {
  if (int rc = check_model(m)) return rc;
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (n_comps < 0 || n_comps > mano::kPca)
    return fail(MANO_EINVAL, "n_comps %d must be in [0, 45] (mano_np.py:55-56)", n_comps);
  if (pca_stride != 0 && pca_stride < n_comps)
    return fail(MANO_EINVAL, "pca_stride %lld < n_comps %d", (long long)pca_stride, n_comps);
  if (rot_stride != 0 && rot_stride < 3)
    return fail(MANO_EINVAL, "rot_stride %lld must be 0 or >= 3", (long long)rot_stride);
  if (!m->dm.has_pca) return fail(MANO_EINVAL, "the model was created without the PCA arrays");
  if (n == 0) return MANO_OK;
  if (!pose || (n_comps > 0 && !pca)) return fail(MANO_EINVAL, "pose / pca pointer is NULL");
  DeviceGuard guard(m->device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  hipError_t e = mano::launch_pose_from_pca(m->dm, n, pca, n_comps, pca_stride, rot, rot_stride,
                                            pose, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "pose_from_pca launch");
  return MANO_OK;
}

int mano_forward_pca(const mano_model* m, int64_t n, const float* betas, int64_t betas_stride,
                     const float* pca, int32_t n_comps, int64_t pca_stride, const float* rot,
                     int64_t rot_stride, const float* trans, float* verts, float* joints,
                     float* pose_out, float* rest_verts, float* rest_joints, float* rot_mats,
                     void* ws, size_t ws_bytes, void* stream) {
  g_last_error.clear();
  if (int rc = check_model(m)) return rc;
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (!m->dm.has_pca) return fail(MANO_EINVAL, "the model was created without the PCA arrays");
  if (n_comps < 0 || n_comps > mano::kPca)
    return fail(MANO_EINVAL, "n_comps %d must be in [0, 45] (mano_np.py:55-56)", n_comps);
  if (pca_stride != 0 && pca_stride < n_comps)
    return fail(MANO_EINVAL, "pca_stride %lld < n_comps %d", (long long)pca_stride, n_comps);
  if (rot_stride != 0 && rot_stride < 3)
    return fail(MANO_EINVAL, "rot_stride %lld must be 0 or >= 3", (long long)rot_stride);
  if (betas_stride != 0 && betas_stride < mano::kShape)
    return fail(MANO_EINVAL, "betas_stride %lld must be 0 or >= 10", (long long)betas_stride);
  if (n == 0) return MANO_OK;
  if (!betas || !verts || (n_comps > 0 && !pca))
    return fail(MANO_EINVAL, "betas, verts and (for n_comps > 0) pca are required");
  if (int rc = check_workspace(m, n, ws, ws_bytes, false)) return rc;
  DeviceGuard guard(m->device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  char* base = static_cast<char*>(ws);
  const mano::PcaInput in{pca, n_comps, pca_stride, rot, rot_stride, pose_out};
  hipError_t e = mano::launch_articulate(
      m->dm, n, betas, betas_stride, nullptr, trans, reinterpret_cast<float*>(base + w.features_off),
      reinterpret_cast<float*>(base + w.transforms_off), joints, rest_joints, rot_mats,
      static_cast<hipStream_t>(stream), &in);
  if (e != hipSuccess) return hip_fail(e, "articulate (pca) launch");
  return mano_stage_blend_skin(m, n, rest_verts, trans, verts, ws, ws_bytes, stream);
}

// ---- device memory and streams without a framework ----
int mano_alloc(int device, size_t bytes, void** out) {
  g_last_error.clear();
  if (!out) return fail(MANO_EINVAL, "out is NULL");
  *out = nullptr;
  if (device < 0) return fail(MANO_EINVAL, "device %d is negative", device);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  if (bytes == 0) return MANO_OK;
  hipError_t e = hipMalloc(out, bytes);  // 256-B aligned (hipMalloc granularity)
  if (e != hipSuccess) {
    *out = nullptr;
    return hip_fail(e, "hipMalloc");
  }
  return MANO_OK;
}

int mano_free(int device, void* ptr) {
  g_last_error.clear();
  if (!ptr) return MANO_OK;
  if (device < 0) return fail(MANO_EINVAL, "device %d is negative", device);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  hipError_t e = hipFree(ptr);
  if (e != hipSuccess) return hip_fail(e, "hipFree");
  return MANO_OK;
}

int mano_memcpy(int device, void* dst, const void* src, size_t bytes, int32_t kind, void* stream) {
  g_last_error.clear();
  hipMemcpyKind k;
  switch (kind) {
    case MANO_MEMCPY_HOST_TO_DEVICE: k = hipMemcpyHostToDevice; break;
    case MANO_MEMCPY_DEVICE_TO_HOST: k = hipMemcpyDeviceToHost; break;
    case MANO_MEMCPY_DEVICE_TO_DEVICE: k = hipMemcpyDeviceToDevice; break;
    default: return fail(MANO_EINVAL, "memcpy kind %d is not a MANO_MEMCPY_* value", kind);
  }
  if (bytes == 0) return MANO_OK;
  if (!dst || !src) return fail(MANO_EINVAL, "memcpy dst / src is NULL");
  if (device < 0) return fail(MANO_EINVAL, "device %d is negative", device);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  hipError_t e = stream ? hipMemcpyAsync(dst, src, bytes, k, static_cast<hipStream_t>(stream))
                        : hipMemcpy(dst, src, bytes, k);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
  return MANO_OK;
}

int mano_synchronize(int device) {
  g_last_error.clear();
  if (device < 0) return fail(MANO_EINVAL, "device %d is negative", device);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
  return MANO_OK;
}

int mano_synthetic_inputs(int device, uint64_t seed, int64_t first, int64_t n, float beta_sigma,
                          float pose_sigma, float trans_range, float* betas, float* pose,
                          float* trans, void* stream) {
  g_last_error.clear();
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (first < 0) return fail(MANO_EINVAL, "first_index %lld < 0", (long long)first);
  if (device < 0) return fail(MANO_EINVAL, "device %d is negative", device);
  if (n == 0 || (!betas && !pose && !trans)) return MANO_OK;
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  hipError_t e = mano::launch_synthetic_inputs(seed, first, n, beta_sigma, pose_sigma, trans_range,
                                               betas, pose, trans, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "synthetic_inputs launch");
  return MANO_OK;
}

int mano_rodrigues(int device, int64_t n, const float* aa, float* rot, void* stream) {
  if (n < 0 || n > kMaxHands * 16) return fail(MANO_EINVAL, "n %lld out of range", (long long)n);
  if (n == 0) return MANO_OK;
  if (!aa || !rot) return fail(MANO_EINVAL, "axis_angle / rot pointer is NULL");
  if (device < 0) return fail(MANO_EINVAL, "device %d is negative", device);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  hipError_t e = mano::launch_rodrigues(n, aa, rot, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "rodrigues launch");
  return MANO_OK;
}

}  // extern "C"
