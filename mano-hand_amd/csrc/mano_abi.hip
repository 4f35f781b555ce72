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
  void* block;            // single device allocation holding every array of dm
  int32_t* status_flags;  // [kStatusFlags] pinned host memory; dm.status is its device address
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

// OR of the raised MANO_DEVICE_* bits (host reads of the pinned flags; no
// wait).  `clear`: each flag is taken with one host atomic exchange, so a
// flag a kernel sets after the exchange stays for the next reader.
int32_t read_flags(const mano_model* m, bool clear) {
  int32_t bits = 0;
  for (int b = 0; b < mano::kStatusFlags; ++b) {
    int32_t* f = m->status_flags + b;
    const int32_t v = clear ? __atomic_exchange_n(f, 0, __ATOMIC_ACQ_REL) : __atomic_load_n(f, __ATOMIC_ACQUIRE);
    if (v) bits |= int32_t(1) << b;
  }
  return bits;
}

// Every launching entry point on a model: a kernel of an earlier launch
// raised a status flag, so its outputs are not valid -- fail loudly until the
// caller has read (and cleared) the flags.
int check_launchable(const mano_model* m) {
  if (int rc = check_model(m)) return rc;
  if (const int32_t bits = read_flags(m, false))
    return fail(MANO_EDEVICE,
                "device status 0x%x: an earlier launch on this model did not write all its outputs "
                "(MANO_DEVICE_SKIN_HANDOFF_TIMEOUT = 1); mano_model_device_status with MANO_STATUS_CLEAR "
                "reads and clears it",
                unsigned(bits));
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

}  // namespace

namespace mano {
// The thread-local message of mano_last_error(), for the other ABI files.
int set_error(int code, const char* msg) {
  g_last_error = msg;
  return code;
}
}  // namespace mano

extern "C" {

int mano_abi_version(void) { return 7; }

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
  mano::HostModel hm;
  std::string err;
  if (!mano::pack_model(n_verts, mesh_template, mesh_shape_basis, mesh_pose_basis, j_regressor,
                        skinning_weights, parents, pose_pca_basis, pose_pca_mean, hm, err))
    return fail(MANO_EINVAL, "%s", err.c_str());

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
  std::vector<float> zeros(64, 0.f);

  // ---- one device block, 256-B aligned sub-arrays ----
  struct Part { const void* src; size_t bytes; size_t off; };
  enum { kBasis, kWeights, kJt, kJs, kParents, kDepth, kPcaB, kPcaM, kZeros, kBasis16, kW16, kBasisH3, kB16V, kW16V, kTilesV, kBh3V, kNParts };
  std::vector<Part> parts(kNParts);
  parts[kBasis] = {hm.tiles.data(), hm.tiles.size() * 4, 0};
  parts[kWeights] = {hm.weights.data(), hm.weights.size() * 4, 0};
  parts[kJt] = {hm.jt.data(), hm.jt.size() * 4, 0};
  parts[kJs] = {hm.js.data(), hm.js.size() * 4, 0};
  parts[kParents] = {parents, kJoints * 4, 0};
  parts[kDepth] = {hm.depth.data(), kJoints * 4, 0};
  parts[kPcaB] = {hm.pca.data(), hm.pca.size() * 4, 0};
  parts[kPcaM] = {hm.pmean.data(), hm.pmean.size() * 4, 0};
  parts[kZeros] = {zeros.data(), zeros.size() * 4, 0};
  parts[kBasis16] = {hm.b16.data(), hm.b16.size() * 4, 0};
  parts[kW16] = {hm.w16.data(), hm.w16.size() * 4, 0};
  parts[kBasisH3] = {hm.bh3.data(), hm.bh3.size() * 2, 0};
  parts[kB16V] = {hm.b16v.data(), hm.b16v.size() * 4, 0};
  parts[kW16V] = {hm.w16v.data(), hm.w16v.size() * 4, 0};
  parts[kTilesV] = {hm.tiles_v.data(), hm.tiles_v.size() * 4, 0};
  parts[kBh3V] = {hm.bh3v.data(), hm.bh3v.size() * 2, 0};
  size_t total = 0;
  for (auto& p : parts) {
    p.off = total;
    total = align256(total + p.bytes);
  }
  void* block = nullptr;
  e = hipMalloc(&block, total);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(model buffer)");
  for (auto& p : parts) {
    if (p.bytes == 0) continue;  // no aligned variants for this V
    e = hipMemcpy(static_cast<char*>(block) + p.off, p.src, p.bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(block);
      return hip_fail(e, "hipMemcpy(model buffer)");
    }
  }
  // The status flags: pinned, coherent host memory the kernels write
  // through its device address (read by the host without a device copy).
  void* flags = nullptr;
  e = hipHostMalloc(&flags, kStatusFlags * sizeof(int32_t), hipHostMallocCoherent);
  if (e != hipSuccess) {
    (void)hipFree(block);
    return hip_fail(e, "hipHostMalloc(status flags)");
  }
  std::memset(flags, 0, kStatusFlags * sizeof(int32_t));
  void* flags_dev = nullptr;
  e = hipHostGetDevicePointer(&flags_dev, flags, 0);
  mano_model* m = e == hipSuccess ? new (std::nothrow) mano_model() : nullptr;
  if (!m) {
    (void)hipHostFree(flags);
    (void)hipFree(block);
    return e != hipSuccess ? hip_fail(e, "hipHostGetDevicePointer(status flags)")
                           : fail(MANO_EINVAL, "out of host memory");
  }
  char* b = static_cast<char*>(block);
  m->magic = kMagic;
  m->device = device;
  m->block = block;
  m->status_flags = static_cast<int32_t*>(flags);
  auto at = [&](int i) { return reinterpret_cast<float*>(b + parts[i].off); };
  m->dm.basis_tiles = at(kBasis);
  m->dm.basis_tiles_v = hm.tiles_v.empty() ? nullptr : at(kTilesV);
  m->dm.weights = at(kWeights);
  m->dm.joint_template = at(kJt);
  m->dm.joint_shape = at(kJs);
  m->dm.parents = reinterpret_cast<int32_t*>(at(kParents));
  m->dm.depth = reinterpret_cast<int32_t*>(at(kDepth));
  m->dm.pca_basis = at(kPcaB);
  m->dm.pca_mean = at(kPcaM);
  m->dm.zeros = at(kZeros);
  m->dm.status = static_cast<int32_t*>(flags_dev);
  m->dm.basis16 = at(kBasis16);
  m->dm.wfrag16 = at(kW16);
  m->dm.basis16v = hm.b16v.empty() ? nullptr : at(kB16V);
  m->dm.wfrag16v = hm.w16v.empty() ? nullptr : at(kW16V);
  m->dm.basis_h3 = reinterpret_cast<uint16_t*>(at(kBasisH3));
  m->dm.basis_h3v = hm.bh3v.empty() ? nullptr : reinterpret_cast<uint16_t*>(at(kBh3V));
  m->dm.h3_vposed_unscale = float(std::ldexp(1.0, -hm.basis_exp));
  m->dm.h3_lbs_unscale = float(std::ldexp(1.0, -(kH3FrameExp + kH3WeightExp)));
  m->dm.precision = MANO_PRECISION_FP32;
  m->dm.has_pca = pose_pca_basis != nullptr;
  m->dm.n_groups16 = hm.n_groups16;
  m->dm.max_depth = hm.max_depth;
  m->dm.n_verts = V;
  m->dm.n_cols = 3 * V;
  m->dm.n_col_tiles = hm.n_col_tiles;
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
  const hipError_t ef = hipHostFree(m->status_flags);
  delete m;
  if (e != hipSuccess) return hip_fail(e, "hipFree(model buffer)");
  if (ef != hipSuccess) return hip_fail(ef, "hipHostFree(status flags)");
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

}  // extern "C"

extern "C" {

int mano_model_device_status(const mano_model* m, int32_t* status, int32_t flags) {
  g_last_error.clear();
  if (int rc = check_model(m)) return rc;
  if (!status) return fail(MANO_EINVAL, "status is NULL");
  if (flags & ~(MANO_STATUS_CLEAR | MANO_STATUS_NO_WAIT))
    return fail(MANO_EINVAL, "flags 0x%x: only MANO_STATUS_CLEAR | MANO_STATUS_NO_WAIT", unsigned(flags));
  if (!(flags & MANO_STATUS_NO_WAIT)) {
    DeviceGuard guard(m->device);
    if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
  }
  // Host reads of the pinned flags: each call takes its own snapshot (no
  // shared device slot, no copy), and with CLEAR each flag goes through one
  // host atomic exchange -- concurrent callers never lose a bit.
  *status = read_flags(m, flags & MANO_STATUS_CLEAR);
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
  if (int rc = check_launchable(m)) return rc;
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
  if (int rc = check_launchable(m)) return rc;
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
  if (int rc = check_launchable(m)) return rc;
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (n == 0) return MANO_OK;
  if (!verts) return fail(MANO_EINVAL, "verts is required");
  if (int rc = check_workspace(m, n, ws, ws_bytes)) return rc;
  DeviceGuard guard(m->device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  char* base = static_cast<char*>(ws);
  float* ws_vp = reinterpret_cast<float*>(base + w.vposed_off);
  const float* vp = rest_verts ? rest_verts : ws_vp;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const float* tr = reinterpret_cast<const float*>(base + w.transforms_off);
  // verts == rest_verts: the LBS in place over its own input (the unfused
  // path's blend GEMM writes v_posed straight into verts).  Any other
  // overlap of the two row ranges has no defined result.
  const size_t bytes = size_t(n) * 3 * size_t(m->dm.n_verts) * sizeof(float);
  const char *src = reinterpret_cast<const char*>(vp), *dst = reinterpret_cast<const char*>(verts);
  const bool in_place = src == dst;
  if (!in_place && src < dst + bytes && dst < src + bytes)
    return fail(MANO_EINVAL, "verts and rest_verts overlap without being the same rows");
  hipError_t e;
  if (in_place && m->dm.precision == MANO_PRECISION_FP32 && mano::skin_in_place_supported(m->dm, n)) {
    e = mano::launch_skin_quad(m->dm, n, tr, vp, trans, verts, s, false, true);
  } else {
    if (in_place) {
      // no in-place kernel for this call (f16x3, a batch below one skin_pair
      // block, a mesh skin_pair does not take): the rows go to the
      // workspace's v_posed first, then the out-of-place LBS
      if (verts == ws_vp) return fail(MANO_EINVAL, "verts is the workspace's own v_posed");
      e = hipMemcpyAsync(ws_vp, vp, bytes, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync");
      vp = ws_vp;
    }
    e = m->dm.precision == MANO_PRECISION_F16X3 ? mano::launch_skin_h3(m->dm, n, tr, vp, trans, verts, s)
                                                 : mano::launch_skin(m->dm, n, tr, vp, trans, verts, s);
  }
  if (e != hipSuccess) return hip_fail(e, "skin launch");
  return MANO_OK;
}

int mano_stage_blend_skin(const mano_model* m, int64_t n, float* rest_verts, const float* trans,
                          float* verts, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = check_launchable(m)) return rc;
  if (n < 0 || n > kMaxHands) return fail(MANO_EINVAL, "n_hands %lld out of range", (long long)n);
  if (n == 0) return MANO_OK;
  if (!verts) return fail(MANO_EINVAL, "verts is required");
  if (int rc = check_workspace(m, n, ws, ws_bytes, false)) return rc;
  DeviceGuard guard(m->device);
  if (guard.err != hipSuccess) return hip_fail(guard.err, "hipSetDevice");
  const mano::Workspace w = mano::workspace_layout(m->dm, n);
  char* base = static_cast<char*>(ws);
  const float* feats = reinterpret_cast<const float*>(base + w.features_off);
  const float* frames = reinterpret_cast<const float*>(base + w.transforms_off);
  // F16X3 covers verts-only calls: the product has no f16x3 kernel that also
  // writes rest_verts (mano_kernels_h3.hip header), so such a call runs the
  // exact-fp32 kernel -- same outputs to ~1e-7 m, more exact.
  hipError_t e = m->dm.precision == MANO_PRECISION_F16X3 && !rest_verts
                     ? mano::launch_blend_skin_h3(m->dm, n, feats, frames, trans, verts,
                                                  static_cast<hipStream_t>(stream))
                     : mano::launch_blend_skin(m->dm, n, feats, frames, trans, verts, rest_verts,
                                               static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "blend_skin launch");
  return MANO_OK;
}

int mano_forward(const mano_model* m, int64_t n, const float* betas, int64_t betas_stride,
                 const float* pose, const float* trans, float* verts, float* joints,
                 float* rest_verts, float* rest_joints, float* rot_mats, void* ws,
                 size_t ws_bytes, void* stream) {
  g_last_error.clear();
  if (int rc = check_launchable(m)) return rc;
  if (n > 0 && !verts) return fail(MANO_EINVAL, "verts is required");
  if (int rc = mano_stage_articulate(m, n, betas, betas_stride, pose, trans, joints, rest_joints,
                                     rot_mats, ws, ws_bytes, stream))
    return rc;
  return mano_stage_blend_skin(m, n, rest_verts, trans, verts, ws, ws_bytes, stream);
}

int mano_pose_from_pca(const mano_model* m, int64_t n, const float* pca, int32_t n_comps,
                       int64_t pca_stride, const float* rot, int64_t rot_stride, float* pose,
                       void* stream) {
  if (int rc = check_launchable(m)) return rc;
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
  if (int rc = check_launchable(m)) return rc;
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

int mano_host_alloc(size_t bytes, void** out) {
  g_last_error.clear();
  if (!out) return fail(MANO_EINVAL, "out is NULL");
  *out = nullptr;
  if (bytes == 0) return MANO_OK;
  // pinned, and mapped into every device's address space at the same
  // address: kernels take it as operands directly
  hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    *out = nullptr;
    return hip_fail(e, "hipHostMalloc");
  }
  return MANO_OK;
}

int mano_host_free(void* ptr) {
  g_last_error.clear();
  if (!ptr) return MANO_OK;
  hipError_t e = hipHostFree(ptr);
  if (e != hipSuccess) return hip_fail(e, "hipHostFree");
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
