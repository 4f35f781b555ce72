// Timing of the fused kernels alone on random operands (diagnostic only):
// the staged blend_skin16 (A fragments + transforms from HBM) and the
// single-launch forward (articulation in the prologue).  WITH_TRANS=1 adds a
// translation.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 fused_ablate.hip
#include "../../mano-hand_amd/csrc/mano_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace mano;
static float* dev_rand(size_t n, float scale) {
  std::vector<float> h(n);
  for (auto& x : h) x = scale * (rand() / (float)RAND_MAX - 0.5f);
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice)); return d;
}
static int32_t* dev_ints(const std::vector<int32_t>& h) {
  int32_t* d; CK(hipMalloc(&d, h.size() * 4)); CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice)); return d;
}
template <class F> static float time_ms(F&& f, int it = 20) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CK(f());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int i = 0; i < it; ++i) CK(f());
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / it;
}
int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 65536;
  DeviceModel m{};
  m.n_verts = 778; m.n_cols = 2334; m.n_col_tiles = 73;
  m.n_groups16 = 49;
  m.basis16 = dev_rand(size_t(147) * kTile16Floats, 0.01f);
  m.wfrag16 = dev_rand(size_t(49) * kWFrag16Floats, 0.1f);
  m.joint_template = dev_rand(48, 0.1f);
  m.joint_shape = dev_rand(480, 0.01f);
  m.parents = dev_ints({-1, 0, 1, 2, 0, 4, 5, 0, 7, 8, 0, 10, 11, 0, 13, 14});
  m.depth = dev_ints({0, 1, 2, 3, 1, 2, 3, 1, 2, 3, 1, 2, 3, 1, 2, 3});
  m.max_depth = 3;
  const long nt16 = (n + 15) / 16;
  float* f16 = dev_rand(size_t(nt16) * kTile16Floats, 1.f);
  float* tf = dev_rand(size_t(n) * kTransformFloats, 1.f);
  float* tr = dev_rand(size_t(n) * 3, 1.f);
  float* betas = dev_rand(size_t(n) * 10, 2.f);
  float* pose = dev_rand(size_t(n) * 48, 1.f);
  float* joints; CK(hipMalloc(&joints, size_t(n) * 48 * 4));
  const bool with_trans = getenv("WITH_TRANS") != nullptr;
  float* verts; CK(hipMalloc(&verts, size_t(n) * 2334 * 4));
  float* t = with_trans ? tr : nullptr;
  const float ms_bs = time_ms([&] { return launch_blend_skin(m, n, f16, tf, t, verts, nullptr, 0); });
  const float ms_fw = time_ms([&] {
    return launch_forward(m, n, betas, 10, pose, t, verts, joints, nullptr, nullptr, nullptr, 0);
  });
  printf("n=%ld trans=%d  blend_skin16 %.3f ms  forward %.3f ms\n", n, int(with_trans), ms_bs, ms_fw);
  return 0;
}
