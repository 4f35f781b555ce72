// Ablation timing of the fused blend_skin kernel (diagnostic only).
// Times launch_blend_skin alone on random operands (WITH_TRANS=1 adds a translation).
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
int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 65536;
  DeviceModel m{};
  m.n_verts = 778; m.n_cols = 2334; m.n_col_tiles = 73;
  m.n_groups16 = 49;
  m.basis16 = dev_rand(size_t(147) * kTile16Floats, 0.01f);
  m.wfrag16 = dev_rand(size_t(49) * kWFrag16Floats, 0.1f);
  const long nt16 = (n + 15) / 16;
  float* f16 = dev_rand(size_t(nt16) * kTile16Floats, 1.f);
  float* t16 = dev_rand(size_t(nt16) * kTFrag16Floats, 1.f);
  float* tr = dev_rand(size_t(n) * 3, 1.f);
  const bool with_trans = getenv("WITH_TRANS") != nullptr;
  float* verts; CK(hipMalloc(&verts, size_t(n) * 2334 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CK(launch_blend_skin(m, n, f16, t16, with_trans ? tr : nullptr, verts, nullptr, 0));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  const int it = 20;
  for (int i = 0; i < it; ++i) CK(launch_blend_skin(m, n, f16, t16, with_trans ? tr : nullptr, verts, nullptr, 0));
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-24s n=%ld  %.3f ms\n", argc > 2 ? argv[2] : "blend_skin16", n, ms / it);
  return 0;
}
