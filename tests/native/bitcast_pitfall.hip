// Fixture of tools/isa_scan.py rule 3 (tests/test_codegen.py): the toolchain
// pitfall behind round 3's wrong sc0 v_posed stores.  bug_kernel passes
// __builtin_bit_cast(unsigned, acc[r]) of an ext_vector_type element to a
// buffer store: hipcc emits element 0 (v0) for every r.  ok_kernel copies the
// element to a scalar first (the product's form, mano_kernels.hip
// store_vposed_tile) and stores v0..v3.  Compiled with -S only, never run.
#include <hip/hip_runtime.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void bug_kernel(float* out, const float* a, int n) {
  f32x4 acc = {};
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[threadIdx.x], a[threadIdx.x + 64], acc, 0, 0, 0);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, n * 4, 0x00020000);
#pragma unroll
  for (int r = 0; r < 4; ++r)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, acc[r]), rs, 4 * (r * 64 + threadIdx.x), 0, 1);
}
__global__ void ok_kernel(float* out, const float* a, int n) {
  f32x4 acc = {};
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[threadIdx.x], a[threadIdx.x + 64], acc, 0, 0, 0);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, n * 4, 0x00020000);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float x = acc[r];
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), rs, 4 * (r * 64 + threadIdx.x), 0, 1);
  }
}
