// Microbenchmark: where should the per-hand skinning transforms live for LBS?
// Build: hipcc --offload-arch=gfx950 -O3 -o skin_variants skin_variants.hip
// Runs every variant on the same synthetic data (65,536 hands x 778 verts),
// checks each against variant 0 and prints the average kernel time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NV = 778, NJ = 16, TF = 192, RUN = 16;

__device__ __forceinline__ void load_w(const float* __restrict__ W, int v, float w[16]) {
  const f32x4* wp = reinterpret_cast<const f32x4*>(W + v * 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) { f32x4 q = wp[i]; w[4*i]=q[0]; w[4*i+1]=q[1]; w[4*i+2]=q[2]; w[4*i+3]=q[3]; }
}

// V1: 4 waves/block, each wave its own hand run, scalar-loaded A, 1 hand per iteration.
__global__ __launch_bounds__(256) void v1(const float* __restrict__ W, const float* __restrict__ A,
    const float* __restrict__ vp, float* __restrict__ out, long n) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int vb = blockIdx.y * 64; if (vb > NV - 64) vb = NV - 64;
  const int v = vb + lane;
  float w[16]; load_w(W, v, w);
  const long h0 = ((long)blockIdx.x * 4 + wave) * RUN;
  for (long h = h0; h < h0 + RUN && h < n; ++h) {
    const float* Ah = A + h * TF;
    float T[12];
#pragma unroll
    for (int m = 0; m < 12; ++m) T[m] = w[0] * Ah[m];
#pragma unroll
    for (int j = 1; j < 16; ++j)
#pragma unroll
      for (int m = 0; m < 12; ++m) T[m] = fmaf(w[j], Ah[j*12+m], T[m]);
    const float* p = vp + h * NV * 3 + 3 * v;
    float p0 = p[0], p1 = p[1], p2 = p[2];
    float* o = out + h * NV * 3 + 3 * v;
    o[0] = fmaf(T[0], p0, fmaf(T[1], p1, fmaf(T[2], p2, T[3])));
    o[1] = fmaf(T[4], p0, fmaf(T[5], p1, fmaf(T[6], p2, T[7])));
    o[2] = fmaf(T[8], p0, fmaf(T[9], p1, fmaf(T[10], p2, T[11])));
  }
}

// V2: 13 waves/block (all vertex groups), the block's hand run of A staged in LDS,
// read back with wave-uniform (broadcast) ds_read_b128; v_posed ping-pong prefetch.
template <int HR>
__global__ __launch_bounds__(832) void v2(const float* __restrict__ W, const float* __restrict__ A,
    const float* __restrict__ vp, float* __restrict__ out, long n) {
  __shared__ f32x4 As[HR * TF / 4];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long h0 = (long)blockIdx.x * HR;
  const int cnt = (int)(n - h0 < HR ? n - h0 : HR);
  const f32x4* src = reinterpret_cast<const f32x4*>(A + h0 * TF);
  for (int i = threadIdx.x; i < cnt * TF / 4; i += 832) As[i] = src[i];
  int vb = wave * 64; if (vb > NV - 64) vb = NV - 64;
  const int v = vb + lane;
  float w[16]; load_w(W, v, w);
  __syncthreads();
  const long stride = NV * 3;
  const float* vrow = vp + h0 * stride + 3 * v;
  float* orow = out + h0 * stride + 3 * v;
  float P[2][3];
#pragma unroll
  for (int u = 0; u < 2; ++u) { const float* q = vrow + min(u, cnt-1) * stride; P[u][0]=q[0]; P[u][1]=q[1]; P[u][2]=q[2]; }
  for (int i = 0; i < cnt; i += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = min(i + u, cnt - 1);
      const f32x4* Ah = As + k * (TF / 4);
      float T[12];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const f32x4 a0 = Ah[3*j], a1 = Ah[3*j+1], a2 = Ah[3*j+2];
        const float a[12] = {a0[0],a0[1],a0[2],a0[3],a1[0],a1[1],a1[2],a1[3],a2[0],a2[1],a2[2],a2[3]};
#pragma unroll
        for (int m = 0; m < 12; ++m) T[m] = j ? fmaf(w[j], a[m], T[m]) : w[0] * a[m];
      }
      const float p0 = P[u][0], p1 = P[u][1], p2 = P[u][2];
      const float* q = vrow + min(i + u + 2, cnt - 1) * stride;
      P[u][0] = q[0]; P[u][1] = q[1]; P[u][2] = q[2];
      float* o = orow + k * stride;
      o[0] = fmaf(T[0], p0, fmaf(T[1], p1, fmaf(T[2], p2, T[3])));
      o[1] = fmaf(T[4], p0, fmaf(T[5], p1, fmaf(T[6], p2, T[7])));
      o[2] = fmaf(T[8], p0, fmaf(T[9], p1, fmaf(T[10], p2, T[11])));
    }
  }
}

// V3: like V2 but each lane blends TWO vertices (v and v+64 of a 128-vertex
// group) so every broadcast LDS read feeds 2 FMAs; 7 waves/block.
template <int HR>
__global__ __launch_bounds__(448) void v3(const float* __restrict__ W, const float* __restrict__ A,
    const float* __restrict__ vp, float* __restrict__ out, long n) {
  __shared__ f32x4 As[HR * TF / 4];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long h0 = (long)blockIdx.x * HR;
  const int cnt = (int)(n - h0 < HR ? n - h0 : HR);
  const f32x4* src = reinterpret_cast<const f32x4*>(A + h0 * TF);
  for (int i = threadIdx.x; i < cnt * TF / 4; i += 448) As[i] = src[i];
  int vb = wave * 128; if (vb > NV - 128) vb = NV - 128;
  const int va = vb + lane, vb2 = vb + 64 + lane;
  float w[16], x[16]; load_w(W, va, w); load_w(W, vb2, x);
  __syncthreads();
  const long stride = NV * 3;
  for (int k = 0; k < cnt; ++k) {
    const f32x4* Ah = As + k * (TF / 4);
    float T[12], U[12];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const f32x4 a0 = Ah[3*j], a1 = Ah[3*j+1], a2 = Ah[3*j+2];
      const float a[12] = {a0[0],a0[1],a0[2],a0[3],a1[0],a1[1],a1[2],a1[3],a2[0],a2[1],a2[2],a2[3]};
#pragma unroll
      for (int m = 0; m < 12; ++m) { T[m] = j ? fmaf(w[j], a[m], T[m]) : w[0] * a[m]; U[m] = j ? fmaf(x[j], a[m], U[m]) : x[0] * a[m]; }
    }
    const float* p = vp + (h0 + k) * stride + 3 * va;
    const float* q = vp + (h0 + k) * stride + 3 * vb2;
    float p0 = p[0], p1 = p[1], p2 = p[2], q0 = q[0], q1 = q[1], q2 = q[2];
    float* o = out + (h0 + k) * stride + 3 * va;
    o[0] = fmaf(T[0], p0, fmaf(T[1], p1, fmaf(T[2], p2, T[3])));
    o[1] = fmaf(T[4], p0, fmaf(T[5], p1, fmaf(T[6], p2, T[7])));
    o[2] = fmaf(T[8], p0, fmaf(T[9], p1, fmaf(T[10], p2, T[11])));
    float* r = out + (h0 + k) * stride + 3 * vb2;
    r[0] = fmaf(U[0], q0, fmaf(U[1], q1, fmaf(U[2], q2, U[3])));
    r[1] = fmaf(U[4], q0, fmaf(U[5], q1, fmaf(U[6], q2, U[7])));
    r[2] = fmaf(U[8], q0, fmaf(U[9], q1, fmaf(U[10], q2, U[11])));
  }
}


// 12 FMAs T[m] += A_J[m] * w, with A_J[m] broadcast from lane J of each 16-lane
// row (DPP row_newbcast): lane k of every row holds joint k's 12 transform values.
#ifndef NOP
#define NOP "s_nop 1\n\t"
#endif
#define FMA_DPP(J)                                                                              \
  asm volatile(NOP                                                                    \
               "v_fmac_f32_dpp %0, %12, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %1, %13, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %2, %14, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %3, %15, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %4, %16, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %5, %17, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %6, %18, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %7, %19, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %8, %20, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %9, %21, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %10, %22, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t" \
               "v_fmac_f32_dpp %11, %23, %24 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"     \
               : "+v"(T[0]), "+v"(T[1]), "+v"(T[2]), "+v"(T[3]), "+v"(T[4]), "+v"(T[5]),        \
                 "+v"(T[6]), "+v"(T[7]), "+v"(T[8]), "+v"(T[9]), "+v"(T[10]), "+v"(T[11])       \
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),   \
                 "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(w[J]))

__device__ __forceinline__ void load_a(const float* __restrict__ Ah, int lane, float a[12]) {
  const f32x4* p = reinterpret_cast<const f32x4*>(Ah + (lane & 15) * 12);
  const f32x4 x = p[0], y = p[1], z = p[2];
  a[0]=x[0]; a[1]=x[1]; a[2]=x[2]; a[3]=x[3]; a[4]=y[0]; a[5]=y[1]; a[6]=y[2]; a[7]=y[3];
  a[8]=z[0]; a[9]=z[1]; a[10]=z[2]; a[11]=z[3];
}

// V5: DPP-broadcast transforms (vector loads, no SGPR/LDS), v_posed + A ping-pong prefetch.
__global__ __launch_bounds__(256) void v5(const float* __restrict__ W, const float* __restrict__ A,
    const float* __restrict__ vp, float* __restrict__ out, long n) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int vb = blockIdx.y * 64; if (vb > NV - 64) vb = NV - 64;
  const int v = vb + lane;
  float w[16]; load_w(W, v, w);
  const long h0 = ((long)blockIdx.x * 4 + wave) * RUN;
  if (h0 >= n) return;
  const int cnt = (int)(n - h0 < RUN ? n - h0 : RUN);
  const long stride = NV * 3;
  const float* vrow = vp + h0 * stride + 3 * v;
  float* orow = out + h0 * stride + 3 * v;
  const float* Ab = A + h0 * TF;
  float P[2][3], AA[2][12];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const float* q = vrow + min(u, cnt-1) * stride; P[u][0]=q[0]; P[u][1]=q[1]; P[u][2]=q[2];
    load_a(Ab + min(u, cnt - 1) * TF, lane, AA[u]);
  }
  for (int i = 0; i < cnt; i += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = min(i + u, cnt - 1);
      float T[12];
#pragma unroll
      for (int m = 0; m < 12; ++m) T[m] = 0.f;
      {
        const float (&a)[12] = AA[u];
        FMA_DPP(0); FMA_DPP(1); FMA_DPP(2); FMA_DPP(3); FMA_DPP(4); FMA_DPP(5); FMA_DPP(6); FMA_DPP(7);
        FMA_DPP(8); FMA_DPP(9); FMA_DPP(10); FMA_DPP(11); FMA_DPP(12); FMA_DPP(13); FMA_DPP(14); FMA_DPP(15);
      }
      const float p0 = P[u][0], p1 = P[u][1], p2 = P[u][2];
      const int kn = min(i + u + 2, cnt - 1);
      const float* q = vrow + kn * stride;
      P[u][0] = q[0]; P[u][1] = q[1]; P[u][2] = q[2];
      load_a(Ab + kn * TF, lane, AA[u]);
      float* o = orow + k * stride;
      o[0] = fmaf(T[0], p0, fmaf(T[1], p1, fmaf(T[2], p2, T[3])));
      o[1] = fmaf(T[4], p0, fmaf(T[5], p1, fmaf(T[6], p2, T[7])));
      o[2] = fmaf(T[8], p0, fmaf(T[9], p1, fmaf(T[10], p2, T[11])));
    }
  }
}

// V4: pure streaming copy of the same bytes (vp in -> out), the HBM ceiling for this shape.
__global__ __launch_bounds__(256) void vcopy(const f32x4* __restrict__ in, f32x4* __restrict__ out, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) out[i] = in[i];
}

int main() {
  const long n = 65536;
  const size_t nvp = n * NV * 3;
  std::vector<float> hW(NV * 16), hA(n * TF);
  srand(1);
  for (int v = 0; v < NV; ++v) { float s = 0; for (int j = 0; j < 16; ++j) { hW[v*16+j] = rand() / (float)RAND_MAX; s += hW[v*16+j]; } for (int j = 0; j < 16; ++j) hW[v*16+j] /= s; }
  for (auto& a : hA) a = rand() / (float)RAND_MAX - 0.5f;
  float *W, *A, *vp, *out, *ref;
  CK(hipMalloc(&W, hW.size() * 4)); CK(hipMalloc(&A, hA.size() * 4));
  CK(hipMalloc(&vp, nvp * 4)); CK(hipMalloc(&out, nvp * 4)); CK(hipMalloc(&ref, nvp * 4));
  CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
  { std::vector<float> hv(nvp); for (auto& x : hv) x = rand() / (float)RAND_MAX - 0.5f; CK(hipMemcpy(vp, hv.data(), nvp * 4, hipMemcpyHostToDevice)); }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch, bool check) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int it = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < it; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
    double maxerr = 0;
    if (check) {
      std::vector<float> a(nvp), b(nvp);
      CK(hipMemcpy(a.data(), out, nvp * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), ref, nvp * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < nvp; i += 7) maxerr = fmax(maxerr, fabs(a[i] - b[i]));
    }
    const double bytes = (double)n * (NV * 3 * 4 * 2 + TF * 4);
    printf("%-28s %8.3f ms  %7.1f GB/s  maxerr %.2e\n", name, ms, bytes / ms / 1e6, maxerr);
  };
  const unsigned runs = (n + 4 * RUN - 1) / (4 * RUN);
  // reference into `ref`
  hipLaunchKernelGGL(v1, dim3(runs, 13), dim3(256), 0, 0, W, A, vp, ref, n);
  CK(hipDeviceSynchronize());
  timeit("v1 scalar A, 1 hand/iter", [&] { hipLaunchKernelGGL(v1, dim3(runs, 13), dim3(256), 0, 0, W, A, vp, out, n); }, true);
  timeit("v2<16> LDS A bcast", [&] { hipLaunchKernelGGL(v2<16>, dim3((n + 15) / 16), dim3(832), 0, 0, W, A, vp, out, n); }, true);
  timeit("v2<32> LDS A bcast", [&] { hipLaunchKernelGGL(v2<32>, dim3((n + 31) / 32), dim3(832), 0, 0, W, A, vp, out, n); }, true);
  timeit("v2<64> LDS A bcast", [&] { hipLaunchKernelGGL(v2<64>, dim3((n + 63) / 64), dim3(832), 0, 0, W, A, vp, out, n); }, true);
  timeit("v3<16> LDS A, 2 vert/lane", [&] { hipLaunchKernelGGL(v3<16>, dim3((n + 15) / 16), dim3(448), 0, 0, W, A, vp, out, n); }, true);
  timeit("v3<32> LDS A, 2 vert/lane", [&] { hipLaunchKernelGGL(v3<32>, dim3((n + 31) / 32), dim3(448), 0, 0, W, A, vp, out, n); }, true);
  timeit("v5 DPP bcast A", [&] { hipLaunchKernelGGL(v5, dim3(runs, 13), dim3(256), 0, 0, W, A, vp, out, n); }, true);
  timeit("copy (HBM ceiling)", [&] { hipLaunchKernelGGL(vcopy, dim3(4096), dim3(256), 0, 0, (const f32x4*)vp, (f32x4*)out, (long)(nvp / 4)); }, false);
  return 0;
}
