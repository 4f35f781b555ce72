// mano_kernels.hip -- gfx950 (MI355X, CDNA4) MFMA kernels of the MANO forward pass.
//
// Reference hot path: MANOModel.update() in /root/reference/mano_np.py:79-115.
// mano_forward is two launches on the caller's stream: articulate
// (mano_articulate.hip: Rodrigues, the chain, the transforms and the X rows),
// then
//
//   blend_skin16  v_posed = [beta | features | 1] . [S ; P ; T] (:81, :87-93) on
//                 v_mfma_f32_16x16x4_f32 with LDS-DMA-staged basis tiles, then
//                 LBS (:112-115) with the per-vertex blended transforms also on
//                 MFMA, v_posed never leaving registers.
//
// The staged API adds the unfused kernels: blend (the same GEMM on
// v_mfma_f32_32x32x2_f32, v_posed to HBM) and skin_span (HBM-streaming LBS
// with the same MFMA transform tiles as blend_skin16, so both paths agree bit
// for bit).  Built with the max-ILP machine scheduler (__graft_entry__.py
// SRC_FLAGS): blend_skin16 0.4902-0.4904 vs 0.4929-0.4932 ms (same box, two
// runs each, identical bits), 142 VGPRs and no spill instead of 168 + 2.
#include <algorithm>

#include "mano_internal.h"
#include "mano_span.h"

// Sector-aligned output rows of blend_skin16 and the unfused blend (mano_layout.h;
// diagnostic builds: 0 = the round-3 layouts, every hand on the plain tiles).
#ifndef MANO_BS_ALIGN
#define MANO_BS_ALIGN 1
#endif

namespace mano {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));  // hand rows: 8-B aligned for odd hands


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

// v_posed leaves as buffer stores with the sc0 cache policy: the unfused blend
// 0.3629-0.3669 vs 0.3676-0.3765 ms with plain global stores, the LBS after it
// 0.288 vs 0.290 (same box, same bits); sc1 took the blend to 0.395
// (profiles/r03q_ab_blend_store_policy.jsonl); nontemporal stores to 0.60
// (partial lines: rows are 9,336 B apart).  The tile's rows are hands
// h0 + (hr << lp), hr < n_valid (residue-class tiles, mano_layout.h); rows
// past n_valid and columns past the row end fall outside the buffer and are
// dropped.
#ifndef MANO_BLEND_STORE_POLICY
#define MANO_BLEND_STORE_POLICY 1  // buffer-store cache policy bits of v_posed (1 = sc0; diagnostic builds: others)
#endif
#ifndef MANO_BLEND_COUNTED
#define MANO_BLEND_COUNTED 0  // blend_kernel: 1 = counted-vmcnt barriers (diagnostic: 0.363 vs 0.359 ms with sc0 stores, 0.387 vs 0.403 nontemporal; profiles/r05/r05b_blend_ab.jsonl)
#endif
__device__ __forceinline__ void store_vposed_tile(float* __restrict__ vposed, const f32x16& acc,
                                                  int64_t h0, int lp, int n_valid, int col, int n_cols,
                                                  int hi) {
  // D[hand][col]: col = lane & 31, hand = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
  const int rstride = n_cols << lp;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(vposed + h0 * n_cols, 0, ((n_valid - 1) * rstride + n_cols) * 4,
                                                    0x00020000);
  // Every lane issues its 16 stores (the blend kernel's counted vmcnt needs
  // an exact per-wave count); a lane past the row end gets an offset beyond
  // the buffer, whose store is dropped.  The sentinel 2^30 is above any
  // num_records here (lp <= 3: < 32 rows x 8 x 2,334 floats x 4 B = 2.4 MB)
  // and leaves room for the row term (4 hr rstride < 2.4 MB), so the signed
  // sum never overflows.
  const int cbase = col < n_cols ? 4 * col : 0x40000000;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int hr = (r & 3) + 8 * (r >> 2) + 4 * hi;
    const float x = acc[r];  // a scalar first: __builtin_bit_cast of a vector element reads element 0
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), rs, cbase + 4 * hr * rstride, 0, MANO_BLEND_STORE_POLICY);
  }
}

// The lane's byte offset is re-materialised at every call (an opaque 32-bit
// value, so the source is SGPR base + VGPR offset): hoisted, hipcc kept a
// 64-bit per-lane pointer live across the group loop and spilled it, and the
// scratch reload's vmcnt(0) then waited for the previous group's stores.
__device__ __forceinline__ void stage_basis_tile16(const float* __restrict__ basis16, int t,
                                                   f32x4* buf, int wave, int lane) {
  unsigned lane_off = unsigned(lane) * 16u;
  asm volatile("" : "+v"(lane_off));
  const char* src = reinterpret_cast<const char*>(basis16 + int64_t(t) * kTile16Floats);
  for (int g = wave; g < kGroups16; g += 4) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + (lane_off + unsigned(g) * 1024u)),
        (__attribute__((address_space(3))) void*)(buf + g * 64), 16, 0, 0);
  }
}

// One block per quad of 4 32-hand tiles (residue classes, mano_layout.h,
// lq = 7): with `aligned` the tiles' rows share one sector phase and the
// block uses column-tile variant sigma_r (shifts >> 4 r & 15), so every
// 32-float row segment a tile stores starts on a sector boundary.
__global__ __launch_bounds__(256, 2) void blend_kernel(
    const float* __restrict__ features, const float* __restrict__ basis_tiles,
    float* __restrict__ vposed, int64_t n, int n_cols, int n_col_tiles, int lp, unsigned shifts, int aligned) {
  __shared__ f32x4 bs[2][kKGroups * 64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // A wave past the batch end recomputes the quad's last tile (identical values).
  const AlignedTile tile = aligned_tile(n, lp, blockIdx.x, wave, 7, 5);
  const int sigma = aligned ? int((shifts >> (4 * tile.cls)) & 15u) : 0;
  const float* tiles = basis_tiles + (aligned ? int64_t(sigma) * n_col_tiles * kTileFloats : 0);

  // A fragments of v_mfma_f32_32x32x2_f32: step s holds X[hand = lane & 31][k =
  // 2 s + (lane >> 5)] (rows past the tile's valid hands repeat its last one).
  float a[kKGroups * 4];
  {
    const int64_t row = tile.h0 + (int64_t(min(lane & 31, tile.n_valid - 1)) << lp);
    const float* x = features + row * kXStride;
#pragma unroll
    for (int s = 0; s < kKGroups * 4; ++s) a[s] = s < kKSteps ? x[x_pos(2 * s + (lane >> 5))] : 0.f;
  }

  stage_basis_tile(tiles, 0, bs[0], wave, lane);
  __syncthreads();

  const int hi = lane >> 5;
  const int col_in_tile = lane & 31;
  auto col_of = [&](int t) { return aligned ? aligned_tile_col(n_cols, sigma, t, col_in_tile) : t * kColTile + col_in_tile; };
  // The template is row k = 145 of the basis (X[:, 145] = 1), so the MFMA chain
  // yields v_posed directly.  Tile t's stores are issued one iteration late,
  // before tile t+2's LDS-DMA, so the barrier's vmcnt(0) only waits on old
  // stores and the DMA the MFMA chain has already hidden.
  f32x16 prev = {};
#if MANO_BLEND_COUNTED
  // Tile t+1's LDS-DMA first, then tile t-1's 16 stores: the barrier waits
  // with vmcnt(16), so those stores stay in flight through the next tile's
  // MFMA chain (in issue order, they must retire before the NEXT barrier's
  // DMA does) instead of gating this one -- a store policy whose completion
  // takes longer (nontemporal) no longer stalls every tile.
  for (int t = 0; t < n_col_tiles; ++t) {
    if (t + 1 < n_col_tiles) stage_basis_tile(tiles, t + 1, bs[(t + 1) & 1], wave, lane);
    asm volatile("" ::: "memory");  // the DMA stays older than the stores (the vmcnt count)
    __builtin_amdgcn_sched_barrier(0);
    if (t > 0) store_vposed_tile(vposed, prev, tile.h0, lp, tile.n_valid, col_of(t - 1), n_cols, hi);
    prev = mfma_tile(a, bs[t & 1], lane);
    if (t == 0) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
#else
  for (int t = 0; t < n_col_tiles; ++t) {
    if (t > 0) store_vposed_tile(vposed, prev, tile.h0, lp, tile.n_valid, col_of(t - 1), n_cols, hi);
    if (t + 1 < n_col_tiles) stage_basis_tile(tiles, t + 1, bs[(t + 1) & 1], wave, lane);
    prev = mfma_tile(a, bs[t & 1], lane);
    __syncthreads();
  }
#endif
  store_vposed_tile(vposed, prev, tile.h0, lp, tile.n_valid, col_of(n_col_tiles - 1), n_cols, hi);
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
// One GEMM tile: 37 dependent v_mfma_f32_16x16x4_f32 (one accumulator), the
// LDS read of K-group g + 1 issued before group g's four MFMAs and pinned
// there by a scheduling barrier.  hook() is issued after K-group kAt (pinned
// between the groups' MFMAs the same way; kAt < 0: none).
// MANO_BS_ACC2=1 (diagnostic builds): two accumulators, K-steps 0..19 and
// 20..36, issued alternately so a wave alone in its MFMA phase is not held to
// one MFMA per 40-cycle dependent latency (the 16x16x4 issue interval is 32),
// summed at the end (changes the rounding order: not bit-identical to the
// unfused blend GEMM).
#ifndef MANO_BS_ACC2
#define MANO_BS_ACC2 0
#endif
template <int kAt, typename Hook>
__device__ __forceinline__ f32x4 mfma16_tile_hook(const float (&a)[kGroups16 * 4],
                                                  const f32x4* __restrict__ b, int lane, Hook&& hook) {
#if MANO_BS_ACC2
  constexpr int kHalf = (kGroups16 + 1) / 2;  // K-groups of the first accumulator
  f32x4 acc0 = {}, acc1 = {};
  f32x4 bn0 = b[lane], bn1 = b[kHalf * 64 + lane];
#pragma unroll
  for (int g = 0; g < kHalf; ++g) {
    const int g1 = kHalf + g;
    const f32x4 bv0 = bn0, bv1 = bn1;
    if (g + 1 < kHalf) bn0 = b[(g + 1) * 64 + lane];
    if (g1 + 1 < kGroups16) bn1 = b[(g1 + 1) * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * g + q], bv0[q], acc0, 0, 0, 0);
      if (g1 < kGroups16 && 4 * g1 + q < kSteps16)
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * g1 + q], bv1[q], acc1, 0, 0, 0);
    }
    if (g == kAt) {
      __builtin_amdgcn_sched_barrier(0);
      hook();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  f32x4 sum;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float s = acc0[r] + acc1[r];
    asm volatile("" : "+v"(s));  // scalar adds (no v_pk_add_f32 beside the MFMAs)
    sum[r] = s;
  }
  return sum;
#else
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
    if (g == kAt) {
      __builtin_amdgcn_sched_barrier(0);
      hook();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  return acc;
#endif
}
__device__ __forceinline__ f32x4 mfma16_tile(const float (&a)[kGroups16 * 4], const f32x4* __restrict__ b,
                                             int lane) {
  return mfma16_tile_hook<-1>(a, b, lane, [] {});
}

// LBS A fragments of a 16-hand tile straight from the [n][16][3][4]
// transforms: F[c * 4 + k][q] = A_j(hand h0 + (lane & 15))[c][k], joint
// j = 4 q + (lane >> 4) (rows past the batch end repeat the last hand).
__device__ __forceinline__ void load_lbs_frags(const float* __restrict__ transforms, int64_t h0,
                                               int64_t n, int lane, float (&F)[12][4]) {
  const int64_t n_left = n - 1 - h0;  // >= 0
  const int hl = min(lane & 15, int(n_left < 15 ? n_left : 15));
  const f32x4* A = reinterpret_cast<const f32x4*>(transforms + h0 * kTransformFloats) +
                   (hl * kTransformFloats + (lane >> 4) * 12) / 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const f32x4 v = A[q * 12 + i];
#pragma unroll
      for (int e = 0; e < 4; ++e) F[4 * i + e][q] = v[e];
    }
  }
}

// load_lbs_frags for a tile of hands base + (i << lp), i < n_valid (rows past
// n_valid repeat the last valid hand): blend_skin16's residue-class tiles.
__device__ __forceinline__ void load_lbs_frags_strided(const float* __restrict__ transforms, int64_t base,
                                                       int lp, int n_valid, int lane, float (&F)[12][4]) {
  const int64_t hand = base + (int64_t(min(lane & 15, n_valid - 1)) << lp);
  const f32x4* A = reinterpret_cast<const f32x4*>(transforms + hand * kTransformFloats) + (lane >> 4) * 3;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const f32x4 v = A[q * 12 + i];
#pragma unroll
      for (int e = 0; e < 4; ++e) F[4 * i + e][q] = v[e];
    }
  }
}

// LBS of one 16-hand x 16-vertex tile (mano_np.py:112-115): the 12 transform
// tiles T_{c,k} = F_{c,k} . W^T (4 MFMAs each, K = 16 joints) applied to the
// rest vertices p[coord] as out_c = T_c3 + T_c2 z + T_c1 y + T_c0 x (fmaf,
// translation column first).  kFence pins the three coordinate rows in order
// so at most 16 T registers are live (hipcc otherwise hoists all 48 MFMAs).
template <bool kFence = false>
__device__ __forceinline__ void lbs_apply16(const float (&F)[12][4], const f32x4& wf,
                                            const f32x4 (&p)[3], f32x4 (&out)[3]) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 3 - kk;
      const float* f = F[c * 4 + k];
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
    if constexpr (kFence) {
      asm volatile("" : "+v"(out[c]));  // materialise row c here (no SLP across rows)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// lbs_apply16 for rest vertices held as per-row points p[r] = (x, y, z) of
// hand row0 + r (the skin kernel's loads); same fmaf order.  Each coordinate
// row is materialised before the next so at most 16 T registers are live.
typedef float f32x3 __attribute__((ext_vector_type(3)));
__device__ __forceinline__ void lbs_apply16_rows(const float (&F)[12][4], const f32x4& wf,
                                                 const f32x3 (&p)[4], f32x4 (&out)[3]) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    f32x4 T[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float* f = F[c * 4 + k];
      T[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[0], wf[0], f32x4{}, 0, 0, 0);
      T[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[1], wf[1], T[k], 0, 0, 0);
      T[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[2], wf[2], T[k], 0, 0, 0);
      T[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[3], wf[3], T[k], 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float o = T[3][r];
      o = fmaf(T[2][r], p[r][2], o);
      o = fmaf(T[1][r], p[r][1], o);
      o = fmaf(T[0][r], p[r][0], o);
      asm volatile("" : "+v"(o));  // one scalar chain per row (no SLP pairing)
      out[c][r] = o;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Work split of the persistent launches: the (tile, vertex group) units are
// cut into gridDim.x (blend_skin16: one range per block of 4 hand tiles) or
// 4 gridDim.x (skin_span: one range per wave) equal contiguous ranges, with the
// grid sized to the resident capacity of the chip, so every SIMD gets the same
// MFMA / HBM work and there is no partially-filled second wave of blocks.
__device__ __forceinline__ void unit_range(int64_t units, int64_t worker, int64_t n_workers,
                                           int64_t& begin, int64_t& end) {
  begin = worker * units / n_workers;
  end = (worker + 1) * units / n_workers;
}

// Workgroup barrier after s_waitcnt vmcnt(N) lgkmcnt(0): every vector-memory
// op of this wave but the N youngest has completed (loads, stores and LDS-DMA
// retire in issue order) and every LDS access.  __syncthreads() would wait
// for vmcnt(0) -- the previous group's output stores too -- and hipcc does
// not count the LDS-DMA as an LDS write.
template <int N>
__device__ __forceinline__ void barrier_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Wave issue priority around a short issue section (s_setprio; 0 = unchanged).
template <int P>
__device__ __forceinline__ void prio_up() {
  if constexpr (P != 0) __builtin_amdgcn_s_setprio(P);
}
template <int P>
__device__ __forceinline__ void prio_down() {
  if constexpr (P != 0) __builtin_amdgcn_s_setprio(0);
}
#ifndef MANO_BS_DMA_PRIO
#define MANO_BS_DMA_PRIO 1    // blend_skin16: priority while issuing the basis LDS-DMA (0.512 -> 0.506 ms)
#endif
#ifndef MANO_BS_STORE_PRIO
#define MANO_BS_STORE_PRIO 0  // blend_skin16: priority while issuing the point stores
#endif
// Diagnostic builds only (tools/debug/bs_ablate.sh): 1 = no output stores
// (a never-taken data-dependent store keeps the work alive), 2 = no LBS
// (v_posed is stored as verts), 3 = both, 4 = the same stores into a
// line-aligned scratch layout (each 192-B hand segment at a 256-B boundary:
// same instructions, bytes, cache policy and deferral, no partially written
// sector; the verts and rest_verts buffers must hold n * n_groups * 256 B,
// tools/debug/align_bound.py reads them back in the reference layout).
#ifndef MANO_BS_ABLATE
#define MANO_BS_ABLATE 0
#endif
// 8 = barriers without s_barrier (waits only; results wrong), 16 = no basis
// DMA after the prologue (results wrong).
template <int N>
__device__ __forceinline__ void bs_barrier() {
#if MANO_BS_ABLATE & 8
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
#else
  barrier_vmcnt<N>();
#endif
}
// blend_skin16's verts point stores are nontemporal when verts is the only
// output stream (same-box A/B at 65,536 hands, tools/debug/time_stages.py:
// 0.493 vs 0.504 ms, identical bits).  With rest_verts as a second stream
// they are plain: nontemporal there took 0.85 vs 0.61 ms, and the unfused
// blend GEMM (0.60 vs 0.37) and blend_skin_h3 (0.40 vs 0.26) lose the same way.
// Either stream alone nontemporal beside the other plain is as bad (0.72-0.74
// vs 0.62 ms, profiles/r03k_ab_nt_rest_verts.jsonl).
#ifndef MANO_BS_NT_STORE
#define MANO_BS_NT_STORE 1
#endif
// With rest_verts: bit 0 = verts nontemporal, bit 1 = rest_verts
// nontemporal.  Round 3, with partial sectors, 0 was best; with the
// sector-aligned rows (round 4) 2 is: the rest_verts kernel 0.5555 / 0.5576
// vs 0.5620 / 0.5667 ms, writes 1,313 vs 1,376 MB per launch (1.07x vs
// 1.12x of 1,224), same digests; 1: no change, 3: 0.65 ms
// (profiles/r04c_ab_path.jsonl, r04d_*).
#ifndef MANO_BS_REST_NT
#define MANO_BS_REST_NT 2
#endif
__device__ __forceinline__ float* byte_at(float* base, unsigned byte_off) {
  return reinterpret_cast<float*>(reinterpret_cast<char*>(base) + byte_off);
}
template <bool kNt>
__device__ __forceinline__ void store_out(float* dst, f32x3 v) {
  if constexpr (kNt) __builtin_nontemporal_store(v, reinterpret_cast<f32x3*>(dst));
  else *reinterpret_cast<f32x3*>(dst) = v;
}

// Fused blend GEMM + LBS.  A block owns a contiguous range of (quad of 4
// hand tiles, vertex group) units; at each quad its waves load their A
// fragments (the X rows written by articulate_kernel) and LBS fragments (the
// transforms), then run that quad's groups: 3 GEMM tiles (x, y, z) per group,
// then the LBS epilogue on MFMA; v_posed never leaves registers.  The basis
// tiles are LDS-DMA-staged two tiles ahead in a ring of 3 slots (tile q of a
// group in slot q), so the barrier after tile t waits for tile t + 1's DMA
// only: it was issued before the previous group's output stores, which stay
// in flight (counted vmcnt, below).
// Diagnostic build only (MANO_BS_STAMP=1, tools/debug/bs_stamps.py): per wave
// the shader clock and the 100-MHz real-time clock at entry and exit, the
// hardware ids and the units it ran, read back by mano_debug_bs_stamps().
#ifndef MANO_BS_STAMP
#define MANO_BS_STAMP 0
#endif
#if MANO_BS_STAMP
constexpr int kStampWaves = 4096;
__device__ unsigned long long g_bs_stamps[kStampWaves * 8];
__device__ __forceinline__ void bs_stamp(int slot, unsigned long long v) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && w < kStampWaves) {
    volatile unsigned long long* p = g_bs_stamps + w * 8 + slot;
    *p = v;
  }
}
#endif

#ifndef MANO_BS_BLOCKS_PER_CU
#define MANO_BS_BLOCKS_PER_CU 3  // resident blocks per CU (diagnostic builds: 1, 2, 4)
#endif
template <bool kTrans, bool kVposed>
__global__ __launch_bounds__(256, MANO_BS_BLOCKS_PER_CU) void blend_skin16_kernel(
    const float* __restrict__ features, const float* __restrict__ transforms,
    const float* __restrict__ basis16, const float* __restrict__ wfrag16,
    const float* __restrict__ trans, float* __restrict__ verts, float* __restrict__ vposed,
    int64_t n, int n_verts, int n_groups, int lp, unsigned shifts, int aligned) {
  // One slot: a basis tile (10 KB) + the group's W fragment (1 KB, with the
  // group's first tile); ring of 3.
  constexpr int kRingF4 = (kGroups16 + 1) * 64;
  constexpr int kSlots = 3;
  constexpr int kStores = (MANO_BS_ABLATE & 1) ? 0 : (kVposed ? 8 : 4);  // dwordx3 point stores per group
  // vmcnt of the barrier after tile t: the wave's memory ops issued after tile
  // t + 1's DMA -- tile t + 2's DMA (at least 2 pieces per wave) and, after a
  // group's first tile, the previous group's stores.
  constexpr int kPieces = kGroups16 / 4;     // LDS-DMA pieces per wave and tile, at least
  constexpr int kDmaPrio = MANO_BS_DMA_PRIO, kStorePrio = MANO_BS_STORE_PRIO;
  // With rest_verts (two output streams) a group's rest_verts points leave
  // right after its GEMM tiles and its verts points inside the next group's
  // first tile chain (after K-group 2), so the 8 stores of a group do not
  // issue as one burst (0.605 vs 0.619 ms, same box; the verts-only kernel
  // spills under the extra live registers and keeps its stores together).
  // (Diagnostic ablation builds store nothing or store elsewhere: no deferral,
  // so `pend` / `poff` are never flushed unassigned.)
  constexpr bool kDefer = kVposed && (MANO_BS_ABLATE == 0 || MANO_BS_ABLATE == 4);
  // the verts-only kernel's stores nontemporal; with rest_verts only the
  // rest_verts stream (MANO_BS_REST_NT above)
  constexpr bool kVertsNt = kVposed ? bool(MANO_BS_REST_NT & 1) : bool(MANO_BS_NT_STORE);
  constexpr bool kRestNt = MANO_BS_REST_NT & 2;
  constexpr int kDeferAt = 2;
  __shared__ f32x4 lds[kSlots * kRingF4];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int vstride32 = 3 * n_verts;
  // Sector-aligned rows (mano_layout.h, `aligned`): hands are taken in
  // residue classes r = h mod P (P = 2^lp); quad (r, j) holds hands
  // 64 P j + P i + r, i = 0..63 (wave w: i = 16 w .. 16 w + 15), whose rows
  // share one sector phase, so the whole block uses one operand variant
  // s_r = shifts >> 4 r & 15.  Quads are numbered class-major: the grid's
  // contiguous eighths (the XCDs, below) each read one or two variants.
  // Without it (lp = 0): quad j = hands 64 j .. 64 j + 63, the plain layout.
  const int64_t n_quads = aligned_n_quads(n, lp);
  int64_t u, u_end;
  // Paired ranges: range r goes to block (r % per) * 8 + r / per (per =
  // gridDim / 8), so ranges r and r + 1 sit on one XCD (blocks are dealt to
  // the XCDs round robin: speed only, nothing depends on it), and odd ranges
  // take their quads last-first.  The quad split between ranges r and r + 1
  // is then the first quad both take (odd r) or the last (even r), so its X
  // rows and transforms are fetched once into that XCD's L2 for both
  // (blend_skin16 reads 132 vs 156 MB per launch at 65,536 hands, same time:
  // profiles/r03m_pmc_paired.json).
  int64_t rng = blockIdx.x;
  bool backward = false;
  if (gridDim.x % 8 == 0) {
    const int64_t per = gridDim.x / 8;
    rng = (blockIdx.x % 8) * per + blockIdx.x / 8;
    backward = rng & 1;
  }
  unit_range(n_quads * n_groups, rng, gridDim.x, u, u_end);
  const int64_t q_first = u / n_groups, q_last = (u_end - 1) / n_groups;
#if MANO_BS_STAMP
  bs_stamp(0, __builtin_amdgcn_s_memtime());
  bs_stamp(2, __builtin_amdgcn_s_memrealtime());
  bs_stamp(4, (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                  ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32));
  bs_stamp(5, (unsigned long long)(u_end - u));
  int n_ranges = 0;
  unsigned long long t_first = 0, t_prologue = 0;  // cycles from a range's start to its first barrier
#endif

  for (int64_t iq = 0; u < u_end && iq <= q_last - q_first; ++iq) {
#if MANO_BS_STAMP
    ++n_ranges;
    const unsigned long long t_range = __builtin_amdgcn_s_memtime();
#endif
    const int64_t quad = backward ? q_last - iq : q_first + iq;
    const int64_t qs = quad * n_groups;
    const int g0 = int((u > qs ? u : qs) - qs);
    const int g1 = int((u_end < qs + n_groups ? u_end : qs + n_groups) - qs);
    // This wave's tile: hands h0 + (i << lp), i < n_valid (mano_layout.h).  A
    // wave past the batch end recomputes the quad's last tile and rewrites
    // its (identical) values, so every store below is unconditional.
    const AlignedTile tile = aligned_tile(n, lp, quad, wave);
    const int64_t h0 = tile.h0;
    const int n_valid = tile.n_valid;
    const int shift = aligned ? int((shifts >> (4 * tile.cls)) & 15u) : 0;
    const float* bvar = basis16 + (aligned ? int64_t(shift) * n_groups * 3 * kTile16Floats : 0);
    const float* wvar = wfrag16 + (aligned ? int64_t(shift) * n_groups * kWFrag16Floats : 0);

    // An opaque lane index per range: keeps hipcc from hoisting lane-dependent
    // addresses out of the range loop, which would hold them in registers --
    // spilled -- across the GEMM.
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    const int row0 = 4 * (lane >> 4);  // D rows (hands) of this lane: row0 + r
    const int col = lane & 15;         // D column (vertex of the group)


    float a[kGroups16 * 4];
    float F[12][4];  // LBS A fragments, tile (c, k) = c * 4 + k, resident for the quad
    // A fragments from the X rows: lane's steps 4g..4g+3 are one dwordx4.
    const int64_t row = h0 + (int64_t(min(lane & 15, n_valid - 1)) << lp);
    const f32x4* src = reinterpret_cast<const f32x4*>(features + row * kXStride) + (lane >> 4);
#pragma unroll
    for (int g = 0; g < kGroups16; ++g) {
      const f32x4 v = src[4 * g];
#pragma unroll
      for (int q = 0; q < 4; ++q) a[4 * g + q] = v[q];
    }
    load_lbs_frags_strided(transforms, h0, lp, n_valid, lane, F);
    // The lane's 4 rows' translations, held in registers for the range (read
    // from an LDS copy at every group: 0.4952 vs 0.4913 ms with trans, same bits)
    float tv[4][3];
    if constexpr (kTrans) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) tv[r][c] = trans[(h0 + (int64_t(min(row0 + r, n_valid - 1)) << lp)) * 3 + c];
    }
    // ABLATE 4: tiles of 16 rows x n_groups x 64 floats (the aligned scratch layout)
    const int64_t tile_floats = MANO_BS_ABLATE == 4 ? int64_t(n_groups) * 64 : int64_t(vstride32);
    float* vtile = verts + h0 * tile_floats;
    float* ptile = kVposed ? vposed + h0 * tile_floats : nullptr;
    const int rstride = vstride32 << lp;  // floats between the tile's rows

    // The W fragment rides in the slot of the group's first tile (LDS-DMA by
    // wave 2, which has the fewest basis pieces): a global load in the loop
    // would make hipcc wait vmcnt(0) -- the tiles in flight -- before the LBS.
    auto stage_w = [&](int grp, f32x4* slot) {
      if (wave == 2) {
        unsigned lane_off = unsigned(lane) * 16u;
        asm volatile("" : "+v"(lane_off));
        const char* src = reinterpret_cast<const char*>(wvar + int64_t(grp) * kWFrag16Floats);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + lane_off),
                                         (__attribute__((address_space(3))) void*)(slot + kGroups16 * 64),
                                         16, 0, 0);
      }
    };
    stage_basis_tile16(bvar, 3 * g0, lds, wave, lane);
    stage_w(g0, lds);
    stage_basis_tile16(bvar, 3 * g0 + 1, lds + kRingF4, wave, lane);
    bs_barrier<0>();  // the first two tiles and every prologue load have landed
#if MANO_BS_STAMP
    {
      const unsigned long long dt = __builtin_amdgcn_s_memtime() - t_range;
      if (n_ranges == 1) t_first = dt;
      t_prologue += dt;
    }
#endif

    f32x3 pend[4];      // kDefer: the previous group's verts points, stored during this group's tile 0
    unsigned poff[4];
    auto flush = [&]() {
#pragma unroll
      for (int r = 0; r < 4; ++r) store_out<kVertsNt>(byte_at(vtile, poff[r]), pend[r]);
    };
    for (int grp = g0; grp < g1; ++grp) {
      const bool more = grp + 1 < g1;
      f32x4 p[3];
      // Tile 3 grp + q in slot q; tile 3 grp + q + 2 goes to slot (q + 2) % 3.
      prio_up<kDmaPrio>();
      if constexpr (!(MANO_BS_ABLATE & 16)) stage_basis_tile16(bvar, 3 * grp + 2, lds + 2 * kRingF4, wave, lane);
      prio_down<kDmaPrio>();
      const f32x4 wf = lds[kGroups16 * 64 + lane];  // read before slot 0 is re-staged
      if (!kDefer || grp == g0) p[0] = mfma16_tile(a, lds, lane);
      else p[0] = mfma16_tile_hook<kDeferAt>(a, lds, lane, flush);
      if (grp == g0) bs_barrier<kPieces>();
      else bs_barrier<kPieces + kStores>();
      if (more) {
        prio_up<kDmaPrio>();
        if constexpr (!(MANO_BS_ABLATE & 16)) stage_basis_tile16(bvar, 3 * grp + 3, lds, wave, lane);
        stage_w(grp + 1, lds);
        prio_down<kDmaPrio>();
      }
      p[1] = mfma16_tile(a, lds + kRingF4, lane);
      if (more) bs_barrier<kPieces>();
      else bs_barrier<0>();
      if (more) {
        prio_up<kDmaPrio>();
        if constexpr (!(MANO_BS_ABLATE & 16)) stage_basis_tile16(bvar, 3 * grp + 4, lds + kRingF4, wave, lane);
        prio_down<kDmaPrio>();
      }
      p[2] = mfma16_tile(a, lds + 2 * kRingF4, lane);
      if (more) bs_barrier<kPieces>();
      else bs_barrier<0>();
      // the lane's vertex in this group (grp, shift uniform: scalar branches)
      int vx;
      if (aligned) {
        vx = aligned_group_vertex(n_verts, shift, grp, col);
      } else {
        const int vb = grp * 16 < n_verts - 16 ? grp * 16 : n_verts - 16;
        vx = vb + col;
      }
      const int voff = 3 * vx;
      // byte offset of row hr's point of this lane from the tile base
      auto row_off = [&](int hr) -> unsigned {
        if constexpr (MANO_BS_ABLATE == 4) return 4u * unsigned(((hr << lp) * n_groups + grp) * 64 + 3 * col);
        else return 4u * unsigned(hr * rstride + voff);
      };
      if constexpr (kVposed) {
        // rest_verts leave before the LBS: their stores drain under its MFMAs
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int hr = min(row0 + r, n_valid - 1);
          store_out<kRestNt>(byte_at(ptile, row_off(hr)), f32x3{p[0][r], p[1][r], p[2][r]});
        }
      }
      f32x4 out[3];
      if constexpr (MANO_BS_ABLATE & 2) {
        out[0] = p[0];
        out[1] = p[1];
        out[2] = p[2];
        (void)wf;
      } else {
        lbs_apply16(F, wf, p, out);
      }
      if constexpr (MANO_BS_ABLATE & 1) {
        if (out[0][0] == 1234.5f && out[1][1] == 2345.5f) vtile[voff] = out[2][2];
        continue;
      }
      prio_up<kStorePrio>();
      // One 12-B point store per row; rows past the batch end rewrite the
      // last hand's identical values.
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hr = min(row0 + r, n_valid - 1);
        float o0 = out[0][r], o1 = out[1][r], o2 = out[2][r];
        if constexpr (kTrans) {
          o0 += tv[r][0];
          o1 += tv[r][1];
          o2 += tv[r][2];
        }
        // 32-bit byte offset from the tile's uniform base (< 16 rows x 9,336 B):
        // the SGPR-base + VGPR-offset store form, no 64-bit address VALU.
        // (opaque: hipcc otherwise hoists the row offsets and spills 10 VGPRs
        // in the verts-only range prologue)
        unsigned boff = row_off(hr);
        asm volatile("" : "+v"(boff));
        if constexpr (kDefer) {
          pend[r] = f32x3{o0, o1, o2};
          poff[r] = boff;
        } else
          store_out<kVertsNt>(byte_at(vtile, boff), f32x3{o0, o1, o2});
      }
      prio_down<kStorePrio>();
    }
    if constexpr (kDefer) flush();  // the range's last group
  }
#if MANO_BS_STAMP
  bs_stamp(1, __builtin_amdgcn_s_memtime());
  bs_stamp(3, __builtin_amdgcn_s_memrealtime());
  bs_stamp(6, (unsigned long long)n_ranges);
  bs_stamp(7, t_first | (t_prologue << 32));
#endif
}

// ---------------------------------------------------------------------------
// skin_span: standalone LBS (mano_np.py:112-115) over a v_posed buffer, the
// span streaming of mano_span.h (16 hands x 64 vertices per wave unit, whole-
// line float4 sweeps through a per-wave LDS stage) with blend_skin16's LBS
// operands and arithmetic: the transform fragments of a tile stay in VGPRs,
// each group runs the same 12 v_mfma_f32_16x16x4_f32 transform tiles and
// fmaf apply order (lbs_apply16_rows), then + trans -- so the staged path
// agrees with blend_skin16 bit for bit.
// ---------------------------------------------------------------------------
template <bool kTrans>
struct SpanLbs16 {
  using W = f32x4;
  static constexpr bool kInPlace = true;
  struct Tile {
    float F[12][4];
    float tr[4][3];
  };
  const float* transforms;
  const float* wfrag16;
  const float* trans;
  Tile cur;

  __device__ __forceinline__ W load_w(int grp, int lane) const {
    return reinterpret_cast<const f32x4*>(wfrag16 + int64_t(grp) * kWFrag16Floats)[lane];
  }
  __device__ __forceinline__ void fetch_tile(int64_t h0, int64_t n, int n_valid, int lane, Tile& t) const {
    load_lbs_frags(transforms, h0, n, lane, t.F);
    if constexpr (kTrans) {
      const int row0 = 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) t.tr[r][c] = trans[(h0 + min(row0 + r, n_valid - 1)) * 3 + c];
    }
  }
  __device__ __forceinline__ void set_tile(const Tile& t) { cur = t; }
  __device__ __forceinline__ void apply(const W& wf, const float (&p)[4][3], float (&o)[4][3]) const {
    f32x3 pr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pr[r] = f32x3{p[r][0], p[r][1], p[r][2]};
    f32x4 out[3];
    lbs_apply16_rows(cur.F, wf, pr, out);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) o[r][c] = kTrans ? out[c][r] + cur.tr[r][c] : out[c][r];
  }
};

template <bool kTrans>
__global__ __launch_bounds__(256, MANO_SPAN_BLOCKS_PER_CU) void skin_span_kernel(
    const float* __restrict__ transforms, const float* __restrict__ wfrag16,
    const float* __restrict__ vposed, const float* __restrict__ trans, float* __restrict__ verts,
    int64_t n, int n_verts, int n_groups) {
  __shared__ f32x4 stage[4 * span::kStageFloats / 4];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SpanLbs16<kTrans> lbs{transforms, wfrag16, trans, {}};
  span::run_units<true, 3, MANO_SPAN_CHUNK>(lbs, vposed, verts, n, n_verts, n_groups, span::xcd_worker(wave),
                  int64_t(gridDim.x) * 4, reinterpret_cast<float*>(stage) + wave * span::kStageFloats,
                  int(threadIdx.x & 63));
}


// ---------------------------------------------------------------------------
// Synthetic workload (include/mano_hip.h mano_synthetic_inputs): Philox-4x32-10
// keyed by the seed, counter (global hand index lo, hi, block, 0).  One lane
// per (hand, block): 16 lanes x 4 words = the hand's 64 words; Box-Muller pairs
// (w[2m], w[2m+1]) never straddle a block.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = uint64_t(0xD2511F53u) * c[0];
    const uint64_t p1 = uint64_t(0xCD9E8D57u) * c[2];
    const uint32_t hi0 = uint32_t(p0 >> 32), lo0 = uint32_t(p0);
    const uint32_t hi1 = uint32_t(p1 >> 32), lo1 = uint32_t(p1);
    c[0] = hi1 ^ c[1] ^ k0;
    c[1] = lo1;
    c[2] = hi0 ^ c[3] ^ k1;
    c[3] = lo0;
  }
}

// u in (0, 1), exactly representable: ((w >> 8) + 0.5) / 2^24.
__device__ __forceinline__ float unit_open(uint32_t w) {
  return (float(w >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

__global__ __launch_bounds__(256) void synthetic_inputs_kernel(
    uint32_t k0, uint32_t k1, int64_t first, int64_t n, float beta_sigma, float pose_sigma,
    float trans_range, float* __restrict__ betas, float* __restrict__ pose,
    float* __restrict__ trans) {
  // Grid-stride over the n * 16 (hand, block) lanes: the grid is bounded
  // (launch_synthetic_inputs), any n up to the ABI's 2^30 hands.
  for (int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x; idx < n * 16;
       idx += int64_t(gridDim.x) * 256) {
    const int64_t h = idx >> 4;
    const int b = int(idx & 15);
    const uint64_t g = uint64_t(first + h);
    uint32_t w[4] = {uint32_t(g), uint32_t(g >> 32), uint32_t(b), 0u};
    philox4x32_10(w, k0, k1);
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int e = 4 * b + 2 * pr;  // element index of the pair's first member
      float v[2];
      if (e < 58) {
        const float r = sqrtf(-2.0f * logf(unit_open(w[2 * pr])));
        float s, c;
        sincospif(2.0f * unit_open(w[2 * pr + 1]), &s, &c);
        v[0] = r * c;
        v[1] = r * s;
      } else {
        v[0] = 2.0f * unit_open(w[2 * pr]) - 1.0f;
        v[1] = 2.0f * unit_open(w[2 * pr + 1]) - 1.0f;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int el = e + q;
        if (el < kShape) {
          if (betas) betas[h * kShape + el] = beta_sigma * v[q];
        } else if (el < 58) {
          if (pose) pose[h * (kJoints * 3) + (el - kShape)] = pose_sigma * v[q];
        } else if (el < 61) {
          if (trans) trans[h * 3 + (el - 58)] = trans_range * v[q];
        }
      }
    }
  }
}

}  // namespace

hipError_t launch_synthetic_inputs(uint64_t seed, int64_t first, int64_t n, float beta_sigma,
                                   float pose_sigma, float trans_range, float* betas, float* pose,
                                   float* trans, hipStream_t stream) {
  const int64_t threads = n * 16;
  const int64_t blocks = std::min<int64_t>((threads + 255) / 256, int64_t(1) << 20);  // grid-stride beyond
  hipLaunchKernelGGL(synthetic_inputs_kernel, dim3(unsigned(blocks)), dim3(256), 0,
                     stream, uint32_t(seed), uint32_t(seed >> 32), first, n, beta_sigma, pose_sigma,
                     trans_range, betas, pose, trans);
  return hipGetLastError();
}

hipError_t launch_blend(const DeviceModel& m, int64_t n, const float* features, float* vposed,
                        hipStream_t stream) {
  // v_posed rows' sector phases (mano_layout.h): class r of the rows starts at
  // float a + 3 V r (mod 8); its column tiles are shifted onto sector
  // boundaries (MANO_BS_ALIGN 0: the plain tiles).
  int lp = 0, aligned = 0;
  unsigned shifts = 0;
  const float* tiles = m.basis_tiles;
  if (MANO_BS_ALIGN && m.basis_tiles_v) {
    lp = aligned_period_log2(m.n_verts);
    shifts = aligned_col_shifts(m.n_verts, unsigned(reinterpret_cast<uintptr_t>(vposed) >> 2) & 7u, lp);
    tiles = m.basis_tiles_v;
    aligned = 1;
  }
  const int64_t blocks = aligned_n_quads(n, lp, 7);
  hipLaunchKernelGGL(blend_kernel, dim3(unsigned(blocks)), dim3(256), 0, stream, features,
                     tiles, vposed, n, m.n_cols, m.n_col_tiles, lp, shifts, aligned);
  return hipGetLastError();
}

namespace {

// Blocks of `kernel` (256 threads) the device holds at once.  Each persistent
// kernel states the blocks per CU it is built for (its __launch_bounds__); the
// occupancy API only caps that, because it reads one block per CU high for
// kernels using 97-112 SGPRs on gfx950 (MI355X_MICROARCH.md, correctness
// boundaries).
constexpr int kBlendSkinBlocksPerCU = MANO_BS_BLOCKS_PER_CU;  // 142 VGPRs: 3 waves per SIMD
constexpr int kSkinBlocksPerCU = MANO_SPAN_BLOCKS_PER_CU;  // skin_span

template <class Kernel>
int64_t resident_blocks(Kernel kernel, const DeviceModel& m, int design_per_cu) {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, 256, 0) != hipSuccess || b < 1) b = 1;
  if (b > design_per_cu) b = design_per_cu;
  return int64_t(b) * (m.n_cu > 0 ? m.n_cu : 1);
}

// At least this many (tile, group) units per worker: below it, splitting a
// tile's groups over more workers costs more operand set-up than it gains --
// except while that would leave CUs empty: small launches (the drop-in's
// batch of 1 is 49 units) spread one block per CU, down to a unit per worker,
// for latency.
constexpr int64_t kMinUnitsPerWorker = 8;

template <class Kernel>
dim3 persistent_grid(Kernel kernel, const DeviceModel& m, int64_t units, int workers_per_block,
                     int design_per_cu) {
  const int64_t want = (units + kMinUnitsPerWorker - 1) / kMinUnitsPerWorker;
  int64_t blocks_wanted = (want + workers_per_block - 1) / workers_per_block;
  const int64_t spread = (units + workers_per_block - 1) / workers_per_block;
  const int64_t n_cu = m.n_cu > 0 ? m.n_cu : 1;
  if (blocks_wanted < n_cu) blocks_wanted = spread < n_cu ? spread : n_cu;
  const int64_t cap = resident_blocks(kernel, m, design_per_cu);
  return dim3{unsigned(blocks_wanted < cap ? blocks_wanted : cap)};
}

}  // namespace

hipError_t launch_blend_skin(const DeviceModel& m, int64_t n, const float* features,
                             const float* transforms, const float* trans, float* verts,
                             float* vposed, hipStream_t stream) {
  // The verts rows' sector phases: class r = h mod 2^lp starts at float
  // a + 3 V r (mod 8), a = the verts address in floats (mod 8); its variant
  // s_r = (-3 c_r) mod 8 puts the groups on sector boundaries.
  int lp = 0, aligned = 0;
  unsigned shifts = 0;
  const float* b16 = m.basis16;
  const float* w16 = m.wfrag16;
  if (MANO_BS_ALIGN && MANO_BS_ABLATE == 0 && m.basis16v && m.wfrag16v) {
    lp = aligned_period_log2(m.n_verts);
    shifts = aligned_shifts(m.n_verts, unsigned(reinterpret_cast<uintptr_t>(verts) >> 2) & 7u, lp);
    b16 = m.basis16v;
    w16 = m.wfrag16v;
    aligned = 1;
  }
  const int64_t n_quads = aligned_n_quads(n, lp);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, persistent_grid(kernel, m, n_quads * m.n_groups16, 1, kBlendSkinBlocksPerCU),
                       dim3(256), 0, stream, features, transforms, b16, w16, trans, verts,
                       vposed, n, m.n_verts, m.n_groups16, lp, shifts, aligned);
  };
  if (trans && vposed) launch(blend_skin16_kernel<true, true>);
  else if (trans) launch(blend_skin16_kernel<true, false>);
  else if (vposed) launch(blend_skin16_kernel<false, true>);
  else launch(blend_skin16_kernel<false, false>);
  return hipGetLastError();
}

// fp32 standalone LBS: skin_quad (mano_skin_quad.hip) by default; skin_span
// (above) for meshes it does not take, or with MANO_SKIN_QUAD=0.
#ifndef MANO_SKIN_QUAD
#define MANO_SKIN_QUAD 1
#endif
hipError_t launch_skin(const DeviceModel& m, int64_t n, const float* transforms,
                       const float* vposed, const float* trans, float* verts,
                       hipStream_t stream) {
#if MANO_SKIN_QUAD
  if (skin_quad_supported(m)) return launch_skin_quad(m, n, transforms, vposed, trans, verts, stream);
#endif
  const int64_t units = (n + 15) / 16 * span::n_spans(m.n_verts);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, persistent_grid(kernel, m, units, 4, kSkinBlocksPerCU), dim3(256), 0,
                       stream, transforms, m.wfrag16, vposed, trans, verts, n, m.n_verts, m.n_groups16);
  };
  if (trans) launch(skin_span_kernel<true>);
  else launch(skin_span_kernel<false>);
  return hipGetLastError();
}

#if MANO_BS_STAMP
}  // namespace mano
extern "C" int mano_debug_bs_stamps(unsigned long long* host, int count) {
  if (count > mano::kStampWaves * 8) count = mano::kStampWaves * 8;
  return int(hipMemcpyFromSymbol(host, HIP_SYMBOL(mano::g_bs_stamps), size_t(count) * 8, 0,
                                 hipMemcpyDeviceToHost));
}
namespace mano {
#endif

}  // namespace mano
