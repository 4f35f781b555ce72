// mano_kernels_h3.hip -- the f16x3 precision mode of the MANO forward pass on
// gfx950 (MI355X): the blend GEMM (mano_np.py:81, :87-93) and the LBS
// transform blend (:112) on v_mfma_f32_16x16x32_f16 with every fp32 operand
// split into two halves (mano_internal.h, "f16x3 precision mode").
//
// gfx950 has no reduced-precision fast path for fp32 inputs (no xf32): an f32
// MFMA runs at 1/16 of the f16 rate.  Three f16 MFMAs per product
// (hi.hi + hi.lo + lo.hi, each exact in the fp32 accumulator) do the same
// contraction at 16/3 x the f32 rate with 22 significant bits per operand:
// measured vertex error vs the float64 reference is the same order as the
// exact-fp32 path (~1e-7 m; tests/test_gpu_parity.py), and the forward pass
// moves from the MFMA roof to the HBM store roof.
//
//   blend_skin_h3  fused: per (16-hand tile, 16-vertex group) 45 GEMM MFMAs
//                  (3 coords x 5 K-steps x 3 split products) on basis pieces
//                  LDS-DMA-staged per group (32 KB, ring of 2, shared by the 4
//                  waves of a block), then 24 LBS MFMAs (12 transform tiles x
//                  2) applied in registers; v_posed never leaves registers.
//   skin_span_h3   standalone LBS over a v_posed buffer (HBM streaming in
//                  64-vertex spans, mano_span.h), the same 24 LBS MFMAs and
//                  apply order as blend_skin_h3.
//
// Packed fp32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) is kept out of
// these kernels: every scalar result the vectorizer could pair goes through
// no_pack(), and the library is built with -fno-slp-vectorize.  Packed fp32
// beside MFMA is also the slower form on gfx950 (MI355X_MICROARCH.md).
//
// The fused kernel has NO rest_verts (v_posed output) instantiation.  Built
// with the vectorizer on, those instantiations -- and only those -- returned
// wrong x coordinates for hand rows 14-15 under load; round 2 localized it to
// a v_pk_fma_f32 with an SGPR-pair multiplier (the LBS output's final
// fma(o, 2^-k, trans)) and excluded wait-state hazards, the counted vmcnt
// barriers, stray stores and spills, but no hardware or compiler rule that
// explains it was found (profiles/r03_f16x3_windows.jsonl).
// Rather than ship a kernel whose correctness rests on a guard nobody can
// explain, the product does not build it: an F16X3 call that asks for
// rest_verts runs the exact-fp32 blend_skin16 (mano_abi.hip), so f16x3
// arithmetic is used for verts-only forwards.  The guards stay (no_pack,
// -fno-slp-vectorize, the ISA scans of tests/test_codegen.py).
//
// CORRECTNESS DEPENDS ON THE BUILD FLAG.  The kernels that remain are correct
// as built with -fno-slp-vectorize (no packed fp32 anywhere in the library);
// the root cause of the packed-FMA miscompute was never found, so nothing
// says the remaining kernels would stay correct if the vectorizer paired
// their scalars again.  Two CPU tests guard it: the flag is on both build
// recipes (test_no_slp_vectorize_flag_on_every_build) and the disassembly
// has no v_pk_*_f32 (test_no_packed_fp32_valu).
//
// FROZEN (round 6).  The mode is opt-in and off the headline: blend_skin_h3
// runs at 0.263 ms = 33 % of 8 TB/s on its 10,744 B/hand (2.67 TB/s, 18 %
// more counter traffic than algorithmic), the sum of a latency-bound GEMM
// phase and a store phase that do not overlap.  The one split left that
// could overlap them (a wave per output coordinate or vertex group with its
// B fragments in registers) was priced by its store order alone at 0.210 ms
// for the stores (profiles/r05/r05w_store_patterns.txt) -- above the 0.20-ms
// mark a rebuild would need -- so no further variant is built.
#include "mano_internal.h"
#include "mano_span.h"

#ifndef MANO_H3_ASM_MFMA
#define MANO_H3_ASM_MFMA 0
#endif
// Sector-aligned output rows (mano_layout.h; diagnostic builds: 0 = plain).
#ifndef MANO_H3_ALIGN
#define MANO_H3_ALIGN 1
#endif

namespace mano {
namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// An opaque scalar: the value leaves the vectorizer's reach (no packed fp32).
// MANO_H3_NO_PACK=0 (debug builds for tools/debug/h3_root_cause.sh only)
// makes it transparent again.
#ifndef MANO_H3_NO_PACK
#define MANO_H3_NO_PACK 1
#endif
__device__ __forceinline__ float no_pack(float x) {
#if MANO_H3_NO_PACK
  asm("" : "+v"(x));
#endif
  return x;
}
// MANO_H3_SCALAR_UNSCALE=1 (debug builds): the LBS output's final
// fma(o, 2^-k, trans) stays scalar even when no_pack is transparent.
#ifndef MANO_H3_SCALAR_UNSCALE
#define MANO_H3_SCALAR_UNSCALE 0
#endif
__device__ __forceinline__ float no_pack_unscale(float x) {
#if MANO_H3_NO_PACK || MANO_H3_SCALAR_UNSCALE
  asm("" : "+v"(x));
#endif
  return x;
}

#if MANO_H3_ASM_MFMA
// Debug form: the MFMAs as inline asm with tied accumulators; results reach
// VALU through mfma_fence (hipcc does not see the asm MFMAs' latency).
__device__ __forceinline__ void mfma_init(f32x4& acc, const f16x8& a, const f16x8& b) {
  asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_acc(f32x4& acc, const f16x8& a, const f16x8& b) {
  asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
template <int N>
__device__ __forceinline__ void mfma_fence(f32x4 (&t)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(t[i]));
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(t[i]));
}
template <int N>
__device__ __forceinline__ void operand_fence(f16x8 (&f)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
  asm volatile("s_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}
#else
__device__ __forceinline__ void mfma_init(f32x4& acc, const f16x8& a, const f16x8& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
}
__device__ __forceinline__ void mfma_acc(f32x4& acc, const f16x8& a, const f16x8& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void mfma_fence(f32x4 (&)[N]) {}
template <int N>
__device__ __forceinline__ void operand_fence(f16x8 (&)[N]) {}
#endif

// Blend-GEMM A fragments of one hand row, split into halves.  Step s, element
// j of lane quarter q = lane >> 4 is X[k = 32 s + 8 q + j]; in the k-permuted
// fp32 row (x_pos) the pair (j = m, j = m + 4) sits at 16 (2 s + (q >> 1)) +
// 4 m + 2 (q & 1), so each step is 4 dwordx2 loads.
__device__ __forceinline__ void load_x_h3(const float* __restrict__ xrow, int q,
                                          f16x8 (&xh)[kH3Steps], f16x8 (&xl)[kH3Steps]) {
#pragma unroll
  for (int s = 0; s < kH3Steps; ++s) {
    const float* blk = xrow + 16 * (2 * s + (q >> 1)) + 2 * (q & 1);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f32x2 v = *reinterpret_cast<const f32x2*>(blk + 4 * m);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const _Float16 h = static_cast<_Float16>(v[e]);
        xh[s][m + 4 * e] = h;
        xl[s][m + 4 * e] = static_cast<_Float16>(no_pack(v[e] - static_cast<float>(h)));
      }
    }
  }
}

// LBS A fragments of a 16-hand tile from the [n][16][3][4] transforms:
// F[c * 4 + k] element j of lane l = part(2^kH3FrameExp A_{8 ((l >> 4) & 1) + j}
// (hand h0 + (l & 15))[c][k]), part = hi for l < 32, lo for l >= 32 (rows past
// the batch end repeat the last hand).  fetch: the lane's 8 joints x 3 rows;
// split: the halves.
__device__ __forceinline__ void fetch_frames_h3(const float* __restrict__ transforms, int64_t h0,
                                                int64_t n, int lane, f32x4 (&raw)[24]) {
  const int64_t n_left = n - 1 - h0;  // >= 0
  const int hl = min(lane & 15, int(n_left < 15 ? n_left : 15));
  const f32x4* A = reinterpret_cast<const f32x4*>(transforms + (h0 + hl) * kTransformFloats) +
                   8 * ((lane >> 4) & 1) * 3;
#pragma unroll
  for (int i = 0; i < 24; ++i) raw[i] = A[i];
}

__device__ __forceinline__ void split_frames_h3(const f32x4 (&raw)[24], int lane, f16x8 (&F)[12]) {
  const bool lo = lane >= 32;
  constexpr float kScale = float(1 << kH3FrameExp);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x = no_pack(raw[3 * j + c][k] * kScale);
        const _Float16 h = static_cast<_Float16>(x);
        F[c * 4 + k][j] = lo ? static_cast<_Float16>(no_pack(x - static_cast<float>(h))) : h;
      }
    }
  }
}

// The fused kernel's tiles: hands h0 + (i << lp), i <= rmax (rows past rmax
// repeat hand rmax; residue-class tiles, mano_layout.h).
__device__ __forceinline__ void load_frames_h3(const float* __restrict__ transforms, int64_t h0,
                                               int lp, int rmax, int lane, f16x8 (&F)[12]) {
  f32x4 raw[24];
  const int64_t hand = h0 + (int64_t(min(lane & 15, rmax)) << lp);
  const f32x4* A = reinterpret_cast<const f32x4*>(transforms + hand * kTransformFloats) + 8 * ((lane >> 4) & 1) * 3;
#pragma unroll
  for (int i = 0; i < 24; ++i) raw[i] = A[i];
  split_frames_h3(raw, lane, F);
}

// LBS of one 16-hand x 16-vertex tile (mano_np.py:112-115): transform tiles
// T_{c,k} = [Fh | Fl].[Wh ; Wh] + [Fh | Fl].[Wl ; 0] (K = 32 each; the 12
// tiles' first MFMAs, then their second, so no MFMA waits on its
// predecessor), applied to the rest vertices p[coord] as out_c =
// fma(T_c3 + T_c2 z + T_c1 y + T_c0 x, 2^-(kH3FrameExp + kH3WeightExp),
// trans_c), translation column first, every rounding spelled out (fmaf) so
// fused and standalone LBS agree bit for bit.
__device__ __forceinline__ void lbs_h3(const f16x8 (&F)[12], const f16x8& w1, const f16x8& w2,
                                       const f32x4 (&p)[3], float t_unscale,
                                       const float (&tr)[4][3], f32x4 (&out)[3]) {
  f32x4 T[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) mfma_init(T[i], F[i], w2);
#pragma unroll
  for (int i = 0; i < 12; ++i) mfma_acc(T[i], F[i], w1);
  mfma_fence(T);
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float o = T[c * 4 + 3][r];
#pragma unroll
      for (int k = 2; k >= 0; --k) o = no_pack(fmaf(T[c * 4 + k][r], p[k][r], o));
      out[c][r] = no_pack_unscale(fmaf(o, t_unscale, tr[r][c]));
    }
}

#ifndef MANO_H3_SKIN_PAIR
#define MANO_H3_SKIN_PAIR 1  // standalone f16x3 LBS: skin_pair's structure (skin_span_h3 for what it does not take)
#endif
#ifndef MANO_H3_DMA_PRIO
#define MANO_H3_DMA_PRIO 0  // blend_skin_h3: wave priority while issuing the next group's LDS-DMA (1 and 3 measured: within noise)
#endif

// Workgroup barrier after s_waitcnt vmcnt(N) lgkmcnt(0): every vector-memory
// op of this wave but the N youngest has completed (loads, stores and LDS-DMA
// count together, in issue order) and every LDS access.  __syncthreads() would
// add the workgroup release fence, i.e. vmcnt(0): a wait on the group's output
// stores that the LDS hand-off does not need.
// MANO_H3_FULL_WAIT=1 (debug builds) waits for every vector-memory op instead.
#ifndef MANO_H3_FULL_WAIT
#define MANO_H3_FULL_WAIT 0
#endif
// MANO_H3_ABLATE (diagnostic builds; results wrong): 1 = waits without
// s_barrier, 2 = no output stores, 4 = no LBS (v_posed stored as verts),
// 8 = no basis DMA after the range prologue.
#ifndef MANO_H3_ABLATE
#define MANO_H3_ABLATE 0
#endif
template <int N>
__device__ __forceinline__ void barrier_vmcnt() {
#if MANO_H3_ABLATE & 1
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(MANO_H3_FULL_WAIT ? 0 : N) : "memory");
#else
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(MANO_H3_FULL_WAIT ? 0 : N) : "memory");
#endif
}

#ifndef MANO_H3_NT_STORE
#define MANO_H3_NT_STORE 0  // nontemporal output point stores (as blend_skin16's)
#endif
__device__ __forceinline__ void store_out_h3(float* dst, f32x3 v) {
  if constexpr (MANO_H3_NT_STORE) __builtin_nontemporal_store(v, reinterpret_cast<f32x3*>(dst));
  else *reinterpret_cast<f32x3*>(dst) = v;
}

__device__ __forceinline__ void unit_range_h3(int64_t units, int64_t worker, int64_t n_workers,
                                              int64_t& begin, int64_t& end) {
  begin = worker * units / n_workers;
  end = (worker + 1) * units / n_workers;
}

#ifndef MANO_H3_WAVES
#define MANO_H3_WAVES 8
#endif
constexpr int kH3Waves = MANO_H3_WAVES;  // waves (16-hand tiles) per blend_skin_h3 block
#ifndef MANO_H3_TPW
#define MANO_H3_TPW 1
#endif
constexpr int kH3TPW = MANO_H3_TPW;  // 16-hand tiles per wave (each B piece read feeds them all)
#ifndef MANO_H3_BLOCKS
#define MANO_H3_BLOCKS 1
#endif
constexpr int kH3BlocksPerCU = MANO_H3_BLOCKS;
#ifndef MANO_H3_RING
#define MANO_H3_RING 2
#endif
#ifndef MANO_H3_SPLIT_ACC
#define MANO_H3_SPLIT_ACC 0  // blend_skin_h3: one LDS read per B fragment, two accumulators
#endif
// LDS slots of blend_skin_h3's basis ring (32 KB each; groups staged ahead =
// kH3Ring - 1).  160 KB of LDS per CU holds at most 4 with one block per CU.
constexpr int kH3Ring = MANO_H3_RING;
static_assert(kH3Ring >= 2 && kH3Ring <= 4 && kH3Ring * 32 * 1024 * kH3BlocksPerCU <= 160 * 1024, "basis ring exceeds the LDS");

// barrier_vmcnt<kBase + d * (DMA ops per group)> for d = later_dmas (a
// runtime value: one branch per count, each an immediate s_waitcnt).
template <int kBase>
__device__ __forceinline__ void ring_barrier(int later_dmas) {
  constexpr int kDma = kH3GroupPieces / kH3Waves;  // global_load_lds per wave per group
  if (later_dmas <= 0) barrier_vmcnt<kBase>();
  else if (later_dmas == 1) barrier_vmcnt<kBase + kDma>();
  else barrier_vmcnt<kBase + 2 * kDma>();
}


// One group's 32 fragment pieces (32 KB), global -> LDS, 32 / kH3Waves per wave.
__device__ __forceinline__ void stage_group_h3(const uint16_t* __restrict__ basis_h3, int grp,
                                               f16x8* slot, int wave, int lane) {
  const uint16_t* src = basis_h3 + int64_t(grp) * kH3GroupHalves + lane * 8;
#pragma unroll
  for (int i = 0; i < kH3GroupPieces / kH3Waves; ++i) {
    const int piece = wave + kH3Waves * i;
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + piece * kH3PieceHalves),
        (__attribute__((address_space(3))) void*)(slot + piece * 64), 16, 0, 0);
  }
  // LDS reads of the ring must not move above the DMA issue.
  asm volatile("" ::: "memory");
}

// Fused blend GEMM + LBS, f16x3, verts only.  A block (kH3Waves waves, kH3TPW
// 16-hand tiles each) owns a contiguous range of (block tile set, vertex group)
// units; the group's basis + weight pieces are LDS-DMA-staged once per block,
// one group ahead (ring of 2 x 32 KB), and every B piece a wave reads feeds its
// kH3TPW tiles.  Each group ends with an explicit vmcnt wait: the next
// group's DMA was issued before this group's kStores output stores, so
// vmcnt(kStores) covers it without waiting for the stores themselves.  Stores
// are branch-free (rows past the batch end rewrite the last hand's identical
// values), so their count is exact.
template <bool kTrans>
__global__ __launch_bounds__(64 * kH3Waves, kH3BlocksPerCU) void blend_skin_h3_kernel(
    const float* __restrict__ features, const float* __restrict__ transforms,
    const uint16_t* __restrict__ basis_h3, const float* __restrict__ trans,
    float* __restrict__ verts, int64_t n, int n_verts, int n_groups,
    float p_unscale, float t_unscale, int lp, unsigned shifts, int aligned) {
  constexpr int kSlot = kH3GroupPieces * 64;                // f16x8 per slot (32 KB)
  constexpr int kStores = (MANO_H3_ABLATE & 2) ? 0 : 4 * kH3TPW;  // global_store_dwordx3 per group
  constexpr int kTiles = kH3Waves * kH3TPW;                 // hand tiles per block unit
  __shared__ f16x8 ring[kH3Ring * kSlot];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  static_assert(kTiles == 8, "residue-class sets of 8 16-hand tiles (mano_layout.h, lq = 7)");
  const int vstride = 3 * n_verts;
  const int rstride = vstride << lp;  // floats between a tile's rows
  // Sector-aligned rows (mano_layout.h, as blend_skin16): a set holds the 128
  // hands of one residue class r, and the block uses basis variant s_r.
  const int64_t n_sets = aligned_n_quads(n, lp, 7);
  int64_t u, u_end;
  unit_range_h3(n_sets * n_groups, blockIdx.x, gridDim.x, u, u_end);

  while (u < u_end) {
    const int64_t set = u / n_groups;
    const int g0 = int(u - set * n_groups);
    const int g1 = int(n_groups - g0 < u_end - u ? n_groups : g0 + (u_end - u));
    u += g1 - g0;

    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));  // keep lane-derived addresses inside the range loop
    const int q = lane >> 4;
    const int col = lane & 15;

    // the set's tiles share one residue class, so one basis variant
    const int shift = aligned ? int((shifts >> (4 * aligned_tile(n, lp, set, wave * kH3TPW, 7, 4).cls)) & 15u) : 0;
    const uint16_t* bvar = basis_h3 + (aligned ? int64_t(shift) * n_groups * kH3GroupHalves : 0);
#pragma unroll
    for (int i = 0; i < kH3Ring - 1; ++i)
      if (g0 + i < g1) stage_group_h3(bvar, g0 + i, ring + i * kSlot, wave, lane);
    f16x8 xh[kH3TPW][kH3Steps], xl[kH3TPW][kH3Steps], F[kH3TPW][12];
    float tr[kH3TPW][4][3] = {};
    unsigned roff[kH3TPW][4];  // D rows (hands 4q + r) of each tile, clamped to the batch
    float* vtile[kH3TPW];
#pragma unroll
    for (int t = 0; t < kH3TPW; ++t) {
      const AlignedTile tile = aligned_tile(n, lp, set, wave * kH3TPW + t, 7, 4);
      // A tile past the batch end recomputes the set's last tile (identical
      // values).  The tile's rows are hands h0 + (i << lp), i <= rmax.
      const int64_t h0 = tile.h0;
      const int rmax = tile.n_valid - 1;  // last row of the tile in the batch
      load_x_h3(features + (h0 + (int64_t(min(col, rmax)) << lp)) * kXStride, q, xh[t], xl[t]);
      load_frames_h3(transforms, h0, lp, rmax, lane, F[t]);
      operand_fence(xh[t]);
      operand_fence(xl[t]);
      operand_fence(F[t]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hr = min(4 * q + r, rmax);
        roff[t][r] = unsigned(hr * rstride);
        if constexpr (kTrans) {
#pragma unroll
          for (int c = 0; c < 3; ++c) tr[t][r][c] = trans[(h0 + (int64_t(hr) << lp)) * 3 + c];
        }
      }
      vtile[t] = verts + h0 * int64_t(vstride);
    }
    // The first kH3Ring - 1 groups' pieces and every prologue load have landed.
    barrier_vmcnt<0>();

    for (int grp = g0, slot = 0; grp < g1; ++grp, slot = slot + 1 < kH3Ring ? slot + 1 : 0) {
      // group grp + kH3Ring - 1 into the slot group grp - 1 left (every wave
      // passed the barrier that ended group grp - 1)
      if (!(MANO_H3_ABLATE & 8) && grp + kH3Ring - 1 < g1) {
        if constexpr (MANO_H3_DMA_PRIO != 0) __builtin_amdgcn_s_setprio(MANO_H3_DMA_PRIO);
        const int ahead = slot + kH3Ring - 1 < kH3Ring ? slot + kH3Ring - 1 : slot - 1;
        stage_group_h3(bvar, grp + kH3Ring - 1, ring + ahead * kSlot, wave, lane);
        if constexpr (MANO_H3_DMA_PRIO != 0) __builtin_amdgcn_s_setprio(0);
      }
      const f16x8* L = ring + slot * kSlot + lane;
      f32x4 p[kH3TPW][3];
#if MANO_H3_SPLIT_ACC
      // Each K-step's two B fragments of a coordinate (lo and hi halves) are
      // read from LDS once and feed all three products: the small ones (hi.lo,
      // lo.hi) into one accumulator, hi.hi into a second, added at the end --
      // 30 fragment reads per group instead of 45.
      {
        f32x4 pb[kH3TPW][3];
        // MANO_H3_SPLIT_ACC 2: step s + 1's six fragments are read before
        // step s's MFMAs (pinned by scheduling barriers), so an MFMA waits on
        // a read issued a whole step earlier, not on the one just before it.
        f16x8 cur_lo[3], cur_hi[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          cur_lo[c] = L[((2 * c + 1) * kH3Steps) * 64];
          cur_hi[c] = L[((2 * c) * kH3Steps) * 64];
        }
#pragma unroll
        for (int s = 0; s < kH3Steps; ++s) {
          f16x8 nxt_lo[3], nxt_hi[3];
          if (MANO_H3_SPLIT_ACC >= 2 && s + 1 < kH3Steps) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              nxt_lo[c] = L[((2 * c + 1) * kH3Steps + s + 1) * 64];
              nxt_hi[c] = L[((2 * c) * kH3Steps + s + 1) * 64];
            }
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const f16x8 b_lo = MANO_H3_SPLIT_ACC >= 2 ? cur_lo[c] : L[((2 * c + 1) * kH3Steps + s) * 64];
            const f16x8 b_hi = MANO_H3_SPLIT_ACC >= 2 ? cur_hi[c] : L[((2 * c) * kH3Steps + s) * 64];
#pragma unroll
            for (int t = 0; t < kH3TPW; ++t) {
              if (s == 0) {
                mfma_init(p[t][c], xh[t][0], b_lo);
                mfma_init(pb[t][c], xh[t][0], b_hi);
              } else {
                mfma_acc(p[t][c], xh[t][s], b_lo);
                mfma_acc(pb[t][c], xh[t][s], b_hi);
              }
              mfma_acc(p[t][c], xl[t][s], b_hi);
            }
          }
          if (MANO_H3_SPLIT_ACC >= 2 && s + 1 < kH3Steps) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              cur_lo[c] = nxt_lo[c];
              cur_hi[c] = nxt_hi[c];
            }
          }
        }
#pragma unroll
        for (int t = 0; t < kH3TPW; ++t) {
          mfma_fence(p[t]);
          mfma_fence(pb[t]);
#pragma unroll
          for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) p[t][c][r] = no_pack(p[t][c][r] + pb[t][c][r]);
        }
      }
#else
      // The coordinates' (and tiles') chains interleaved (independent
      // accumulators), each summing hi.lo, lo.hi, then hi.hi over the 5 K-steps.
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const f16x8 b = L[((2 * c + 1) * kH3Steps) * 64];
#pragma unroll
        for (int t = 0; t < kH3TPW; ++t) mfma_init(p[t][c], xh[t][0], b);
      }
#pragma unroll
      for (int s = 1; s < kH3Steps; ++s)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const f16x8 b = L[((2 * c + 1) * kH3Steps + s) * 64];
#pragma unroll
          for (int t = 0; t < kH3TPW; ++t) mfma_acc(p[t][c], xh[t][s], b);
        }
#pragma unroll
      for (int s = 0; s < kH3Steps; ++s)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const f16x8 b = L[((2 * c) * kH3Steps + s) * 64];
#pragma unroll
          for (int t = 0; t < kH3TPW; ++t) mfma_acc(p[t][c], xl[t][s], b);
        }
#pragma unroll
      for (int s = 0; s < kH3Steps; ++s)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const f16x8 b = L[((2 * c) * kH3Steps + s) * 64];
#pragma unroll
          for (int t = 0; t < kH3TPW; ++t) mfma_acc(p[t][c], xh[t][s], b);
        }
#endif
      // the lane's vertex in this group (grp, shift uniform: scalar branches)
      int vx;
      if (aligned) {
        vx = aligned_group_vertex(n_verts, shift, grp, col);
      } else {
        vx = (grp * 16 < n_verts - 16 ? grp * 16 : n_verts - 16) + col;
      }
      const int voff = 3 * vx;
      const f16x8 w1 = L[kH3WPiece * 64];
      const f16x8 w2 = L[(kH3WPiece + 1) * 64];
#pragma unroll
      for (int t = 0; t < kH3TPW; ++t) {
        mfma_fence(p[t]);
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) p[t][c][r] = no_pack(p[t][c][r] * p_unscale);
        f32x4 out[3];
        if constexpr (MANO_H3_ABLATE & 4) {
          out[0] = p[t][0];
          out[1] = p[t][1];
          out[2] = p[t][2];
        } else {
          lbs_h3(F[t], w1, w2, p[t], t_unscale, tr[t], out);
        }
        if constexpr (MANO_H3_ABLATE & 2) {
          if (out[0][0] == 1234.5f && out[1][1] == 2345.5f) vtile[t][roff[t][0] + unsigned(voff)] = out[2][2];
          continue;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          store_out_h3(vtile[t] + (roff[t][r] + unsigned(voff)), f32x3{out[0][r], out[1][r], out[2][r]});
        }
      }
      // Group grp + 1 has landed in LDS (every wave's pieces) and every wave
      // is done reading this slot, which the next iteration re-stages.  The
      // ops younger than group grp + 1's DMA (issued kH3Ring - 2 iterations
      // ago, or in the prologue) are the kH3Ring - 1 groups' stores and the
      // DMAs of groups grp + 2 .. grp + kH3Ring - 1 that exist in the range.
      const int later_dmas = min(kH3Ring - 2, max(0, g1 - grp - 2));
      ring_barrier<(kH3Ring - 1) * kStores>(later_dmas);
    }
  }
}

// Standalone LBS, f16x3: the span streaming of mano_span.h with skin_h3's
// operands -- the tile's split transform fragments in VGPRs, each group's
// weight pieces from basis_h3 -- and lbs_h3 itself, so it agrees with
// blend_skin_h3's LBS bit for bit.
template <bool kTrans>
struct SpanLbsH3 {
  static constexpr bool kInPlace = false;
  struct W {
    f16x8 w1, w2;
  };
  struct Tile {
    f32x4 raw[24];
    float tr[4][3];
  };
  const float* transforms;
  const uint16_t* basis_h3;
  const float* trans;
  float t_unscale;
  int lane;
  f16x8 F[12];
  float tr[4][3];

  __device__ __forceinline__ W load_w(int grp, int ln) const {
    const f16x8* wg = reinterpret_cast<const f16x8*>(basis_h3) + int64_t(grp) * (kH3GroupPieces * 64) + ln;
    return W{wg[kH3WPiece * 64], wg[(kH3WPiece + 1) * 64]};
  }
  __device__ __forceinline__ void fetch_tile(int64_t h0, int64_t n, int n_valid, int ln, Tile& t) const {
    fetch_frames_h3(transforms, h0, n, ln, t.raw);
    const int row0 = 4 * (ln >> 4);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        t.tr[r][c] = kTrans ? trans[(h0 + min(row0 + r, n_valid - 1)) * 3 + c] : 0.f;
  }
  __device__ __forceinline__ void set_tile(const Tile& t) {
    split_frames_h3(t.raw, lane, F);
    operand_fence(F);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) tr[r][c] = t.tr[r][c];
  }
  __device__ __forceinline__ void apply(const W& w, const float (&p)[4][3], float (&o)[4][3]) const {
    f32x4 pk[3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) pk[c][r] = p[r][c];
    f32x4 out[3];
    lbs_h3(F, w.w1, w.w2, pk, t_unscale, tr, out);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) o[r][c] = out[c][r];
  }
};

#ifndef MANO_SPAN_H3_STRIDE
#define MANO_SPAN_H3_STRIDE false  // skin_span_h3: tile-major per-wave ranges (split operands built once per tile)
#endif
#ifndef MANO_SPAN_H3_PRIO
#define MANO_SPAN_H3_PRIO 0
#endif
template <bool kTrans>
__global__ __launch_bounds__(256, MANO_SPAN_H3_BLOCKS_PER_CU) void skin_span_h3_kernel(
    const float* __restrict__ transforms, const uint16_t* __restrict__ basis_h3,
    const float* __restrict__ vposed, const float* __restrict__ trans, float* __restrict__ verts,
    int64_t n, int n_verts, int n_groups, float t_unscale) {
  __shared__ f32x4 stage[4 * span::kStageFloats / 4];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SpanLbsH3<kTrans> lbs{transforms, basis_h3, trans, t_unscale, int(threadIdx.x & 63), {}, {}};
  span::run_units<MANO_SPAN_H3_STRIDE, MANO_SPAN_H3_PRIO, 1>(
      lbs, vposed, verts, n, n_verts, n_groups,
      MANO_SPAN_H3_STRIDE ? span::xcd_worker(wave) : int64_t(blockIdx.x) * 4 + wave,
                  int64_t(gridDim.x) * 4, reinterpret_cast<float*>(stage) + wave * span::kStageFloats,
                  int(threadIdx.x & 63));
}

constexpr int kBlendSkinH3BlocksPerCU = kH3BlocksPerCU;  // 64 KB of LDS per block
constexpr int kSkinH3BlocksPerCU = MANO_SPAN_H3_BLOCKS_PER_CU;
constexpr int64_t kMinUnitsPerWorkerH3 = 8;

template <class Kernel>
dim3 persistent_grid_h3(Kernel kernel, const DeviceModel& m, int64_t units, int workers_per_block,
                        int design_per_cu, int block_threads = 256) {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, block_threads, 0) != hipSuccess || b < 1) b = 1;
  if (b > design_per_cu) b = design_per_cu;
  const int64_t cap = int64_t(b) * (m.n_cu > 0 ? m.n_cu : 1);
  const int64_t want = (units + kMinUnitsPerWorkerH3 - 1) / kMinUnitsPerWorkerH3;
  const int64_t blocks_wanted = (want + workers_per_block - 1) / workers_per_block;
  return dim3{unsigned(blocks_wanted < cap ? blocks_wanted : cap)};
}

}  // namespace

hipError_t launch_blend_skin_h3(const DeviceModel& m, int64_t n, const float* features,
                                const float* transforms, const float* trans, float* verts,
                                hipStream_t stream) {
  // Sector-aligned rows as launch_blend_skin (mano_layout.h): verts phase
  // classes and the basis variant of each (MANO_H3_ALIGN 0: the plain layout).
  int lp = 0, aligned = 0;
  unsigned shifts = 0;
  const uint16_t* bh3 = m.basis_h3;
  if (MANO_H3_ALIGN && m.basis_h3v) {
    lp = aligned_period_log2(m.n_verts);
    shifts = aligned_shifts(m.n_verts, unsigned(reinterpret_cast<uintptr_t>(verts) >> 2) & 7u, lp);
    bh3 = m.basis_h3v;
    aligned = 1;
  }
  const int64_t units = aligned_n_quads(n, lp, 7) * m.n_groups16;
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, persistent_grid_h3(kernel, m, units, 1, kBlendSkinH3BlocksPerCU, 64 * kH3Waves),
                       dim3(64 * kH3Waves), 0, stream, features, transforms, bh3, trans, verts,
                       n, m.n_verts, m.n_groups16, m.h3_vposed_unscale, m.h3_lbs_unscale, lp, shifts, aligned);
  };
  if (trans) launch(blend_skin_h3_kernel<true>);
  else launch(blend_skin_h3_kernel<false>);
  return hipGetLastError();
}

hipError_t launch_skin_h3(const DeviceModel& m, int64_t n, const float* transforms,
                          const float* vposed, const float* trans, float* verts,
                          hipStream_t stream) {
#if MANO_H3_SKIN_PAIR
  // skin_pair's memory / compute waves with the f16x3 LBS (mano_skin_quad.hip)
  if (skin_quad_supported(m)) {
    const hipError_t e = launch_skin_quad(m, n, transforms, vposed, trans, verts, stream, true);
    if (e != hipErrorNotSupported) return e;  // not supported: a batch below one block
  }
#endif
  const int64_t units = (n + 15) / 16 * span::n_spans(m.n_verts);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, persistent_grid_h3(kernel, m, units, 4, kSkinH3BlocksPerCU), dim3(256),
                       0, stream, transforms, m.basis_h3, vposed, trans, verts, n, m.n_verts,
                       m.n_groups16, m.h3_lbs_unscale);
  };
  if (trans) launch(skin_span_h3_kernel<true>);
  else launch(skin_span_h3_kernel<false>);
  return hipGetLastError();
}

}  // namespace mano
