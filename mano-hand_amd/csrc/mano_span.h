// mano_span.h -- the span tiling of the standalone LBS kernels (skin_span in
// mano_kernels.hip, skin_span_h3 in mano_kernels_h3.hip): LBS
// (mano_np.py:112-115) over a v_posed buffer in HBM, streamed with whole-line
// float4 accesses.
//
// A wave's unit is (16-hand tile, span of 64 vertices): 16 hand rows x 768 B
// of v_posed.  The wave reads them as 12 float4 per lane in one flat
// row-major sweep (each 64-lane load is 1 KB of consecutive row segments),
// drops them into its own LDS stage, reads them back in the 16x16 MFMA D
// layout (lane (q, col): hands 4q + r, vertex 16 g + col; 4-B reads, which
// hit 32 distinct banks per half-wave with the 196-float row stride), skins
// them in registers, writes the results back in place and streams the stage
// out with the same flat float4 sweep.  The next unit's rows are loaded while
// the current one is skinned.
//
// Vertices past the last full span (n_verts % 64 of them) are the tail unit
// of each tile: its 16-vertex groups take the per-group path (point loads and
// stores straight from HBM, the last group shifted to end at n_verts).
#pragma once
#include "mano_internal.h"

namespace mano {
namespace span {

typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// A float4 at 4-B alignment: hand rows are 9,336 B apart, so every other row
// starts 8 B off a 16-B boundary (multi-dword global accesses need dword
// alignment only).
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));

#ifndef MANO_SPAN_VERTS
#define MANO_SPAN_VERTS 64
#endif
#ifndef MANO_SPAN_CHUNK
#define MANO_SPAN_CHUNK 1             // skin_span: consecutive units per grid-stride step
#endif
#ifndef MANO_SPAN_BLOCKS_PER_CU
#define MANO_SPAN_BLOCKS_PER_CU 2     // skin_span: <= 256 VGPRs, 2 waves per SIMD
#endif
#ifndef MANO_SPAN_H3_BLOCKS_PER_CU
#define MANO_SPAN_H3_BLOCKS_PER_CU 1  // skin_span_h3: the split operands need > 256 VGPRs
#endif
constexpr int kVerts = MANO_SPAN_VERTS;     // vertices per span
constexpr int kGroups = kVerts / 16;        // 16-vertex MFMA groups per span
constexpr int kRowF4 = 3 * kVerts / 4;      // float4 per hand row of a span (48)
constexpr int kStride = 3 * kVerts + 4;     // LDS row stride, floats (+16 B per row)
constexpr int kStageFloats = 16 * kStride;  // one wave's stage: 12,544 B
constexpr int kF4 = 16 * kRowF4 / 64;       // float4 per lane per unit (12)

// Units per 16-hand tile: the full spans, plus the tail unit if n_verts % 64.
__host__ __device__ constexpr int n_spans(int n_verts) {
  return n_verts / kVerts + (n_verts % kVerts ? 1 : 0);
}

// Compiler barrier between a wave's LDS hand-offs.  A wave's LDS accesses
// execute in issue order, so no wait is needed, only that hipcc keeps the
// program order of accesses whose data other lanes produced.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// (row, float4 column) of the lane's float4 i in the flat sweep of a tile.
__device__ __forceinline__ void sweep_slot(int i, int lane, int& row, int& c4) {
  const int idx = 64 * i + lane;
  row = idx / kRowF4;
  c4 = idx - kRowF4 * row;
}

// The 16 rows of a span, HBM -> registers (rows past the batch end re-read
// the tile's last hand).  MANO_SPAN_NT_LOAD: non-temporal (read-once) loads.
#ifndef MANO_SPAN_NT_LOAD
#define MANO_SPAN_NT_LOAD 0
#endif
__device__ __forceinline__ void load_rows(const float* __restrict__ tile, int vstride, int v0,
                                          int n_valid, int lane, f32x4u (&buf)[kF4]) {
#pragma unroll
  for (int i = 0; i < kF4; ++i) {
    int row, c4;
    sweep_slot(i, lane, row, c4);
    const unsigned off = unsigned(min(row, n_valid - 1) * vstride + 4 * c4);
    const f32x4u* src = reinterpret_cast<const f32x4u*>(tile + 3 * v0 + off);
    if constexpr (MANO_SPAN_NT_LOAD) buf[i] = __builtin_nontemporal_load(src);
    else buf[i] = *src;
  }
}

__device__ __forceinline__ void put_rows(float* stage, int lane, const f32x4u (&buf)[kF4]) {
#pragma unroll
  for (int i = 0; i < kF4; ++i) {
    int row, c4;
    sweep_slot(i, lane, row, c4);
    *reinterpret_cast<f32x4*>(stage + row * kStride + 4 * c4) = buf[i];
  }
}

// Stage -> HBM.  A row past the batch end holds the last hand's results and
// re-writes them (identical bits) to that hand's row.
#ifndef MANO_SPAN_ABLATE
#define MANO_SPAN_ABLATE 0  // diagnostic: 1 = tile operands / weights fetched once, 2 = no LBS, 4 = NT stores
#endif
__device__ __forceinline__ void store_rows(const float* stage, float* __restrict__ tile, int vstride,
                                           int v0, int n_valid, int lane) {
#pragma unroll
  for (int i = 0; i < kF4; ++i) {
    int row, c4;
    sweep_slot(i, lane, row, c4);
    const f32x4 v = *reinterpret_cast<const f32x4*>(stage + row * kStride + 4 * c4);
    const unsigned off = unsigned(min(row, n_valid - 1) * vstride + 4 * c4);
    if constexpr (MANO_SPAN_ABLATE & 4) __builtin_nontemporal_store(v, reinterpret_cast<f32x4u*>(tile + 3 * v0 + off));
    else *reinterpret_cast<f32x4u*>(tile + 3 * v0 + off) = v;
  }
}

// Diagnostic (MANO_SPAN_ABLATE & 8): registers -> HBM in the same sweep.
__device__ __forceinline__ void store_regs(const f32x4u (&buf)[kF4], float* __restrict__ tile, int vstride,
                                           int v0, int n_valid, int lane) {
#pragma unroll
  for (int i = 0; i < kF4; ++i) {
    int row, c4;
    sweep_slot(i, lane, row, c4);
    const unsigned off = unsigned(min(row, n_valid - 1) * vstride + 4 * c4);
    *reinterpret_cast<f32x4u*>(tile + 3 * v0 + off) = buf[i];
  }
}

// The lane's points of group g in the MFMA D layout: p[r] = vertex 16 g + col
// of hand row 4q + r.
__device__ __forceinline__ void read_points(const float* stage, int lane, int g, float (&p)[4][3]) {
  const float* s = stage + 4 * (lane >> 4) * kStride + 48 * g + 3 * (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) p[r][c] = s[r * kStride + c];
}

__device__ __forceinline__ void write_points(float* stage, int lane, int g, const float (&o)[4][3]) {
  float* s = stage + 4 * (lane >> 4) * kStride + 48 * g + 3 * (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) s[r * kStride + c] = o[r][c];
}

// Worker id of the calling wave for the grid-stride unit order: consecutive
// ids on one XCD (blocks are dispatched round-robin over the 8 XCDs, so block
// b runs on XCD b % 8 -- an assumption made for L2 locality only), so the
// spans of a tile, and their shared transforms, stay in one L2.
__device__ __forceinline__ int64_t xcd_worker(int wave) {
  const int64_t b = blockIdx.x, nb = gridDim.x;
  if (nb % 8) return b * 4 + wave;
  return ((b % 8) * (nb / 8) + b / 8) * 4 + wave;
}

// The unit loop of a skin_span kernel.  With kStride, worker w (one per
// wave) takes units w, w + n_workers, w + 2 n_workers, ...: at any moment the
// chip works on n_workers consecutive units, a compact window of v_posed and
// verts (this order measured 5.3 TB/s on a plain copy of the span pattern
// where contiguous per-wave ranges reached 3.1-4.0,
// tools/microbench/span_patterns), at the price of fetching the tile's LBS
// operands for every unit.  Without it, each wave runs a contiguous
// tile-major range and fetches them once per tile (the f16x3 operands are
// split in registers, which makes the per-unit fetch cost more than the
// locality gains).
// A unit's rows are loaded one unit ahead; its tile's LBS operands and its
// groups' weights are loaded at its start and made current BEFORE the next
// rows are prefetched (vmcnt retires in issue order: waiting for a load
// issued after the prefetch would wait for the prefetch too; and the f16x3
// operands are split in registers, which needs them landed), their latency
// covered by the other wave on the SIMD.  kPrio != 0 raises the wave's issue
// priority while it issues a unit's row loads and stores, so the HBM stream is
// not held behind the sibling wave's MFMAs (fp32 skin_span: 0.305 -> 0.297 ms
// at kPrio 3; the f16x3 kernel, one wave per SIMD, gains nothing).  Lbs supplies:
//   typename Lbs::W, Lbs::Tile          one group's weights, one tile's operands
//   W    load_w(int grp, int lane)
//   void fetch_tile(int64_t h0, int64_t n, int n_valid, int lane, Tile&)
//   void set_tile(const Tile&)           make them the current operands
//   Tile cur; static constexpr bool kInPlace  fetch_tile may write cur directly
//   void apply(const W&, const float (&p)[4][3], float (&o)[4][3])
template <bool kStride, int kPrio, int kChunk, class Lbs>
__device__ __forceinline__ void run_units(Lbs& lbs, const float* __restrict__ vposed,
                                          float* __restrict__ verts, int64_t n, int n_verts,
                                          int n_groups, int64_t worker, int64_t n_workers,
                                          float* stage, int lane) {
  const int vstride = 3 * n_verts;
  const int n_full = n_verts / kVerts;
  const int n_tail = n_groups - kGroups * n_full;  // 0..4 groups past the full spans
  const int spans = n_spans(n_verts);
  const int64_t units = (n + 15) / 16 * spans;
  const int row0 = 4 * (lane >> 4);
  const int col = lane & 15;
  auto rows_of = [&](int64_t t) {
    const int64_t left = n - 16 * t;
    return int(left < 16 ? left : 16);
  };
  // A tail unit's points ride in the row registers: group g, row r, coord c
  // at float 12 g + 3 r + c.
  auto tail_offset = [&](int n_valid, int g, int r) {
    const int vb = min(16 * (kGroups * n_full + g), n_verts - 16);
    return unsigned(min(row0 + r, n_valid - 1) * vstride + 3 * (vb + col));
  };
  f32x4u buf[kF4];
  auto fetch_rows = [&](int64_t uu) {
    if (uu >= units) return;
    const int64_t t = uu / spans;
    const int sp = int(uu - t * spans);
    const int n_valid = rows_of(t);
    const float* src = vposed + t * 16 * vstride;
    if (sp < n_full) {
      load_rows(src, vstride, kVerts * sp, n_valid, lane, buf);
    } else {
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        if (g < n_tail) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const f32x3 v = *reinterpret_cast<const f32x3*>(src + tail_offset(n_valid, g, r));
#pragma unroll
            for (int c = 0; c < 3; ++c) buf[(12 * g + 3 * r + c) >> 2][(12 * g + 3 * r + c) & 3] = v[c];
          }
        }
      }
    }
  };
  // kStride: units worker + k n_workers (operands fetched per unit);
  // otherwise the contiguous range [u_begin, u_end), tile-major (operands
  // fetched when the tile changes).
  // kStride with kChunk > 1: chunks of kChunk consecutive units in the
  // grid-stride order (the spans of a chunk mostly share a tile, whose
  // operands are then fetched once).
  const int64_t u_begin = kStride ? worker * kChunk : worker * units / n_workers;
  const int64_t u_end = kStride ? units : (worker + 1) * units / n_workers;
  auto next_unit = [&](int64_t uu) -> int64_t {
    if (!kStride || kChunk == 1) return uu + (kStride ? n_workers : 1);
    return (uu + 1) % kChunk ? uu + 1 : uu + 1 + (n_workers - 1) * kChunk;
  };
  int64_t cur_tile = -1;
  typename Lbs::W w_once[kGroups];
  if constexpr ((MANO_SPAN_ABLATE & 1) && Lbs::kInPlace) {
    lbs.fetch_tile(0, n, 16, lane, lbs.cur);
#pragma unroll
    for (int g = 0; g < kGroups; ++g) w_once[g] = lbs.load_w(g, lane);
  }
  fetch_rows(u_begin);
  for (int64_t uu = u_begin; uu < u_end; uu = next_unit(uu)) {
    const int64_t tile = uu / spans;
    const int s = int(uu - tile * spans);
    const int64_t h0 = tile * 16;
    const int n_valid = rows_of(tile);
    const bool full = s < n_full;
    const bool new_tile = (kStride && kChunk == 1) || tile != cur_tile;
    cur_tile = tile;
    // Lbs::kInPlace: the operands load straight into the current ones (the
    // previous unit's are dead here), so no second copy is live.
    typename Lbs::Tile tops;
    if (new_tile && !((MANO_SPAN_ABLATE & 1) && Lbs::kInPlace)) {
      if constexpr (Lbs::kInPlace) lbs.fetch_tile(h0, n, n_valid, lane, lbs.cur);
      else lbs.fetch_tile(h0, n, n_valid, lane, tops);
    }
    typename Lbs::W w[kGroups];
#pragma unroll
    for (int g = 0; g < kGroups; ++g)
      if constexpr ((MANO_SPAN_ABLATE & 1) && Lbs::kInPlace) w[g] = w_once[g];
      else if (full || g < n_tail) w[g] = lbs.load_w(kGroups * (full ? s : n_full) + g, lane);
    if constexpr ((MANO_SPAN_ABLATE & 8) && Lbs::kInPlace) {
      if (full) {  // plain copy of the unit's rows, no LDS, no LBS
        f32x4u cp[kF4];
#pragma unroll
        for (int i = 0; i < kF4; ++i) cp[i] = buf[i];
        if (next_unit(uu) < u_end) fetch_rows(next_unit(uu));
        store_regs(cp, verts + h0 * vstride, vstride, kVerts * s, n_valid, lane);
        continue;
      }
    }
    if (full) {
      put_rows(stage, lane, buf);
      if (!Lbs::kInPlace && new_tile) lbs.set_tile(tops);
      if constexpr (kPrio != 0) __builtin_amdgcn_s_setprio(kPrio);
      if (next_unit(uu) < u_end) fetch_rows(next_unit(uu));
      if constexpr (kPrio != 0) __builtin_amdgcn_s_setprio(0);
      wave_sync();
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        float p[4][3], o[4][3];
        read_points(stage, lane, g, p);
        if constexpr ((MANO_SPAN_ABLATE & 2) && Lbs::kInPlace) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) o[r][c] = p[r][c] + w[g][r];
        } else {
          lbs.apply(w[g], p, o);
        }
        write_points(stage, lane, g, o);
        __builtin_amdgcn_sched_barrier(0);  // one group's LBS temporaries live at a time
      }
      wave_sync();
      if constexpr (kPrio != 0) __builtin_amdgcn_s_setprio(kPrio);
      store_rows(stage, verts + h0 * vstride, vstride, kVerts * s, n_valid, lane);
      if constexpr (kPrio != 0) __builtin_amdgcn_s_setprio(0);
      wave_sync();
    } else {
      float p[kGroups][4][3];
#pragma unroll
      for (int g = 0; g < kGroups; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 3; ++c) p[g][r][c] = buf[(12 * g + 3 * r + c) >> 2][(12 * g + 3 * r + c) & 3];
      if (!Lbs::kInPlace && new_tile) lbs.set_tile(tops);
      if (next_unit(uu) < u_end) fetch_rows(next_unit(uu));
      float* dst = verts + h0 * vstride;
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        if (g < n_tail) {
          float o[4][3];
          lbs.apply(w[g], p[g], o);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            *reinterpret_cast<f32x3*>(dst + tail_offset(n_valid, g, r)) = f32x3{o[r][0], o[r][1], o[r][2]};
        }
      }
    }
  }
}

}  // namespace span
}  // namespace mano
