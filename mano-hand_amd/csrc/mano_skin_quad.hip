// mano_skin_quad.hip -- the standalone fp32 LBS (mano_np.py:112-115) over a
// v_posed buffer in HBM: verts = sum_j W[v][j] A_j [v_posed; 1] (+ trans).
//
// Layout of the work.  A wave's unit is 4 hands x one 64-vertex span: four
// 768-B row segments of v_posed (3 KB), read as 3 float4 per lane in one flat
// sweep and written back the same way.  Units go to the waves in grid-stride
// order (consecutive worker ids on one XCD), so the chip streams a compact,
// in-order window of v_posed and verts.  tools/microbench/span_rows.hip: such
// 3-KB units copy at 5.7 TB/s, where skin_span's 16-hand x 64-vertex units
// (12 KB) reach 5.0 -- the fewer bytes each wave holds in flight, the closer
// the stream gets to a flat copy.
//
// The transform blend is turned around from blend_skin16's: the MFMA D rows
// are the 48 (hand, c, k) entries of the unit's 4 hands (3 row tiles of 16),
// the columns the 16 vertices of a group,
//     T[(hh, c, k)][v] = sum_j A_{h0+hh, j}[c][k] W[v][j]   (3 tiles x 4 MFMAs),
// so lane (q, v) of tile tau holds the 4 k-entries of one (hand, coordinate)
// pair in its 4 accumulator registers and applies them itself:
//     out = T_3 + T_2 z + T_1 y + T_0 x (+ trans)   (fmaf, blend_skin16's order).
// Same 48 MFMAs per 16 x 16 (hand, vertex) block as blend_skin16's LBS, same
// B fragments (wfrag16), the same fmaf chains -- the results are bit-identical
// to the fused kernel's (tests/test_gpu_parity.py fused == unfused).
//
// Per block (one per CU, kQWaves waves): every group's W fragment resident in
// LDS (n_groups16 KB, loaded once), and per wave a stage of the unit's rows
// (row stride 196 floats) and its 4 hands' transforms.  The next unit's rows,
// transforms and translations are loaded into registers before the current
// unit is skinned.  Vertices past the last full span (n_verts % 64) form the
// tail unit of each hand quad: its 16-vertex groups (the last one shifted to
// end at n_verts, as the packed W fragments are) load and store their points
// straight from HBM.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mano_internal.h"

namespace mano {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x3 __attribute__((ext_vector_type(3)));
// Hand rows are 9,336 B apart, so half of them start 8 B off a 16-B boundary
// (multi-dword global accesses need dword alignment only).
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));

#ifndef MANO_QUAD_WAVES
#define MANO_QUAD_WAVES 8  // waves per block, one block per CU: 2 waves per SIMD
#endif
constexpr int kQWaves = MANO_QUAD_WAVES;
#ifndef MANO_QUAD_ABLATE
#define MANO_QUAD_ABLATE 0  // diagnostic builds only: 1 = no LBS
#endif
constexpr int kQHands = 4;
constexpr int kQVerts = 64;                                  // vertices per full span
constexpr int kQRowF4 = 3 * kQVerts / 4;                     // 48 float4 per row segment
constexpr int kQF4 = kQHands * kQRowF4 / 64;                 // 3 float4 per lane per unit
constexpr int kQStride = 3 * kQVerts + 4;                    // LDS row stride, floats
constexpr int kQTrF4PerHand = kTransformFloats / 4;          // 48
constexpr int kQTrF4 = kQHands * kQTrF4PerHand / 64;         // 3 float4 per lane
#ifndef MANO_QUAD_MAX_GROUPS
#define MANO_QUAD_MAX_GROUPS 56  // W resident in LDS: V <= 896 (16 waves' stages + 56 KB fit 160 KB)
#endif
constexpr int kQMaxGroups = MANO_QUAD_MAX_GROUPS;
static_assert(kQHands * kQRowF4 % 64 == 0 && kQHands * kQTrF4PerHand % 64 == 0, "whole sweeps");

struct QuadStage {
  float rows[kQHands * kQStride];         // the unit's v_posed rows, then its verts
  float tr[kQHands * kTransformFloats];   // the 4 hands' [16][3][4] transforms
  float trans[16];                        // the 4 hands' translations (12 used)
};

// c ? a : b on values (a select of array elements can become a select of
// their addresses, which sends the arrays to scratch).
__device__ __forceinline__ int pick(bool c, int a, int b) {
  const int m = -int(c);
  return (a & m) | (b & ~m);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// One (hand, coordinate) output of lane (q, v): the 4 MFMAs of its tile's
// transform blend over K = 16 joints, then the apply in blend_skin16's order.
__device__ __forceinline__ float lbs_quad(const float (&a)[4], const f32x4& wf, float x, float y,
                                          float z) {
  f32x4 T = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], wf[0], f32x4{}, 0, 0, 0);
  T = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], wf[1], T, 0, 0, 0);
  T = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], wf[2], T, 0, 0, 0);
  T = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], wf[3], T, 0, 0, 0);
  float o = T[3];
  o = fmaf(T[2], z, o);
  o = fmaf(T[1], y, o);
  o = fmaf(T[0], x, o);
  return o;
}

template <bool kTrans>
__global__ __launch_bounds__(64 * kQWaves, 1) void skin_quad_kernel(
    const float* __restrict__ transforms, const float* __restrict__ wfrag16,
    const float* __restrict__ vposed, const float* __restrict__ trans, float* __restrict__ verts,
    int64_t n, int n_verts, int n_groups) {
  __shared__ f32x4 w_lds[kQMaxGroups * 64];
  __shared__ QuadStage stages[kQWaves];
  for (int i = threadIdx.x; i < n_groups * 64; i += 64 * kQWaves)
    w_lds[i] = reinterpret_cast<const f32x4*>(wfrag16)[i];
  __syncthreads();

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  QuadStage& st = stages[wave];
  const int vstride = 3 * n_verts;
  const int n_full = n_verts / kQVerts;
  const int n_tail = n_groups - 4 * n_full;  // groups past the full spans (0..4)
  const int spans = n_full + (n_tail > 0 ? 1 : 0);
  const int64_t n_quads = (n + kQHands - 1) / kQHands;
  // Worker ids: consecutive on one XCD (blocks go round-robin over the 8
  // XCDs -- assumed for L2 locality only), so the spans of a hand quad, and
  // its transforms, stay in one L2.  Worker w takes units w, w + n_workers,
  // ... of the (quad, span) sequence, stepped without divisions.
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int64_t blk = (nb % 8) ? b : (b % 8) * (nb / 8) + b / 8;
  const int64_t worker = blk * kQWaves + wave, n_workers = nb * kQWaves;
  const int64_t step_q = n_workers / spans;
  const int step_s = int(n_workers - step_q * spans);
  auto advance = [&](int64_t& qd, int& s) {
    qd += step_q;
    s += step_s;
    if (s >= spans) {
      s -= spans;
      ++qd;
    }
  };

  // Lane roles.  Tile tau, lane (q, v): accumulator rows 4q..4q+3 are the
  // k = 0..3 entries of (hand hh[tau], coordinate cc[tau]); the A operand
  // of step s is row m = 16 tau + v, joint 4 s + q.
  const int q = lane >> 4, v = lane & 15;
  int hh[3], cc[3], a_off[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int m0 = 16 * t + 4 * q, m = 16 * t + v;
    hh[t] = m0 / 12;
    cc[t] = (m0 % 12) / 4;
    a_off[t] = (m / 12) * kTransformFloats + 12 * q + m % 12;
  }
  // Row-segment sweeps: a full span is 48 float4 per row, the tail segment
  // (vertices tail_v0 .. n_verts) 3 * tail_len / 4; sweep slot i of the lane
  // is float4 idx = 64 i + lane of the unit's rows, clamped to the last one,
  // so every unit issues the same 3 loads and 3 stores (duplicates rewrite
  // identical bits) and hipcc's wait counts see no conditional memory op.
  // Per slot: the row, the float offset in the row segment and in the stage.
  const int tail_v0 = min(kQVerts * n_full, n_verts - 16);
  const int tail_rf4 = 3 * (n_verts - tail_v0) / 4;
  // (separate full / tail arrays: a runtime-indexed [2][] array goes to scratch)
  int frow[kQF4], fcol[kQF4], fst[kQF4], trow[kQF4], tcol4[kQF4], tst[kQF4];
#pragma unroll
  for (int i = 0; i < kQF4; ++i) {
    const int idx = 64 * i + lane;
    frow[i] = idx / kQRowF4;
    fcol[i] = 4 * (idx % kQRowF4);
    fst[i] = frow[i] * kQStride + fcol[i];
    const int it = min(idx, kQHands * tail_rf4 - 1);
    trow[i] = it / tail_rf4;
    tcol4[i] = 4 * (it % tail_rf4);
    tst[i] = trow[i] * kQStride + tcol4[i];
  }
  int thand[kQTrF4], tcol[kQTrF4];  // transforms sweep: hand, float4 within the hand
#pragma unroll
  for (int i = 0; i < kQTrF4; ++i) {
    thand[i] = (64 * i + lane) / kQTrF4PerHand;
    tcol[i] = (64 * i + lane) % kQTrF4PerHand;
  }
  const int trh = min(lane, 11) / 3, trc = min(lane, 11) % 3;

  f32x4u rb[kQF4];
  f32x4 tb[kQTrF4];
  float trb = 0.f;
  auto fetch = [&](int64_t qd, int s) {
    const int64_t h0 = qd * kQHands;
    const int last = int(n - h0 < kQHands ? n - h0 : kQHands) - 1;  // hands past it re-read it
    const bool full = s < n_full;
    const f32x4* T = reinterpret_cast<const f32x4*>(transforms + h0 * kTransformFloats);
#pragma unroll
    for (int i = 0; i < kQTrF4; ++i) tb[i] = T[unsigned(min(thand[i], last) * kQTrF4PerHand + tcol[i])];
    if constexpr (kTrans) trb = trans[h0 * 3 + unsigned(min(trh, last) * 3 + trc)];
    const float* src = vposed + h0 * vstride + 3 * (full ? kQVerts * s : tail_v0);
    unsigned off[kQF4];
    if (full) {
#pragma unroll
      for (int i = 0; i < kQF4; ++i) off[i] = unsigned(min(frow[i], last) * vstride + fcol[i]);
    } else {
#pragma unroll
      for (int i = 0; i < kQF4; ++i) off[i] = unsigned(min(trow[i], last) * vstride + tcol4[i]);
    }
#pragma unroll
    for (int i = 0; i < kQF4; ++i) rb[i] = *reinterpret_cast<const f32x4u*>(src + off[i]);
  };
  auto stage_unit = [&](int s) {
    const bool full = s < n_full;
#pragma unroll
    for (int i = 0; i < kQTrF4; ++i) reinterpret_cast<f32x4*>(st.tr)[64 * i + lane] = tb[i];
    if constexpr (kTrans) {
      if (lane < 12) st.trans[lane] = trb;
    }
    int so[kQF4];
    if (full) {
#pragma unroll
      for (int i = 0; i < kQF4; ++i) so[i] = fst[i];
    } else {
#pragma unroll
      for (int i = 0; i < kQF4; ++i) so[i] = tst[i];
    }
#pragma unroll
    for (int i = 0; i < kQF4; ++i) *reinterpret_cast<f32x4*>(st.rows + so[i]) = rb[i];
  };
  // One group's LBS: points from the stage, outputs back in place (every
  // lane's points are read -- in-order LDS -- before any output lands).
  auto skin_group = [&](const float (&a)[3][4], const float (&tr3)[3], int wgrp, int lv) {
    const f32x4 wf = w_lds[wgrp * 64 + lane];
    float p[3][3], o[3];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int c = 0; c < 3; ++c) p[t][c] = st.rows[hh[t] * kQStride + 3 * (lv + v) + c];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      o[t] = lbs_quad(a[t], wf, p[t][0], p[t][1], p[t][2]);
      if constexpr (kTrans) o[t] = o[t] + tr3[t];
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) st.rows[hh[t] * kQStride + 3 * (lv + v) + cc[t]] = o[t];
    __builtin_amdgcn_sched_barrier(0);
  };

  // Unit (qd, s): its operands and rows go registers -> LDS stage, the next
  // unit is fetched, the unit is skinned and stored.  The next unit's stage
  // hand-off sits after this unit's stores, so its wait (vmcnt(3): all but
  // the 3 stores) never waits for them.
  int64_t qd = worker / spans;
  int s = int(worker - qd * spans);
  int64_t qn = qd;
  int sn = s;
  advance(qn, sn);
  if (qd < n_quads) {
    fetch(qd, s);
    stage_unit(s);
    if (qn < n_quads) fetch(qn, sn);
  }
  while (qd < n_quads) {
    const int64_t h0 = qd * kQHands;
    const int last = int(n - h0 < kQHands ? n - h0 : kQHands) - 1;
    const bool full = s < n_full;
    const int v0 = full ? kQVerts * s : tail_v0;  // first vertex of the unit's segment
    wave_sync();
    float a[3][4], tr3[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
#pragma unroll
      for (int k = 0; k < 4; ++k) a[t][k] = st.tr[a_off[t] + 4 * 12 * k];
      tr3[t] = kTrans ? st.trans[3 * hh[t] + cc[t]] : 0.f;
    }
    if (MANO_QUAD_ABLATE & 1) {
      // diagnostic: no LBS (the stage streams out unchanged)
    } else if (full) {
      // The unit's 4 groups at once: 12 independent 4-MFMA chains issued
      // step-major (no chain waits on its own previous MFMA), every point
      // and W fragment read up front -- one wave per SIMD has the registers,
      // and its compute per unit must stay under the row stream's latency.
      f32x4 wf[4];
      float p[4][3][3];
#pragma unroll
      for (int g = 0; g < 4; ++g) wf[g] = w_lds[(4 * s + g) * 64 + lane];
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int c = 0; c < 3; ++c) p[g][t][c] = st.rows[hh[t] * kQStride + 48 * g + 3 * v + c];
      f32x4 T[4][3];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int t = 0; t < 3; ++t)
            T[g][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][k], wf[g][k], k == 0 ? f32x4{} : T[g][t], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          float o = T[g][t][3];
          o = fmaf(T[g][t][2], p[g][t][2], o);
          o = fmaf(T[g][t][1], p[g][t][1], o);
          o = fmaf(T[g][t][0], p[g][t][0], o);
          if constexpr (kTrans) o = o + tr3[t];
          st.rows[hh[t] * kQStride + 48 * g + 3 * v + cc[t]] = o;
        }
    } else {
      // the tail's groups, at the packed W fragments' placement (the mesh's
      // last group shifted to end at n_verts)
      for (int g = 0; g < n_tail; ++g)
        skin_group(a, tr3, 4 * n_full + g, min(16 * (4 * n_full + g), n_verts - 16) - tail_v0);
    }
    wave_sync();
    float* dst = verts + h0 * vstride + 3 * v0;
    int so[kQF4];
    unsigned go[kQF4];
    if (full) {
#pragma unroll
      for (int i = 0; i < kQF4; ++i) {
        so[i] = fst[i];
        go[i] = unsigned(min(frow[i], last) * vstride + fcol[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < kQF4; ++i) {
        so[i] = tst[i];
        go[i] = unsigned(min(trow[i], last) * vstride + tcol4[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < kQF4; ++i)
      *reinterpret_cast<f32x4u*>(dst + go[i]) = *reinterpret_cast<const f32x4*>(st.rows + so[i]);
    wave_sync();  // the stage reads are issued before the next unit's writes
    qd = qn;
    s = sn;
    if (qd < n_quads) {
      advance(qn, sn);
      stage_unit(s);
      if (qn < n_quads) fetch(qn, sn);
    }
  }
}


// ---------------------------------------------------------------------------
// skin_quad_direct (MANO_QUAD_DIRECT): the same units and transposed blend,
// but each lane loads exactly what it uses straight into registers -- per
// group and tile the 12-B point of its (hand, vertex) (a wave's load covers
// the 192-B row segments of 1-2 hands; the lanes of one vertex's three
// coordinates read the same 12 B), its 12 A-operand words and its
// translation word -- and stores its one output word per group and tile.  No
// LDS staging: the next unit's loads are issued before this unit's MFMAs
// (ping-pong register sets), every unit issues the same loads and stores
// (tail groups and hands past the batch end are clamped duplicates that
// rewrite identical bits), so hipcc's wait before a unit's MFMAs leaves the
// previous unit's stores and the next unit's loads in flight.
// ---------------------------------------------------------------------------
#ifndef MANO_QUAD_DIRECT
#define MANO_QUAD_DIRECT 0
#endif
#ifndef MANO_QUAD_DIRECT_WAVES
#define MANO_QUAD_DIRECT_WAVES 4  // one wave per SIMD
#endif
constexpr int kQdWaves = MANO_QUAD_DIRECT_WAVES;

struct QuadRegs {
  f32x3 p[4][3];  // point of (hand hh[t], vertex vb_g + v)
  float a[3][4];  // A operand of step k: transforms of row 16 t + v, joint 4 k + q
  float tr[3];    // translation of (hand hh[t], coordinate cc[t])
};

template <bool kTrans>
__global__ __launch_bounds__(64 * kQdWaves, 1) void skin_quad_direct_kernel(
    const float* __restrict__ transforms, const float* __restrict__ wfrag16,
    const float* __restrict__ vposed, const float* __restrict__ trans, float* __restrict__ verts,
    int64_t n, int n_verts, int n_groups) {
  __shared__ f32x4 w_lds[kQMaxGroups * 64];
  for (int i = threadIdx.x; i < n_groups * 64; i += 64 * kQdWaves)
    w_lds[i] = reinterpret_cast<const f32x4*>(wfrag16)[i];
  __syncthreads();

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int vstride = 3 * n_verts;
  const int n_full = n_verts / kQVerts;
  const int n_tail = n_groups - 4 * n_full;
  const int spans = n_full + (n_tail > 0 ? 1 : 0);
  const int64_t n_quads = (n + kQHands - 1) / kQHands;
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int64_t blk = (nb % 8) ? b : (b % 8) * (nb / 8) + b / 8;
  const int64_t worker = blk * kQdWaves + wave, n_workers = nb * kQdWaves;
  const int64_t step_q = n_workers / spans;
  const int step_s = int(n_workers - step_q * spans);

  const int q = lane >> 4, v = lane & 15;
  int hh[3], cc[3], ah[3], aoff[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int m0 = 16 * t + 4 * q, m = 16 * t + v;
    hh[t] = m0 / 12;
    cc[t] = (m0 % 12) / 4;
    ah[t] = m / 12;
    aoff[t] = 12 * q + m % 12;
  }
  auto group_of = [&](int s, int g) { return s < n_full ? 4 * s + g : 4 * n_full + min(g, n_tail - 1); };
  auto vbase_of = [&](int G) { return min(16 * G, n_verts - 16); };

  // Buffer resources per unit (SGPR base = the quad's first row), per-lane
  // 32-bit voffsets, per-group soffsets: the addressing costs a few scalar
  // ops and one VALU op per tile, not 64-bit VALU address math per load.
  constexpr int kRsrcFlags = 0x00020000;  // gfx9 raw buffer, 32-bit dwords
  auto rsrc = [&](const float* base, int64_t floats) {
    const int64_t bytes = floats * 4;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0,
                                             int(bytes < 0x7fffffff ? bytes : 0x7fffffff), kRsrcFlags);
  };
  auto fetch = [&](int64_t qd, int s, QuadRegs& r) {
    const int64_t h0 = qd * kQHands;
    const int last = int(n - h0 < kQHands ? n - h0 : kQHands) - 1;
    const auto rv = rsrc(vposed + h0 * vstride, int64_t(last + 1) * vstride);
    const auto rt = rsrc(transforms + h0 * kTransformFloats, int64_t(last + 1) * kTransformFloats);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int voff = 4 * (min(hh[t], last) * vstride + 3 * v);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        r.p[g][t] = __builtin_bit_cast(f32x3, __builtin_amdgcn_raw_buffer_load_b96(
                                                  rv, voff, 12 * vbase_of(group_of(s, g)), 0));
      const int aofs = 4 * (min(ah[t], last) * kTransformFloats + aoff[t]);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        r.a[t][k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rt, aofs, 4 * 48 * k, 0));
      if constexpr (kTrans) {
        const auto rr = rsrc(trans + h0 * 3, int64_t(last + 1) * 3);
        r.tr[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, 4 * (min(hh[t], last) * 3 + cc[t]), 0, 0));
      }
    }
  };

  // The stored words and their voffsets stay live until after the next
  // fetch (keep_live), so the next unit's loads never land in a register a
  // store still reads (hipcc would wait for that store first).
  float out[12];
  int out_off[3];
  auto keep_live = [&] {
#pragma unroll
    for (int i = 0; i < 12; ++i) asm volatile("" ::"v"(out[i]));
#pragma unroll
    for (int i = 0; i < 3; ++i) asm volatile("" ::"v"(out_off[i]));
  };
  auto compute = [&](int64_t qd, int s, const QuadRegs& r) {
    const int64_t h0 = qd * kQHands;
    const int last = int(n - h0 < kQHands ? n - h0 : kQHands) - 1;
    const auto ro = rsrc(verts + h0 * vstride, int64_t(last + 1) * vstride);
    f32x4 wf[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) wf[g] = w_lds[group_of(s, g) * 64 + lane];
    f32x4 T[4][3];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 3; ++t)
          T[g][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(r.a[t][k], wf[g][k], k == 0 ? f32x4{} : T[g][t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      out_off[t] = 4 * (min(hh[t], last) * vstride + 3 * v + cc[t]);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float o = T[g][t][3];
        o = fmaf(T[g][t][2], r.p[g][t][2], o);
        o = fmaf(T[g][t][1], r.p[g][t][1], o);
        o = fmaf(T[g][t][0], r.p[g][t][0], o);
        if constexpr (kTrans) o = o + r.tr[t];
        out[4 * t + g] = o;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), ro, out_off[t],
                                              12 * vbase_of(group_of(s, g)), 0);
      }
    }
  };

  auto advance = [&](int64_t& aq, int& as) {
    aq += step_q;
    as += step_s;
    if (as >= spans) {
      as -= spans;
      ++aq;
    }
  };
  // Program order of the memory operations, kept by the IR passes (memory
  // clobber) and the machine scheduler (sched_barrier).
  auto order_point = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  int64_t qd = worker / spans;
  int s = int(worker - qd * spans);
  if (qd >= n_quads) return;
  // Ping-pong register sets; the next unit's fetch is unconditional (past the
  // end it re-fetches the current unit), so every step issues the same loads.
  QuadRegs ra, rb;
#pragma unroll
  for (int i = 0; i < 12; ++i) out[i] = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) out_off[i] = 0;
  fetch(qd, s, ra);
  for (;;) {
    int64_t q1 = qd;
    int s1 = s;
    advance(q1, s1);
    const bool more1 = q1 < n_quads;
    fetch(more1 ? q1 : qd, more1 ? s1 : s, rb);
    keep_live();
    order_point();  // the next unit's loads go out before this unit's MFMAs
    compute(qd, s, ra);
    order_point();
    if (!more1) break;
    qd = q1;
    s = s1;
    advance(q1, s1);
    const bool more2 = q1 < n_quads;
    fetch(more2 ? q1 : qd, more2 ? s1 : s, ra);
    keep_live();
    order_point();
    compute(qd, s, rb);
    order_point();
    if (!more2) break;
    qd = q1;
    s = s1;
  }
}

}  // namespace

bool skin_quad_supported(const DeviceModel& m) {
  // the tail segment must be whole float4 per row
  const int tail_v0 = std::min(kQVerts * (m.n_verts / kQVerts), m.n_verts - 16);
  return m.n_verts >= 16 && m.n_groups16 <= kQMaxGroups && (3 * (m.n_verts - tail_v0)) % 4 == 0;
}

hipError_t launch_skin_quad(const DeviceModel& m, int64_t n, const float* transforms,
                            const float* vposed, const float* trans, float* verts,
                            hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int spans = m.n_verts / kQVerts + (m.n_verts % kQVerts ? 1 : 0);
  const int64_t units = (n + kQHands - 1) / kQHands * spans;
  int64_t blocks = (units + kQWaves - 1) / kQWaves;
  const int64_t cap = m.n_cu > 0 ? m.n_cu : 1;
  if (blocks > cap) blocks = cap;
#if MANO_QUAD_DIRECT
  blocks = std::min<int64_t>((units + kQdWaves - 1) / kQdWaves, cap);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, dim3(unsigned(blocks)), dim3(64 * kQdWaves), 0, stream, transforms,
                       m.wfrag16, vposed, trans, verts, n, m.n_verts, m.n_groups16);
  };
  if (trans) launch(skin_quad_direct_kernel<true>);
  else launch(skin_quad_direct_kernel<false>);
  return hipGetLastError();
#else
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, dim3(unsigned(blocks)), dim3(64 * kQWaves), 0, stream, transforms,
                       m.wfrag16, vposed, trans, verts, n, m.n_verts, m.n_groups16);
  };
  if (trans) launch(skin_quad_kernel<true>);
  else launch(skin_quad_kernel<false>);
  return hipGetLastError();
#endif
}

}  // namespace mano
