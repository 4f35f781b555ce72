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
// Two kernels share these units and this arithmetic:
//   skin_pair_kernel (default): per SIMD one memory wave (v_posed rows and
//     the 4 hands' transforms LDS-DMA'd into a stage slot; skinned slot ->
//     verts) and two compute waves (slot -> MFMA -> slot, alternate units),
//     four slots per memory wave handed over through LDS counters -- the HBM
//     stream runs at one streaming wave per SIMD, the span_rows optimum,
//     with the MFMA work beside it.  0.252-0.258 ms at 65,536 hands (trans),
//     61-63 % of 8 TB/s (tools/debug/time_skin.py).
//   skin_quad_kernel (MANO_QUAD_PAIR=0): every wave does both roles for its
//     own units, 2 waves per SIMD: 0.286-0.291 ms.
// Per block (one per CU): every group's W fragment resident in LDS (n_groups16
// KB, loaded once) and per unit a stage of its rows (row stride 196 floats)
// and its 4 hands' transforms.  Vertices past the last full span
// (n_verts % 64) form the tail unit of each hand quad: its segment starts at
// min(64 n_full, n_verts - 16) and its 16-vertex groups sit where the packed
// W fragments put them (the mesh's last group shifted to end at n_verts).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>

#include "../../include/mano_hip.h"
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
#ifndef MANO_QUAD_P_EARLY
#define MANO_QUAD_P_EARLY 1  // issue a unit's point reads before its transform-blend MFMAs
#endif
#ifndef MANO_QUAD_GROUP_MAJOR
#define MANO_QUAD_GROUP_MAJOR 1  // transform-blend MFMAs and apply group by group (fewer live registers)
#endif
#ifndef MANO_QUAD_ABLATE
#define MANO_QUAD_ABLATE 0  // diagnostic builds only: 1 = no LBS (skin_quad), 2 = no compute (skin_pair), 4 = no transform DMA (skin_pair)
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

template <int kStride>
struct StageT {
  static constexpr int kRowStride = kStride;
  float rows[kQHands * kStride];          // the unit's v_posed rows, then its verts
  float tr[kQHands * kTransformFloats];   // the 4 hands' [16][3][4] transforms
  float trans[16];                        // the 4 hands' translations (12 used)
};
using QuadStage = StageT<kQStride>;

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

// NG groups (G[0..NG)): the full units and a 1-group tail skip the
// duplicates a multi-group tail needs.
template <bool kTrans, int NG = 4, class Stage = QuadStage>
__device__ __forceinline__ void skin_unit4_w(Stage& st, const f32x4 (&wf)[4], const float (&a)[3][4],
                                             const float (&tr3)[3], const int (&lv)[4], const int (&hh)[3],
                                             const int (&cc)[3], int v) {
  float p[NG][3][3];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int c = 0; c < 3; ++c) p[g][t][c] = st.rows[hh[t] * Stage::kRowStride + 3 * (lv[g] + v) + c];
#if MANO_QUAD_P_EARLY
  // The point reads issue before the MFMAs and land behind them (hipcc would
  // sink them below the MFMAs to save registers, exposing their latency).
  __builtin_amdgcn_sched_barrier(0);
#endif
#if MANO_QUAD_GROUP_MAJOR
  // Group by group: its 3 chains of 4 MFMAs, then its apply -- 12 transform
  // registers live instead of 48 (3 independent chains keep the f32 MFMA pipe
  // full; the apply's VALU shares that datapath, so nothing overlaps anyway).
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    f32x4 T[3];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        T[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][k], wf[g][k], k == 0 ? f32x4{} : T[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float o = T[t][3];
      o = fmaf(T[t][2], p[g][t][2], o);
      o = fmaf(T[t][1], p[g][t][1], o);
      o = fmaf(T[t][0], p[g][t][0], o);
      if constexpr (kTrans) o = o + tr3[t];
      st.rows[hh[t] * Stage::kRowStride + 3 * (lv[g] + v) + cc[t]] = o;
    }
  }
#else
  f32x4 T[NG][3];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        T[g][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][k], wf[g][k], k == 0 ? f32x4{} : T[g][t], 0, 0, 0);
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float o = T[g][t][3];
      o = fmaf(T[g][t][2], p[g][t][2], o);
      o = fmaf(T[g][t][1], p[g][t][1], o);
      o = fmaf(T[g][t][0], p[g][t][0], o);
      if constexpr (kTrans) o = o + tr3[t];
      st.rows[hh[t] * Stage::kRowStride + 3 * (lv[g] + v) + cc[t]] = o;
    }
#endif
}

// skin_unit4_w with the groups' W fragments read from the block's LDS copy.
template <bool kTrans, int NG = 4, class Stage = QuadStage>
__device__ __forceinline__ void skin_unit4(Stage& st, const f32x4* w_lds, const float (&a)[3][4],
                                           const float (&tr3)[3], const int (&G)[4], const int (&lv)[4],
                                           const int (&hh)[3], const int (&cc)[3], int v, int lane) {
  f32x4 wf[4];
#pragma unroll
  for (int g = 0; g < NG; ++g) wf[g] = w_lds[G[g] * 64 + lane];
  skin_unit4_w<kTrans, NG, Stage>(st, wf, a, tr3, lv, hh, cc, v);
}

// The f16x3 precision mode (mano_kernels_h3.hip) on the same units: the
// transform blend T[(hand, c, k)][v] = sum_j A_j[c][k] W[v][j] as two
// v_mfma_f32_16x16x32_f16 per tile with every operand split into halves --
// A = [Ah | Al] (x 2^kH3FrameExp, hi in lanes 0-31, lo in 32-63), W pieces
// w1 = [Wh ; Wh], w2 = [Wl ; 0] (x 2^kH3WeightExp): T = A.w2 then += A.w1,
// blend_skin_h3's products in its order -- then its apply:
// out = fma(T3 + T2 z + T1 y + T0 x, 2^-(kH3FrameExp + kH3WeightExp), trans).
// wl: per group 64 x 16 B, entries 0-31 = w1's lanes 0-31 (lanes 32-63 are
// the same), 32-63 = w2's lanes 0-31 (lanes 32-63 are zero).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <bool kTrans, int NG = 4, class Stage = QuadStage>
__device__ __forceinline__ void skin_unit4_h3(Stage& st, const f16x8* wl, const f16x8 (&a)[3],
                                              const float (&tr3)[3], const int (&G)[4], const int (&lv)[4],
                                              const int (&hh)[3], const int (&cc)[3], int v, int lane,
                                              float t_unscale) {
  float p[NG][3][3];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int c = 0; c < 3; ++c) p[g][t][c] = st.rows[hh[t] * Stage::kRowStride + 3 * (lv[g] + v) + c];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const f16x8 w1 = wl[G[g] * 64 + (lane & 31)];
    const f16x8 w2l = wl[G[g] * 64 + 32 + (lane & 31)];
    const f16x8 w2 = lane < 32 ? w2l : f16x8{};
    f32x4 T[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) T[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], w2, f32x4{}, 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 3; ++t) T[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], w1, T[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float o = T[t][3];
      o = fmaf(T[t][2], p[g][t][2], o);
      o = fmaf(T[t][1], p[g][t][1], o);
      o = fmaf(T[t][0], p[g][t][0], o);
      st.rows[hh[t] * Stage::kRowStride + 3 * (lv[g] + v) + cc[t]] = fmaf(o, t_unscale, kTrans ? tr3[t] : 0.f);
    }
  }
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
    if (!(MANO_QUAD_ABLATE & 1)) {  // diagnostic 1: no LBS (the stage streams out unchanged)
      if (full) {
        const int G[4] = {4 * s, 4 * s + 1, 4 * s + 2, 4 * s + 3};
        const int lv[4] = {0, 16, 32, 48};
        skin_unit4<kTrans>(st, w_lds, a, tr3, G, lv, hh, cc, v, lane);
      } else {
        int G[4], lv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          G[g] = 4 * n_full + min(g, n_tail - 1);
          lv[g] = min(16 * G[g], n_verts - 16) - tail_v0;
        }
        if (n_tail == 1) skin_unit4<kTrans, 1>(st, w_lds, a, tr3, G, lv, hh, cc, v, lane);
        else skin_unit4<kTrans>(st, w_lds, a, tr3, G, lv, hh, cc, v, lane);
      }
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
// skin_pair_kernel: skin_quad's units with the roles split per SIMD.  Memory
// wave w (0..3), step k: once unit k's DMA into slot k % kPairSlots has
// landed it signals full = k + 1, then stores unit k - kPairCompute once that
// slot's done counter says it is skinned, then DMAs unit k + 2 into the slot
// just read out; compute wave c of pair w (wave 4 + 4c + w, same SIMD) skins
// units c, c + kPairCompute, ... in place and sets the slot's done counter.
// Staging unit k BEFORE waiting for unit k - 2 gives each unit two memory
// steps of compute (the poll stamps).  Measured (65,536
// hands, trans): 0.252-0.258 ms; register staging instead of LDS-DMA 0.262;
// the wait before the stage 0.275; one compute wave per memory wave
// 0.335-0.374; the memory waves alone (no LBS) 0.241-0.265.
// ---------------------------------------------------------------------------
#ifndef MANO_QUAD_PAIR
#define MANO_QUAD_PAIR 1  // the default standalone LBS; 0 = skin_quad_kernel
#endif
#ifndef MANO_QUAD_PAIR_COMPUTE
#define MANO_QUAD_PAIR_COMPUTE 2  // compute waves per memory wave (same SIMD)
#endif
// memory waves 0..3, compute waves 4..; wave w runs on SIMD w % 4
#ifndef MANO_QUAD_PAIR_PRIO
#define MANO_QUAD_PAIR_PRIO 0  // issue priority of the memory waves
#endif
constexpr int kPairs = 4;
constexpr int kPairCompute = MANO_QUAD_PAIR_COMPUTE;
#ifndef MANO_PAIR_SLOTS
#define MANO_PAIR_SLOTS 4  // stage slots per memory wave (LDS-DMA path: units k + 1 .. k + SLOTS - 2 in flight)
#endif
constexpr int kPairSlots = MANO_PAIR_SLOTS;

constexpr int kPairWaves = kPairs * (1 + kPairCompute);
// Hand quads in reverse order: the unfused path's blend GEMM writes v_posed
// in hand order, so its last ~256 MB are still dirty in the Infinity Cache
// when the LBS starts; taken last-first, those rows are read (and their
// lines retired) before the stream pushes them out to HBM.
#ifndef MANO_PAIR_REVERSE
#define MANO_PAIR_REVERSE 0
#endif
constexpr bool kPairReverse = MANO_PAIR_REVERSE;
constexpr int kPairMaxGroups = 52;  // W in LDS beside the slots: V <= 832
// (Rows packed at 192 floats, DMA'd as 3 full-wave instructions per unit
// instead of 4 three-quarter-wave ones: measured no faster, commit 05d3853,
// profiles/r03n_ab_skin_packed.jsonl.)
using PairStage = QuadStage;
constexpr int kPStride = PairStage::kRowStride;
constexpr int kPairRowDmas = kQHands;

struct PairShared {
  PairStage slot[kPairs][kPairSlots];
  int full[kPairs];               // units staged
  int done[kPairs][kPairSlots];   // per slot: 1 + the last unit skinned in it
};

// The hand-over counters are read and written with inline ds_read/ds_write:
// a volatile C++ access would make hipcc wait for every outstanding memory
// operation (vmcnt(0)) -- the memory wave's loads and stores in flight.
__device__ __forceinline__ unsigned lds_addr(const int* p) {
  typedef const __attribute__((address_space(3))) int* lds_ptr;
  return unsigned(reinterpret_cast<uintptr_t>((lds_ptr)p));  // generic -> LDS address (32 bit)
}
// Bounded: false after kPairPollLimit polls (2^20: tens of ms), and the
// caller then stops -- a lost hand-over never hangs the kernel (every wave
// reaches its exit); it raises MANO_DEVICE_SKIN_HANDOFF_TIMEOUT among the
// model's status flags, and the memory wave drops the stores of every unit
// it could not confirm as skinned, so no un-skinned row reaches verts.  The
// waves of a workgroup are co-resident, so the bound is reached only by a
// broken hand-over protocol (the diagnostic 1-poll build forces it); the
// host then sees it: every later launch on the model returns MANO_EDEVICE
// until mano_model_device_status clears the flag (include/mano_hip.h).
#ifndef MANO_PAIR_POLL_LIMIT
#define MANO_PAIR_POLL_LIMIT (1 << 20)  // diagnostic builds: tiny limits force the timeout path
#endif
constexpr int kPairPollLimit = MANO_PAIR_POLL_LIMIT;
#ifndef MANO_PAIR_SLEEP_MEM
#define MANO_PAIR_SLEEP_MEM 1  // s_sleep between the memory wave's polls (0 = none)
#endif
#ifndef MANO_PAIR_SLEEP_CMP
#define MANO_PAIR_SLEEP_CMP 1  // s_sleep between a compute wave's polls
#endif
template <int kSleep = 1>
__device__ __forceinline__ bool pair_wait_ge(const int* flag, int target) {
  const unsigned a = lds_addr(flag);
  for (int it = 0; it < kPairPollLimit; ++it) {
    int x;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(a) : "memory");
    if (__builtin_amdgcn_readfirstlane(x) >= target) return true;
    if constexpr (kSleep > 0) __builtin_amdgcn_s_sleep(kSleep);
  }
  return false;
}
// A hand-over wait gave up: one lane sets the bit's flag among the model's
// status flags -- pinned host memory mapped into the device, one word per
// MANO_DEVICE_* bit, so raising it is a plain vector store at system scope
// (no read-modify-write across the host link).  The host reads and clears
// the flags (mano_model_device_status), and every later launch on the model
// fails with MANO_EDEVICE until then.
__device__ __forceinline__ void raise_status(int* flags, int bit) {
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_store(flags + __builtin_ctz(unsigned(bit)), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void pair_signal(int* flag, int value) {
  // the slot's LDS writes have landed before the counter moves
  asm volatile("s_waitcnt lgkmcnt(0)\n\tds_write_b32 %0, %1" ::"v"(lds_addr(flag)), "v"(value) : "memory");
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// LDS-DMA buffer loads (device-only helpers: the host pass of a kernel
// template cannot instantiate this builtin and would silently drop the stub).
template <int kAux = 0>
__device__ __forceinline__ void buffer_load_lds16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_byte_addr, int voffset,
                                                  int soffset) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, reinterpret_cast<__attribute__((address_space(3))) void*>(uintptr_t(lds_byte_addr)),
                                           16, voffset, soffset, 0, kAux);
}
// Cache policy of skin_pair's v_posed row DMA (bit 0) and verts stores (bit 1):
// set = nontemporal (diagnostic builds; the product streams with the default
// policy -- with partial-sector rows nontemporal made no difference, round 2).
#ifndef MANO_PAIR_NT
#define MANO_PAIR_NT 0
#endif
constexpr int kPairRowAux = (MANO_PAIR_NT & 1) ? 2 : 0, kPairStoreAux = (MANO_PAIR_NT & 2) ? 2 : 0;
__device__ __forceinline__ void buffer_load_lds4(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_byte_addr, int voffset,
                                                 int soffset) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, reinterpret_cast<__attribute__((address_space(3))) void*>(uintptr_t(lds_byte_addr)),
                                           4, voffset, soffset, 0, 0);
}

// Diagnostic build only (MANO_PAIR_STAMP=1, tools/debug/pair_stamps.py): per
// wave the shader-clock cycles from entry to exit, the cycles spent in the
// hand-over polls and the units handled, read back by mano_debug_pair_stamps().
#ifndef MANO_PAIR_STAMP
#define MANO_PAIR_STAMP 0
#endif
#if MANO_PAIR_STAMP
constexpr int kPairStampWaves = 256 * 12;
__device__ unsigned long long g_pair_stamps[kPairStampWaves * 8];
struct PairStamp {
  unsigned long long t0, wait = 0, units = 0, t_stage = 0, t_store = 0, t_fetch = 0;
  __device__ PairStamp() : t0(__builtin_amdgcn_s_memtime()) {}
  __device__ void done(int wave) {
    const int w = blockIdx.x * 12 + wave;
    if ((threadIdx.x & 63) == 0 && w < kPairStampWaves) {
      volatile unsigned long long* p = g_pair_stamps + w * 8;
      p[0] = __builtin_amdgcn_s_memtime() - t0;
      p[1] = wait;
      p[2] = units;
      p[3] = 1;
      p[4] = t_stage;
      p[5] = t_store;
      p[6] = t_fetch;
    }
  }
};
#define PAIR_TIMED(expr, st) ({ const unsigned long long _t = __builtin_amdgcn_s_memtime(); auto _r = (expr); st.wait += __builtin_amdgcn_s_memtime() - _t; _r; })
#define PAIR_TIMED_STMT(stmt, field) do { const unsigned long long _t = __builtin_amdgcn_s_memtime(); stmt; stamp.field += __builtin_amdgcn_s_memtime() - _t; } while (0)
#else
struct PairStamp {
  unsigned long long units = 0;
  __device__ void done(int) {}
};
#define PAIR_TIMED(expr, st) (expr)
#define PAIR_TIMED_STMT(stmt, field) stmt
#endif

// kH3: the f16x3 mode (skin_unit4_h3, W halves from basis_h3's pieces 30 /
// 31, t_unscale); otherwise fp32 (wfrag16).
//
// kAlign (fp32): sector-aligned units (mano_layout.h).  A unit's 4 hands are
// of one residue class of the rows' 32-B sector phase (hands c + P (4 q + r),
// P = 2^lp), blocks are dealt to the classes round robin (block b serves
// class b mod P), and a class's 64-vertex spans start at its shift s
// (vertices s + 64 k), so every full span's four 768-B row segments start on
// a sector boundary and their float4 loads and stores are 16-B aligned.  The
// W fragments in LDS are variant s's groups 0 .. 4 n_full - 1 (wfrag16v)
// followed by the plain first and last groups; the edge unit of a hand quad
// stages vertices [0, 16) and [V - 16, V) side by side in its rows (24
// float4 per row, lanes 0-11 and 12-23 of one DMA) and skins them as two
// groups -- the rows' first and last sectors, which neighbouring hands share
// in any layout, and the aligned spans' edges rewritten with identical values.
//
// kInPlace (fp32, plain units): verts == vposed, the LBS overwrites its own
// input (the unfused path's blend GEMM writes v_posed into the verts buffer).
// Units are disjoint except the tail: its segment starts d = 64 n_full -
// tail_v0 vertices inside the last full span (V = 778: d = 6), whose unit
// owns them.  So the tail unit stores only its own rows' floats ov = 3 d ..:
// whole float4 past ov, and the float4 straddling ov as a b32 (dword 1 or 3)
// plus a b64 (dwords 2-3) from its sweep-0 lane -- every unit issues those two
// extra stores (dropped: an offset past num_records), so the step's
// vector-memory op count stays fixed.  The tail's reads of the d shared
// vertices may then see the span's skinned values; they feed only the d
// outputs it does not store.  The blend GEMM's last ~256 MB of v_posed are
// still dirty in the Infinity Cache when the LBS starts -- with all its
// blocks resident at once (n <= 65,536), the last ~42 % of EVERY row -- so
// the LBS reads those lines as hits and overwrites them in the cache instead
// of having them written back first, provided the rest of its stream does
// not evict them: the cold spans go nontemporal (MANO_PAIR_INPLACE_HOT
// below).  Hand quads go last-first (for larger batches the hot lines are the
// last hands' rows).  (In place,
// `vposed` and `verts` alias despite their __restrict__: the kernel touches
// both only through buffer intrinsics on resource descriptors -- the rows'
// LDS-DMA and the memory wave's stores, ordered by its counted vmcnt -- never
// through the pointers themselves, and distinct units' bytes are disjoint
// apart from the tail reads above.)
#ifndef MANO_PAIR_INPLACE_FORWARD
#define MANO_PAIR_INPLACE_FORWARD 0  // diagnostic builds: 1 = in-place units in hand order
#endif
#ifndef MANO_PAIR_INPLACE_ORDER
#define MANO_PAIR_INPLACE_ORDER 0  // diagnostic builds: 1 = in-place units span-major, last span first
#endif
// In place, the spans the launcher estimates cold (below hot_span0: their
// v_posed already left the Infinity Cache) are read AND written nontemporal,
// so streaming them does not push out the hot spans' dirty lines before the
// LBS overwrites them: 0.2555-0.2581 vs 0.2717-0.2727 ms in the unfused path
// (62 vs 58.6 % of 8 TB/s), bit-identical; either bit alone gains nothing
// (stores only 0.271) or loses (reads only 0.285), profiles/r06/r06q_*,
// r06r_*.  (Diagnostic builds: bit 0 = reads, bit 1 = stores.)
#ifndef MANO_PAIR_INPLACE_HOT
#define MANO_PAIR_INPLACE_HOT 3
#endif
template <bool kTrans, bool kH3 = false, bool kAlign = false, bool kInPlace = false>
__global__ __launch_bounds__(64 * kPairWaves, 1) void skin_pair_kernel(
    const float* __restrict__ transforms, const float* __restrict__ wfrag16,
    const float* __restrict__ vposed, const float* __restrict__ trans, float* __restrict__ verts,
    int64_t n, int n_verts, int n_groups, const uint16_t* __restrict__ basis_h3, float t_unscale,
    int* __restrict__ status, const float* __restrict__ wfrag16v, int lp, unsigned shifts, int hot_span0) {
  static_assert(!(kAlign && kH3), "aligned units: fp32 only");
  static_assert(!(kInPlace && (kAlign || kH3)), "in-place units: fp32 plain units only");
  __shared__ f32x4 w_lds[kPairMaxGroups * 64];
  __shared__ PairShared sh;
  const int P = kAlign ? 1 << lp : 1;
  const int bcls = kAlign ? int(blockIdx.x) & (P - 1) : 0;  // this block's residue class
  const int shift = kAlign ? int((shifts >> (4 * bcls)) & 15u) : 0;
  const int n_full = n_verts / kQVerts;
  if constexpr (kAlign) {
    const int n_al = 4 * n_full;  // variant groups, then the plain first and last group
    const f32x4* wv = reinterpret_cast<const f32x4*>(wfrag16v + int64_t(shift) * n_groups * kWFrag16Floats);
    const f32x4* wp = reinterpret_cast<const f32x4*>(wfrag16);
    for (int i = threadIdx.x; i < (n_al + 2) * 64; i += 64 * kPairWaves) {
      const int grp = i >> 6, e = i & 63;
      w_lds[i] = grp < n_al ? wv[i] : wp[(grp == n_al ? 0 : n_groups - 1) * 64 + e];
    }
  } else {
    for (int i = threadIdx.x; i < n_groups * 64; i += 64 * kPairWaves) {
      if constexpr (kH3) {
        const int grp = i >> 6, e = i & 63;
        w_lds[i] = reinterpret_cast<const f32x4*>(basis_h3 + int64_t(grp) * kH3GroupHalves +
                                                  (kH3WPiece + (e >> 5)) * kH3PieceHalves)[e & 31];
      } else {
        w_lds[i] = reinterpret_cast<const f32x4*>(wfrag16)[i];
      }
    }
  }

  if (threadIdx.x < kPairs) sh.full[threadIdx.x] = 0;
  if (threadIdx.x < kPairs * kPairSlots) sh.done[threadIdx.x / kPairSlots][threadIdx.x % kPairSlots] = 0;
  __syncthreads();

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave & (kPairs - 1);
  const bool is_mem = wave < kPairs;
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int vstride = 3 * n_verts;
  const int rstride = vstride * P;  // floats between a unit's rows
  const int n_tail = n_groups - 4 * n_full;
  const int spans = n_full + (kAlign || n_tail > 0 ? 1 : 0);
  // hand quads of this block's class (all hands without kAlign)
  const int64_t n_hands_c = kAlign ? (n > bcls ? (n - 1 - bcls) / P + 1 : 0) : n;
  const int64_t n_quads = (n_hands_c + kQHands - 1) / kQHands;
  const int64_t b = kAlign ? int64_t(blockIdx.x) / P : int64_t(blockIdx.x);
  const int64_t nb = kAlign ? int64_t(gridDim.x) / P : int64_t(gridDim.x);
  const int64_t blk = (nb % 8) ? b : (b % 8) * (nb / 8) + b / 8;
  const int64_t worker = blk * kPairs + pair, n_workers = nb * kPairs;
  const int64_t step_q = n_workers / spans;
  const int step_s = int(n_workers - step_q * spans);
  auto advance = [&](int64_t& aq, int& as) {
    aq += step_q;
    as += step_s;
    if (as >= spans) {
      as -= spans;
      ++aq;
    }
  };
  const int tail_v0 = min(kQVerts * n_full, n_verts - 16);
  // Unit (q, s) of the worker sequence -> the unit it stands for: itself, or
  // with the span-major in-place order unit u = q spans + s is span
  // spans - 1 - u / n_quads of quad u % n_quads (a bijection on the units).
  constexpr bool kSpanMajor = kInPlace && MANO_PAIR_INPLACE_ORDER == 1;
  auto unit_of = [&](int64_t uq, int us, int64_t& q2, int& s2) {
    if constexpr (kSpanMajor) {
      const uint64_t u = uint64_t(uq) * uint64_t(spans) + uint64_t(us);
      const uint64_t k = u / uint64_t(n_quads);
      s2 = spans - 1 - int(k);
      q2 = int64_t(u - k * uint64_t(n_quads));
    } else {
      q2 = uq;
      s2 = us;
    }
  };
  int* full_flag = &sh.full[pair];
  int64_t qd = worker / spans;
  int s = int(worker - qd * spans);
  if (qd >= n_quads) return;

  static_assert(kPairSlots >= 2 * kPairCompute, "slot count: the two units being skinned and one in flight");
  PairStamp stamp;
  if (is_mem) {
    if (MANO_QUAD_PAIR_PRIO) __builtin_amdgcn_s_setprio(MANO_QUAD_PAIR_PRIO);
    // The memory wave with LDS-DMA loads: unit k + 2's rows, transforms
    // and translations go straight from HBM into its stage slot (buffer
    // loads with the lds bit: lane i's 16 B land at M0 + 16 i), so a step
    // has no register staging: wait until unit k's DMA has landed, signal,
    // store unit k - 2 once skinned, then DMA unit k + 2 into the slot the
    // store has just read out.  Each row is one DMA of its 48 (full span)
    // or tail_rf4 (tail) float4, so the stage keeps its padded row stride.
    // Rows and hands past the batch end fall outside num_records: their
    // loads write zeros, their stores are dropped.
    // the tail unit's float4 per row (kAlign: the edge unit's two 16-vertex pieces)
    const int tail_rf4 = kAlign ? 24 : 3 * (n_verts - tail_v0) / 4;
    // an edge-unit float4 at column tc of its staged row: head piece (tc < 48)
    // at the row start, tail piece at vertex V - 16
    auto edge_col = [&](int tc) { return tc < 48 ? tc : 3 * (n_verts - 16) + (tc - 48); };
    int fvo[kQF4], tvo[kQF4];                 // store sweep: global byte offsets in the unit's rows
    unsigned fso[kQF4], tso[kQF4];            // store sweep: LDS byte addresses in slot 0
    const unsigned slot0 = lds_addr(reinterpret_cast<const int*>(&sh.slot[pair][0]));
#pragma unroll
    for (int i = 0; i < kQF4; ++i) {
      const int idx = 64 * i + lane;
      const int fr = idx / kQRowF4, fc = 4 * (idx % kQRowF4);
      const int it = min(idx, kQHands * tail_rf4 - 1);
      const int tr = it / tail_rf4, tc = 4 * (it % tail_rf4);
      fvo[i] = 4 * (fr * rstride + fc);
      tvo[i] = 4 * (tr * rstride + (kAlign ? edge_col(tc) : tc));
      fso[i] = slot0 + unsigned(offsetof(PairStage, rows)) + 4u * unsigned(fr * kPStride + fc);
      tso[i] = slot0 + unsigned(offsetof(PairStage, rows)) + 4u * unsigned(tr * kPStride + tc);
    }
    // kInPlace: the tail unit's store offsets (floats before ov dropped) and
    // the straddling float4's b32 / b64 pieces (sweep-0 lanes only)
    constexpr int kDrop = 0x40000000;  // past any num_records here: the store is dropped
    const int ov = kInPlace ? 3 * (kQVerts * n_full - tail_v0) : 0;
    int tvo_ip[kQF4];
    int p32o = kDrop, p64o = kDrop;
#pragma unroll
    for (int i = 0; i < kQF4; ++i) {
      const int idx = 64 * i + lane;
      const int it = min(idx, kQHands * tail_rf4 - 1);
      const int tc = 4 * (it % tail_rf4);
      tvo_ip[i] = tc >= ov ? tvo[i] : kDrop;
      if (kInPlace && i == 0 && idx == it && tc < ov && ov < tc + 4) {
        p32o = (ov & 3) == 2 ? kDrop : tvo[0] + 4 * ((ov & 3) == 1 ? 1 : 3);
        p64o = (ov & 3) <= 2 ? tvo[0] + 8 : kDrop;
      }
    }
    int rvo[kPairRowDmas];  // DMA j: the lane's byte offset in the unit's rows
    int evo[kPairRowDmas];  // kAlign, edge unit: head piece (lanes 0-11), tail piece (12-23)
#pragma unroll
    for (int j = 0; j < kPairRowDmas; ++j) {
      rvo[j] = 4 * j * rstride + 16 * lane;
      evo[j] = 4 * j * rstride + 4 * edge_col(4 * lane);
    }
    // transforms: lane's 16 B of sweep i (3 KB of the unit's 4 hands, each
    // 768 B; kAlign: the hands are P rows apart), translations: lane < 12
    int tro[kQTrF4];
#pragma unroll
    for (int i = 0; i < kQTrF4; ++i) {
      const int bb = 1024 * i + 16 * lane;
      tro[i] = (bb / 768) * P * 768 + bb % 768;
    }
    const int xo = 4 * ((lane / 3) * P * 3 + lane % 3);
    // first hand and hands in the batch of hand quad fq (rows P apart)
    constexpr bool kReverse = kPairReverse || (kInPlace && !MANO_PAIR_INPLACE_FORWARD && !kSpanMajor);
    auto unit_hands = [&](int64_t fq, int64_t& h0, int& valid) {
      const int64_t qq = kReverse ? n_quads - 1 - fq : fq;
      h0 = kAlign ? bcls + int64_t(P) * kQHands * qq : qq * kQHands;
      const int64_t left = kAlign ? (n - 1 - h0) / P + 1 : n - h0;
      valid = int(left < kQHands ? left : kQHands);
    };
    constexpr int kRsrcFlags = 0x00020000;  // gfx9 raw buffer
    auto rsrc = [&](const float* base, int64_t floats) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, int(floats * 4), kRsrcFlags);
    };
    const unsigned slot0_s = __builtin_amdgcn_readfirstlane(slot0);
    auto lds_at = [&](int slot, unsigned byte_off) {
      return slot0_s + unsigned(slot) * unsigned(sizeof(PairStage)) + byte_off;
    };
    // VMEM ops per DMA: 4 rows + 3 transform sweeps (+ 1 translations)
    // (diagnostic MANO_QUAD_ABLATE & 4: no transform DMA -- stale operands, timing only)
    constexpr int kTrOps = (MANO_QUAD_ABLATE & 4) ? 0 : kQTrF4;
    constexpr int kDmaOps = kPairRowDmas + kTrOps + (kTrans ? 1 : 0);
    constexpr int kStoreOps = 3 + (kInPlace ? 2 : 0);  // per store call, on every path
    // in place: spans below hot_span0 (full spans only; the launcher's
    // estimate of what the blend GEMM left in the Infinity Cache) stream
    // nontemporal, the hot ones with the default policy
    constexpr bool kColdNtRead = kInPlace && (MANO_PAIR_INPLACE_HOT & 1);
    constexpr bool kColdNtStore = kInPlace && (MANO_PAIR_INPLACE_HOT & 2);
    auto dma = [&](int64_t fq0, int fs0, int slot) {
      int64_t fq, h0;
      int fs, valid;
      unit_of(fq0, fs0, fq, fs);
      unit_hands(fq, h0, valid);
      // rows / hands past the batch end are outside num_records (loads give 0)
      const auto rv = rsrc(vposed + h0 * vstride, kAlign ? int64_t(valid - 1) * rstride + vstride : int64_t(valid) * vstride);
      const auto rt = rsrc(transforms + h0 * kTransformFloats,
                           kAlign ? int64_t(valid - 1) * P * kTransformFloats + kTransformFloats
                                  : int64_t(valid) * kTransformFloats);
      const bool full = fs < n_full;
      const int soff = kAlign ? (full ? 4 * 3 * (shift + kQVerts * fs) : 0) : 4 * 3 * (full ? kQVerts * fs : tail_v0);
      const int row_f4 = full ? kQRowF4 : tail_rf4;
#pragma unroll
      for (int i = 0; i < kTrOps; ++i) {
        if constexpr (kAlign)
          buffer_load_lds16(rt, lds_at(slot, unsigned(offsetof(PairStage, tr)) + 1024u * i), tro[i], 0);
        else
          buffer_load_lds16(rt, lds_at(slot, unsigned(offsetof(PairStage, tr)) + 1024u * i), 16 * lane,
                                         1024 * i);
      }
      if constexpr (kTrans) {
        const auto rr = rsrc(trans + h0 * 3, kAlign ? int64_t(valid - 1) * P * 3 + 3 : int64_t(valid) * 3);
        if (lane < 12)
          buffer_load_lds4(rr, lds_at(slot, unsigned(offsetof(PairStage, trans))), kAlign ? xo : 4 * lane, 0);
      }
      if (kColdNtRead && __builtin_amdgcn_readfirstlane(fs) < hot_span0) {  // a uniform (scalar) branch
        // a cold span (its v_posed left the Infinity Cache): read around it,
        // so the stream does not push the hot spans' dirty lines out
#pragma unroll
        for (int r = 0; r < kQHands; ++r)
          if (lane < row_f4)
            buffer_load_lds16<2>(rv, lds_at(slot, unsigned(offsetof(PairStage, rows)) + 4u * r * kPStride), rvo[r],
                                 soff);
      } else {
#pragma unroll
        for (int r = 0; r < kQHands; ++r)
          if (lane < row_f4)
            buffer_load_lds16<kPairRowAux>(rv, lds_at(slot, unsigned(offsetof(PairStage, rows)) + 4u * r * kPStride),
                                           kAlign && !full ? evo[r] : rvo[r], soff);
      }
    };
    auto ds_read4 = [](unsigned addr) {
      return *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(uintptr_t(addr));
    };
    constexpr unsigned kSlotBytes = sizeof(PairStage);
    auto store = [&](int64_t fq0, int fs0, unsigned slot, bool real) {
      const unsigned so = slot * kSlotBytes;
      int64_t fq, h0;
      int fs, valid;
      unit_of(fq0, fs0, fq, fs);
      unit_hands(fq, h0, valid);
      // not real: num_records 0, every store dropped
      const auto ro = rsrc(verts + h0 * vstride, !real ? 0 : kAlign ? int64_t(valid - 1) * rstride + vstride
                                                                    : int64_t(valid) * vstride);
      const bool full = fs < n_full;
      const int soff = kAlign ? (full ? 4 * 3 * (shift + kQVerts * fs) : 0) : 4 * 3 * (full ? kQVerts * fs : tail_v0);
      f32x4 sdata[kQF4];
#pragma unroll
      for (int i = 0; i < kQF4; ++i) sdata[i] = ds_read4((full ? fso[i] : tso[i]) + so);
      if (kColdNtStore && __builtin_amdgcn_readfirstlane(fs) < hot_span0) {  // a uniform (scalar) branch
#pragma unroll
        for (int i = 0; i < kQF4; ++i)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, sdata[i]), ro, fvo[i], soff, 2);
      } else {
#pragma unroll
        for (int i = 0; i < kQF4; ++i)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, sdata[i]), ro,
                                                 full ? fvo[i] : (kInPlace ? tvo_ip[i] : tvo[i]), soff,
                                                 kPairStoreAux);
      }
      if constexpr (kInPlace) {
        // scalars first (a bit cast of a vector element reads element 0)
        const float e1 = sdata[0][1], e2 = sdata[0][2], e3 = sdata[0][3];
        const float e = (ov & 3) == 1 ? e1 : e3;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(e), ro, full ? kDrop : p32o, soff, kPairStoreAux);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(e2), __float_as_uint(e3)}, ro,
                                              full ? kDrop : p64o, soff, kPairStoreAux);
      }
    };
    // Units k + 1 .. k + kAhead - 1 are in flight while unit k is skinned;
    // unit k + kAhead goes into unit k - 2's slot once that is stored.
    constexpr int kAhead = kPairSlots - kPairCompute;
    int64_t pend_q[kPairCompute + 1];
    int pend_s[kPairCompute + 1];
    int k = 0;
    bool ok = true;
    int64_t qa = qd;  // unit k + kAhead (past the end: the current unit again)
    int sa = s;
    // Prologue: DMA units 0 .. kAhead - 1 with kStoreOps (dropped) stores
    // after each, so at every step's wait the ops issued after unit k's DMA
    // are the same: kAhead - 1 times (kStoreOps stores + a DMA).
    // (straight-line: no branch between the prologue's DMA groups, so every
    // control-flow path into the step's wait has the same op sequence --
    // tools/isa_scan.py checks it on the disassembly)
    dma(qa, sa, 0);
    advance(qa, sa);
#pragma unroll
    for (int j = 1; j < kAhead; ++j) {
      store(qd, s, 0, false);
      // the dropped stores stay ahead of the next DMA group (nothing else
      // orders them: no data dependence, no exec-masked block in between)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      dma(qa < n_quads ? qa : qd, qa < n_quads ? sa : s, j);
      advance(qa, sa);
    }
    const int64_t n_units = (n_quads * spans - worker + n_workers - 1) / n_workers;  // >= 2
    for (int64_t i = 0; i < n_units; ++i) {
      // unit k = (qd, s) in slot k % kPairSlots: its DMA has landed once at
      // most (kAhead - 1) (kStoreOps + kDmaOps) younger VMEM ops are outstanding.
      PAIR_TIMED_STMT(asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kAhead - 1) * (kStoreOps + kDmaOps)) : "memory"),
                      t_stage);
      pair_signal(full_flag, k + 1);
#pragma unroll
      for (int j = kPairCompute; j > 0; --j) pend_q[j] = pend_q[j - 1], pend_s[j] = pend_s[j - 1];
      pend_q[0] = qd;
      pend_s[0] = s;
      // One store call on every path (its buffer resource drops the bytes
      // when `real` is false), so the step's vector-memory op sequence has
      // no branch: 3 stores, then the DMA.
      const bool drained = k >= kPairCompute;  // unit k - 2 exists
      const int ku = k - kPairCompute;
      if (drained && ok) {
        ok = PAIR_TIMED(pair_wait_ge<MANO_PAIR_SLEEP_MEM>(&sh.done[pair][ku % kPairSlots], ku + 1), stamp);
        if (!ok) raise_status(status, MANO_DEVICE_SKIN_HANDOFF_TIMEOUT);
      }
      stamp.units += drained;
      // after a lost hand-over the stores are issued dropped (same op count)
      PAIR_TIMED_STMT(store(drained ? pend_q[kPairCompute] : qd, drained ? pend_s[kPairCompute] : s,
                            drained ? unsigned(ku % kPairSlots) : 0u, drained && ok), t_store);
      // the store's LDS reads have returned (its data is in registers), so
      // unit k - 2's slot is free for unit k + kAhead
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      PAIR_TIMED_STMT(dma(qa < n_quads ? qa : qd, qa < n_quads ? sa : s, (k + kAhead) % kPairSlots), t_fetch);
      advance(qa, sa);
      advance(qd, s);
      ++k;
    }
    // the last min(k, 2) units
    for (int i = min(k, kPairCompute) - 1; ok && i >= 0; --i) {
      const int ku = k - 1 - i;
      if (!pair_wait_ge<MANO_PAIR_SLEEP_MEM>(&sh.done[pair][ku % kPairSlots], ku + 1)) {
        raise_status(status, MANO_DEVICE_SKIN_HANDOFF_TIMEOUT);
        break;
      }
      store(pend_q[i], pend_s[i], unsigned(ku % kPairSlots), true);
    }
    // no LDS-DMA may still be writing when the workgroup's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp.done(wave);
    return;
  }

  // compute wave
  const int q = lane >> 4, v = lane & 15;
  int hh[3], cc[3], a_off[3], h3_off[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int m0 = 16 * t + 4 * q, m = 16 * t + v;
    hh[t] = m0 / 12;
    cc[t] = (m0 % 12) / 4;
    a_off[t] = (m / 12) * kTransformFloats + 12 * q + m % 12;
    h3_off[t] = (m / 12) * kTransformFloats + 12 * 8 * (q & 1) + m % 12;  // f16x3: joints 8 (q & 1) + j
  }
  // compute wave c of the pair takes the pair's units k = c, c + kPairCompute, ...
  const int cw = (wave - kPairs) / kPairs;
  for (int i = 0; i < cw; ++i) advance(qd, s);
  for (int k = cw; qd < n_quads; k += kPairCompute) {
    if (!PAIR_TIMED(pair_wait_ge<MANO_PAIR_SLEEP_CMP>(full_flag, k + 1), stamp)) {
      raise_status(status, MANO_DEVICE_SKIN_HANDOFF_TIMEOUT);
      return;
    }
    ++stamp.units;
    PairStage& st = sh.slot[pair][k % kPairSlots];
    int64_t q_unit;
    int s_unit;
    unit_of(qd, s, q_unit, s_unit);
    (void)q_unit;
    if (MANO_QUAD_ABLATE & 2) {  // diagnostic: no compute (the memory waves alone)
      pair_signal(&sh.done[pair][k % kPairSlots], k + 1);
#pragma unroll
      for (int i = 0; i < kPairCompute; ++i) advance(qd, s);
      continue;
    }
    float tr3[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) tr3[t] = kTrans ? st.trans[3 * hh[t] + cc[t]] : 0.f;
    // The unit's 4 groups (a tail unit: its n_tail groups, the last repeated
    // -- duplicates rewrite identical bits).  Every point is read before any
    // output lands: the tail's last group is shifted onto its neighbour's
    // vertices when n_verts % 16 != 0, and the skinning is in place.  Full
    // units get compile-time group offsets (LDS immediates).
    if constexpr (kH3) {
      // A operands: row m = 16 t + (lane & 15) is (hand m / 12, c, k), K
      // element j of the lane is joint 8 ((lane >> 4) & 1) + j, the hi half
      // in lanes 0-31 and the lo half in 32-63 (blend_skin_h3's split).
      f16x8 ah[3];
      const bool lo = lane >= 32;
      constexpr float kScale = float(1 << kH3FrameExp);
#pragma unroll
      for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = st.tr[h3_off[t] + 12 * j] * kScale;
          const _Float16 h = static_cast<_Float16>(x);
          ah[t][j] = lo ? static_cast<_Float16>(x - static_cast<float>(h)) : h;
        }
      }
      const f16x8* wl = reinterpret_cast<const f16x8*>(w_lds);
      if (s_unit < n_full) {
        const int G[4] = {4 * s_unit, 4 * s_unit + 1, 4 * s_unit + 2, 4 * s_unit + 3};
        const int lv[4] = {0, 16, 32, 48};
        skin_unit4_h3<kTrans, 4, PairStage>(st, wl, ah, tr3, G, lv, hh, cc, v, lane, t_unscale);
      } else {
        int G[4], lv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          G[g] = 4 * n_full + min(g, n_tail - 1);
          lv[g] = min(16 * G[g], n_verts - 16) - tail_v0;
        }
        if (n_tail == 1) skin_unit4_h3<kTrans, 1, PairStage>(st, wl, ah, tr3, G, lv, hh, cc, v, lane, t_unscale);
        else skin_unit4_h3<kTrans, 4, PairStage>(st, wl, ah, tr3, G, lv, hh, cc, v, lane, t_unscale);
      }
    } else {
      float a[3][4];
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) a[t][kk] = st.tr[a_off[t] + 4 * 12 * kk];
      if (s_unit < n_full) {
        const int G[4] = {4 * s_unit, 4 * s_unit + 1, 4 * s_unit + 2, 4 * s_unit + 3};
        const int lv[4] = {0, 16, 32, 48};
        skin_unit4<kTrans, 4, PairStage>(st, w_lds, a, tr3, G, lv, hh, cc, v, lane);
      } else if constexpr (kAlign) {
        // the edge unit: vertices [0, 16) and [V - 16, V), staged side by side
        const int G[4] = {4 * n_full, 4 * n_full + 1, 4 * n_full + 1, 4 * n_full + 1};
        const int lv[4] = {0, 16, 16, 16};
        skin_unit4<kTrans, 2, PairStage>(st, w_lds, a, tr3, G, lv, hh, cc, v, lane);
      } else {
        int G[4], lv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          G[g] = 4 * n_full + min(g, n_tail - 1);
          lv[g] = min(16 * G[g], n_verts - 16) - tail_v0;
        }
        if (n_tail == 1) skin_unit4<kTrans, 1, PairStage>(st, w_lds, a, tr3, G, lv, hh, cc, v, lane);
        else skin_unit4<kTrans, 4, PairStage>(st, w_lds, a, tr3, G, lv, hh, cc, v, lane);
      }
    }
    pair_signal(&sh.done[pair][k % kPairSlots], k + 1);
#pragma unroll
    for (int i = 0; i < kPairCompute; ++i) advance(qd, s);
  }
  stamp.done(wave);
}

}  // namespace

#if MANO_PAIR_STAMP
}  // namespace mano
extern "C" int mano_debug_pair_stamps(unsigned long long* host, int count) {
  if (count > mano::kPairStampWaves * 8) count = mano::kPairStampWaves * 8;
  return int(hipMemcpyFromSymbol(host, HIP_SYMBOL(mano::g_pair_stamps), size_t(count) * 8, 0,
                                 hipMemcpyDeviceToHost));
}
namespace mano {
#endif

// skin_pair's sector-aligned units (kAlign) for this mesh: the variants
// exist, every shift's 64-vertex spans end inside the row with at most 16
// vertices after them, and the W fragments (4 n_full variant groups + 2)
// fit the block's LDS.
#ifndef MANO_PAIR_ALIGN
#define MANO_PAIR_ALIGN 0
#endif
bool pair_align_ok(const DeviceModel& m) {
  const int V = m.n_verts, n_full = V / kQVerts;
  if (!m.wfrag16v || V < 32 || 4 * n_full + 2 > kPairMaxGroups) return false;
  for (int s = 0; s < kAlignVariants; ++s)
    if (s + kQVerts * n_full > V || V - (s + kQVerts * n_full) > 16 || 4 * n_full > (V - s) / 16) return false;
  return true;
}

// The in-place form's launch: skin_pair's fp32 plain units (a batch large
// enough for one block of them).
bool skin_in_place_supported(const DeviceModel& m, int64_t n) {
#if MANO_QUAD_PAIR
  if (!skin_quad_supported(m) || n <= 0) return false;
  const int spans = m.n_verts / kQVerts + (m.n_verts % kQVerts ? 1 : 0);
  const int64_t units = (n + kQHands - 1) / kQHands * spans;
  return units / (2 * kPairs) >= 1;
#else
  (void)m;
  (void)n;
  return false;
#endif
}

bool skin_quad_supported(const DeviceModel& m) {
#if MANO_QUAD_PAIR
  if (m.n_groups16 > kPairMaxGroups) return false;
#endif
  // the tail segment must be whole float4 per row
  const int tail_v0 = std::min(kQVerts * (m.n_verts / kQVerts), m.n_verts - 16);
  return m.n_verts >= 16 && m.n_groups16 <= kQMaxGroups && (3 * (m.n_verts - tail_v0)) % 4 == 0;
}

// skin_pair (fp32, or f16x3 with h3) for the meshes skin_quad_supported
// takes; a batch too small for one skin_pair block runs skin_quad_kernel
// (fp32) or returns hipErrorNotSupported (f16x3: the caller's skin_span_h3).
hipError_t launch_skin_quad(const DeviceModel& m, int64_t n, const float* transforms,
                            const float* vposed, const float* trans, float* verts,
                            hipStream_t stream, bool h3, bool in_place) {
  if (n <= 0) return hipSuccess;
  if (in_place) {
#if MANO_QUAD_PAIR
    if (h3 || !skin_in_place_supported(m, n)) return hipErrorNotSupported;
    const int64_t units = (n + kQHands - 1) / kQHands * (m.n_verts / kQVerts + (m.n_verts % kQVerts ? 1 : 0));
    const int64_t blocks_ip = std::min<int64_t>(units / (2 * kPairs), m.n_cu > 0 ? m.n_cu : 1);
    // The spans the blend GEMM's v_posed most likely left dirty in the
    // 256-MB Infinity Cache: blend_kernel's blocks walk the column tiles
    // together, so when they all fit the chip at once (n / 128 blocks <= 2
    // per CU) the last-written bytes are the LAST fraction of every row;
    // spans wholly before it are cold.  (More blocks than that: the last
    // hands are the hot ones, and the quads' last-first order serves them.)
    constexpr double kMallBytes = 256.0 * 1024.0 * 1024.0;
    const double row_bytes = double(n) * 3.0 * m.n_verts * 4.0;
    const int64_t blend_blocks = (n + 127) / 128;
    int hot_span0 = 0;
    if (blend_blocks <= 2 * int64_t(m.n_cu > 0 ? m.n_cu : 1) && row_bytes > kMallBytes)
      hot_span0 = int((1.0 - kMallBytes / row_bytes) * m.n_verts) / kQVerts;
    auto launch_ip = [&](auto kernel) {
      hipLaunchKernelGGL(kernel, dim3(unsigned(blocks_ip)), dim3(64 * kPairWaves), 0, stream, transforms,
                         m.wfrag16, vposed, trans, verts, n, m.n_verts, m.n_groups16, m.basis_h3,
                         m.h3_lbs_unscale, m.status, nullptr, 0, 0u, hot_span0);
    };
    if (trans) launch_ip(skin_pair_kernel<true, false, false, true>);
    else launch_ip(skin_pair_kernel<false, false, false, true>);
    return hipGetLastError();
#else
    return hipErrorNotSupported;
#endif
  }
  const int spans = m.n_verts / kQVerts + (m.n_verts % kQVerts ? 1 : 0);
  const int64_t units = (n + kQHands - 1) / kQHands * spans;
  int64_t blocks = (units + kQWaves - 1) / kQWaves;
  const int64_t cap = m.n_cu > 0 ? m.n_cu : 1;
  if (blocks > cap) blocks = cap;
#if MANO_QUAD_PAIR
  // at least 2 units per memory wave (its prologue stages two); a batch too
  // small for one block of those runs skin_quad_kernel
  blocks = std::min<int64_t>(units / (2 * kPairs), cap);
  if (blocks < 1 && h3) return hipErrorNotSupported;
  if (blocks < 1) {
    auto launch1 = [&](auto kernel) {
      hipLaunchKernelGGL(kernel, dim3(1), dim3(64 * kQWaves), 0, stream, transforms, m.wfrag16, vposed,
                         trans, verts, n, m.n_verts, m.n_groups16);
    };
    if (trans) launch1(skin_quad_kernel<true>);
    else launch1(skin_quad_kernel<false>);
    return hipGetLastError();
  }
  // Sector-aligned units (fp32): every class must give each memory wave at
  // least 2 units with whole classes of blocks.
  if (!h3 && MANO_PAIR_ALIGN && pair_align_ok(m)) {
    const int lp = aligned_period_log2(m.n_verts), P = 1 << lp;
    const unsigned shifts = aligned_shifts(m.n_verts, unsigned(reinterpret_cast<uintptr_t>(verts) >> 2) & 7u, lp);
    const int spans_al = m.n_verts / kQVerts + 1;
    int64_t units_min = -1;
    for (int r = 0; r < P; ++r) {
      const int64_t hands = n > r ? (n - 1 - r) / P + 1 : 0;
      const int64_t u = (hands + kQHands - 1) / kQHands * spans_al;
      units_min = units_min < 0 || u < units_min ? u : units_min;
    }
    const int64_t per_class = std::min<int64_t>(units_min / (2 * kPairs), cap / P);
    if (per_class >= 1) {
      auto launch_al = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, dim3(unsigned(per_class * P)), dim3(64 * kPairWaves), 0, stream, transforms,
                           m.wfrag16, vposed, trans, verts, n, m.n_verts, m.n_groups16, m.basis_h3,
                           m.h3_lbs_unscale, m.status, m.wfrag16v, lp, shifts, 0);
      };
      if (trans) launch_al(skin_pair_kernel<true, false, true>);
      else launch_al(skin_pair_kernel<false, false, true>);
      return hipGetLastError();
    }
  }
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, dim3(unsigned(blocks)), dim3(64 * kPairWaves), 0, stream, transforms,
                       m.wfrag16, vposed, trans, verts, n, m.n_verts, m.n_groups16, m.basis_h3,
                       m.h3_lbs_unscale, m.status, nullptr, 0, 0u, 0);
  };
  if (h3) {
    if (trans) launch(skin_pair_kernel<true, true>);
    else launch(skin_pair_kernel<false, true>);
  } else {
    if (trans) launch(skin_pair_kernel<true>);
    else launch(skin_pair_kernel<false>);
  }
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
