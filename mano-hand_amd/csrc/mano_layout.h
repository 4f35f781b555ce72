// mano_layout.h -- the model-buffer and workspace layouts (constants), and
// the host-side packing of a dump_model.py model into them.  Plain C++ (no
// HIP): the library compiles it with hipcc, and tests/test_pack_sanitize.py
// compiles the packing with g++ under AddressSanitizer / UBSan on the CPU.
// Not installed.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "mano_diag.h"

#if !defined(__HIP__) && !defined(__host__)
#define __host__
#define __device__
#endif

namespace mano {

constexpr int kJoints = 16;                    // mano_np.py:35
constexpr int kShape = 10;                     // mano_np.py:36
constexpr int kPoseFeats = 9 * (kJoints - 1);  // 135, mano_np.py:87-91
constexpr int kPca = 45;                       // dump_model.py:8

// Blend GEMM operand geometry (v_mfma_f32_32x32x2_f32: one K-pair per step).
// Row k of the combined basis: k < 10 shape direction k, 10 <= k < 145 pose
// direction k - 10, k = 145 zero pad.
constexpr int kK = kShape + kPoseFeats;        // 145
constexpr int kKSteps = (kK + 1) / 2;          // 73 MFMA steps (K padded to 146)
constexpr int kKGroups = (kKSteps + 3) / 4;    // 19 float4 groups per lane
constexpr int kTileFloats = kKGroups * 64 * 4; // 4864 floats = 19,456 B per tile
constexpr int kHandTile = 32;                  // hands per MFMA row tile
constexpr int kColTile = 32;                   // basis columns per MFMA col tile
constexpr int kTransformFloats = kJoints * 12; // 3x4 skinning transform per joint
// Blend GEMM A operand X (the per-hand row [beta | features | 1 | 0 ...]) in
// the workspace: one row of kXStride floats per hand, k-permuted within each
// block of 16 so that a v_mfma_f32_16x16x4_f32 A-fragment lane reads its four
// consecutive steps with one dwordx4: row position 16 g + 4 r + q holds
//   k = 16 g + 4 q + r        (r = lane >> 4 of the reading lane, q = step % 4)
// i.e. x_pos(k) = 16 (k >> 4) + 4 (k & 3) + ((k >> 2) & 3).  K is padded to
// 160 with zeros (X[:, 145] = 1 multiplies the template row of the basis).
constexpr int kXStride = 160;
__host__ __device__ constexpr int x_pos(int k) { return 16 * (k >> 4) + 4 * (k & 3) + ((k >> 2) & 3); }
// Fused blend_skin kernel operands (v_mfma_f32_16x16x4_f32, 16-hand tiles,
// 16-vertex groups; the LBS transforms T_{c,k}[hand][v] = sum_j A_j[c][k] W[v][j]
// are one 16x16 tile per (c, k) over K = 16 joints):
//   A fragments (from X) per 16 hands, lane l, step s = 4g + q:
//       X[16 t + (l & 15)][k = 4 s + (l >> 4)]            (K padded to 160)
//   basis16 per vertex group (3 tiles x, y, z): [10][64][4]:
//       B[k = 4 s + (l >> 4)][3 (vb + (l & 15)) + coord]
//   LBS A fragments per 16 hands (read from the [n][16][3][4] transforms):
//       F_{c,k}[q] = A_{4 q + (l >> 4)}(16 t + (l & 15))[c][k]
//   wfrag16 per vertex group: [64][4]: W[vb + (l & 15)][4 s + (l >> 4)]
constexpr int kSteps16 = (kK + 1 + 3) / 4;     // 37 MFMA steps (K = 146 -> 148)
constexpr int kGroups16 = (kSteps16 + 3) / 4;  // 10 float4 groups per lane
constexpr int kTile16Floats = kGroups16 * 64 * 4;   // 2560 floats = 10 KB
constexpr int kWFrag16Floats = 64 * 4;         // 256 floats per 16-vertex group

// Sector-aligned output rows of blend_skin16 (round 4).  Hand h's verts row
// starts at float a + 3 V h (a = (verts address / 4) mod 8), so its phase
// within a 32-B sector, c_h = (a + 3 V h) mod 8, repeats with a period of
// P = 8 / gcd(3 V, 8) hands (4 for V = 778: rows are 9,336 B apart).  With the
// 16-vertex groups of hand h shifted by s = (-3 c_h) mod 8 vertices
// (3 s + c_h = 0 mod 8), every group's 48 floats start and end on a sector
// boundary, and its 16 point stores write 6 whole sectors (the round-3
// layout wrote a partial sector at both ends of a group for 3 hands in 4:
// WRITE_SIZE 1.15x of the verts bytes, 1.23x with rest_verts).  Variant s of
// the fused kernel's B and W fragments (basis16v / wfrag16v, kAlignVariants
// of them) maps lane column col of group g to
//   g <  ga = (V - s) / 16:  vertex s + 16 g + col
//   g == ga (the edge group): col < s ? col : min(16 ga + col, V - 1)
// i.e. the edge group holds the row's first s vertices and its last
// (V - s) mod 16, the row's first and last sectors -- which it shares with
// the neighbouring hands' rows in any layout.  Duplicate columns (clamped to
// V - 1) store identical values.  A variant is usable when its edge fits one
// group and the group count equals n_groups16 (every s for V = 778).
constexpr int kAlignVariants = 8;
__host__ __device__ constexpr int aligned_group_vertex(int V, int s, int g, int col) {
  return g < (V - s) / 16 ? s + 16 * g + col
         : col < s        ? col
                          : (16 * ((V - s) / 16) + col < V - 1 ? 16 * ((V - s) / 16) + col : V - 1);
}
constexpr bool aligned_variant_ok(int V, int s, int n_groups16) {
  return V >= s + 16 && s + (V - s) % 16 <= 16 &&
         (V - s) / 16 + ((V - s) % 16 != 0 || s > 0 ? 1 : 0) == n_groups16;
}
// log2 of the period P (hands) of the sector phase of rows of V vertices.
constexpr int aligned_period_log2(int V) {
  return (3 * V) % 8 == 0 ? 0 : (3 * V * 2) % 8 == 0 ? 1 : (3 * V * 4) % 8 == 0 ? 2 : 3;
}
// Variant of class r's hands for a verts row base at float phase a (mod 8):
// s_r = (-3 c_r) mod 8 with c_r = (a + 3 V r) mod 8, four bits per class.
constexpr unsigned aligned_shifts(int V, unsigned a, int lp) {
  unsigned code = 0;
  for (int r = 0; r < (1 << lp); ++r) {
    const unsigned c = (a + 3u * unsigned(V) * unsigned(r)) & 7u;
    code |= ((8u - (3u * c) % 8u) % 8u) << (4 * r);
  }
  return code;
}
// The hand tiles of the kernels that use the variants, in residue classes
// (P = 2^lp; lp = 0 is the plain layout): a block's quad (r, j) holds the
// 2^lq hands 2^lq P j + P i + r, i < 2^lq, wave w of the block the tile of
// T = 2^lt hands with i = T w .. T w + T - 1 (blend_skin16: lq = 6, lt = 4, 4
// waves; blend: lq = 7, lt = 5, 4 waves; blend_skin_h3: lq = 7, lt = 4, 8
// waves).  Quads are numbered class-major.
__host__ __device__ inline int64_t aligned_class_quads(int64_t n, int lp, int r, int lq = 6) {
  return n > r ? ((n - 1 - r) >> (lq + lp)) + 1 : 0;
}
__host__ __device__ inline int64_t aligned_n_quads(int64_t n, int lp, int lq = 6) {
  int64_t q = 0;
  for (int r = 0; r < (1 << lp); ++r) q += aligned_class_quads(n, lp, r, lq);
  return q;
}
// Wave `wave`'s tile of quad `quad`: its first hand h0 (hands h0 + (i << lp),
// i < n_valid, are in the batch) and the quad's class.  A wave whose tile is
// past the batch end takes the quad's last tile (it recomputes and rewrites
// identical values).
struct AlignedTile {
  int64_t h0;
  int n_valid;
  int cls;
};
__host__ __device__ inline AlignedTile aligned_tile(int64_t n, int lp, int64_t quad, int wave, int lq = 6,
                                                   int lt = 4) {
  int cls = 0;
  int64_t j = quad;
  while (cls + 1 < (1 << lp) && j >= aligned_class_quads(n, lp, cls, lq))
    j -= aligned_class_quads(n, lp, cls++, lq);
  const int64_t qbase = (j << (lq + lp)) + cls;
  int64_t h0 = qbase + (int64_t(wave << lt) << lp);
  if (h0 >= n) h0 = qbase + (int64_t((int(((n - 1 - qbase) >> lp) >> lt)) << lt) << lp);
  const int64_t left = ((n - 1 - h0) >> lp) + 1;
  return AlignedTile{h0, int(left < (1 << lt) ? left : (1 << lt)), cls};
}
// The unfused blend GEMM's column tiles (v_mfma_f32_32x32x2_f32, 32 floats of
// a v_posed row each) on sector boundaries: for a row at float phase c the
// tiles are shifted by sigma = (8 - c) mod 8 floats; variant sigma's tile t
// column j is
//   t <  ta = (C - sigma) / 32:  sigma + 32 t + j
//   t == ta (the edge tile):     j < sigma ? j : 32 ta + j   (>= C: not stored)
// (C = 3 V columns).  Usable when the edge fits one tile and the tile count
// equals n_col_tiles (every sigma for V = 778: 73 tiles).
__host__ __device__ constexpr int aligned_tile_col(int C, int sigma, int t, int j) {
  return t < (C - sigma) / 32 ? sigma + 32 * t + j : j < sigma ? j : 32 * ((C - sigma) / 32) + j;
}
constexpr bool aligned_col_variant_ok(int C, int sigma, int n_col_tiles) {
  return C >= sigma + 32 && sigma + (C - sigma) % 32 <= 32 &&
         (C - sigma) / 32 + ((C - sigma) % 32 != 0 || sigma > 0 ? 1 : 0) == n_col_tiles;
}
// Column shift of class r's rows for a row base at float phase a (mod 8).
constexpr unsigned aligned_col_shifts(int V, unsigned a, int lp) {
  unsigned code = 0;
  for (int r = 0; r < (1 << lp); ++r) code |= ((8u - ((a + 3u * unsigned(V) * unsigned(r)) & 7u)) & 7u) << (4 * r);
  return code;
}

// f16x3 precision mode (mano_kernels_h3.hip): every fp32 operand x is carried
// as an unevaluated pair of halves x = hi + lo (hi = f16(x), lo = f16(x - hi),
// 22 significant bits) and each product as hi.hi + hi.lo + lo.hi on
// v_mfma_f32_16x16x32_f16: the three partial products are exact in the fp32
// accumulator, only lo.lo (< 2^-22 relative) is dropped.  Operands are scaled
// by powers of two so their lo halves stay normal (scaling is exact).
//   A operand of the blend GEMM: the X rows (unscaled), read from the same
//     k-permuted fp32 rows the fp32 path uses and split in registers.
//   B operand: the basis x 2^basis_exp, pre-split at model load into
//     basis_h3[group][piece][64 lanes][8 halves], one 1-KB piece per
//     (coord c, part hi/lo, K-step s of 32) = (2c + part) * 5 + s, pieces 30/31
//     the LBS weight fragments [Wh ; Wh] and [Wl ; 0] (x 2^kH3WeightExp).
//     Lane l of a K-step-s piece holds B[k = 32 s + 8 (l >> 4) + j][vertex
//     vb + (l & 15)], j = 0..7 (the 16x16x32 operand map).
//   LBS A operand: transforms x 2^kH3FrameExp, split per lane at load:
//     lane l holds [Fh | Fl](hand l & 15)[k = 8 (l >> 4) + j] with k < 16 the
//     hi halves of joints 0..15 and k >= 16 the lo halves, so
//     [Fh | Fl] . [Wh ; Wh] + [Fh | Fl] . [Wl ; 0] = Fh Wh + Fl Wh + Fh Wl.
constexpr int kH3Steps = 5;                          // K = 160 = 5 x 32
constexpr int kH3PieceHalves = 64 * 8;               // one 1-KB fragment piece
constexpr int kH3WPiece = 6 * kH3Steps;              // 30: [Wh ; Wh], 31: [Wl ; 0]
constexpr int kH3GroupPieces = kH3WPiece + 2;        // 32 KB per 16-vertex group
constexpr int kH3GroupHalves = kH3GroupPieces * kH3PieceHalves;
constexpr int kH3FrameExp = 6;                       // transforms x 64 (|A| < 1000)
constexpr int kH3WeightExp = 14;                     // weights x 16384 (|W| <= 1)

// The device block's arrays as built on the host by pack_model (float32 /
// f16 bits in the kernels' fragment layouts; see DeviceModel for each).
struct HostModel {
  std::vector<float> tiles;     // blend_kernel B fragments [n_col_tiles][kKGroups][64][4]
  std::vector<float> tiles_v;   // their sector-aligned variants [kAlignVariants][n_col_tiles][...]
                                //   (empty when some variant does not fit V)
  std::vector<float> b16;       // blend_skin16 B fragments [n_groups16][3][kTile16Floats]
  std::vector<float> w16;       // LBS weight fragments [n_groups16][kWFrag16Floats]
  std::vector<float> b16v;      // sector-aligned variants [kAlignVariants][n_groups16][3][kTile16Floats]
  std::vector<float> w16v;      //   and their W fragments [kAlignVariants][n_groups16][kWFrag16Floats]
                                //   (empty when some variant does not fit V)
  std::vector<uint16_t> bh3;    // f16x3 pieces [n_groups16][kH3GroupHalves]
  std::vector<uint16_t> bh3v;   // their sector-aligned variants [kAlignVariants][n_groups16][...]
  std::vector<float> weights;   // [V][16]
  std::vector<float> jt, js;    // J_regressor . template [16][3], . shapedirs [16][3][10]
  std::vector<float> pca, pmean;  // [45][45], [45] (zeros without PCA arrays)
  std::vector<int32_t> depth;   // [16]
  int max_depth = 0, n_groups16 = 0, n_col_tiles = 0, basis_exp = 0;
};

// Validate the parents and pack the float64 dump-layout arrays
// (dump_model.py:8-18; pose_pca_basis / pose_pca_mean nullable) for V
// vertices.  The joint regression is folded in float64 here
// (J = Jreg.T + (Jreg.S).beta, mano_np.py:83).  Returns false with a message
// on a bad argument; touches no GPU.
bool pack_model(int n_verts, const double* mesh_template, const double* mesh_shape_basis,
                const double* mesh_pose_basis, const double* j_regressor,
                const double* skinning_weights, const int32_t* parents,
                const double* pose_pca_basis, const double* pose_pca_mean, HostModel& out,
                std::string& error);

// IEEE binary16 bits of a float (round to nearest even) and back; the
// f16x3 split x = hi + lo with hi = f16(x), lo = f16(x - hi).
uint16_t f16_bits(float f);
float f16_value(uint16_t h);

}  // namespace mano
