// mano_pack.cpp -- host-side packing of a dump_model.py model into the device
// block's layouts (mano_layout.h).  Replaces the array binding of
// MANOModel.__init__ (mano_np.py:17-33) and folds the joint regression
// (mano_np.py:83) in float64.  Plain C++: no HIP call, so the CPU suite runs it
// under AddressSanitizer / UBSan (tests/test_pack_sanitize.py).
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "mano_layout.h"

namespace mano {

// IEEE binary16 bits of a float, round to nearest even (host side of the
// f16x3 operand split; overflow saturates to infinity, tiny values go
// subnormal).
uint16_t f16_bits(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) return uint16_t(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0u));
  if (absx >= 0x477ff000u) return uint16_t(sign | 0x7c00u);  // rounds past 65504
  if (absx < 0x38800000u) {  // below the smallest normal half (2^-14): subnormal or zero
    const float a = std::fabs(f) * 16777216.0f;  // units of 2^-24, exact scaling
    const float r = std::nearbyint(a);           // default rounding mode: to nearest even
    return uint16_t(sign | uint32_t(r));
  }
  const uint32_t mant = absx & 0x7fffffu;
  uint32_t h = ((absx >> 23) - 112u) << 10 | (mant >> 13);
  const uint32_t rest = mant & 0x1fffu;
  if (rest > 0x1000u || (rest == 0x1000u && (h & 1u))) ++h;
  return uint16_t(sign | h);
}

float f16_value(uint16_t h) {
  const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  float v = e == 0 ? std::ldexp(float(m), -24) : std::ldexp(float(m | 0x400u), int(e) - 25);
  if (e == 31) v = m ? NAN : INFINITY;
  return (h & 0x8000u) ? -v : v;
}

namespace {

__attribute__((format(printf, 2, 3))) bool set_error(std::string& error, const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  error = buf;
  return false;
}

void split_f16(double x, uint16_t& hi, uint16_t& lo) {
  const float xf = float(x);
  hi = f16_bits(xf);
  lo = f16_bits(xf - f16_value(hi));
}

}  // namespace

bool pack_model(int n_verts, const double* mesh_template, const double* mesh_shape_basis,
                const double* mesh_pose_basis, const double* j_regressor,
                const double* skinning_weights, const int32_t* parents,
                const double* pose_pca_basis, const double* pose_pca_mean, HostModel& out,
                std::string& error) {
  if (n_verts < 32 || n_verts > (1 << 24)) return set_error(error, "n_verts %d out of range [32, 2^24]", n_verts);
  if (!mesh_template || !mesh_shape_basis || !mesh_pose_basis || !j_regressor || !skinning_weights ||
      !parents)
    return set_error(error, "a required model array is NULL");
  if ((pose_pca_basis == nullptr) != (pose_pca_mean == nullptr))
    return set_error(error, "pose_pca_basis and pose_pca_mean must both be given or both NULL");
  if (parents[0] != -1) return set_error(error, "parents[0] must be -1 (root)");
  std::vector<int32_t> depth(kJoints, 0);
  int max_depth = 0;
  for (int i = 1; i < kJoints; ++i) {
    if (parents[i] < 0 || parents[i] >= i)
      return set_error(error, "parents[%d] = %d must satisfy 0 <= p < %d", i, parents[i], i);
    depth[i] = depth[parents[i]] + 1;
    if (depth[i] > max_depth) max_depth = depth[i];
  }

  const int V = n_verts;
  const int n_cols = 3 * V;
  const int n_col_tiles = (n_cols + kColTile - 1) / kColTile;

  // ---- host float64 folds (J regression into beta space, mano_np.py:83) ----
  std::vector<float> jt(kJoints * 3), js(kJoints * 3 * kShape);
  for (int j = 0; j < kJoints; ++j) {
    for (int c = 0; c < 3; ++c) {
      double acc = 0.0;
      for (int v = 0; v < V; ++v) acc += j_regressor[size_t(j) * V + v] * mesh_template[size_t(v) * 3 + c];
      jt[j * 3 + c] = float(acc);
      for (int s = 0; s < kShape; ++s) {
        double a2 = 0.0;
        for (int v = 0; v < V; ++v)
          a2 += j_regressor[size_t(j) * V + v] * mesh_shape_basis[(size_t(v) * 3 + c) * kShape + s];
        js[(j * 3 + c) * kShape + s] = float(a2);
      }
    }
  }

  // ---- blend basis as MFMA B-fragment tiles ----
  // tile t, group g, lane l, slot q  <-  Basis[k = 2(4g+q) + (l>>5)][col = 32t + (l&31)]
  auto fill_tiles = [&](auto col_of, float* tiles) {
    for (int t = 0; t < n_col_tiles; ++t)
      for (int g = 0; g < kKGroups; ++g)
        for (int l = 0; l < 64; ++l)
          for (int q = 0; q < 4; ++q) {
            const int k = 2 * (4 * g + q) + (l >> 5);
            const int col = col_of(t, l & 31);
            float v = 0.f;
            if (col < n_cols) {
              if (k < kShape)
                v = float(mesh_shape_basis[size_t(col) * kShape + k]);
              else if (k < kK)
                v = float(mesh_pose_basis[size_t(col) * kPoseFeats + (k - kShape)]);
              else if (k == kK)
                v = float(mesh_template[col]);  // multiplied by X[:, 145] = 1
            }
            tiles[((size_t(t) * kKGroups + g) * 64 + l) * 4 + q] = v;
          }
  };
  std::vector<float> tiles(size_t(n_col_tiles) * kTileFloats, 0.f);
  fill_tiles([&](int t, int j) { return t * kColTile + j; }, tiles.data());
  // ... and their sector-aligned variants (mano_layout.h aligned_tile_col)
  bool col_variants_ok = true;
  for (int sg = 0; sg < kAlignVariants; ++sg)
    col_variants_ok = col_variants_ok && aligned_col_variant_ok(n_cols, sg, n_col_tiles);
  std::vector<float> tiles_v;
  if (col_variants_ok) {
    tiles_v.assign(size_t(kAlignVariants) * tiles.size(), 0.f);
    for (int sg = 0; sg < kAlignVariants; ++sg)
      fill_tiles([&](int t, int j) { return aligned_tile_col(n_cols, sg, t, j); }, tiles_v.data() + sg * tiles.size());
  }
  // 16x16x4 fused layout: group g = 16 vertices from min(16g, V-16); and
  // the sector-aligned variants (mano_layout.h aligned_group_vertex).
  const int n_groups16 = (V + 15) / 16;
  auto fill16 = [&](auto vertex_of, float* b16, float* w16) {
    for (int g = 0; g < n_groups16; ++g) {
      for (int l = 0; l < 64; ++l) {
        const int v = vertex_of(g, l & 15);
        for (int st = 0; st < 4; ++st)
          if (v < V)
            w16[size_t(g) * kWFrag16Floats + l * 4 + st] =
                float(skinning_weights[size_t(v) * kJoints + 4 * st + (l >> 4)]);
        for (int q = 0; q < 3; ++q)
          for (int gg = 0; gg < kGroups16; ++gg)
            for (int qq = 0; qq < 4; ++qq) {
              const int k = 4 * (4 * gg + qq) + (l >> 4);
              float val = 0.f;
              if (k <= kK && v < V) {
                const size_t colv = size_t(v) * 3 + q;
                val = k < kShape ? float(mesh_shape_basis[colv * kShape + k])
                      : k < kK   ? float(mesh_pose_basis[colv * kPoseFeats + (k - kShape)])
                                 : float(mesh_template[colv]);
              }
              b16[((size_t(g) * 3 + q) * kGroups16 + gg) * 256 + l * 4 + qq] = val;
            }
      }
    }
  };
  std::vector<float> b16(size_t(n_groups16) * 3 * kTile16Floats, 0.f);
  std::vector<float> w16(size_t(n_groups16) * kWFrag16Floats, 0.f);
  fill16([&](int g, int col) { return std::max(0, std::min(16 * g, V - 16)) + col; }, b16.data(), w16.data());
  bool variants_ok = true;
  for (int sh = 0; sh < kAlignVariants; ++sh) variants_ok = variants_ok && aligned_variant_ok(V, sh, n_groups16);
  std::vector<float> b16v, w16v;
  if (variants_ok) {
    b16v.assign(size_t(kAlignVariants) * b16.size(), 0.f);
    w16v.assign(size_t(kAlignVariants) * w16.size(), 0.f);
    for (int sh = 0; sh < kAlignVariants; ++sh)
      fill16([&](int g, int col) { return aligned_group_vertex(V, sh, g, col); }, b16v.data() + sh * b16.size(),
             w16v.data() + sh * w16.size());
  }
  // f16x3 pieces (mano_internal.h): basis x 2^basis_exp with the largest
  // entry at most 2^14, split hi/lo; weights x 2^kH3WeightExp.
  double bmax = 0.0;
  for (size_t i = 0; i < size_t(V) * 3 * kShape; ++i) bmax = std::max(bmax, std::fabs(mesh_shape_basis[i]));
  for (size_t i = 0; i < size_t(V) * 3 * kPoseFeats; ++i) bmax = std::max(bmax, std::fabs(mesh_pose_basis[i]));
  for (size_t i = 0; i < size_t(V) * 3; ++i) bmax = std::max(bmax, std::fabs(mesh_template[i]));
  const int basis_exp = bmax > 0.0 ? 14 - int(std::ceil(std::log2(bmax))) : 0;
  const double bscale = std::ldexp(1.0, basis_exp), wscale = std::ldexp(1.0, kH3WeightExp);
  auto fill_h3 = [&](auto vertex_of, uint16_t* bh3) {
    for (int g = 0; g < n_groups16; ++g) {
      uint16_t* G = bh3 + size_t(g) * kH3GroupHalves;
      for (int l = 0; l < 64; ++l) {
        const int v = vertex_of(g, l & 15);
        for (int j = 0; j < 8; ++j) {
          const int kq = 8 * (l >> 4) + j;  // K index inside a 32-step
          for (int c = 0; c < 3; ++c)
            for (int s = 0; s < kH3Steps; ++s) {
              const int k = 32 * s + kq;
              double val = 0.0;
              if (k <= kK && v < V) {
                const size_t colv = size_t(v) * 3 + c;
                val = k < kShape ? mesh_shape_basis[colv * kShape + k]
                      : k < kK   ? mesh_pose_basis[colv * kPoseFeats + (k - kShape)]
                                 : mesh_template[colv];
              }
              uint16_t hi, lo;
              split_f16(val * bscale, hi, lo);
              G[(size_t((2 * c) * kH3Steps + s) * 64 + l) * 8 + j] = hi;
              G[(size_t((2 * c + 1) * kH3Steps + s) * 64 + l) * 8 + j] = lo;
            }
          uint16_t hi, lo;
          split_f16(skinning_weights[size_t(v) * kJoints + (kq & 15)] * wscale, hi, lo);
          G[(size_t(kH3WPiece) * 64 + l) * 8 + j] = hi;                       // [Wh ; Wh]
          G[(size_t(kH3WPiece + 1) * 64 + l) * 8 + j] = kq < 16 ? lo : 0;     // [Wl ; 0]
        }
      }
    }
  };
  std::vector<uint16_t> bh3(size_t(n_groups16) * kH3GroupHalves, 0);
  fill_h3([&](int g, int col) { return std::max(0, std::min(16 * g, V - 16)) + col; }, bh3.data());
  std::vector<uint16_t> bh3v;
  if (variants_ok) {
    bh3v.assign(size_t(kAlignVariants) * bh3.size(), 0);
    for (int sh = 0; sh < kAlignVariants; ++sh)
      fill_h3([&](int g, int col) { return aligned_group_vertex(V, sh, g, col); }, bh3v.data() + sh * bh3.size());
  }
  std::vector<float> wts(size_t(V) * kJoints);
  for (size_t i = 0; i < wts.size(); ++i) wts[i] = float(skinning_weights[i]);
  std::vector<float> pca(kPca * kPca, 0.f), pmean(kPca, 0.f);
  if (pose_pca_basis) {
    for (int i = 0; i < kPca * kPca; ++i) pca[i] = float(pose_pca_basis[i]);
    for (int i = 0; i < kPca; ++i) pmean[i] = float(pose_pca_mean[i]);
  }


  out.tiles = std::move(tiles);
  out.tiles_v = std::move(tiles_v);
  out.b16 = std::move(b16);
  out.w16 = std::move(w16);
  out.b16v = std::move(b16v);
  out.w16v = std::move(w16v);
  out.bh3 = std::move(bh3);
  out.bh3v = std::move(bh3v);
  out.weights = std::move(wts);
  out.jt = std::move(jt);
  out.js = std::move(js);
  out.pca = std::move(pca);
  out.pmean = std::move(pmean);
  out.depth = std::move(depth);
  out.max_depth = max_depth;
  out.n_groups16 = n_groups16;
  out.n_col_tiles = n_col_tiles;
  out.basis_exp = basis_exp;
  return true;
}

}  // namespace mano
