// pack_check.cpp -- CPU check of the host-side model packing (mano_pack.cpp),
// built by tests/test_pack_sanitize.py with g++ -fsanitize=address,undefined.
//
// For several mesh sizes (the 778-vertex MANO mesh and small meshes that hit
// every tail-group case) it packs a random dump-layout model and decodes every
// fragment layout back to the model arrays it came from (mano_layout.h):
// blend_kernel tiles, blend_skin16 basis / weight fragments, the f16x3 pieces
// (hi + lo == the scaled value to 2^-22 relative), the float64 J folds
// (mano_np.py:83), then checks the argument errors.  Exit status 0 = all good.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mano_layout.h"

using namespace mano;

namespace {

int g_fail = 0;
#define EXPECT(cond, ...)                     \
  do {                                        \
    if (!(cond)) {                            \
      if (g_fail < 20) {                      \
        printf("FAIL %s:%d: ", __FILE__, __LINE__); \
        printf(__VA_ARGS__);                  \
        printf("\n");                         \
      }                                       \
      ++g_fail;                               \
    }                                         \
  } while (0)

struct Rng {
  uint64_t s;
  double uniform() {  // [-1, 1)
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return double(s >> 11) / double(1ull << 52) - 1.0;
  }
};

const int32_t kParents[16] = {-1, 0, 1, 2, 0, 4, 5, 0, 7, 8, 0, 10, 11, 0, 13, 14};

void check_mesh(int V, uint64_t seed) {
  Rng rng{seed};
  std::vector<double> tmpl(size_t(V) * 3), sd(size_t(V) * 3 * kShape), pd(size_t(V) * 3 * kPoseFeats),
      jr(size_t(kJoints) * V), w(size_t(V) * kJoints), pca(kPca * kPca), mean(kPca);
  for (auto& x : tmpl) x = 0.05 * rng.uniform();
  for (auto& x : sd) x = 5e-3 * rng.uniform();
  for (auto& x : pd) x = 2e-3 * rng.uniform();
  for (auto& x : jr) x = std::fabs(rng.uniform()) / V;
  for (auto& x : w) x = std::fabs(rng.uniform()) / kJoints;
  for (auto& x : pca) x = rng.uniform();
  for (auto& x : mean) x = 0.1 * rng.uniform();
  HostModel hm;
  std::string err;
  const bool ok = pack_model(V, tmpl.data(), sd.data(), pd.data(), jr.data(), w.data(), kParents, pca.data(),
                             mean.data(), hm, err);
  EXPECT(ok, "V=%d pack_model failed: %s", V, err.c_str());
  if (!ok) return;
  const int n_cols = 3 * V, n_groups = (V + 15) / 16;
  EXPECT(hm.n_groups16 == n_groups && hm.n_col_tiles == (n_cols + 31) / 32 && hm.max_depth == 3,
         "V=%d geometry %d %d %d", V, hm.n_groups16, hm.n_col_tiles, hm.max_depth);
  // Row k of the combined basis [S ; P ; template] at column col = 3 v + c.
  auto basis = [&](int k, int col) -> double {
    if (k < kShape) return sd[size_t(col) * kShape + k];
    if (k < kK) return pd[size_t(col) * kPoseFeats + (k - kShape)];
    if (k == kK) return tmpl[col];
    return 0.0;
  };
  // blend_kernel tiles: tile t, group g, lane l, slot q <- B[k = 2(4g+q) + (l>>5)][32t + (l&31)]
  EXPECT(hm.tiles.size() == size_t(hm.n_col_tiles) * kTileFloats, "tiles size");
  for (int t = 0; t < hm.n_col_tiles; ++t)
    for (int g = 0; g < kKGroups; ++g)
      for (int l = 0; l < 64; ++l)
        for (int q = 0; q < 4; ++q) {
          const int k = 2 * (4 * g + q) + (l >> 5), col = 32 * t + (l & 31);
          const float want = col < n_cols ? float(basis(k, col)) : 0.f;
          const float got = hm.tiles[((size_t(t) * kKGroups + g) * 64 + l) * 4 + q];
          EXPECT(got == want, "V=%d tile %d g %d l %d q %d: %g vs %g", V, t, g, l, q, got, want);
        }
  // the blend tiles' sector-aligned variants: present iff every sigma fits;
  // variant sigma tile t lane j holds aligned_tile_col's column (zero past
  // the row end); every column is covered exactly once; for a row at float
  // phase c the tiles t < ta of variant (8 - c) mod 8 start on a sector
  bool cols_ok = true;
  for (int sg = 0; sg < kAlignVariants; ++sg) cols_ok = cols_ok && aligned_col_variant_ok(n_cols, sg, hm.n_col_tiles);
  EXPECT(cols_ok == !hm.tiles_v.empty(), "V=%d column variants present %d", V, int(cols_ok));
  if (V == 778) EXPECT(cols_ok, "V=778 must have every column variant");
  for (int sg = 0; sg < kAlignVariants && !hm.tiles_v.empty(); ++sg) {
    std::vector<int> cnt(n_cols, 0);
    for (int t = 0; t < hm.n_col_tiles; ++t)
      for (int l = 0; l < 64; ++l) {
        const int col = aligned_tile_col(n_cols, sg, t, l & 31);
        if (l < 32 && col < n_cols) ++cnt[col];
        if (t < (n_cols - sg) / 32 && l == 0) EXPECT((unsigned(col) + 8u - unsigned(sg)) % 8 == 0, "col phase");
        for (int g = 0; g < kKGroups; ++g)
          for (int q = 0; q < 4; ++q) {
            const int k = 2 * (4 * g + q) + (l >> 5);
            const float want = col < n_cols ? float(basis(k, col)) : 0.f;
            EXPECT(hm.tiles_v[(((size_t(sg) * hm.n_col_tiles + t) * kKGroups + g) * 64 + l) * 4 + q] == want,
                   "V=%d tiles_v s %d t %d l %d k %d", V, sg, t, l, k);
          }
      }
    for (int c = 0; c < n_cols; ++c) EXPECT(cnt[c] == 1, "V=%d sigma %d column %d covered %d times", V, sg, c, cnt[c]);
  }
  for (unsigned phase = 0; phase < 8; ++phase) {
    const int sg = int(aligned_col_shifts(V, phase, 0) & 15u);
    EXPECT((phase + unsigned(sg)) % 8 == 0, "V=%d column shift of phase %u", V, phase);
  }
  // blend_skin16 fragments: group g covers vertices vb..vb+15, vb = min(16g, V-16)
  EXPECT(hm.b16.size() == size_t(n_groups) * 3 * kTile16Floats && hm.w16.size() == size_t(n_groups) * 256,
         "b16/w16 size");
  for (int g = 0; g < n_groups; ++g) {
    const int vb = std::min(16 * g, V - 16);
    for (int l = 0; l < 64; ++l) {
      const int v = vb + (l & 15);
      for (int st = 0; st < 4; ++st) {
        const float want = float(w[size_t(v) * kJoints + 4 * st + (l >> 4)]);
        EXPECT(hm.w16[size_t(g) * 256 + l * 4 + st] == want, "V=%d w16 g %d l %d", V, g, l);
      }
      for (int c = 0; c < 3; ++c)
        for (int gg = 0; gg < kGroups16; ++gg)
          for (int qq = 0; qq < 4; ++qq) {
            const int k = 4 * (4 * gg + qq) + (l >> 4);
            const float want = k <= kK ? float(basis(k, 3 * v + c)) : 0.f;
            const float got = hm.b16[((size_t(g) * 3 + c) * kGroups16 + gg) * 256 + l * 4 + qq];
            EXPECT(got == want, "V=%d b16 g %d c %d k %d: %g vs %g", V, g, c, k, got, want);
          }
    }
  }
  // sector-aligned variants (mano_layout.h): present iff every shift fits V;
  // variant s group g lane col holds aligned_group_vertex's vertex; the
  // groups of a variant cover every vertex; for a row at float phase c the
  // groups g < ga of variant (-3 c) mod 8 start on a sector boundary.
  bool all_ok = true;
  for (int sh = 0; sh < kAlignVariants; ++sh) all_ok = all_ok && aligned_variant_ok(V, sh, n_groups);
  EXPECT(all_ok == !hm.b16v.empty() && hm.b16v.size() == hm.w16v.size() * 3 * kTile16Floats / kWFrag16Floats,
         "V=%d variants present %d, sizes %zu %zu", V, int(all_ok), hm.b16v.size(), hm.w16v.size());
  if (V == 778) EXPECT(all_ok, "V=778 must have every aligned variant");
  for (int sh = 0; sh < kAlignVariants && !hm.b16v.empty(); ++sh) {
    const int ga = (V - sh) / 16;
    std::vector<int> seen(V, 0);
    for (int g = 0; g < n_groups; ++g)
      for (int l = 0; l < 64; ++l) {
        const int v = aligned_group_vertex(V, sh, g, l & 15);
        EXPECT(v >= 0 && v < V, "V=%d s %d g %d col %d vertex %d", V, sh, g, l & 15, v);
        if (v < 0 || v >= V) continue;
        seen[v] = 1;
        if (g < ga) EXPECT(v == sh + 16 * g + (l & 15), "V=%d s %d aligned group %d", V, sh, g);
        for (int st = 0; st < 4; ++st)
          EXPECT(hm.w16v[(size_t(sh) * n_groups + g) * 256 + l * 4 + st] ==
                     float(w[size_t(v) * kJoints + 4 * st + (l >> 4)]), "V=%d w16v s %d g %d l %d", V, sh, g, l);
        for (int c = 0; c < 3; ++c)
          for (int gg = 0; gg < kGroups16; ++gg)
            for (int qq = 0; qq < 4; ++qq) {
              const int k = 4 * (4 * gg + qq) + (l >> 4);
              const float want = k <= kK ? float(basis(k, 3 * v + c)) : 0.f;
              EXPECT(hm.b16v[(((size_t(sh) * n_groups + g) * 3 + c) * kGroups16 + gg) * 256 + l * 4 + qq] == want,
                     "V=%d b16v s %d g %d c %d k %d", V, sh, g, c, k);
            }
      }
    for (int v = 0; v < V; ++v) EXPECT(seen[v], "V=%d s %d vertex %d not covered", V, sh, v);
  }
  for (unsigned phase = 0; phase < 8; ++phase) {
    const int sh = int(aligned_shifts(V, phase, 0) & 15u);
    for (int g = 0; g < (V - sh) / 16; ++g)
      EXPECT((phase + 3 * unsigned(aligned_group_vertex(V, sh, g, 0))) % 8 == 0, "V=%d phase %u group %d", V, phase, g);
  }
  // blend_skin16's residue-class hand tiles: over every quad and wave, the
  // rows cover each hand of the batch, only hands of the batch, and a
  // quad's rows all share one class; rows of class r sit at the phase its
  // shift aligns.
  const int lp = aligned_period_log2(V);
  const int kGeom[3][3] = {{6, 4, 4}, {7, 5, 4}, {7, 4, 8}};  // lq, lt, waves: blend_skin16, blend, blend_skin_h3
  for (const auto& geo : kGeom)
  for (int64_t n : {1, 2, 3, 5, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 1000, 1027, 4097}) {
    const int lq = geo[0], lt = geo[1], waves = geo[2];
    std::vector<int> hit(size_t(n), 0);
    const int64_t nq = aligned_n_quads(n, lp, lq);
    const int T = 1 << lt;
    for (int64_t q = 0; q < nq; ++q)
      for (int wv = 0; wv < waves; ++wv) {
        const AlignedTile t = aligned_tile(n, lp, q, wv, lq, lt);
        EXPECT(t.n_valid >= 1 && t.n_valid <= T && t.h0 >= 0 && t.h0 < n, "V=%d n %lld q %lld w %d", V,
               (long long)n, (long long)q, wv);
        for (int i = 0; i < T; ++i) {
          const int64_t h = t.h0 + (int64_t(i < t.n_valid ? i : t.n_valid - 1) << lp);
          EXPECT(h >= 0 && h < n && (h & ((1 << lp) - 1)) == t.cls, "V=%d n %lld hand %lld", V, (long long)n,
                 (long long)h);
          if (h >= 0 && h < n) hit[size_t(h)] = 1;
        }
      }
    for (int64_t h = 0; h < n; ++h) EXPECT(hit[size_t(h)], "V=%d n %lld hand %lld not covered", V, (long long)n, (long long)h);
    for (unsigned a = 0; a < 8; ++a) {
      const unsigned code = aligned_shifts(V, a, lp);
      for (int64_t h = 0; h < 64 && h < n; ++h) {
        const int sh = int((code >> (4 * (h & ((1 << lp) - 1)))) & 15u);
        EXPECT((a + 3u * unsigned(V) * unsigned(h) + 3u * unsigned(sh)) % 8 == 0, "V=%d a %u hand %lld", V, a,
               (long long)h);
      }
    }
  }
  // f16x3 pieces: hi + lo of the basis x 2^basis_exp and of the weights x 2^kH3WeightExp
  const double bscale = std::ldexp(1.0, hm.basis_exp), wscale = std::ldexp(1.0, kH3WeightExp);
  EXPECT(hm.bh3.size() == size_t(n_groups) * kH3GroupHalves, "bh3 size");
  double worst = 0.0;
  for (int g = 0; g < n_groups; ++g) {
    const int vb = std::min(16 * g, V - 16);
    const uint16_t* G = hm.bh3.data() + size_t(g) * kH3GroupHalves;
    for (int l = 0; l < 64; ++l) {
      const int v = vb + (l & 15);
      for (int j = 0; j < 8; ++j) {
        const int kq = 8 * (l >> 4) + j;
        for (int c = 0; c < 3; ++c)
          for (int s = 0; s < kH3Steps; ++s) {
            const int k = 32 * s + kq;
            const double x = (k <= kK ? basis(k, 3 * v + c) : 0.0) * bscale;
            const double hi = f16_value(G[(size_t((2 * c) * kH3Steps + s) * 64 + l) * 8 + j]);
            const double lo = f16_value(G[(size_t((2 * c + 1) * kH3Steps + s) * 64 + l) * 8 + j]);
            const double e = std::fabs(hi + lo - x);
            worst = std::max(worst, e / std::max(std::fabs(x), 1e-30));
            EXPECT(e <= std::ldexp(std::fabs(x), -21) + std::ldexp(1.0, -24), "V=%d h3 basis g %d k %d: %g vs %g",
                   V, g, k, hi + lo, x);
          }
        const double x = w[size_t(v) * kJoints + (kq & 15)] * wscale;
        const double hi = f16_value(G[(size_t(kH3WPiece) * 64 + l) * 8 + j]);
        const double lo = f16_value(G[(size_t(kH3WPiece + 1) * 64 + l) * 8 + j]);
        EXPECT(std::fabs(hi - f16_value(f16_bits(float(x)))) == 0.0, "V=%d h3 Wh", V);
        if (kq < 16) EXPECT(std::fabs(hi + lo - x) <= std::ldexp(std::fabs(x), -21) + std::ldexp(1.0, -24), "V=%d h3 W", V);
        else EXPECT(lo == 0.0, "V=%d h3 [Wl ; 0] upper half", V);
      }
    }
  }
  EXPECT(hm.bh3.size() > 0 && std::ldexp(1.0, 14 - hm.basis_exp) >= 5e-3, "basis_exp %d", hm.basis_exp);
  // f16x3 sector-aligned variants: present with the fp32 ones; piece entries
  // of variant s decode to aligned_group_vertex's vertex
  EXPECT(hm.bh3v.empty() == hm.b16v.empty() && (hm.bh3v.empty() || hm.bh3v.size() == kAlignVariants * hm.bh3.size()),
         "V=%d bh3v size %zu", V, hm.bh3v.size());
  for (int sh = 0; sh < kAlignVariants && !hm.bh3v.empty(); ++sh)
    for (int g = 0; g < n_groups; ++g) {
      const uint16_t* G = hm.bh3v.data() + (size_t(sh) * n_groups + g) * kH3GroupHalves;
      for (int l = 0; l < 64; ++l) {
        const int v = aligned_group_vertex(V, sh, g, l & 15);
        for (int j = 0; j < 8; ++j) {
          const int kq = 8 * (l >> 4) + j;
          for (int c = 0; c < 3; ++c)
            for (int st = 0; st < kH3Steps; ++st) {
              const int k = 32 * st + kq;
              const double x = (k <= kK ? basis(k, 3 * v + c) : 0.0) * bscale;
              const double hi = f16_value(G[(size_t((2 * c) * kH3Steps + st) * 64 + l) * 8 + j]);
              const double lo = f16_value(G[(size_t((2 * c + 1) * kH3Steps + st) * 64 + l) * 8 + j]);
              EXPECT(std::fabs(hi + lo - x) <= std::ldexp(std::fabs(x), -21) + std::ldexp(1.0, -24),
                     "V=%d bh3v s %d g %d k %d", V, sh, g, k);
            }
          const double wx = w[size_t(v) * kJoints + (kq & 15)] * wscale;
          EXPECT(f16_value(G[(size_t(kH3WPiece) * 64 + l) * 8 + j]) == f16_value(f16_bits(float(wx))),
                 "V=%d bh3v Wh s %d g %d", V, sh, g);
        }
      }
    }
  // J folds in float64 (mano_np.py:83)
  for (int j = 0; j < kJoints; ++j)
    for (int c = 0; c < 3; ++c) {
      double acc = 0.0;
      for (int v = 0; v < V; ++v) acc += jr[size_t(j) * V + v] * tmpl[size_t(v) * 3 + c];
      EXPECT(hm.jt[j * 3 + c] == float(acc), "jt");
      for (int s = 0; s < kShape; ++s) {
        double a2 = 0.0;
        for (int v = 0; v < V; ++v) a2 += jr[size_t(j) * V + v] * sd[(size_t(v) * 3 + c) * kShape + s];
        EXPECT(hm.js[(j * 3 + c) * kShape + s] == float(a2), "js");
      }
    }
  EXPECT(hm.pca[7] == float(pca[7]) && hm.pmean[44] == float(mean[44]), "pca copy");
  printf("V=%4d ok: %zu tile + %zu b16 + %zu bh3 entries decoded, f16x3 worst rel %.2e\n", V, hm.tiles.size(),
         hm.b16.size(), hm.bh3.size(), worst);
}

void check_errors() {
  std::vector<double> a(size_t(64) * 3 * kPoseFeats, 0.0);
  HostModel hm;
  std::string err;
  int32_t bad_par[16];
  for (int i = 0; i < 16; ++i) bad_par[i] = kParents[i];
  bad_par[5] = 9;
  EXPECT(!pack_model(64, a.data(), a.data(), a.data(), a.data(), a.data(), bad_par, nullptr, nullptr, hm, err) &&
             err.find("parents[5]") != std::string::npos, "bad parents: %s", err.c_str());
  EXPECT(!pack_model(31, a.data(), a.data(), a.data(), a.data(), a.data(), kParents, nullptr, nullptr, hm, err),
         "V < 32 accepted");
  EXPECT(!pack_model(64, nullptr, a.data(), a.data(), a.data(), a.data(), kParents, nullptr, nullptr, hm, err),
         "NULL template accepted");
  EXPECT(!pack_model(64, a.data(), a.data(), a.data(), a.data(), a.data(), kParents, a.data(), nullptr, hm, err),
         "PCA basis without mean accepted");
  EXPECT(pack_model(64, a.data(), a.data(), a.data(), a.data(), a.data(), kParents, nullptr, nullptr, hm, err) &&
             hm.pca.size() == size_t(kPca * kPca) && hm.pca[0] == 0.f,
         "model without PCA arrays: %s", err.c_str());
  // f16 conversions at the edges
  EXPECT(f16_bits(65504.f) == 0x7bff && f16_bits(1e6f) == 0x7c00 && f16_bits(-0.f) == 0x8000, "f16 edges");
  EXPECT(f16_value(f16_bits(std::ldexp(1.f, -24))) == std::ldexp(1.f, -24), "f16 subnormal");
  printf("argument errors ok\n");
}

}  // namespace

int main() {
  for (int V : {32, 50, 64, 100, 130, 200, 778}) check_mesh(V, 1000 + V);
  check_errors();
  if (g_fail) printf("%d failures\n", g_fail);
  return g_fail ? 1 : 0;
}
