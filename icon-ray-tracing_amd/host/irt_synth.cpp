// irt_synth.cpp -- synthetic RnBk icosahedral ICON grids in the `.ic` record format.
//
// Real DWD ICON data (netCDF grid + HHL + fields) is not available offline and the
// reference's converter (tools/convert_icon/convert_icon.cpp) needs netCDF, so benches and
// tests use this generator.  Construction (deterministic, double precision, then rounded
// to float like convert_icon.cpp:356-358 does for clat/clon):
//  - icosahedron from (0,+-1,+-phi) and its cyclic permutations, normalised; faces oriented
//    counter-clockwise seen from outside (the orientation sample()'s "> 0 => outside"
//    plane tests expect, ICONGrid.h:201-203);
//  - root split: every face into rootN^2 triangles on a barycentric lattice, vertices
//    projected to the unit sphere; then `bisections` rounds of 4-way edge-midpoint
//    splitting (midpoints normalised).  20*rootN^2*4^bisections triangles (R2B07: 1.31 M);
//  - corners: lat = asin(z), lon = atan2(y, x) (toSpherical, ICONGrid.h:36-42);
//  - levels: H_l = R + top*(l/L)^2, R = 6.371229e6 m (convert_icon.cpp:359), HSURF = 0;
//  - value of layer l of a column with centre c: 0.5 + 0.35 sin(4cx+3cy) cos(5cz)(1-h)
//    + 0.1 h + noise*(hash(column,l)-0.5), h = (l+0.5)/L, normalised to [0,1] over the
//    grid (convert_icon.cpp:317-328 normalises its fields the same way);
//  - records of <= 31 layers (MAX_LAYERS 32, ICONGrid.h:57), bottom to top, consecutive
//    per column, the layer boundary height shared by neighbouring records
//    (convert_icon.cpp:362-388).
// Terrain (terrainHeight > 0, irt_synth_grid_terrain): synthetic DWD-like fields run through
// convert_icon's `.ic` branch (convert_icon.cpp:353-391) expression by expression --
//  - HSURF per column: terrainHeight * max(0, m)^1.5 of a smooth field m of the column centre
//    plus hash noise, clamped to [0, 1] (~60 % of the columns are land, 0 m elsewhere);
//  - HHL of half level k = 1..levels above the ground: z_k + HSURF (1 - z_k / Zd)^2 (z_k < Zd,
//    Zd = min(top, 20 km)), z_k = top (k/L)^2: terrain-following near the ground, flat above
//    (SLEVE-like), monotone in k since 2 HSURF < Zd;
//  - records as convert_icon writes them: H[0] = R + HSURF for the first record of a column
//    (prevH, 361), H[j] = R + HHL - HSURF (371, double arithmetic rounded to float), so the
//    first layer of every land column is inverted (H[0] > H[1]); the last record of a column gets
//    levels % 32 - 1 layers (365: 90 levels -> 31 + 31 + 25); levels % 32 == 0 is refused (the
//    reference writes numLayers = -1, which irt_load_ic rejects).

#include <math.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "irt_internal.h"

namespace {

struct D3 {
  double x, y, z;
};
inline D3 add(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline D3 mul(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline double dotd(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline D3 crossd(D3 u, D3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
inline D3 unit(D3 a) { return mul(a, 1.0 / sqrt(dotd(a, a))); }

struct Tri {
  D3 a, b, c;
};

// Triangle `leaf` of the depth-first 4-way bisection of root t: children (a,ab,ca),
// (ab,b,bc), (ca,bc,c), (ab,bc,ca), the first level's choice in the leaf index's highest
// base-4 digit.  Every midpoint is computed from the same parent doubles as a recursive
// descent would, so any leaf comes out identical without generating the others.
Tri descend(Tri t, int depth, size_t leaf) {
  for (int d = depth - 1; d >= 0; --d) {
    const int c = (int)((leaf >> (2 * d)) & 3);
    const D3 ab = unit(add(t.a, t.b)), bc = unit(add(t.b, t.c)), ca = unit(add(t.c, t.a));
    if (c == 0) t = {t.a, ab, ca};
    else if (c == 1) t = {ab, t.b, bc};
    else if (c == 2) t = {ca, bc, t.c};
    else t = {ab, bc, ca};
  }
  return t;
}

inline uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// The grid generator: root triangles, level heights and the value normalisation once; then
// any range of records on demand (irt_create_synth streams them into HBM chunk by chunk).
struct SynthGen {
  int rootN = 0, bisections = 0, levels = 0, recsPerCol = 0;
  float noise = 0.f;
  uint32_t seed = 0;
  double terrain = 0.0, top = 0.0, zd = 0.0;  // terrain: max HSURF (0: flat grid)
  size_t numTris = 0, total = 0;
  std::vector<Tri> roots;
  std::vector<float> H;
  double vmin = INFINITY, vmax = -INFINITY, vscale = 0.0;

  int init(int rn, int bis, int lev, float topHeight, float nz, uint32_t sd, float terrainHeight = 0.f) {
    using irt::set_error;
    if (rn < 1 || bis < 0 || bis > 12 || lev < 1 || lev > 100000 || !(terrainHeight >= 0.f) ||
        (terrainHeight > 0.f && (lev % 32 == 0 || !(topHeight > 0.f) ||
                                 2.0 * terrainHeight >= std::min(20000.0, (double)topHeight)))) {
      set_error("irt_synth_grid: bad argument");
      return IRT_E_INVALID;
    }
    rootN = rn, bisections = bis, levels = lev, noise = nz, seed = sd;
    terrain = terrainHeight;
    top = topHeight;
    zd = std::min(20000.0, (double)topHeight);
    numTris = 20ull * rootN * rootN * (1ull << (2 * bisections));
    recsPerCol = (levels + 30) / 31;
    total = numTris * recsPerCol;
    const double phi = (1.0 + sqrt(5.0)) / 2.0;
    const D3 V[12] = {{-1, phi, 0}, {1, phi, 0}, {-1, -phi, 0}, {1, -phi, 0},
                      {0, -1, phi}, {0, 1, phi}, {0, -1, -phi}, {0, 1, -phi},
                      {phi, 0, -1}, {phi, 0, 1}, {-phi, 0, -1}, {-phi, 0, 1}};
    const int F[20][3] = {{0, 11, 5}, {0, 5, 1},  {0, 1, 7},   {0, 7, 10}, {0, 10, 11},
                          {1, 5, 9},  {5, 11, 4}, {11, 10, 2}, {10, 7, 6}, {7, 1, 8},
                          {3, 9, 4},  {3, 4, 2},  {3, 2, 6},   {3, 6, 8},  {3, 8, 9},
                          {4, 9, 5},  {2, 4, 11}, {6, 2, 10},  {8, 6, 7},  {9, 8, 1}};
    roots.clear();
    roots.reserve(20 * rootN * rootN);
    for (int f = 0; f < 20; ++f) {
      D3 a = unit(V[F[f][0]]), b = unit(V[F[f][1]]), c = unit(V[F[f][2]]);
      if (dotd(crossd(sub(b, a), sub(c, a)), add(add(a, b), c)) < 0) std::swap(b, c);
      auto P = [&](int i, int j) {  // barycentric lattice point, on the sphere
        double s = (double)i / rootN, t = (double)j / rootN;
        return unit(add(a, add(mul(sub(b, a), s), mul(sub(c, a), t))));
      };
      for (int j = 0; j < rootN; ++j)
        for (int i = 0; i + j < rootN; ++i) {
          roots.push_back({P(i, j), P(i + 1, j), P(i, j + 1)});
          if (i + j + 1 < rootN) roots.push_back({P(i + 1, j), P(i + 1, j + 1), P(i, j + 1)});
        }
    }
    const float R = 6.371229E6f;
    H.assign(levels + 1, 0.f);
    for (int l = 0; l <= levels; ++l) {
      double f = (double)l / levels;
      H[l] = (float)((double)R + (double)topHeight * f * f);
    }
    // value range over the whole grid (min/max: any evaluation order gives the same)
    const int threads = irt::default_threads();
    std::vector<double> lo(threads, INFINITY), hi(threads, -INFINITY);
    std::vector<std::thread> ts;
    const size_t chunk = (numTris + threads - 1) / threads;
    for (int t = 0; t < threads; ++t)
      ts.emplace_back([&, t] {
        std::vector<double> v(levels);
        double l = INFINITY, h = -INFINITY;  // thread-local: no false sharing
        for (size_t k = t * chunk; k < std::min(numTris, (t + 1) * chunk); ++k) {
          values(k, v.data());
          for (double x : v) {
            l = std::min(l, x);
            h = std::max(h, x);
          }
        }
        lo[t] = l;
        hi[t] = h;
      });
    for (auto &t : ts) t.join();
    for (int t = 0; t < threads; ++t) {
      vmin = std::min(vmin, lo[t]);
      vmax = std::max(vmax, hi[t]);
    }
    vscale = vmax > vmin ? 1.0 / (vmax - vmin) : 0.0;
    return IRT_OK;
  }

  Tri tri(size_t t) const {
    const size_t per = (size_t)1 << (2 * bisections);
    return descend(roots[t / per], bisections, t % per);
  }

  // un-normalised values of column t's layers
  void values(size_t t, double *v) const {
    const Tri tr = tri(t);
    D3 c = unit(add(add(tr.a, tr.b), tr.c));
    double base = sin(4 * c.x + 3 * c.y) * cos(5 * c.z);
    for (int l = 0; l < levels; ++l) {
      double h = (l + 0.5) / levels;
      double x = 0.5 + 0.35 * base * (1 - h) + 0.1 * h;
      if (noise != 0.f) {
        uint32_t k = hash32((uint32_t)t * 2654435761u ^ hash32((uint32_t)l + seed * 97u));
        x += (double)noise * ((k >> 8) * (1.0 / 16777216.0) - 0.5);
      }
      v[l] = x;
    }
  }

  // HSURF of column t (terrain grids)
  double hsurf(size_t t) const {
    const Tri tr = tri(t);
    const D3 c = unit(add(add(tr.a, tr.b), tr.c));
    double m = 0.5 * (sin(11 * c.x + 2) * cos(9 * c.y - 1) + sin(7 * c.z + 3 * c.x) * cos(13 * c.y)) + 0.1;
    const uint32_t k = hash32((uint32_t)t * 0x9E3779B1u ^ (seed * 131u + 7u));
    m += 0.15 * ((k >> 8) * (1.0 / 16777216.0) - 0.5);
    m = std::min(m, 1.0);
    return m > 0.0 ? terrain * pow(m, 1.5) : 0.0;
  }
  // HHL of half level k (1..levels) above the ground of a column with surface height hs
  double hhl(int k, double hs) const {
    const double f = (double)k / levels, z = top * f * f;
    const double d = z < zd ? 1.0 - z / zd : 0.0;
    return z + hs * d * d;
  }
  // the column's records as convert_icon.cpp:356-388 writes them (terrain grids)
  void terrain_column(size_t t, const double *v, const float *lat, const float *lon, size_t first,
                      size_t count, irt_icon_cell *out) const {
    constexpr float R = 6.371229E6f;
    const double hs = hsurf(t);
    int valueIt = 0, hhlIt = 0;
    float prevH = R + hs;  // (361)
    for (int i = 0; i < recsPerCol; ++i) {
      int nl = 31;
      if ((i + 1) * nl > levels) nl = levels % 32 - 1;  // (364-366)
      float H[32] = {};
      float val[32] = {};
      H[0] = prevH;
      for (int j = 1; j <= nl; ++j) {
        ++hhlIt;
        H[j] = R + hhl(hhlIt, hs) - hs;  // (371): float + double - double, rounded to float
        prevH = H[j];
      }
      for (int j = 0; j < nl; ++j) val[j] = (float)((v[valueIt++] - vmin) * vscale);
      const size_t r = t * recsPerCol + i;
      if (r < first || r >= first + count) continue;
      irt_icon_cell &cell = out[r - first];
      memset(&cell, 0, sizeof(cell));
      memcpy(cell.lat, lat, 3 * sizeof(float));
      memcpy(cell.lon, lon, 3 * sizeof(float));
      cell.numLayers = nl;
      memcpy(cell.height, H, sizeof(H));
      memcpy(cell.value, val, sizeof(val));
    }
  }

  // records [first, first + count), in parallel over columns
  void fill(size_t first, size_t count, irt_icon_cell *out) const {
    if (!count) return;
    const size_t t0 = first / recsPerCol, t1 = (first + count - 1) / recsPerCol + 1;
    const int threads = count < 4096 ? 1 : irt::default_threads();
    std::vector<std::thread> ts;
    const size_t chunk = (t1 - t0 + threads - 1) / threads;
    for (int th = 0; th < threads; ++th)
      ts.emplace_back([&, th] {
        std::vector<double> v(levels);
        for (size_t t = t0 + th * chunk; t < std::min(t1, t0 + (th + 1) * chunk); ++t) {
          const Tri tr = tri(t);
          const D3 cs[3] = {tr.a, tr.b, tr.c};
          float lat[3], lon[3];
          for (int k = 0; k < 3; ++k) {
            double z = std::max(-1.0, std::min(1.0, cs[k].z));
            lat[k] = (float)asin(z);
            lon[k] = (float)atan2(cs[k].y, cs[k].x);
          }
          values(t, v.data());
          if (terrain > 0.0) {
            terrain_column(t, v.data(), lat, lon, first, count, out);
            continue;
          }
          for (int rc = 0; rc < recsPerCol; ++rc) {
            const size_t r = t * recsPerCol + rc;
            if (r < first || r >= first + count) continue;
            irt_icon_cell &cell = out[r - first];
            memset(&cell, 0, sizeof(cell));
            memcpy(cell.lat, lat, sizeof(lat));
            memcpy(cell.lon, lon, sizeof(lon));
            const int l0 = rc * 31;
            const int nl = std::min(31, levels - l0);
            cell.numLayers = nl;
            for (int j = 0; j <= nl; ++j) cell.height[j] = H[l0 + j];
            for (int j = 0; j < nl; ++j) cell.value[j] = (float)((v[l0 + j] - vmin) * vscale);
          }
        }
      });
    for (auto &t : ts) t.join();
  }
};

}  // namespace

namespace irt {
int synth_open(int rootN, int bisections, int levels, float topHeight, float noise, uint32_t seed,
               float terrainHeight, void **gen, size_t *total) {
  SynthGen *g = new SynthGen();
  int rc = g->init(rootN, bisections, levels, topHeight, noise, seed, terrainHeight);
  if (rc) {
    delete g;
    return rc;
  }
  *gen = g;
  *total = g->total;
  return IRT_OK;
}
void synth_fill(const void *gen, size_t first, size_t count, irt_icon_cell *out) {
  static_cast<const SynthGen *>(gen)->fill(first, count, out);
}
void synth_close(void *gen) { delete static_cast<SynthGen *>(gen); }
}  // namespace irt

extern "C" int irt_synth_grid_terrain(int rootN, int bisections, int levels, float topHeight,
                                      float noise, uint32_t seed, float terrainHeight,
                                      irt_icon_cell *out, size_t capacity, size_t *count) {
  using irt::set_error;
  if (!count) {
    set_error("irt_synth_grid: bad argument");
    return IRT_E_INVALID;
  }
  if (!out) {  // the count only: no value pass
    if (rootN < 1 || bisections < 0 || bisections > 12 || levels < 1 || levels > 100000) {
      set_error("irt_synth_grid: bad argument");
      return IRT_E_INVALID;
    }
    *count = 20ull * rootN * rootN * (1ull << (2 * bisections)) * ((levels + 30) / 31);
    return IRT_OK;
  }
  SynthGen g;
  int rc = g.init(rootN, bisections, levels, topHeight, noise, seed, terrainHeight);
  if (rc) return rc;
  *count = g.total;
  if (capacity < g.total) {
    set_error("irt_synth_grid: capacity %zu < %zu", capacity, g.total);
    return IRT_E_INVALID;
  }
  g.fill(0, g.total, out);
  return IRT_OK;
}

extern "C" int irt_synth_grid(int rootN, int bisections, int levels, float topHeight,
                              float noise, uint32_t seed, irt_icon_cell *out, size_t capacity,
                              size_t *count) {
  return irt_synth_grid_terrain(rootN, bisections, levels, topHeight, noise, seed, 0.f, out,
                                capacity, count);
}
