// irt_scene.cpp -- host preparation of the HBM-resident scene for the gfx950 kernels.
//
//  1. per record: the three side planes sample() builds on every call
//     (icon_rt/ICONGrid.h:187-199), computed ONCE here with the same glibc cosf/sinf and
//     the same float expression order, so the kernel's plane tests are bit-identical to
//     the reference's -- and the 12 sin/cos per cell test disappear from the hot loop;
//  2. per record: a 256-B height/value block for findHeight/getValue (ICONGrid.h:117-164);
//  3. the point locator replacing the reference's cell location (CPU: linear scan,
//     deviceCode.cu:116-123; GPU: OptiX/cuBQL, 58-115): a gnomonic cube map with G x G
//     cells per face, each cell listing every record whose column can contain a point of
//     that direction, sorted by record index.  Conservative by construction:
//       - the region sample() accepts is {r in [h0,hN]} x the cone of its three side
//         planes, i.e. the geodesic triangle of the corners (or, for clockwise corners,
//         its antipode -- handled);
//       - geodesic triangles are straight-edged under the gnomonic projection, so each is
//         rasterised per face by a separating-axis test against every grid cell, padded by
//         1e-5 in face coordinates (~60 m on the Earth; float error of the kernel's
//         direction->cell mapping and of the plane rounding is < 1e-6);
//       - triangles with an angular radius > 15 degrees (R1B00/R2B00-class grids) use a
//         cone-vs-cell test; degenerate records go into every list.
//     With lists sorted by index, the first list entry passing sample() IS the
//     reference's "lowest index wins" answer (deviceCode.cu:119-122).

#include <math.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>
#include <vector>

#include "irt_internal.h"

namespace irt {

namespace {

struct V3 {
  float x, y, z;
};
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 u, V3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
// toCartesian (ICONGrid.h:44-54)
inline V3 toCartesian(float r, float lat, float lon) {
  float x = r * cosf(lat) * cosf(lon);
  float y = r * cosf(lat) * sinf(lon);
  float z = r * sinf(lat);
  return {x, y, z};
}
// makePlane (ICONGrid.h:170-174)
inline Plane4 makePlane(V3 a, V3 b, V3 c) {
  V3 N = cross(b - a, c - a);
  return {N.x, N.y, N.z, dot(a, N)};
}
// evalPlane (ICONGrid.h:176-179)
inline float evalPlane(const Plane4 &p, float px, float py, float pz) {
  return (px * p.x + py * p.y + pz * p.z) - p.w;
}

struct D3 {
  double x, y, z;
};
inline double dotd(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline D3 unitd(D3 a) {
  double l = sqrt(dotd(a, a));
  return {a.x / l, a.y / l, a.z / l};
}
inline double comp(const D3 &d, int a) { return a == 0 ? d.x : a == 1 ? d.y : d.z; }

constexpr double kPadUV = 1e-5;          // face-coordinate padding
constexpr double kBigCap = 0.2617993878;  // 15 degrees

// Face f: axis f/2, sign +1 for even f; (u, v) axes as in cubemap_cell (irt_common.h).
inline void face_axes(int f, int &ax, int &ua, int &va, double &s) {
  ax = f / 2;
  s = (f % 2 == 0) ? 1.0 : -1.0;
  ua = ax == 0 ? 1 : 0;
  va = ax == 2 ? 1 : 2;
}

// Direction of the centre / corners of grid cell (i,j) of face f.
inline D3 face_dir(int f, double u, double v) {
  int ax, ua, va;
  double s;
  face_axes(f, ax, ua, va, s);
  double c[3];
  c[ax] = s;
  c[ua] = u;
  c[va] = v;
  return unitd({c[0], c[1], c[2]});
}

// Triangle (grid coordinates) vs axis-aligned box, separating axis test.
inline bool tri_box_overlap(const double tx[3], const double ty[3], double bx0, double by0,
                            double bx1, double by1) {
  // box axes
  double mnx = std::min(tx[0], std::min(tx[1], tx[2])), mxx = std::max(tx[0], std::max(tx[1], tx[2]));
  double mny = std::min(ty[0], std::min(ty[1], ty[2])), mxy = std::max(ty[0], std::max(ty[1], ty[2]));
  if (mxx < bx0 || mnx > bx1 || mxy < by0 || mny > by1) return false;
  const double cx = 0.5 * (bx0 + bx1), cy = 0.5 * (by0 + by1);
  const double hx = 0.5 * (bx1 - bx0), hy = 0.5 * (by1 - by0);
  for (int k = 0; k < 3; ++k) {
    const int k1 = (k + 1) % 3;
    const double nx = -(ty[k1] - ty[k]), ny = tx[k1] - tx[k];
    double p0 = nx * tx[0] + ny * ty[0], p1 = nx * tx[1] + ny * ty[1], p2 = nx * tx[2] + ny * ty[2];
    double tmin = std::min(p0, std::min(p1, p2)), tmax = std::max(p0, std::max(p1, p2));
    double bc = nx * cx + ny * cy, br = hx * fabs(nx) + hy * fabs(ny);
    if (tmax < bc - br || tmin > bc + br) return false;
  }
  return true;
}

struct Rasterizer {
  int G;
  // Append grid cells overlapped by the geodesic triangle with unit corner directions d[3].
  void triangle(const D3 d[3], std::vector<uint32_t> &cells) const {
    const D3 c = unitd({d[0].x + d[1].x + d[2].x, d[0].y + d[1].y + d[2].y,
                        d[0].z + d[1].z + d[2].z});
    double rho = 0;
    for (int k = 0; k < 3; ++k) rho = std::max(rho, acos(std::max(-1.0, std::min(1.0, dotd(c, d[k])))));
    if (!(rho < kBigCap)) {
      cap(c, rho, cells);
      return;
    }
    const double padG = kPadUV * 0.5 * G;
    for (int f = 0; f < 6; ++f) {
      int ax, ua, va;
      double s;
      face_axes(f, ax, ua, va, s);
      double tx[3], ty[3];
      bool front = true;
      for (int k = 0; k < 3; ++k) {
        const double w = s * comp(d[k], ax);
        if (!(w > 1e-6)) {
          front = false;
          break;
        }
        tx[k] = (comp(d[k], ua) / w + 1.0) * 0.5 * G;
        ty[k] = (comp(d[k], va) / w + 1.0) * 0.5 * G;
      }
      if (!front) continue;
      double mnx = std::min(tx[0], std::min(tx[1], tx[2])) - padG;
      double mxx = std::max(tx[0], std::max(tx[1], tx[2])) + padG;
      double mny = std::min(ty[0], std::min(ty[1], ty[2])) - padG;
      double mxy = std::max(ty[0], std::max(ty[1], ty[2])) + padG;
      int i0 = std::max(0, (int)floor(mnx)), i1 = std::min(G - 1, (int)floor(mxx));
      int j0 = std::max(0, (int)floor(mny)), j1 = std::min(G - 1, (int)floor(mxy));
      for (int j = j0; j <= j1; ++j)
        for (int i = i0; i <= i1; ++i)
          if (tri_box_overlap(tx, ty, i - padG, j - padG, i + 1 + padG, j + 1 + padG))
            cells.push_back((uint32_t)f * G * G + (uint32_t)j * G + (uint32_t)i);
    }
  }
  // Cone of half-angle rho around c versus every grid cell's bounding cone.
  void cap(const D3 &c, double rho, std::vector<uint32_t> &cells) const {
    const double padA = 3 * kPadUV;
    for (int f = 0; f < 6; ++f)
      for (int j = 0; j < G; ++j)
        for (int i = 0; i < G; ++i) {
          const double u0 = 2.0 * i / G - 1, u1 = 2.0 * (i + 1) / G - 1;
          const double v0 = 2.0 * j / G - 1, v1 = 2.0 * (j + 1) / G - 1;
          const D3 g = face_dir(f, 0.5 * (u0 + u1), 0.5 * (v0 + v1));
          double delta = 0;
          const double us[2] = {u0, u1}, vs[2] = {v0, v1};
          for (double uu : us)
            for (double vv : vs)
              delta = std::max(delta, acos(std::max(-1.0, std::min(1.0, dotd(g, face_dir(f, uu, vv))))));
          const double ang = acos(std::max(-1.0, std::min(1.0, dotd(c, g))));
          if (ang <= rho + delta + padA) cells.push_back((uint32_t)f * G * G + (uint32_t)j * G + (uint32_t)i);
        }
  }
  void all(std::vector<uint32_t> &cells) const {
    for (uint32_t k = 0; k < 6u * G * G; ++k) cells.push_back(k);
  }
};

inline bool finite_geometry(const irt_icon_cell &c) {
  for (int k = 0; k < 3; ++k)
    if (!std::isfinite(c.lat[k]) || !std::isfinite(c.lon[k])) return false;
  for (int j = 0; j <= c.numLayers; ++j)
    if (!std::isfinite(c.height[j])) return false;
  return true;
}

// LocEntry::meta: numLayers | (height[1..numLayers] non-decreasing) << 31.  For sorted
// heights findHeight's lower_bound equals the count of height[1..nl] < r, which the
// kernel evaluates from one 128-B line in registers.
inline uint32_t entry_meta(const irt_icon_cell &c) {
  bool sorted = true;
  for (int j = 2; j <= c.numLayers; ++j)
    if (!(c.height[j - 1] <= c.height[j])) sorted = false;
  return (uint32_t)c.numLayers | (sorted ? 0x80000000u : 0u);
}

inline bool same_column(const irt_icon_cell &a, const irt_icon_cell &b) {
  return memcmp(a.lat, b.lat, sizeof(a.lat)) == 0 && memcmp(a.lon, b.lon, sizeof(a.lon)) == 0;
}

}  // namespace

int build_scene(const irt_icon_cell *cells, size_t n, HostScene &S, int threads) {
  if (n > 0xFFFFFFF0ull) {
    set_error("too many cells (%zu)", n);
    return IRT_E_INVALID;
  }
  for (size_t i = 0; i < n; ++i) {
    if (cells[i].numLayers < 0 || cells[i].numLayers > 31) {
      set_error("cell %zu: numLayers %d outside [0,31] (MAX_LAYERS 32, ICONGrid.h:57)", i,
                cells[i].numLayers);
      return IRT_E_DATA;
    }
    if (!finite_geometry(cells[i])) {
      set_error("cell %zu: non-finite lat/lon/height", i);
      return IRT_E_DATA;
    }
  }
  if (threads <= 0) threads = default_threads();
  S = HostScene();
  S.n = n;
  compute_volume_info(cells, n, S.info);

  // --- per-record planes and height/value blocks
  S.hv.assign(n * kHV, 0.f);
  S.planes.resize(n * 3);
  S.trig.resize(n * 12);
  {
    std::vector<std::thread> ts;
    const size_t chunk = (n + threads - 1) / std::max(threads, 1);
    for (int t = 0; t < threads; ++t) {
      const size_t b = t * chunk, e = std::min(n, b + chunk);
      if (b >= e) break;
      ts.emplace_back([&, b, e] {
        for (size_t i = b; i < e; ++i) {
          const irt_icon_cell &c = cells[i];
          const float h0 = c.height[0], hN = c.height[c.numLayers];
          V3 bv[3], tv[3];
          for (int k = 0; k < 3; ++k) {
            bv[k] = toCartesian(h0, c.lat[k], c.lon[k]);
            tv[k] = toCartesian(hN, c.lat[k], c.lon[k]);
          }
          S.planes[3 * i + 0] = makePlane(bv[0], bv[1], tv[1]);
          S.planes[3 * i + 1] = makePlane(bv[1], bv[2], tv[2]);
          S.planes[3 * i + 2] = makePlane(bv[2], bv[0], tv[0]);
          for (int k = 0; k < 3; ++k) {
            float *t = &S.trig[12 * i + 4 * k];
            t[0] = cosf(c.lat[k]);
            t[1] = sinf(c.lat[k]);
            t[2] = cosf(c.lon[k]);
            t[3] = sinf(c.lon[k]);
          }
          float *hv = &S.hv[i * kHV];
          memcpy(hv, c.height, 32 * sizeof(float));
          memcpy(hv + 32, c.value, 31 * sizeof(float));
          int32_t nl = c.numLayers;
          memcpy(hv + 63, &nl, 4);
        }
      });
    }
    for (auto &t : ts) t.join();
  }

  // --- columns: runs of consecutive records with identical corners
  std::vector<size_t> runStart;
  for (size_t i = 0; i < n; ++i)
    if (i == 0 || !same_column(cells[i], cells[i - 1])) runStart.push_back(i);
  const size_t numRuns = runStart.size();
  runStart.push_back(n);

  double scale = 1.5;
  if (const char *e = getenv("IRT_LOCATOR_SCALE")) scale = atof(e);
  int G = (int)llround(sqrt((double)std::max<size_t>(numRuns, 1) / 6.0) * scale);
  G = std::max(4, std::min(G, 4096));
  if (const char *e = getenv("IRT_LOCATOR_G")) G = std::max(1, std::min(4096, atoi(e)));
  S.G = G;
  const uint32_t numGridCells = 6u * G * G;
  Rasterizer R{G};

  // --- rasterise runs in parallel; each thread owns a contiguous range of runs so the
  //     concatenated (cell, record) pairs stay in record order
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> parts(threads);
  {
    std::vector<std::thread> ts;
    const size_t chunk = (numRuns + threads - 1) / std::max(threads, 1);
    for (int t = 0; t < threads; ++t) {
      const size_t b = t * chunk, e = std::min(numRuns, b + chunk);
      if (b >= e) break;
      ts.emplace_back([&, t, b, e] {
        std::vector<uint32_t> gc;
        auto &out = parts[t];
        for (size_t r = b; r < e; ++r) {
          const size_t i0 = runStart[r], i1 = runStart[r + 1];
          const irt_icon_cell &c = cells[i0];
          D3 d[3];
          for (int k = 0; k < 3; ++k) {
            const double la = c.lat[k], lo = c.lon[k];
            d[k] = {cos(la) * cos(lo), cos(la) * sin(lo), sin(la)};
          }
          // Which cone do the float planes carve out?  Probe the centroid direction
          // (and its antipode) at the record's mid radius.
          const D3 cd = unitd({d[0].x + d[1].x + d[2].x, d[0].y + d[1].y + d[2].y,
                               d[0].z + d[1].z + d[2].z});
          gc.clear();
          int mode = 2;  // 0 normal, 1 antipodal, 2 degenerate
          for (size_t i = i0; i < i1 && mode == 2; ++i) {
            const irt_icon_cell &ci = cells[i];
            // only records with a positive radial extent carve out a cone (inverted ones
            // never pass the radial test; zero-thickness ones are spheres, see below)
            if (!(ci.height[0] < ci.height[ci.numLayers])) continue;
            const double rm = 0.5 * ((double)ci.height[0] + (double)ci.height[ci.numLayers]);
            for (int sgn = 0; sgn < 2 && mode == 2; ++sgn) {
              const double s = sgn ? -rm : rm;
              const float px = (float)(cd.x * s), py = (float)(cd.y * s), pz = (float)(cd.z * s);
              bool in = true;
              for (int k = 0; k < 3; ++k)
                if (evalPlane(S.planes[3 * i + k], px, py, pz) > 0.f) in = false;
              if (in) mode = sgn;
            }
          }
          if (std::isnan(cd.x) || std::isnan(cd.y) || std::isnan(cd.z)) mode = 2;
          if (mode == 2) {
            R.all(gc);
          } else {
            D3 dd[3] = {d[0], d[1], d[2]};
            if (mode == 1)
              for (auto &q : dd) q = {-q.x, -q.y, -q.z};
            R.triangle(dd, gc);
          }
          std::sort(gc.begin(), gc.end());
          gc.erase(std::unique(gc.begin(), gc.end()), gc.end());
          for (size_t i = i0; i < i1; ++i) {
            const irt_icon_cell &ci = cells[i];
            // inverted: the radial test never passes; zero thickness: the sphere table
            if (!(ci.height[0] < ci.height[ci.numLayers])) continue;
            for (uint32_t g : gc) out.emplace_back(g, (uint32_t)i);
          }
        }
      });
    }
    for (auto &t : ts) t.join();
  }

  // --- zero-thickness records (height[0] == height[numLayers], e.g. the numLayers == 0
  //     records convert_icon writes for numLayers % 32 == 1, convert_icon.cpp:363-365):
  //     their bottom and top corners coincide, so every side plane has N == 0 and
  //     sample() accepts ANY direction at r == height[0] exactly -- a sphere.  They are
  //     kept out of the cell lists, in a table sorted by (radius, record).
  {
    std::vector<std::pair<float, uint32_t>> sph;
    for (size_t i = 0; i < n; ++i)
      if (cells[i].height[0] == cells[i].height[cells[i].numLayers])
        sph.emplace_back(cells[i].height[0], (uint32_t)i);
    std::sort(sph.begin(), sph.end());
    S.sphR.clear();
    S.sphOff.assign(1, 0u);
    S.sphRec.clear();
    for (size_t k = 0; k < sph.size(); ++k) {
      if (k == 0 || sph[k].first != sph[k - 1].first) {
        if (k) S.sphOff.push_back((uint32_t)S.sphRec.size());
        S.sphR.push_back(sph[k].first);
      }
      S.sphRec.push_back(sph[k].second);
    }
    if (!sph.empty()) S.sphOff.push_back((uint32_t)S.sphRec.size());
    S.sphBits.assign(kSphBitWords, 0u);
    for (float r : S.sphR) {
      const uint32_t h = sph_hash(r);
      S.sphBits[h >> 5] |= 1u << (h & 31);
    }
  }

  // --- stable counting sort by grid cell -> CSR
  S.offsets.assign(numGridCells + 1, 0);
  size_t total = 0;
  for (auto &p : parts) {
    total += p.size();
    for (auto &e : p) S.offsets[e.first + 1]++;
  }
  for (uint32_t k = 0; k < numGridCells; ++k) S.offsets[k + 1] += S.offsets[k];
  if (total > 0xFFFFFFF0ull) {
    set_error("locator too large (%zu entries)", total);
    return IRT_E_INVALID;
  }
  S.entries.resize(total);
  {
    std::vector<uint32_t> cursor(S.offsets.begin(), S.offsets.end() - 1);
    for (auto &p : parts)
      for (auto &e : p) {
        const irt_icon_cell &c = cells[e.second];
        S.entries[cursor[e.first]++] = {c.height[0], c.height[c.numLayers], e.second,
                                        entry_meta(c)};
      }
  }
  S.info.locatorFaceRes = G;
  S.info.locatorEntries = total;
  return build_bins(S, threads);
}

// ---------------------------------------------------------------- radially binned lists
namespace {

// Open bin (lo, hi) membership of a record with radial extent [h0, hN] (irt_common.h).
inline bool in_bin(float h0, float hN, float lo, float hi) {
  return (h0 < hi && hN > lo) || (h0 == hN && h0 == hi);
}

// Expected number of list entries a radius drawn uniformly from the cell's radial extent
// meets, for the given edges: sum over bins of (bin length within [rmin, rmax]) * count.
double bin_cost(const std::vector<LocEntry> &E, const float *edges, int ne, double rmin,
                double rmax) {
  double cost = 0;
  for (int k = 0; k <= ne; ++k) {
    const float lo = k ? edges[k - 1] : -INFINITY, hi = k < ne ? edges[k] : INFINITY;
    const double a = std::max(rmin, (double)lo), b = std::min(rmax, (double)hi);
    if (!(b > a)) continue;
    size_t cnt = 0;
    for (const LocEntry &e : E) cnt += in_bin(e.h0, e.hN, lo, hi) ? 1 : 0;
    cost += (b - a) * (double)cnt;
  }
  return cost;
}

// Up to kMaxEdges edges for one cell, greedily, among the records' bottom heights.
int choose_edges(const std::vector<LocEntry> &E, float *edges) {
  if (E.size() <= 2) return 0;
  double rmin = INFINITY, rmax = -INFINITY;
  std::vector<float> cand;
  for (const LocEntry &e : E) {
    rmin = std::min(rmin, (double)e.h0);
    rmax = std::max(rmax, (double)e.hN);
    cand.push_back(e.h0);
  }
  std::sort(cand.begin(), cand.end());
  cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
  std::vector<float> c2;
  for (float v : cand)
    if (v > rmin && v < rmax) c2.push_back(v);
  if (c2.size() > 48) {  // bound the search: 48 quantiles
    std::vector<float> q;
    for (int k = 0; k < 48; ++k) q.push_back(c2[(size_t)k * c2.size() / 48]);
    q.erase(std::unique(q.begin(), q.end()), q.end());
    c2.swap(q);
  }
  int ne = 0;
  double best = bin_cost(E, edges, 0, rmin, rmax);
  while (ne < kMaxEdges) {
    int bi = -1;
    double bc = best;
    for (size_t i = 0; i < c2.size(); ++i) {
      float tr[kMaxEdges];
      int m = 0;
      bool dup = false;
      for (int k = 0; k < ne; ++k) {
        if (edges[k] == c2[i]) dup = true;
        tr[m++] = edges[k];
      }
      if (dup) continue;
      tr[m++] = c2[i];
      std::sort(tr, tr + m);
      const double c = bin_cost(E, tr, m, rmin, rmax);
      if (c < bc * 0.98) {
        bc = c;
        bi = (int)i;
      }
    }
    if (bi < 0) break;
    edges[ne++] = c2[bi];
    std::sort(edges, edges + ne);
    best = bc;
  }
  return ne;
}

}  // namespace

int build_bins(HostScene &S, int threads) {
  const uint32_t numGridCells = 6u * S.G * S.G;
  // per-record height/value blocks
  S.blocks.assign(S.n * (size_t)kBlk4 * 4, 0.f);
  for (size_t i = 0; i < S.n; ++i) {
    float *B = &S.blocks[i * (size_t)kBlk4 * 4];
    const float *hv = &S.hv[i * kHV];
    for (int j = 0; j < 32; ++j) B[blk_height_pos(j)] = hv[j];
    for (int c = 0; c < 31; ++c) B[blk_value_pos(c)] = hv[32 + c];
  }
  // pass 1: edges and per-bin counts per cell
  S.binHdr.assign((size_t)numGridCells * kBinHdrWords, 0u);
  std::vector<uint64_t> cellCount(numGridCells + 1, 0);
  auto parallel = [&](auto &&fn) {
    std::vector<std::thread> ts;
    const uint32_t chunk = (numGridCells + threads - 1) / std::max(threads, 1);
    for (int t = 0; t < threads; ++t) {
      const uint32_t b = t * chunk, e = std::min(numGridCells, b + chunk);
      if (b >= e) break;
      ts.emplace_back([&, b, e] { fn(b, e); });
    }
    for (auto &t : ts) t.join();
  };
  parallel([&](uint32_t b, uint32_t e) {
    std::vector<LocEntry> E;
    for (uint32_t cell = b; cell < e; ++cell) {
      E.assign(S.entries.begin() + S.offsets[cell], S.entries.begin() + S.offsets[cell + 1]);
      float edges[kMaxEdges];
      const int ne = choose_edges(E, edges);
      uint32_t *H = &S.binHdr[(size_t)cell * kBinHdrWords];
      uint32_t cum = 0;
      for (int k = 0; k < kMaxEdges; ++k) H[k] = f2u(k < ne ? edges[k] : INFINITY);
      for (int k = 0; k <= kMaxEdges; ++k) {
        if (k <= ne) {
          const float lo = k ? edges[k - 1] : -INFINITY, hi = k < ne ? edges[k] : INFINITY;
          for (const LocEntry &x : E) cum += in_bin(x.h0, x.hN, lo, hi) ? 1u : 0u;
        }
        H[4 + k] = cum;
      }
      cellCount[cell + 1] = cum;
    }
  });
  for (uint32_t k = 0; k < numGridCells; ++k) cellCount[k + 1] += cellCount[k];
  const uint64_t total = cellCount[numGridCells];
  if (total > 0xFFFFFFF0ull) {
    set_error("binned locator too large (%llu entries)", (unsigned long long)total);
    return IRT_E_INVALID;
  }
  S.binEntries = total;
  S.fat.assign(total * kFat4 * 4, 0.f);
  // pass 2: fill the fat entries
  parallel([&](uint32_t b, uint32_t e) {
    for (uint32_t cell = b; cell < e; ++cell) {
      uint32_t *H = &S.binHdr[(size_t)cell * kBinHdrWords];
      H[3] = (uint32_t)cellCount[cell];
      size_t at = cellCount[cell];
      const float edges[kMaxEdges] = {u2f(H[0]), u2f(H[1]), u2f(H[2])};
      int ne = 0;
      while (ne < kMaxEdges && edges[ne] != INFINITY) ++ne;
      for (int k = 0; k <= ne; ++k) {
        const float lo = k ? edges[k - 1] : -INFINITY, hi = k < ne ? edges[k] : INFINITY;
        for (uint32_t q = S.offsets[cell]; q < S.offsets[cell + 1]; ++q) {
          const LocEntry &x = S.entries[q];
          if (!in_bin(x.h0, x.hN, lo, hi)) continue;
          float *F = &S.fat[at++ * kFat4 * 4];
          memcpy(F, &S.planes[3 * (size_t)x.idx], 12 * sizeof(float));
          F[12] = x.h0;
          F[13] = x.hN;
          F[14] = u2f(x.idx);
          F[15] = u2f(x.meta);
          const float *hv = &S.hv[(size_t)x.idx * kHV];
          F[16] = hv[7];
          F[17] = hv[15];
          F[18] = hv[23];
          F[19] = hv[31];
        }
      }
    }
  });
  return IRT_OK;
}

namespace {
// sample() of one fat entry (ICONGrid.h:181-208), value from the record's blocks
bool test_fat(const HostScene &s, const float *F, float px, float py, float pz, float r,
              float &value) {
  if (r < F[12] || r > F[13]) return false;  // ICONGrid.h:184
  for (int k = 0; k < 3; ++k) {
    const Plane4 p = {F[4 * k], F[4 * k + 1], F[4 * k + 2], F[4 * k + 3]};
    if (evalPlane(p, px, py, pz) > 0.f) return false;  // ICONGrid.h:201-203
  }
  const uint32_t rec = f2u(F[14]), meta = f2u(F[15]);
  const int nl = (int)(meta & 0x7fffffffu);
  const float *B = &s.blocks[(size_t)rec * kBlk4 * 4];
  if (meta >> 31) {
    const int b = rec_coarse_block(F[16], F[17], F[18], F[19], nl, r);
    const float *Q = B + 16 * b;
    const int m = rec_block_index(Q[0], Q[1], Q[2], Q[3], Q[4], Q[5], Q[6], b, nl, r);
    value = select8(m, Q[8], Q[9], Q[10], Q[11], Q[12], Q[13], Q[14], Q[15]);
  } else {
    int first = 0, count = nl;  // findHeight, literally (ICONGrid.h:117-145)
    while (count > 0) {
      const int stp = count / 2, it = first + stp;
      if (!(r <= B[blk_height_pos(it + 1)])) {
        first = it + 1;
        count -= stp + 1;
      } else {
        count = stp;
      }
    }
    value = B[blk_value_pos(first)];
  }
  return true;
}
// getValue (ICONGrid.h:147-164) of a zero-thickness record: literal findHeight
float sphere_value(const HostScene &s, uint32_t rec, float r) {
  const float *hv = &s.hv[(size_t)rec * kHV];
  int32_t nl;
  memcpy(&nl, hv + 63, 4);
  return hv[32 + find_height(hv, nl, r)];
}
}  // namespace

int locate_bins_host(const HostScene &s, float px, float py, float pz, float &value,
                     uint32_t *record, uint32_t *tested) {
  if (tested) *tested = 0;
  if (s.n == 0 || s.G == 0) return 0;
  const float r = sqrtf(px * px + py * py + pz * pz);
  const uint32_t cell = cubemap_cell(px, py, pz, s.G);
  const uint32_t *H = &s.binHdr[(size_t)cell * kBinHdrWords];
  const float e[3] = {u2f(H[0]), u2f(H[1]), u2f(H[2])};
  const int b = bin_of(r, e[0], e[1], e[2]);
  int hit = 0;
  uint32_t best = 0;
  float bestV = 0.f;
  const int last = (b < kMaxEdges && r == e[b]) ? b + 1 : b;  // exactly on an edge
  for (int k = b; k <= last; ++k) {
    const uint32_t beg = H[3] + (k ? H[4 + k - 1] : 0), end = H[3] + H[4 + k];
    for (uint32_t q = beg; q < end; ++q) {
      const float *F = &s.fat[(size_t)q * kFat4 * 4];
      if (hit && f2u(F[14]) >= best) break;
      if (tested) ++*tested;
      float v;
      if (test_fat(s, F, px, py, pz, r, v)) {
        hit = 1;
        best = f2u(F[14]);
        bestV = v;
        break;
      }
    }
  }
  // sphere records at exactly this radius (see build_scene)
  if (!s.sphR.empty()) {
    const auto it = std::lower_bound(s.sphR.begin(), s.sphR.end(), r);
    if (it != s.sphR.end() && *it == r) {
      const uint32_t rec = s.sphRec[s.sphOff[it - s.sphR.begin()]];  // lowest index
      if (!hit || rec < best) {
        hit = 1;
        best = rec;
        bestV = sphere_value(s, rec, r);
      }
    }
  }
  if (hit) {
    value = bestV;
    if (record) *record = best;
  }
  return hit;
}

// sample() (ICONGrid.h:181-208) with the precomputed planes; lat/lon of toSpherical are
// dead in sample() and skipped.
void build_records(const HostScene &s, std::vector<float> &out) {
  out.assign(s.n * (size_t)kRec4 * 4, 0.f);
  for (size_t i = 0; i < s.n; ++i) {
    float *R = &out[i * (size_t)kRec4 * 4];
    const float *hv = &s.hv[i * kHV];
    for (int k = 0; k < 3; ++k) {
      const Plane4 &p = s.planes[3 * i + k];
      R[4 * k + 0] = p.x;
      R[4 * k + 1] = p.y;
      R[4 * k + 2] = p.z;
      R[4 * k + 3] = p.w;
    }
    R[12] = hv[7];
    R[13] = hv[15];
    R[14] = hv[23];
    R[15] = hv[31];
    for (int j = 0; j < 32; ++j) R[rec_height_pos(j)] = hv[j];
    for (int c = 0; c < 31; ++c) R[rec_value_pos(c)] = hv[32 + c];
    // value[-1] stays 0 (never selected: the block-0 answer index is >= 1)
  }
}

int sample_host(const HostScene &s, uint32_t rec, float px, float py, float pz, float &value) {
  const float r = sqrtf(px * px + py * py + pz * pz);
  const float *hv = &s.hv[(size_t)rec * kHV];
  int32_t nl;
  memcpy(&nl, hv + 63, 4);
  if (r < hv[0] || r > hv[nl]) return 0;
  for (int k = 0; k < 3; ++k)
    if (evalPlane(s.planes[3 * (size_t)rec + k], px, py, pz) > 0.f) return 0;
  value = hv[32 + find_height(hv, nl, r)];
  return 1;
}

int locate_host(const HostScene &s, float px, float py, float pz, float &value,
                uint32_t *record) {
  if (s.n == 0 || s.G == 0) return 0;
  const float r = sqrtf(px * px + py * py + pz * pz);
  const uint32_t cell = cubemap_cell(px, py, pz, s.G);
  for (uint32_t e = s.offsets[cell]; e < s.offsets[cell + 1]; ++e) {
    const LocEntry &E = s.entries[e];
    if (r < E.h0 || r > E.hN) continue;
    if (sample_host(s, E.idx, px, py, pz, value)) {
      if (record) *record = E.idx;
      return 1;
    }
  }
  return 0;
}

// ---------------------------------------------------------------- CUBQL_MODE wedges
namespace {

// toCartesian (ICONGrid.h:44-54) from the corner's glibc trig, the same float expression
inline V3 wedge_vertex(float r, const float *t) { return {(r * t[0]) * t[2], (r * t[0]) * t[3], r * t[1]}; }

// getValue (ICONGrid.h:147-164)
inline float cell_value(const irt_icon_cell &c, float h) {
  return c.value[find_height(c.height, c.numLayers, h)];
}

// The wedge of layer h of record c (hostCode.cu:562-590) and its primBounds (534-552).
inline void make_wedge(const irt_icon_cell &c, const float *trig, int h, WV4 V[6], float lo[3],
                       float hi[3]) {
  const float bv = h == 0 ? cell_value(c, c.height[h])
                          : (cell_value(c, c.height[h - 1]) + cell_value(c, c.height[h])) * 0.5f;
  for (int k = 0; k < 3; ++k) {
    const V3 b = wedge_vertex(c.height[h], trig + 4 * k), t = wedge_vertex(c.height[h + 1], trig + 4 * k);
    V[k] = {b.x, b.y, b.z, bv};
    V[k + 3] = {t.x, t.y, t.z, bv};
  }
  lo[0] = lo[1] = lo[2] = 1e31f;
  hi[0] = hi[1] = hi[2] = -1e31f;
  for (int k = 0; k < 6; ++k) {
    lo[0] = fminf(lo[0], V[k].x);
    lo[1] = fminf(lo[1], V[k].y);
    lo[2] = fminf(lo[2], V[k].z);
    hi[0] = fmaxf(hi[0], V[k].x);
    hi[1] = fmaxf(hi[1], V[k].y);
    hi[2] = fmaxf(hi[2], V[k].z);
  }
}

// Grid cells of the cube map that can hold the direction of a point of box [lo, hi]:
// per face, the gnomonic projection of the box (all corners in front of the face) is the
// convex hull of its projected corners; a box straddling a face's plane takes the whole
// face; a box holding the origin takes every cell.
void rasterize_box(const double lo[3], const double hi[3], int G, std::vector<uint32_t> &out) {
  if (lo[0] <= 0 && hi[0] >= 0 && lo[1] <= 0 && hi[1] >= 0 && lo[2] <= 0 && hi[2] >= 0) {
    for (uint32_t k = 0; k < 6u * G * G; ++k) out.push_back(k);
    return;
  }
  const double padG = kPadUV * 0.5 * G;
  for (int f = 0; f < 6; ++f) {
    int ax, ua, va;
    double sgn;
    face_axes(f, ax, ua, va, sgn);
    int front = 0, behind = 0;
    double mnu = 1e300, mxu = -1e300, mnv = 1e300, mxv = -1e300;
    for (int c = 0; c < 8; ++c) {
      const double p[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
      const double w = sgn * p[ax];
      if (w > 0) {
        ++front;
        const double u = p[ua] / w, v = p[va] / w;
        mnu = std::min(mnu, u);
        mxu = std::max(mxu, u);
        mnv = std::min(mnv, v);
        mxv = std::max(mxv, v);
      } else {
        ++behind;
      }
    }
    if (front == 0) continue;
    int i0 = 0, i1 = G - 1, j0 = 0, j1 = G - 1;
    if (behind == 0) {
      i0 = std::max(0, (int)floor((mnu + 1.0) * 0.5 * G - padG));
      i1 = std::min(G - 1, (int)floor((mxu + 1.0) * 0.5 * G + padG));
      j0 = std::max(0, (int)floor((mnv + 1.0) * 0.5 * G - padG));
      j1 = std::min(G - 1, (int)floor((mxv + 1.0) * 0.5 * G + padG));
    }
    for (int j = j0; j <= j1; ++j)
      for (int i = i0; i <= i1; ++i) out.push_back((uint32_t)f * G * G + (uint32_t)j * G + (uint32_t)i);
  }
}

}  // namespace

int build_wedges(const irt_icon_cell *cells, size_t n, WedgeScene &W, int threads) {
  if (threads <= 0) threads = default_threads();
  W = WedgeScene();
  W.trig.resize(n * 12);
  W.box.assign(n * 8, 0.f);
  size_t numRuns = 0;
  for (size_t i = 0; i < n; ++i)
    if (i == 0 || !same_column(cells[i], cells[i - 1])) ++numRuns;
  int G = (int)llround(sqrt((double)std::max<size_t>(numRuns, 1) / 6.0) * 1.5);
  G = std::max(4, std::min(G, 4096));
  W.G = G;
  const uint32_t numGridCells = 6u * G * G;
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> parts(threads);
  std::vector<std::thread> ts;
  const size_t chunk = (n + threads - 1) / std::max(threads, 1);
  for (int t = 0; t < threads; ++t) {
    const size_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    ts.emplace_back([&, t, b, e] {
      std::vector<uint32_t> gc;
      for (size_t i = b; i < e; ++i) {
        const irt_icon_cell &c = cells[i];
        float *tr = &W.trig[12 * i];
        for (int k = 0; k < 3; ++k) {
          tr[4 * k + 0] = cosf(c.lat[k]);
          tr[4 * k + 1] = sinf(c.lat[k]);
          tr[4 * k + 2] = cosf(c.lon[k]);
          tr[4 * k + 3] = sinf(c.lon[k]);
        }
        float lo[3] = {1e31f, 1e31f, 1e31f}, hi[3] = {-1e31f, -1e31f, -1e31f};
        // the bottom triangle (TRIANGLE_MODE's geometry, hostCode.cu:445-450), also of
        // records without layers
        for (int k = 0; k < 3; ++k) {
          const V3 b = wedge_vertex(c.height[0], tr + 4 * k);
          lo[0] = fminf(lo[0], b.x), lo[1] = fminf(lo[1], b.y), lo[2] = fminf(lo[2], b.z);
          hi[0] = fmaxf(hi[0], b.x), hi[1] = fmaxf(hi[1], b.y), hi[2] = fmaxf(hi[2], b.z);
        }
        for (int h = 0; h < c.numLayers; ++h) {
          WV4 V[6];
          float wl[3], wh[3];
          make_wedge(c, tr, h, V, wl, wh);
          for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], wl[a]);
            hi[a] = fmaxf(hi[a], wh[a]);
          }
        }
        float *bx = &W.box[8 * i];
        int32_t nl = c.numLayers;
        bx[0] = lo[0], bx[1] = lo[1], bx[2] = lo[2];
        memcpy(bx + 3, &nl, 4);
        bx[4] = hi[0], bx[5] = hi[1], bx[6] = hi[2];
        // pad the union box by a relative 1e-6 against the double evaluation
        double dl[3], dh[3];
        for (int a = 0; a < 3; ++a) {
          const double m = 1e-6 * std::max(fabs((double)lo[a]), fabs((double)hi[a])) + 1e-3;
          dl[a] = (double)lo[a] - m;
          dh[a] = (double)hi[a] + m;
        }
        gc.clear();
        rasterize_box(dl, dh, G, gc);
        for (uint32_t g : gc) parts[t].emplace_back(g, (uint32_t)i);
      }
    });
  }
  for (auto &th : ts) th.join();
  W.offsets.assign(numGridCells + 1, 0);
  size_t total = 0;
  for (auto &p : parts) {
    total += p.size();
    for (auto &e : p) W.offsets[e.first + 1]++;
  }
  if (total > 0xFFFFFFF0ull) {
    set_error("wedge locator too large (%zu entries)", total);
    return IRT_E_INVALID;
  }
  for (uint32_t k = 0; k < numGridCells; ++k) W.offsets[k + 1] += W.offsets[k];
  W.recs.resize(total);
  std::vector<uint32_t> cursor(W.offsets.begin(), W.offsets.end() - 1);
  for (auto &p : parts)
    for (auto &e : p) W.recs[cursor[e.first]++] = e.second;
  return IRT_OK;
}

bool triangle_locate_host(const WedgeScene &W, const irt_icon_cell *cells, float px, float py,
                          float pz, float &value, uint32_t *record) {
  if (W.G == 0) return false;
  // ray.direction = -normalize(pos) (deviceCode.cu:67; vecmath normalize = u / |u|)
  const float len = sqrtf(px * px + py * py + pz * pz);
  const float dx = -(px / len), dy = -(py / len), dz = -(pz / len);
  const uint32_t cell = cubemap_cell(px, py, pz, W.G);
  float best = INFINITY;
  uint32_t hit = 0xFFFFFFFFu;
  for (uint32_t q = W.offsets[cell]; q < W.offsets[cell + 1]; ++q) {
    const uint32_t rec = W.recs[q];
    const float *tr = &W.trig[12 * (size_t)rec];
    float v[3][3];
    for (int k = 0; k < 3; ++k) {
      const V3 b = wedge_vertex(cells[rec].height[0], tr + 4 * k);
      v[k][0] = b.x, v[k][1] = b.y, v[k][2] = b.z;
    }
    float t;
    if (ray_triangle(px, py, pz, dx, dy, dz, v[0], v[1], v[2], t) && t < best) {
      best = t;
      hit = rec;
    }
  }
  if (hit == 0xFFFFFFFFu) return false;
  const irt_icon_cell &c = cells[hit];
  if (len < c.height[0] || len > c.height[c.numLayers]) return false;
  value = cell_value(c, len);
  if (record) *record = hit;
  return true;
}

bool wedge_locate_host(const WedgeScene &W, const irt_icon_cell *cells, float px, float py,
                       float pz, float &value) {
  if (W.G == 0) return false;
  const uint32_t cell = cubemap_cell(px, py, pz, W.G);
  for (uint32_t q = W.offsets[cell]; q < W.offsets[cell + 1]; ++q) {
    const uint32_t rec = W.recs[q];
    const float *bx = &W.box[8 * (size_t)rec];
    if (!(bx[0] <= px && px <= bx[4] && bx[1] <= py && py <= bx[5] && bx[2] <= pz && pz <= bx[6]))
      continue;
    const irt_icon_cell &c = cells[rec];
    for (int h = 0; h < c.numLayers; ++h) {
      WV4 V[6];
      float lo[3], hi[3];
      make_wedge(c, &W.trig[12 * (size_t)rec], h, V, lo, hi);
      // box3f::contains (vecmath.h:1088-1092) of the wedge's primBounds
      if (!(lo[0] <= px && px <= hi[0] && lo[1] <= py && py <= hi[1] && lo[2] <= pz && pz <= hi[2]))
        continue;
      if (intersect_wedge(value, px, py, pz, V)) return true;
    }
  }
  return false;
}

}  // namespace irt
