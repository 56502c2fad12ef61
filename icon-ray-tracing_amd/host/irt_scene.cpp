// irt_scene.cpp -- the host restatement of the scene build (csrc/irt_build.h, run on the
// device by csrc/irt_build.hip): per-record planes and height/value blocks, and the
// cube-map point locator with radial bins and sub-cell candidate masks.  Used by the
// host-side checks (include/icon_rt_hip_debug.h) and as the byte-for-byte reference of the
// device build (tests/test_gpu_build.py).  Also the CUBQL_MODE / TRIANGLE_MODE wedge
// locator (below).
//
// toCartesian's cosf/sinf are the host glibc's (trig), exactly as the reference computes
// them (icon_rt/ICONGrid.h:44-54); everything derived from them is IEEE arithmetic that the
// device rounds the same way.

#include <math.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>
#include <vector>

#include "irt_build.h"
#include "irt_internal.h"

namespace irt {

namespace {

struct V3 {
  float x, y, z;
};

inline bool finite_geometry(const irt_icon_cell &c) {
  for (int k = 0; k < 3; ++k)
    if (!std::isfinite(c.lat[k]) || !std::isfinite(c.lon[k])) return false;
  for (int j = 0; j <= c.numLayers; ++j)
    if (!std::isfinite(c.height[j])) return false;
  return true;
}

inline bool same_column(const irt_icon_cell &a, const irt_icon_cell &b) {
  return same_corners(a.lat, a.lon, b.lat, b.lon);
}

template <typename F>
void parallel_ranges(size_t n, int threads, F &&fn) {
  std::vector<std::thread> ts;
  const size_t chunk = (n + threads - 1) / std::max(threads, 1);
  for (int t = 0; t < threads; ++t) {
    const size_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    ts.emplace_back([&fn, t, b, e] { fn(t, b, e); });
  }
  for (auto &t : ts) t.join();
}

}  // namespace

// Cube-map cells per face edge: about one column per cell (scale 1.0).  Finer maps test fewer
// candidates per sample (C3: 1.29 at scale 1.5, 1.45 at 1.0) but read more distinct header
// lines; with the wave-wide candidate scan the coarser map is faster (C3 kernel 0.1014 ->
// 0.0985 ms, comb TF 2.05 -> 2.01 ms; profiles/r02h_locator_scale/).
int locator_resolution(size_t numRuns) {
  double scale = 1.0;
  if (const char *e = getenv("IRT_LOCATOR_SCALE")) scale = atof(e);
  int G = (int)llround(sqrt((double)std::max<size_t>(numRuns, 1) / 6.0) * scale);
  G = std::max(4, std::min(G, 4096));
  if (const char *e = getenv("IRT_LOCATOR_G")) G = std::max(1, std::min(4096, atoi(e)));
  return G;
}

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

  // --- per record: glibc corner trig, planes, radial range, meta, blocks
  S.hv.assign(n * kHV, 0.f);
  S.trig.resize(n * 12);
  S.planes.resize(n * 12);
  S.rng.resize(n * 2);
  S.meta.resize(n);
  S.blocks.resize(n * (size_t)kBlk4 * 4);
  parallel_ranges(n, threads, [&](int, size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      const irt_icon_cell &c = cells[i];
      float *t = &S.trig[12 * i];
      for (int k = 0; k < 3; ++k) {
        t[4 * k + 0] = cosf(c.lat[k]);
        t[4 * k + 1] = sinf(c.lat[k]);
        t[4 * k + 2] = cosf(c.lon[k]);
        t[4 * k + 3] = sinf(c.lon[k]);
      }
      const float h0 = c.height[0], hN = c.height[c.numLayers];
      record_planes(h0, hN, t, &S.planes[12 * i]);
      S.rng[2 * i] = h0;
      S.rng[2 * i + 1] = hN;
      S.meta[i] = record_meta(c.height, c.numLayers);
      record_block(c.height, c.value, &S.blocks[i * (size_t)kBlk4 * 4]);
      float *hv = &S.hv[i * kHV];
      memcpy(hv, c.height, 32 * sizeof(float));
      memcpy(hv + 32, c.value, 31 * sizeof(float));
      int32_t nl = c.numLayers;
      memcpy(hv + 63, &nl, 4);
    }
  });

  // --- columns: runs of consecutive records with identical corners
  std::vector<size_t> runStart;
  for (size_t i = 0; i < n; ++i)
    if (i == 0 || !same_column(cells[i], cells[i - 1])) runStart.push_back(i);
  const size_t numRuns = runStart.size();
  runStart.push_back(n);
  const int G = locator_resolution(numRuns);
  S.G = G;
  const uint32_t numGridCells = 6u * G * G;

  // --- rasterise runs in parallel; each thread owns a contiguous range of runs so the
  //     concatenated (cell, record, mask) triples stay in record order
  struct Item {
    uint32_t cell, rec, sub;
  };
  std::vector<std::vector<Item>> parts(threads);
  parallel_ranges(numRuns, threads, [&](int t, size_t b, size_t e) {
    std::vector<std::pair<uint32_t, uint32_t>> gc;
    auto &out = parts[t];
    for (size_t r = b; r < e; ++r) {
      const uint32_t i0 = (uint32_t)runStart[r], i1 = (uint32_t)runStart[r + 1];
      BD3 d[3], centre;
      corner_dirs(&S.trig[12 * (size_t)i0], d);
      double cosRho = 1.0;
      const int kind = run_kind(d, S.planes.data(), S.rng.data(), i0, i1, cosRho, centre);
      gc.clear();
      auto emit = [&gc](uint32_t cell, uint32_t mask) { gc.emplace_back(cell, mask); };
      if (kind == kRunTri) {
        raster_triangle(d, G, emit);
      } else if (kind == kRunCap) {
        for (uint32_t k = 0; k < numGridCells; ++k)
          if (cap_hits_cell(centre, cosRho, G, k)) emit(k, kFullMask);
      } else if (kind == kRunAll) {
        for (uint32_t k = 0; k < numGridCells; ++k) emit(k, kFullMask);
      }
      for (uint32_t i = i0; i < i1; ++i) {
        // inverted: the radial test never passes; zero thickness: the sphere table
        if (!(S.rng[2 * i] < S.rng[2 * i + 1])) continue;
        for (const auto &g : gc) out.push_back({g.first, i, g.second});
      }
    }
  });

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
    for (auto &e : p) S.offsets[e.cell + 1]++;
  }
  if (total > 0xFFFFFFF0ull) {
    set_error("locator too large (%zu entries)", total);
    return IRT_E_INVALID;
  }
  for (uint32_t k = 0; k < numGridCells; ++k) S.offsets[k + 1] += S.offsets[k];
  S.entryRec.resize(total);
  S.entrySub.resize(total);
  {
    std::vector<uint32_t> cursor(S.offsets.begin(), S.offsets.end() - 1);
    for (auto &p : parts)
      for (auto &e : p) {
        const uint32_t q = cursor[e.cell]++;
        S.entryRec[q] = e.rec;
        S.entrySub[q] = e.sub;
      }
  }
  S.info.locatorFaceRes = G;
  S.info.locatorEntries = total;
  return build_bins(S, threads);
}

// ---------------------------------------------------------------- radially binned lists
namespace {
// irt_build.h entry accessor over a cell's CSR range
struct CellEntries {
  const HostScene &S;
  uint32_t q0;
  float h0(int k) const { return S.rng[2 * (size_t)S.entryRec[q0 + k]]; }
  float hN(int k) const { return S.rng[2 * (size_t)S.entryRec[q0 + k] + 1]; }
  uint32_t sub(int k) const { return S.entrySub[q0 + k]; }
};
}  // namespace

int build_bins(HostScene &S, int threads) {
  const uint32_t numGridCells = 6u * S.G * S.G;
  S.binHdr.assign((size_t)numGridCells * kBinHdrWords, 0u);
  std::vector<uint64_t> cellCount(numGridCells + 1, 0);
  // pass 1: edges, per-bin counts and sub-cell masks per cell (irt_build.h)
  parallel_ranges(numGridCells, threads, [&](int, size_t b, size_t e) {
    std::vector<float> cand;
    for (size_t cell = b; cell < e; ++cell) {
      const uint32_t q0 = S.offsets[cell], n = S.offsets[cell + 1] - q0;
      const CellEntries en{S, q0};
      cand.resize(n);
      double rmin, rmax;
      const int nc = cell_candidates(en, (int)n, cand.data(), rmin, rmax);
      float edges[kMaxEdges] = {0.f, 0.f, 0.f};
      const int ne = choose_edges(en, (int)n, cand.data(), nc, rmin, rmax, edges);
      cellCount[cell + 1] = cell_header(en, (int)n, edges, ne, &S.binHdr[cell * kBinHdrWords]);
    }
  });
  for (uint32_t k = 0; k < numGridCells; ++k) cellCount[k + 1] += cellCount[k];
  const uint64_t total = cellCount[numGridCells];
  if (total > 0xFFFFFFF0ull) {
    set_error("binned locator too large (%llu entries)", (unsigned long long)total);
    return IRT_E_INVALID;
  }
  S.binEntries = total;
  S.fat.assign(total * kFatStride4 * 4, 0.f);
  // pass 2: the fat entries, bin by bin
  parallel_ranges(numGridCells, threads, [&](int, size_t b, size_t e) {
    for (size_t cell = b; cell < e; ++cell) {
      uint32_t *H = &S.binHdr[cell * kBinHdrWords];
      H[3] = (uint32_t)cellCount[cell];
      size_t at = cellCount[cell];
      const float edges[kMaxEdges] = {u2f(H[0]), u2f(H[1]), u2f(H[2])};
      int ne = 0;
      while (ne < kMaxEdges && edges[ne] != INFINITY) ++ne;
      for (int k = 0; k <= ne; ++k) {
        const float lo = k ? edges[k - 1] : -INFINITY, hi = k < ne ? edges[k] : INFINITY;
        for (uint32_t q = S.offsets[cell]; q < S.offsets[cell + 1]; ++q) {
          const uint32_t rec = S.entryRec[q];
          if (!in_bin(S.rng[2 * (size_t)rec], S.rng[2 * (size_t)rec + 1], lo, hi)) continue;
          fat_entry(rec, S.planes.data(), S.rng.data(), S.meta.data(), &S.fat[at++ * kFatStride4 * 4]);
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
  for (int k = 0; k < 3; ++k)
    if (eval_plane(F + 4 * k, px, py, pz) > 0.f) return false;  // ICONGrid.h:201-203
  const uint32_t rec = f2u(F[14]);
  value = record_value_host(s, rec, record_path(f2u(F[15]), F[12], F[13], r), r);
  return true;
}
}  // namespace

// getValue of record rec at radius r along its path (irt_common.h record_path), as the
// kernel's record_value reads it from the blocks
float record_value_host(const HostScene &s, uint32_t rec, uint32_t path, float r) {
  const int nl = (int)(path & 31u);
  const float *B = &s.blocks[(size_t)rec * kBlk4 * 4];
  float value;
  if (path & kPathBlock) {
    int b = (int)((path >> 5) & 3u);
    if (path & kPathExactKeys)
      b = rec_coarse_block(B[blk_height_pos(7)], B[blk_height_pos(15)], B[blk_height_pos(23)], INFINITY,
                           nl, r);
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
  return value;
}

namespace {
// getValue (ICONGrid.h:147-164) of a zero-thickness record: literal findHeight
float sphere_value(const HostScene &s, uint32_t rec, float r) {
  const float *hv = &s.hv[(size_t)rec * kHV];
  int32_t nl;
  memcpy(&nl, hv + 63, 4);
  return hv[32 + find_height(hv, nl, r)];
}
}  // namespace

// The kernel's sampleVolume over the binned lists (irt_render.hip locate_hdr), restated.
int locate_bins_host(const HostScene &s, float px, float py, float pz, float &value,
                     uint32_t *record, uint32_t *tested) {
  if (tested) *tested = 0;
  if (s.n == 0 || s.G == 0) return 0;
  const float r = sqrtf(px * px + py * py + pz * pz);
  uint32_t sub = 0;
  const uint32_t cell = cubemap_cell_sub(px, py, pz, s.G, sub);
  const uint32_t *H = &s.binHdr[(size_t)cell * kBinHdrWords];
  const float e[3] = {u2f(H[0]), u2f(H[1]), u2f(H[2])};
  const int b = bin_of(r, e[0], e[1], e[2]);
  int hit = 0;
  uint32_t best = 0;
  float bestV = 0.f;
  // outside the radial range of every record that can reach the point's quad (the header's
  // bounds, irt_build.h cell_header): no candidate can pass, none is tested (the miss-mode kernels'
  // quad-bound test, irt_render.hip locate_wave)
  const int q = quad_of(sub);
  const bool outside = r > u2f(H[kBoundWord + 2 * q]) || r < u2f(H[kBoundWord + 1 + 2 * q]);
  const int last = outside ? b - 1 : (b < kMaxEdges && r == e[b]) ? b + 1 : b;  // exactly on an edge
  for (int k = b; k <= last; ++k) {
    const uint32_t beg = H[3] + (k ? H[4 + k - 1] : 0), end = H[3] + H[4 + k];
    const uint32_t mask = (H[8 + sub] >> (8 * k)) & 0xFFu;
    for (uint32_t j = 0; beg + j < end; ++j) {
      if (j < (uint32_t)kMaskCand) {  // skip candidates that cannot reach this sub-cell
        const uint32_t m = mask >> j;
        if (!m) {
          j = kMaskCand - 1;
          continue;
        }
        j += (uint32_t)__builtin_ctz(m);
        if (beg + j >= end) break;
      }
      const float *F = &s.fat[(size_t)(beg + j) * kFatStride4 * 4];
      if (hit && f2u(F[14]) >= best) break;  // the second bin: only lower records
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
int sample_host(const HostScene &s, uint32_t rec, float px, float py, float pz, float &value) {
  const float r = sqrtf(px * px + py * py + pz * pz);
  const float *hv = &s.hv[(size_t)rec * kHV];
  int32_t nl;
  memcpy(&nl, hv + 63, 4);
  if (r < hv[0] || r > hv[nl]) return 0;
  for (int k = 0; k < 3; ++k)
    if (eval_plane(&s.planes[12 * (size_t)rec + 4 * k], px, py, pz) > 0.f) return 0;
  value = hv[32 + find_height(hv, nl, r)];
  return 1;
}

int locate_host(const HostScene &s, float px, float py, float pz, float &value,
                uint32_t *record) {
  if (s.n == 0 || s.G == 0) return 0;
  const float r = sqrtf(px * px + py * py + pz * pz);
  const uint32_t cell = cubemap_cell(px, py, pz, s.G);
  for (uint32_t e = s.offsets[cell]; e < s.offsets[cell + 1]; ++e) {
    const uint32_t rec = s.entryRec[e];
    if (r < s.rng[2 * (size_t)rec] || r > s.rng[2 * (size_t)rec + 1]) continue;
    if (sample_host(s, rec, px, py, pz, value)) {
      if (record) *record = rec;
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
