// irt_build.h -- the scene build (per-record planes and height blocks, the cube-map point
// locator) as per-element functions shared by the device build (csrc/irt_build.hip) and
// its host restatement (host/irt_scene.cpp).  Floats follow the reference's expressions;
// the locator geometry is double arithmetic restricted to + - * / sqrt and comparisons,
// which both sides round correctly (no contraction: -ffp-contract=off on both), so the
// device and host builds produce the same bytes (tests/test_gpu_build.py).
//
// The locator replaces the reference's cell location (CPU: linear scan over all cells,
// icon_rt/deviceCode.cu:116-123; GPU: OptiX / cuBQL, 58-115).  A gnomonic cube map with
// G x G cells per face; each cell lists every record whose column can contain a point of
// that direction, split radially into up to four bins, each bin sorted by record index, so
// the first record passing sample() is the reference's "lowest index wins" answer
// (deviceCode.cu:119-122).  Each cell is further split into kSub x kSub sub-cells; for the
// first kMaskCand candidates of every bin the cell header holds, per sub-cell, which of them
// can reach it, and the kernel tests only those (plus any beyond the first kMaskCand).
//
// Conservative by construction:
//   - sample()'s accepting region is {r in [h0,hN]} x the cone of its three side planes,
//     i.e. the geodesic triangle of the corners (or, for clockwise corners, its antipode);
//   - geodesic triangles are straight-edged under the gnomonic projection, so each is
//     rasterised per face by a separating-axis test against every sub-cell, padded by 1e-5
//     in face coordinates (~60 m on the Earth; the float error of the kernel's
//     direction -> cell mapping and of the plane rounding is < 1e-6);
//   - triangles with an angular radius over 15 degrees (R1B00/R2B00-class grids) use a
//     cone-versus-cell test; records whose planes carve out no cone go into every cell.
#pragma once

#include <math.h>

#include "irt_common.h"

namespace irt {

constexpr int kSub = kSubCells;     // sub-cells per cell edge
constexpr double kPadUV = 1e-5;     // face-coordinate padding
constexpr double kCosBigCap = 0.96592582628906831;  // cos(15 degrees)
constexpr double kCapSlack = 1e-4;  // cone test slack (>= the padding's angle + rounding)
constexpr uint32_t kFullMask = (1u << (kSub * kSub)) - 1u;

// ---------------------------------------------------------------- double 3-vectors
struct BD3 {
  double x, y, z;
};
IRT_HD BD3 bd3(double x, double y, double z) {
  BD3 r;
  r.x = x;
  r.y = y;
  r.z = z;
  return r;
}
IRT_HD double bdot(const BD3 &a, const BD3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
IRT_HD BD3 bunit(const BD3 &a) {
  const double l = sqrt(bdot(a, a));
  return bd3(a.x / l, a.y / l, a.z / l);
}
IRT_HD double bcomp(const BD3 &d, int a) { return a == 0 ? d.x : (a == 1 ? d.y : d.z); }
IRT_HD double dmin(double a, double b) { return b < a ? b : a; }  // std::min
IRT_HD double dmax(double a, double b) { return a < b ? b : a; }  // std::max
IRT_HD bool bnan(const BD3 &a) { return a.x != a.x || a.y != a.y || a.z != a.z; }

// Face f: axis f/2, sign +1 for even f; (u, v) axes as in cubemap_cell (irt_common.h).
IRT_HD void face_axes(int f, int &ax, int &ua, int &va, double &s) {
  ax = f / 2;
  s = (f % 2 == 0) ? 1.0 : -1.0;
  ua = ax == 0 ? 1 : 0;
  va = ax == 2 ? 1 : 2;
}

// Unit direction through face coordinates (u, v) of face f.
IRT_HD BD3 face_dir(int f, double u, double v) {
  int ax, ua, va;
  double s;
  face_axes(f, ax, ua, va, s);
  double c[3];
  c[ax] = s;
  c[ua] = u;
  c[va] = v;
  return bunit(bd3(c[0], c[1], c[2]));
}

// Triangle (face grid coordinates) vs axis-aligned box: separating axis test.
IRT_HD bool tri_box_overlap(const double tx[3], const double ty[3], double bx0, double by0,
                            double bx1, double by1) {
  const double mnx = dmin(tx[0], dmin(tx[1], tx[2])), mxx = dmax(tx[0], dmax(tx[1], tx[2]));
  const double mny = dmin(ty[0], dmin(ty[1], ty[2])), mxy = dmax(ty[0], dmax(ty[1], ty[2]));
  if (mxx < bx0 || mnx > bx1 || mxy < by0 || mny > by1) return false;
  const double cx = 0.5 * (bx0 + bx1), cy = 0.5 * (by0 + by1);
  const double hx = 0.5 * (bx1 - bx0), hy = 0.5 * (by1 - by0);
  for (int k = 0; k < 3; ++k) {
    const int k1 = (k + 1) % 3;
    const double nx = -(ty[k1] - ty[k]), ny = tx[k1] - tx[k];
    const double p0 = nx * tx[0] + ny * ty[0], p1 = nx * tx[1] + ny * ty[1],
                 p2 = nx * tx[2] + ny * ty[2];
    const double tmin = dmin(p0, dmin(p1, p2)), tmax = dmax(p0, dmax(p1, p2));
    const double bc = nx * cx + ny * cy;
    const double br = hx * (nx < 0 ? -nx : nx) + hy * (ny < 0 ? -ny : ny);
    if (tmax < bc - br || tmin > bc + br) return false;
  }
  return true;
}

// ---------------------------------------------------------------- per record
// Per record the kernel-side arrays (all indexed by record i):
//   planes[3 i + k]  float4 side plane k (n.xyz, w) of sample()     ICONGrid.h:187-203
//   rng[i]           {height[0], height[numLayers]}                  ICONGrid.h:184
//   meta[i]          numLayers, coarse flag, quantised coarse findHeight keys (record_meta)
//   blocks[16 i ..]  the height/value block (irt_common.h kBlk4)
// trig[3 i + k] = {cosf lat, sinf lat, cosf lon, sinf lon} of corner k, from the host's
// glibc -- so toCartesian (ICONGrid.h:44-54) here rounds exactly as the reference's.

// toCartesian(r, lat, lon) = (r cos(lat) cos(lon), r cos(lat) sin(lon), r sin(lat)), left to
// right as the reference evaluates it
IRT_HD void to_cartesian_trig(float r, const float *t, float &x, float &y, float &z) {
  x = (r * t[0]) * t[2];
  y = (r * t[0]) * t[3];
  z = r * t[1];
}

// makePlane (ICONGrid.h:170-174): N = (b - a) x (c - a), w = a . N
IRT_HD void make_plane(const float *a, const float *b, const float *c, float *out4) {
  const float ux = b[0] - a[0], uy = b[1] - a[1], uz = b[2] - a[2];
  const float vx = c[0] - a[0], vy = c[1] - a[1], vz = c[2] - a[2];
  const float nx = uy * vz - uz * vy, ny = uz * vx - ux * vz, nz = ux * vy - uy * vx;
  out4[0] = nx;
  out4[1] = ny;
  out4[2] = nz;
  out4[3] = a[0] * nx + a[1] * ny + a[2] * nz;
}

// The three side planes sample() builds (ICONGrid.h:187-199): bottom corners at height[0],
// top corners at height[numLayers]; planes (b1,b2,t2), (b2,b3,t3), (b3,b1,t1).
IRT_HD void record_planes(float h0, float hN, const float *trig12, float *out12) {
  float b[3][3], t[3][3];
  for (int k = 0; k < 3; ++k) {
    to_cartesian_trig(h0, trig12 + 4 * k, b[k][0], b[k][1], b[k][2]);
    to_cartesian_trig(hN, trig12 + 4 * k, t[k][0], t[k][1], t[k][2]);
  }
  make_plane(b[0], b[1], t[1], out12);
  make_plane(b[1], b[2], t[2], out12 + 4);
  make_plane(b[2], b[0], t[0], out12 + 8);
}

// evalPlane (ICONGrid.h:176-179)
IRT_HD float eval_plane(const float *p, float px, float py, float pz) {
  return (px * p[0] + py * p[1] + pz * p[2]) - p[3];
}

// meta word (irt_common.h): numLayers, the coarse flag, the quantised coarse keys
IRT_HD uint32_t record_meta(const float *height, int nl) {
  // height[1..numLayers] non-decreasing in float_key order (which implies float order; a -0/+0
  // pair in the wrong order takes the literal path).  findHeight never reads height[0]
  // (ICONGrid.h:125-135 compares hpos with *(it+1) only), so height[0] may sit above
  // height[1]: convert_icon's first record of a land column, H[0] = R + HSURF over
  // H[1] = R + HHL - HSURF (convert_icon.cpp:361, 371).  Keys below height[0] are a prefix of
  // the sorted keys; the radial test (r >= height[0]) makes every one of them count, so only
  // their number is kept (bits 30-31).
  bool coarse = nl >= 1 && float_key(height[0]) <= float_key(height[nl]);
  for (int j = 2; j <= nl; ++j)
    if (!(float_key(height[j - 1]) <= float_key(height[j]))) coarse = false;
  uint32_t m = (uint32_t)nl;
  if (coarse) {
    m |= kMetaCoarse;
    const uint32_t k0 = float_key(height[0]), S = meta_quantum(k0, float_key(height[nl]));
    uint32_t below = 0;
    for (int j = 0; j < 3 && 8 * j + 7 <= nl; ++j) {
      const uint32_t kj = float_key(height[8 * j + 7]);
      if (kj < k0)
        ++below;
      else
        m |= ((kj - k0) / S) << (6 + 8 * j);
    }
    m |= below << kMetaBelowShift;
  }
  return m;
}

// The height/value block (kBlk4 float4): block b = {height[8b..8b+3]}, {height[8b+4..8b+7]},
// {value[8b-1..8b+2]}, {value[8b+3..8b+6]}; value[31] sits in block 0's value[-1] slot
// (blk_value_pos), which the block path never selects.
IRT_HD void record_block(const float *height, const float *value, float *out64) {
  for (int j = 0; j < 64; ++j) out64[j] = 0.f;
  for (int j = 0; j < 32; ++j) out64[blk_height_pos(j)] = height[j];
  for (int c = 0; c < 32; ++c) out64[blk_value_pos(c)] = value[c];
}

// Two records belong to the same column (one locator run) when their corners are equal bit
// for bit.
IRT_HD bool same_corners(const float *latA, const float *lonA, const float *latB, const float *lonB) {
  for (int k = 0; k < 3; ++k)
    if (f2u(latA[k]) != f2u(latB[k]) || f2u(lonA[k]) != f2u(lonB[k])) return false;
  return true;
}

// ---------------------------------------------------------------- per run (column)
// Corner directions of a column from its glibc trig (the float products are exact in
// double), normalised.
IRT_HD void corner_dirs(const float *trig12, BD3 d[3]) {
  for (int k = 0; k < 3; ++k) {
    const double cl = trig12[4 * k], sl = trig12[4 * k + 1], co = trig12[4 * k + 2],
                 so = trig12[4 * k + 3];
    d[k] = bunit(bd3(cl * co, cl * so, sl));
  }
}

enum : int { kRunTri = 0, kRunCap = 1, kRunAll = 2, kRunNone = 3 };

// How a column is rasterised.  Which cone do the records' float planes carve out?  Probe
// the centroid direction (and its antipode) at each record's mid radius; the first record
// with a positive radial extent that accepts one of them decides (inverted records never
// pass the radial test; zero-thickness ones are spheres, kept out of the lists).  Returns
// the kind; d is flipped for the antipodal cone; cosRho = cos of the cone's angular radius.
IRT_HD int run_kind(BD3 d[3], const float *planes /*12 per record*/, const float *rng /*2 per
                     record*/, uint32_t i0, uint32_t i1, double &cosRho, BD3 &centre) {
  bool any = false;
  for (uint32_t i = i0; i < i1; ++i)
    if (rng[2 * i] < rng[2 * i + 1]) any = true;
  if (!any) return kRunNone;
  const BD3 cd = bunit(bd3(d[0].x + d[1].x + d[2].x, d[0].y + d[1].y + d[2].y, d[0].z + d[1].z + d[2].z));
  int mode = 2;  // 0 normal, 1 antipodal, 2 degenerate
  for (uint32_t i = i0; i < i1 && mode == 2; ++i) {
    const float h0 = rng[2 * i], hN = rng[2 * i + 1];
    if (!(h0 < hN)) continue;
    const double rm = 0.5 * ((double)h0 + (double)hN);
    for (int sgn = 0; sgn < 2 && mode == 2; ++sgn) {
      const double s = sgn ? -rm : rm;
      const float px = (float)(cd.x * s), py = (float)(cd.y * s), pz = (float)(cd.z * s);
      bool in = true;
      for (int k = 0; k < 3; ++k)
        if (eval_plane(planes + 12 * (size_t)i + 4 * k, px, py, pz) > 0.f) in = false;
      if (in) mode = sgn;
    }
  }
  if (bnan(cd) || mode == 2) return kRunAll;
  if (mode == 1)
    for (int k = 0; k < 3; ++k) d[k] = bd3(-d[k].x, -d[k].y, -d[k].z);
  centre = mode == 1 ? bd3(-cd.x, -cd.y, -cd.z) : cd;
  cosRho = 1.0;
  for (int k = 0; k < 3; ++k) cosRho = dmin(cosRho, bdot(centre, d[k]));
  return cosRho > kCosBigCap ? kRunTri : kRunCap;
}

// Rasterise a geodesic triangle (unit corner directions d) into (cell, sub-cell mask)
// pairs; emit(cell, mask) is called once per overlapped cell.
template <class Emit>
IRT_HD void raster_triangle(const BD3 d[3], int G, Emit &emit) {
  const int GS = G * kSub;
  const double padF = kPadUV * 0.5 * (double)GS;
  for (int f = 0; f < 6; ++f) {
    int ax, ua, va;
    double s;
    face_axes(f, ax, ua, va, s);
    double tx[3], ty[3];
    bool front = true;
    for (int k = 0; k < 3; ++k) {
      const double w = s * bcomp(d[k], ax);
      if (!(w > 1e-6)) {
        front = false;
        break;
      }
      tx[k] = (bcomp(d[k], ua) / w + 1.0) * 0.5 * (double)GS;
      ty[k] = (bcomp(d[k], va) / w + 1.0) * 0.5 * (double)GS;
    }
    if (!front) continue;
    // fine-grid bounding box, clamped before the int conversion
    const double lim = (double)GS;
    const double mnx = dmax(-1.0, dmin(lim, dmin(tx[0], dmin(tx[1], tx[2])) - padF));
    const double mxx = dmax(-1.0, dmin(lim, dmax(tx[0], dmax(tx[1], tx[2])) + padF));
    const double mny = dmax(-1.0, dmin(lim, dmin(ty[0], dmin(ty[1], ty[2])) - padF));
    const double mxy = dmax(-1.0, dmin(lim, dmax(ty[0], dmax(ty[1], ty[2])) + padF));
    int i0 = (int)floor(mnx), i1 = (int)floor(mxx), j0 = (int)floor(mny), j1 = (int)floor(mxy);
    i0 = i0 < 0 ? 0 : i0;
    j0 = j0 < 0 ? 0 : j0;
    i1 = i1 > GS - 1 ? GS - 1 : i1;
    j1 = j1 > GS - 1 ? GS - 1 : j1;
    if (i0 > i1 || j0 > j1) continue;
    for (int cj = j0 / kSub; cj <= j1 / kSub; ++cj)
      for (int ci = i0 / kSub; ci <= i1 / kSub; ++ci) {
        uint32_t mask = 0;
        for (int sj = 0; sj < kSub; ++sj) {
          const int j = cj * kSub + sj;
          if (j < j0 || j > j1) continue;
          for (int si = 0; si < kSub; ++si) {
            const int i = ci * kSub + si;
            if (i < i0 || i > i1) continue;
            if (tri_box_overlap(tx, ty, i - padF, j - padF, i + 1 + padF, j + 1 + padF))
              mask |= 1u << (sj * kSub + si);
          }
        }
        if (mask) emit((uint32_t)f * G * G + (uint32_t)cj * G + (uint32_t)ci, mask);
      }
  }
}

// Cone of the triangle (centre, cos of its angular radius) versus cell k's bounding cone,
// without inverse trigonometry: angle(c, g) <= rho + delta  <=>  c.g >= cos(rho + delta)
// = cosRho cosDelta - sinRho sinDelta (always true once rho + delta >= pi).
IRT_HD bool cap_hits_cell(const BD3 &c, double cosRho, int G, uint32_t k) {
  const uint32_t GG = (uint32_t)G * (uint32_t)G;
  const int f = (int)(k / GG), j = (int)((k % GG) / (uint32_t)G), i = (int)(k % (uint32_t)G);
  const double u0 = 2.0 * i / G - 1, u1 = 2.0 * (i + 1) / G - 1;
  const double v0 = 2.0 * j / G - 1, v1 = 2.0 * (j + 1) / G - 1;
  const BD3 g = face_dir(f, 0.5 * (u0 + u1), 0.5 * (v0 + v1));
  double cosDelta = 1.0;
  cosDelta = dmin(cosDelta, bdot(g, face_dir(f, u0, v0)));
  cosDelta = dmin(cosDelta, bdot(g, face_dir(f, u1, v0)));
  cosDelta = dmin(cosDelta, bdot(g, face_dir(f, u0, v1)));
  cosDelta = dmin(cosDelta, bdot(g, face_dir(f, u1, v1)));
  if (cosDelta + cosRho <= 0.0) return true;
  const double sinRho = sqrt(dmax(0.0, 1.0 - cosRho * cosRho));
  const double sinDelta = sqrt(dmax(0.0, 1.0 - cosDelta * cosDelta));
  return bdot(c, g) >= cosRho * cosDelta - sinRho * sinDelta - kCapSlack;
}

// ---------------------------------------------------------------- per cell: radial bins
// Open bin (lo, hi) membership of a record with radial extent [h0, hN] (irt_common.h).
IRT_HD bool in_bin(float h0, float hN, float lo, float hi) {
  return (h0 < hi && hN > lo) || (h0 == hN && h0 == hi);
}


// Expected number of list entries a radius drawn uniformly from [rmin, rmax] meets, for
// the given edges: sum over bins of (bin length within [rmin, rmax]) * count.
// Entries are read through an accessor E: e.h0(k), e.hN(k) (radial extent of the cell's k-th
// entry, record order) and e.sub(k) (its sub-cell mask) -- host vectors or device arrays.
template <class E>
IRT_HD double bin_cost(const E &en, int n, const float *edges, int ne, double rmin, double rmax) {
  double cost = 0;
  for (int k = 0; k <= ne; ++k) {
    const float lo = k ? edges[k - 1] : -__builtin_inff(), hi = k < ne ? edges[k] : __builtin_inff();
    const double a = dmax(rmin, (double)lo), b = dmin(rmax, (double)hi);
    if (!(b > a)) continue;
    int cnt = 0;
    for (int e = 0; e < n; ++e) cnt += in_bin(en.h0(e), en.hN(e), lo, hi) ? 1 : 0;
    cost += (b - a) * (double)cnt;
  }
  return cost;
}

// Up to kMaxEdges radial edges for one cell, greedily among the records' bottom heights.
// cand: the distinct bottom heights strictly inside (rmin, rmax), ascending (float_key
// order), nc of them.  Returns the number of edges, ascending in edges[].
template <class E>
IRT_HD int choose_edges(const E &en, int n, const float *cand, int nc, double rmin, double rmax,
                        float *edges) {
  if (n <= 2) return 0;
  // bound the search: 48 quantiles
  float q[48];
  int nq = 0;
  const bool quant = nc > 48;
  for (int k = 0; k < (quant ? 48 : nc); ++k) {
    const float v = quant ? cand[(size_t)k * nc / 48] : cand[k];
    if (nq == 0 || !(q[nq - 1] == v)) q[nq++] = v;
  }
  int ne = 0;
  double best = bin_cost(en, n, edges, 0, rmin, rmax);
  while (ne < kMaxEdges) {
    int bi = -1;
    double bc = best;
    for (int i = 0; i < nq; ++i) {
      float tr[kMaxEdges];
      int m = 0;
      bool dup = false;
      for (int k = 0; k < ne; ++k) {
        if (edges[k] == q[i]) dup = true;
        tr[m++] = edges[k];
      }
      if (dup) continue;
      // insert q[i] in order
      int at = m;
      while (at > 0 && float_key(tr[at - 1]) > float_key(q[i])) {
        tr[at] = tr[at - 1];
        --at;
      }
      tr[at] = q[i];
      ++m;
      const double c = bin_cost(en, n, tr, m, rmin, rmax);
      if (c < bc * 0.98) {
        bc = c;
        bi = i;
      }
    }
    if (bi < 0) break;
    int at = ne;
    while (at > 0 && float_key(edges[at - 1]) > float_key(q[bi])) {
      edges[at] = edges[at - 1];
      --at;
    }
    edges[at] = q[bi];
    ++ne;
    best = bc;
  }
  return ne;
}

// The radial range a cell's entries span and its distinct bottom heights strictly inside
// it, ascending (float_key order; insertion sort, so cand needs room for n).
template <class E>
IRT_HD int cell_candidates(const E &en, int n, float *cand, double &rmin, double &rmax) {
  rmin = __builtin_inf();
  rmax = -__builtin_inf();
  for (int e = 0; e < n; ++e) {
    rmin = dmin(rmin, (double)en.h0(e));
    rmax = dmax(rmax, (double)en.hN(e));
  }
  int nc = 0;
  for (int e = 0; e < n; ++e) {
    const float v = en.h0(e);
    if (!((double)v > rmin && (double)v < rmax)) continue;
    bool dup = false;
    for (int k = 0; k < nc; ++k)
      if (cand[k] == v) dup = true;
    if (dup) continue;
    int at = nc;
    while (at > 0 && float_key(cand[at - 1]) > float_key(v)) {
      cand[at] = cand[at - 1];
      --at;
    }
    cand[at] = v;
    ++nc;
  }
  return nc;
}

// Cell header, kBinHdrWords u32 = 128 B:
//   [0..2]   edges e0 < e1 < e2 (float bits; unused = +inf)
//   [3]      base: index of the cell's first fat entry
//   [4..7]   cumulative ends of bins 0..3 (relative to base)
//   [8..23]  per sub-cell s (kSub x kSub, s = sj*kSub + si): byte k = which of the first
//            kMaskCand candidates of bin k can reach sub-cell s
//   [24..31] per quad q of 2 x 2 sub-cells (kQuads of them, quad_of): words 24 + 2q, 25 + 2q =
//            the highest height[numLayers] and the lowest height[0] of the cell's records whose
//            column can reach the quad (-inf / +inf: none).  No point of the quad outside
//            [lowest, highest] passes sample()'s radial test (ICONGrid.h:184) for any record
//            listed here, and every record that can contain it is listed: such a sample is
//            outside every cell without a candidate test.  convert_icon grids have such voids
//            over every land column (its top H[j] = R + HHL - HSURF, convert_icon.cpp:371, lies
//            HSURF below the ocean's) and under it (H[0] = R + HSURF, 361).
// The kernel loads words 0..7 and word 8+s from the same line (and the quad's words 24..).
//
// Fills every word but the base from a cell's n entries (in record order: bottom/top
// heights and sub-cell masks) and its ne edges; returns the cell's number of fat entries.
IRT_HD uint32_t quad_mask(int q) {  // the sub-cells of quad q
  uint32_t m = 0u;
  for (uint32_t s = 0; s < (uint32_t)(kSub * kSub); ++s)
    if (quad_of(s) == q) m |= 1u << s;
  return m;
}

template <class E>
IRT_HD uint32_t cell_header(const E &en, int n, const float *edges, int ne, uint32_t *H) {
  for (int w = 0; w < kBinHdrWords; ++w) H[w] = 0u;
  // words 24..31: the radial range of the records that can reach each quad
  for (int q = 0; q < kQuads; ++q) {
    const uint32_t qm = quad_mask(q);
    float hi = -__builtin_inff(), lo = __builtin_inff();
    for (int e = 0; e < n; ++e) {
      if (!(en.sub(e) & qm)) continue;
      const float a = en.h0(e), b = en.hN(e);
      hi = b > hi ? b : hi;
      lo = a < lo ? a : lo;
    }
    H[kBoundWord + 2 * q] = f2u(hi);
    H[kBoundWord + 1 + 2 * q] = f2u(lo);
  }
  for (int k = 0; k < kMaxEdges; ++k) H[k] = f2u(k < ne ? edges[k] : __builtin_inff());
  uint32_t cum = 0;
  for (int k = 0; k <= kMaxEdges; ++k) {
    if (k <= ne) {
      const float lo = k ? edges[k - 1] : -__builtin_inff(), hi = k < ne ? edges[k] : __builtin_inff();
      int j = 0;
      for (int e = 0; e < n; ++e) {
        if (!in_bin(en.h0(e), en.hN(e), lo, hi)) continue;
        if (j < kMaskCand) {
          const uint32_t sm = en.sub(e);
          for (int s = 0; s < kSub * kSub; ++s)
            if ((sm >> s) & 1u) H[8 + s] |= 1u << (8 * k + j);
        }
        ++j;
        ++cum;
      }
    }
    H[4 + k] = cum;
  }
  return cum;
}

// One fat entry (kFat4 float4, irt_common.h) of record i.
IRT_HD void fat_entry(uint32_t i, const float *planes, const float *rng, const uint32_t *meta,
                      float *F) {
  for (int k = 0; k < 12; ++k) F[k] = planes[12 * (size_t)i + k];
  F[12] = rng[2 * (size_t)i];
  F[13] = rng[2 * (size_t)i + 1];
  F[14] = u2f(i);
  F[15] = u2f(meta[i]);
}

}  // namespace irt
