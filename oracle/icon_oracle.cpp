// icon_oracle.cpp -- CPU ORACLE for the ICON Woodcock-tracking hot path.
//
// TEST INFRASTRUCTURE ONLY.  This file restates, in plain C++, the reference's
// CPU render path (szellmann/icon-ray-tracing, non-RTCORE build) so the MI355X
// product can be checked against it.  It is compiled into oracle/liboracle.so and
// may only be loaded by tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg.  Nothing under icon-ray-tracing_amd/ uses it.
//
// Pinning: oracle/ref_harness.cpp, compiled into oracle/_ref/ by `make -C oracle ref`,
// includes the reference's own headers from /root/reference as they are (vecmath.h,
// dvr_course-common-both.h, dvr_course-common.h, ICONGrid.h, ShellAccel.h, DDA.h,
// UElems.h, camera.h, thread_pool.h, for_each.h) and restates only the ~60 lines of
// deviceCode.cu raygen glue and the host shell build (Params.h needs the absent cuBQL, so
// deviceCode.cu itself does not compile; pipeline.cu / fb.cu / transfunc.cu are not
// compiled either).  tests/golden/ holds fixtures generated from it and
// tests/test_oracle_golden.py checks this restatement against them bit for bit.
//
// Locators (the `fast` argument of oracle_render*): 0 the reference's literal linear scan
// (deviceCode.cu:116-123, sample() recomputing its planes), 1 the same scan over
// precomputed planes, 2 a direction-voxel locator (DirGrid below, the CPU baseline's
// "BVH or column locator" of BASELINE.md): the same first-index-wins answer, each sample
// testing only the records listed for its voxel.
//
// Numerics: every float expression keeps the reference's evaluation order;
// libm calls (asinf, atan2f, sinf, cosf, logf, powf, tanf, atanf, log10f) go to
// the host glibc exactly where the reference calls them; build with
// -ffp-contract=off.  float->int conversions use x86 cvttss2si semantics
// (out-of-range / NaN -> INT_MIN), which is what the reference's g++ build does.

#include "icon_oracle.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <thread>
#include <string>
#include <vector>

namespace {

struct V3 { float x, y, z; };
struct V4 { float x, y, z, w; };
struct I3 { int x, y, z; };
struct B1 { float lower, upper; };
struct B3 { V3 lower, upper; };

inline V3 v3(float s) { return {s, s, s}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator/(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
// vecmath.h:536-538
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vecmath.h:541-548
inline V3 cross(V3 u, V3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
// vecmath.h:550-557
inline V3 normalize(V3 u) { return u / sqrtf(dot(u, u)); }
inline float length(V3 u) { return sqrtf(dot(u, u)); }
inline V3 vmin(V3 a, V3 b) { return {fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)}; }
inline V3 vmax(V3 a, V3 b) { return {fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)}; }
// vecmath.h:512-533
inline float reduce_min(V3 u) { return fminf(fminf(u.x, u.y), u.z); }
inline float reduce_max(V3 u) { return fmaxf(fmaxf(u.x, u.y), u.z); }
// vecmath.h:46-54
inline int imin(int a, int b) { return a < b ? a : b; }
inline int imax(int a, int b) { return b < a ? a : b; }
// vecmath.h:1338-1341
inline int iclamp(int x, int a, int b) { return imax(a, imin(x, b)); }

// float -> int the way the reference's x86-64 g++ build converts (cvttss2si):
// truncation toward zero, INT_MIN for NaN and for anything outside int range.
inline int f2i(float f) {
  if (!(f > -2147483904.0f && f < 2147483648.0f)) return INT32_MIN;
  return (int)f;
}

inline V3 toV3(oc_vec3 v) { return {v.x, v.y, v.z}; }
inline oc_vec3 toOc(V3 v) { return {v.x, v.y, v.z}; }
inline B3 toB3(oc_box3 b) { return {toV3(b.lower), toV3(b.upper)}; }

// ---------------------------------------------------------------- RNG
// LCG<4> (common/dvr_course-common-both.h:41-86)
struct LCG {
  uint32_t state;
  uint64_t draws = 0;
  LCG(uint32_t val0, uint32_t val1) {
    uint32_t v0 = val0, v1 = val1, s0 = 0;
    for (unsigned n = 0; n < 4; n++) {
      s0 += 0x9e3779b9u;
      v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
      v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    state = v0;
  }
  float operator()() {
    state = 1664525u * state + 1013904223u;
    ++draws;
    return (state & 0x00FFFFFFu) / (float)0x01000000;
  }
};

// ---------------------------------------------------------------- geometry
// ICONGrid.h:36-42
inline V3 toSpherical(V3 c) {
  float r = length(c);
  float lat = asinf(c.z / r);
  float lon = atan2f(c.y, c.x);
  return {r, lat, lon};
}
// ICONGrid.h:44-54
inline V3 toCartesian(V3 s) {
  const float r = s.x, lat = s.y, lon = s.z;
  float x = r * cosf(lat) * cosf(lon);
  float y = r * cosf(lat) * sinf(lon);
  float z = r * sinf(lat);
  return {x, y, z};
}
// ICONGrid.h:170-179 (Plane == vec4f(N, dot(a,N)))
inline V4 makePlane(V3 a, V3 b, V3 c) {
  V3 N = cross(b - a, c - a);
  return {N.x, N.y, N.z, dot(a, N)};
}
inline float evalPlane(const V4 &p, V3 pos) { return dot(pos, V3{p.x, p.y, p.z}) - p.w; }

// ICONGrid.h:117-145 (std::lower_bound over height[1..numLayers])
inline int findHeight(const oc_cell &c, float hpos) {
  int first = 0;
  int count = c.numLayers;
  while (count > 0) {
    int it = first;
    int step = count / 2;
    it = it + step;
    if (!(hpos <= c.height[it + 1])) {
      first = ++it;
      count -= step + 1;
    } else {
      count = step;
    }
  }
  return first;
}
// ICONGrid.h:147-164
inline float getValue(const oc_cell &c, float hpos) { return c.value[findHeight(c, hpos)]; }

// The six corners of a cell column (ICONGrid.h:188-195).
inline void corners(const oc_cell &cell, V3 b[3], V3 t[3]) {
  const float h0 = cell.height[0], hN = cell.height[cell.numLayers];
  for (int k = 0; k < 3; ++k) {
    b[k] = toCartesian({h0, cell.lat[k], cell.lon[k]});
    t[k] = toCartesian({hN, cell.lat[k], cell.lon[k]});
  }
}

struct CellPlanes { V4 p[3]; };
inline CellPlanes cellPlanes(const oc_cell &cell) {
  V3 b[3], t[3];
  corners(cell, b, t);
  CellPlanes P;
  P.p[0] = makePlane(b[0], b[1], t[1]);
  P.p[1] = makePlane(b[1], b[2], t[2]);
  P.p[2] = makePlane(b[2], b[0], t[0]);
  return P;
}

// sample(cell,pos,value) (ICONGrid.h:181-208), literal: toSpherical first,
// corners and planes recomputed per call.
inline bool sampleLiteral(const oc_cell &cell, V3 pos, float &value) {
  const V3 spherical = toSpherical(pos);
  if (spherical.x < cell.height[0] || spherical.x > cell.height[cell.numLayers]) return false;
  CellPlanes P = cellPlanes(cell);
  if (evalPlane(P.p[0], pos) > 0.f) return false; /* ccw */
  if (evalPlane(P.p[1], pos) > 0.f) return false;
  if (evalPlane(P.p[2], pos) > 0.f) return false;
  value = getValue(cell, spherical.x);
  return true;
}
// Same predicate, same result: lat/lon of toSpherical are dead in sample(), and
// the planes depend only on the cell, so they can be precomputed.
inline bool sampleFast(const oc_cell &cell, const CellPlanes &P, V3 pos, float &value) {
  const float r = length(pos);
  if (r < cell.height[0] || r > cell.height[cell.numLayers]) return false;
  if (evalPlane(P.p[0], pos) > 0.f) return false;
  if (evalPlane(P.p[1], pos) > 0.f) return false;
  if (evalPlane(P.p[2], pos) > 0.f) return false;
  value = getValue(cell, r);
  return true;
}

// ICONGrid.h:78-115
inline B3 getBounds(const oc_cell &c) {
  B3 bounds{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
  V3 bv1 = toCartesian({c.height[0], c.lat[0], c.lon[0]});
  V3 bv2 = toCartesian({c.height[0], c.lat[1], c.lon[1]});
  V3 bv3 = toCartesian({c.height[0], c.lat[2], c.lon[2]});
  bounds.lower = vmin(bounds.lower, bv1); bounds.upper = vmax(bounds.upper, bv1);
  bounds.lower = vmin(bounds.lower, bv2); bounds.upper = vmax(bounds.upper, bv2);
  bounds.lower = vmin(bounds.lower, bv3); bounds.upper = vmax(bounds.upper, bv3);
  V3 tv1 = toCartesian({c.height[c.numLayers], c.lat[0], c.lon[0]});
  V3 tv2 = toCartesian({c.height[c.numLayers], c.lat[1], c.lon[1]});
  V3 tv3 = toCartesian({c.height[c.numLayers], c.lat[2], c.lon[2]});
  V3 bary = (tv1 + tv2 + tv3) / 3.f;
  float R = c.height[c.numLayers];
  float D = R - length(bary);
  float off = D / R;
  tv1 = tv1 + tv1 * off;
  tv2 = tv2 + tv2 * off;
  tv3 = tv3 + tv3 * off;
  bounds.lower = vmin(bounds.lower, tv1); bounds.upper = vmax(bounds.upper, tv1);
  bounds.lower = vmin(bounds.lower, tv2); bounds.upper = vmax(bounds.upper, tv2);
  bounds.lower = vmin(bounds.lower, tv3); bounds.upper = vmax(bounds.upper, tv3);
  return bounds;
}

// ---------------------------------------------------------------- ray / shell
struct Ray { V3 org; float tmin; V3 dir; float tmax; };
inline V3 eval(const Ray &r, float t) { return r.org + r.dir * t; }

// vecmath.h:1926-1937
inline bool boxTest(const Ray &ray, const B3 &box, float &t0, float &t1) {
  const V3 t_lo = (box.lower - ray.org) / ray.dir;
  const V3 t_hi = (box.upper - ray.org) / ray.dir;
  const V3 t_nr = vmin(t_lo, t_hi);
  const V3 t_fr = vmax(t_lo, t_hi);
  t0 = fmaxf(ray.tmin, reduce_max(t_nr));
  t1 = fminf(ray.tmax, reduce_min(t_fr));
  return t0 < t1;
}

// ShellAccel.h:34-53
inline bool intersectSphere(const Ray &ray, float radius, float &tnear, float &tfar) {
  float A = dot(ray.dir, ray.dir);
  float B = dot(ray.dir, ray.org) * 2.f;
  float C = dot(ray.org, ray.org) - radius * radius;
  float d = B * B - 4.f * A * C;
  if (d < 0.f) return false;
  d = sqrtf(d);
  float q = B < 0.f ? -0.5f * (B - d) : -0.5f * (B + d);
  float t1 = q / A;
  float t2 = C / q;
  tnear = fminf(t1, t2);
  tfar = fmaxf(t1, t2);
  return true;
}

// ShellAccel.h:57-68 (note dims-1)
inline I3 projectToSphericalGrid(V3 sph, const int dims[3], const B3 &sb) {
  const float radSize = sb.upper.x - sb.lower.x;
  const float latSize = sb.upper.y - sb.lower.y;
  const float lonSize = sb.upper.z - sb.lower.z;
  return {f2i((sph.x - sb.lower.x) / radSize * (dims[0] - 1)),
          f2i((sph.y - sb.lower.y) / latSize * (dims[1] - 1)),
          f2i((sph.z - sb.lower.z) / lonSize * (dims[2] - 1))};
}
// ShellAccel.h:71-80
inline I3 normalizeGridCoord(I3 c, const int dims[3]) {
  while (c.x < 0) c.x += dims[0];
  while (c.x >= dims[0]) c.x -= dims[0];
  while (c.y < 0) c.y += dims[1];
  while (c.y >= dims[1]) c.y -= dims[1];
  while (c.z < 0) c.z += dims[2];
  while (c.z >= dims[2]) c.z -= dims[2];
  return c;
}
// DDA.h:15-21
inline size_t linearIndex(I3 i, const int dims[3]) {
  return i.z * size_t(dims[0]) * dims[1] + i.y * dims[0] + i.x;
}

// sdda (ShellAccel.h:82-229), literal -- including the degenerate r=0 planes.
template <typename Func>
inline void sdda(Ray ray, const int dims[3], const B3 &sb, const Func &func) {
  const float sceneEPS = sb.lower.x * 1e-6f;
  float t1 = 0.f, t2 = 0.f, t3 = 0.f, t4 = 0.f;
  bool s1 = intersectSphere(ray, sb.upper.x, t1, t4);
  bool s2 = intersectSphere(ray, sb.lower.x, t2, t3);
  if (!s1 && !s2) return;
  if (t4 < ray.tmin) return;
  B1 ranges[2] = {{INFINITY, -INFINITY}, {INFINITY, -INFINITY}};
  if (s1 && !s2) {
    ranges[0] = {t1, t4};
  } else if (ray.tmin < t2) {
    ranges[0] = {t1, t2};
    ranges[1] = {t3, t4};
  } else {
    ranges[0] = {t3, t4};
  }
  for (int i = 0; i < 2; ++i) {
    if (ranges[i].upper <= ranges[i].lower) break;  // box1f::empty (vecmath.h:981)
    V3 P1 = eval(ray, ranges[i].lower + sceneEPS);
    V3 P2 = eval(ray, ranges[i].upper - sceneEPS);
    V3 SP1 = toSpherical(P1);
    V3 SP2 = toSpherical(P2);
    const B1 radBounds{sb.lower.x, sb.upper.x};
    const B1 latBounds{sb.lower.y, sb.upper.y};
    const B1 lonBounds{sb.lower.z, sb.upper.z};
    const float radInc = (radBounds.upper - radBounds.lower) / float(dims[0]);
    const float latInc = (latBounds.upper - latBounds.lower) / float(dims[1]);
    const float lonInc = (lonBounds.upper - lonBounds.lower) / float(dims[2]);
    I3 cellID = projectToSphericalGrid(SP1, dims, sb);
    const I3 step = {SP1.x < SP2.x ? 1 : -1, SP1.y < SP2.y ? 1 : -1, SP1.z < SP2.z ? 1 : -1};
    I3 stop = projectToSphericalGrid(SP2, dims, sb);
    stop = {stop.x + step.x, stop.y + step.y, stop.z + step.z};
    float radOff = (cellID.x + step.x) * radInc;
    float latOff = (cellID.y + step.y) * latInc;
    float lonOff = (cellID.z + step.z) * lonInc;
    float radius = step.x == 1 ? sb.lower.x + radOff : sb.upper.x + radOff;
    float sphereT1, sphereT2;
    bool sphereHit = intersectSphere(ray, radius, sphereT1, sphereT2);
    if (!sphereHit) sphereT1 = ranges[i].upper;
    (void)sphereT1;
    V4 latPlane = makePlane(v3(0.f), toCartesian({0.f, latOff, latBounds.lower}),
                            toCartesian({0.f, latOff, latBounds.upper}));
    V4 lonPlane = makePlane(v3(0.f), toCartesian({0.f, lonBounds.lower, lonOff}),
                            toCartesian({0.f, lonBounds.upper, lonOff}));
    V3 tnext = {ranges[i].upper, evalPlane(latPlane, eval(ray, ranges[i].lower)),
                evalPlane(lonPlane, eval(ray, ranges[i].lower))};
    float t = ranges[i].lower;
    while (1) {
      V3 P = ray.org + ray.dir * t;
      float tt1 = FLT_MAX;
      if (tnext.x < tt1 && tnext.x >= t) tt1 = tnext.x;
      if (tnext.y < tt1 && tnext.y >= t) tt1 = tnext.y;
      if (tnext.z < tt1 && tnext.z >= t) tt1 = tnext.z;
      int leafID = (int)linearIndex(normalizeGridCoord(cellID, dims), dims);
      if (!func(leafID, t, tt1)) return;
      const float t_closest = reduce_min(tnext);
      if (tnext.x == t_closest) {
        cellID.x += step.x;
        if (cellID.x == stop.x) break;
      }
      if (tnext.y == t_closest) {
        cellID.y += step.y;
        if (cellID.y == stop.y) break;
        V4 plane = makePlane(v3(0.f), toCartesian({0.f, cellID.y * latInc, latBounds.lower}),
                             toCartesian({0.f, cellID.y * latInc, latBounds.upper}));
        tnext.y = evalPlane(plane, P);
      }
      if (tnext.z == t_closest) {
        cellID.z += step.z;
        if (cellID.z == stop.z) break;
        V4 plane = makePlane(v3(0.f), toCartesian({0.f, lonBounds.lower, cellID.z * lonInc}),
                             toCartesian({0.f, lonBounds.upper, cellID.z * lonInc}));
        tnext.z = evalPlane(plane, P);
      }
      t = t_closest;
    }
  }
}

// projectOnGrid (DDA.h:23-31)
inline I3 projectOnGrid(V3 V, const int dims[3], const B3 &wb) {
  const V3 V01 = (V - wb.lower) / (wb.upper - wb.lower);
  const V3 Vs = V01 * V3{(float)dims[0], (float)dims[1], (float)dims[2]};
  return {iclamp(f2i(Vs.x), 0, dims[0] - 1), iclamp(f2i(Vs.y), 0, dims[1] - 1),
          iclamp(f2i(Vs.z), 0, dims[2] - 1)};
}

// dda3 (DDA.h:35-136) as the reference's g++ CPU build compiles it: vecmath.h declares no
// float min, so `min(reduce_min(tnext), ray.tmax)` (96) resolves to int min(int, int)
// (vecmath.h:46-49): both operands truncated, the result converted back to float.
template <typename Func>
inline void dda3(Ray ray, const int dims[3], const B3 &modelBounds, const Func &func) {
  const float ray_tmin = ray.tmin;
  ray.org = ray.org + v3(ray.tmin) * ray.dir;
  ray.tmin = 0.f;
  ray.tmax -= ray_tmin;
  const V3 rcp_dir = v3(1.f) / ray.dir;
  const V3 lo = (modelBounds.lower - ray.org) * rcp_dir;
  const V3 hi = (modelBounds.upper - ray.org) * rcp_dir;
  V3 tnear = vmin(lo, hi);
  const V3 tfar = vmax(lo, hi);
  if (ray.dir.x == 0.f) tnear.x = FLT_MAX;
  if (ray.dir.y == 0.f) tnear.y = FLT_MAX;
  if (ray.dir.z == 0.f) tnear.z = FLT_MAX;
  I3 cellID = projectOnGrid(ray.org, dims, modelBounds);
  const V3 dist = vmax(v3(0.f), (tfar - tnear) / V3{(float)dims[0], (float)dims[1], (float)dims[2]});
  const I3 step = {ray.dir.x > 0.f ? 1 : -1, ray.dir.y > 0.f ? 1 : -1, ray.dir.z > 0.f ? 1 : -1};
  const I3 stop = {ray.dir.x > 0.f ? dims[0] : -1, ray.dir.y > 0.f ? dims[1] : -1,
                   ray.dir.z > 0.f ? dims[2] : -1};
  V3 tnext = {ray.dir.x > 0.f ? tnear.x + float(cellID.x + 1) * dist.x
                              : tnear.x + float(dims[0] - cellID.x) * dist.x,
              ray.dir.y > 0.f ? tnear.y + float(cellID.y + 1) * dist.y
                              : tnear.y + float(dims[1] - cellID.y) * dist.y,
              ray.dir.z > 0.f ? tnear.z + float(cellID.z + 1) * dist.z
                              : tnear.z + float(dims[2] - cellID.z) * dist.z};
  float t0 = 0.f;
  while (1) {
    const float t1 = (float)imin(f2i(reduce_min(tnext)), f2i(ray.tmax));
    if (!func((int)linearIndex(cellID, dims), ray_tmin + t0, ray_tmin + t1)) return;
    const float t_closest = reduce_min(tnext);
    if (tnext.x == t_closest) {
      tnext.x += dist.x;
      cellID.x += step.x;
      if (cellID.x == stop.x) break;
    }
    if (tnext.y == t_closest) {
      tnext.y += dist.y;
      cellID.y += step.y;
      if (cellID.y == stop.y) break;
    }
    if (tnext.z == t_closest) {
      tnext.z += dist.z;
      cellID.z += step.z;
      if (cellID.z == stop.z) break;
    }
    t0 = t1;
  }
}

// ---------------------------------------------------------------- shading
// dvr_course-common-both.h:30-35
inline float linear_to_srgb(float x) {
  if (x <= 0.0031308f) return 12.92f * x;
  return 1.055f * powf(x, 1.f / 2.4f) - 0.055f;
}
// dvr_course-common-both.h:89-92
inline uint32_t make_8bit(const float f) {
  return (uint32_t)fminf(255, fmaxf(0, (float)f2i(f * 256.f)));
}
// dvr_course-common-both.h:103-110
inline uint32_t make_rgba(V4 c) {
  return (make_8bit(c.x) << 0) + (make_8bit(c.y) << 8) + (make_8bit(c.z) << 16) +
         (make_8bit(c.w) << 24);
}

// postClassify (deviceCode.cu:127-135)
inline V4 postClassify(const oc_params &p, float v) {
  v = (v - p.tf_lower) / (p.tf_upper - p.tf_lower);
  int idx = f2i(v * (p.lut_size));
  float frac = (v * p.lut_size) - idx;
  const float *v1 = p.lut + 4 * iclamp(idx, 0, p.lut_size - 1);
  const float *v2 = p.lut + 4 * iclamp(idx + 1, 0, p.lut_size - 1);
  const float om = 1.f - frac;
  return {v1[0] * frac + v2[0] * om * 1.f, v1[1] * frac + v2[1] * om * 1.f,
          v1[2] * frac + v2[2] * om * 1.f, v1[3] * frac + v2[3] * om * p.opacityScale};
}

// ---------------------------------------------------------------- CUBQL_MODE wedges
// The unstructured-element sampler (deviceCode.cu:90-115): wedges built per (cell, layer)
// as buildCuBQLAccel does (hostCode.cu:557-600), each sample the first wedge whose
// primBounds (534-552) contain the point and whose intersectWedgeEXT (UElems.h:214-311)
// accepts it.  cuBQL's traversal order is unpinned (the submodule is absent); "first"
// here is the lowest wedge index, the order a linear scan of the build would give.
struct Wedge {
  V4 v[6];
  B3 box;
};

// determinant(mat3f) (vecmath.h:733-748) of make_LinearSpace3f(c0, c1, c2) (UElems.h:20-28):
// m(row, col) is component `row` of column `col`
inline float det3(V3 c0, V3 c1, V3 c2) {
  auto det2 = [](float m00, float m01, float m10, float m11) { return m00 * m11 - m10 * m01; };
  const float a00 = det2(c1.y, c2.y, c1.z, c2.z);
  const float a01 = det2(c0.y, c2.y, c0.z, c2.z);
  const float a02 = det2(c0.y, c1.y, c0.z, c1.z);
  return c0.x * a00 - c1.x * a01 + c2.x * a02;
}

// intersectWedgeEXT (UElems.h:176-311), the OpenVKL Newton inversion.  Quirks kept:
// norm2(bbox.size()) binds to norm2(vec2f) through vec2f's converting constructor
// (vecmath.h:317, 386-389), so the tolerance ignores z; WEDGE_CONVERGED /
// WEDGE_OUTSIDE_CELL_TOLERANCE are double literals (compared / folded in double).
inline bool intersectWedgeEXT(float &value, V3 P, const V4 V[6]) {
  B3 bbox{v3(1e31f), v3(-1e31f)};
  for (int i = 0; i < 6; ++i) {
    bbox.lower = vmin(bbox.lower, V3{V[i].x, V[i].y, V[i].z});
    bbox.upper = vmax(bbox.upper, V3{V[i].x, V[i].y, V[i].z});
  }
  const V3 sz = bbox.upper - bbox.lower;
  const float determinantTolerance = (sz.x * sz.x + sz.y * sz.y) * 1e-6f;
  float pc[3] = {.5f, .5f, .5f};
  float w[6], dv[18];
  bool converged = false;
  for (int it = 0; !converged && it < 10; ++it) {
    w[0] = (1.f - pc[0] - pc[1]) * (1.f - pc[2]);  // wedgeInterpolationFunctions (176-184)
    w[1] = pc[0] * (1.f - pc[2]);
    w[2] = pc[1] * (1.f - pc[2]);
    w[3] = (1.f - pc[0] - pc[1]) * pc[2];
    w[4] = pc[0] * pc[2];
    w[5] = pc[1] * pc[2];
    dv[0] = -1.f + pc[2];  // wedgeInterpolationDerivs (187-212)
    dv[1] = 1.f - pc[2];
    dv[2] = 0.f;
    dv[3] = -pc[2];
    dv[4] = pc[2];
    dv[5] = 0.f;
    dv[6] = -1.f + pc[2];
    dv[7] = 0.f;
    dv[8] = 1.f - pc[2];
    dv[9] = -pc[2];
    dv[10] = 0.f;
    dv[11] = pc[2];
    dv[12] = -1.f + pc[0] + pc[1];
    dv[13] = -pc[0];
    dv[14] = -pc[1];
    dv[15] = 1.f - pc[0] - pc[1];
    dv[16] = pc[0];
    dv[17] = pc[1];
    V3 f = v3(0.f), r = v3(0.f), s = v3(0.f), t = v3(0.f);
    for (int i = 0; i < 6; ++i) {
      const V3 pt{V[i].x, V[i].y, V[i].z};
      f = f + pt * w[i];
      r = r + pt * dv[i];
      s = s + pt * dv[i + 6];
      t = t + pt * dv[i + 12];
    }
    f = f - P;
    const float d = det3(r, s, t);
    if (fabsf(d) < determinantTolerance) return false;
    const float d0 = det3(f, s, t) / d;
    const float d1 = det3(r, f, t) / d;
    const float d2 = det3(r, s, f) / d;
    pc[0] = pc[0] - d0;
    pc[1] = pc[1] - d1;
    pc[2] = pc[2] - d2;
    if (((double)fabsf(d0) < 1e-4) & ((double)fabsf(d1) < 1e-4) & ((double)fabsf(d2) < 1e-4)) {
      converged = true;
    } else if ((fabsf(pc[0]) > 1e6) | (fabsf(pc[1]) > 1e6) | (fabsf(pc[2]) > 1e6)) {
      return false;
    }
  }
  if (!converged) return false;
  const float lo = (float)(0.f - 1e-6), hi = (float)(1.f + 1e-6);
  if (pc[0] >= lo && pc[0] <= hi && pc[1] >= lo && pc[1] <= hi && pc[2] >= lo && pc[2] <= hi &&
      pc[0] + pc[1] <= hi) {
    float val = 0.f;
    for (int i = 0; i < 6; ++i) val += w[i] * V[i].w;
    value = val;
    return true;
  }
  return false;
}

// buildCuBQLAccel's wedges (hostCode.cu:557-600) and computeBounds (534-552)
void buildWedges(const oc_cell *cells, size_t n, std::vector<Wedge> &out) {
  out.clear();
  for (size_t i = 0; i < n; ++i) {
    const oc_cell &cell = cells[i];
    for (int h = 0; h < cell.numLayers; ++h) {
      Wedge wd;
      const float bv = h == 0 ? getValue(cell, cell.height[h])
                              : (getValue(cell, cell.height[h - 1]) + getValue(cell, cell.height[h])) * 0.5f;
      for (int k = 0; k < 3; ++k) {
        const V3 b = toCartesian({cell.height[h], cell.lat[k], cell.lon[k]});
        const V3 t = toCartesian({cell.height[h + 1], cell.lat[k], cell.lon[k]});
        wd.v[k] = {b.x, b.y, b.z, bv};
        wd.v[k + 3] = {t.x, t.y, t.z, bv};  // `#if 1`: the top takes bv too (574-577)
      }
      wd.box = B3{v3(1e31f), v3(-1e31f)};
      for (int k = 0; k < 6; ++k) {
        wd.box.lower = vmin(wd.box.lower, V3{wd.v[k].x, wd.v[k].y, wd.v[k].z});
        wd.box.upper = vmax(wd.box.upper, V3{wd.v[k].x, wd.v[k].y, wd.v[k].z});
      }
      out.push_back(wd);
    }
  }
}

inline bool boxContains(const B3 &b, V3 p) {  // box3f::contains (vecmath.h:1088-1092)
  return b.lower.x <= p.x && p.x <= b.upper.x && b.lower.y <= p.y && p.y <= b.upper.y &&
         b.lower.z <= p.z && p.z <= b.upper.z;
}

// ---------------------------------------------------------------- TRIANGLE_MODE
// deviceCode.cu:61-76 with buildTriangleAccel's triangles (hostCode.cu:445-450): a ray from
// the sample toward the Earth's centre, back faces culled, the closest hit's cell, then its
// radial range and getValue.  OptiX's triangle test is not available: Moller-Trumbore (the
// product's definition, csrc/irt_common.h ray_triangle; parity unpinned), the lowest index
// winning equal distances.
inline bool rayTriangle(V3 o, V3 d, V3 a, V3 b, V3 c, float &t) {
  const V3 e1 = b - a, e2 = c - a;
  const V3 p{d.y * e2.z - d.z * e2.y, d.z * e2.x - d.x * e2.z, d.x * e2.y - d.y * e2.x};
  const float det = e1.x * p.x + e1.y * p.y + e1.z * p.z;
  if (!(det > 0.f)) return false;
  const V3 tv = o - a;
  const float u = tv.x * p.x + tv.y * p.y + tv.z * p.z;
  if (u < 0.f || u > det) return false;
  const V3 q{tv.y * e1.z - tv.z * e1.y, tv.z * e1.x - tv.x * e1.z, tv.x * e1.y - tv.y * e1.x};
  const float v = d.x * q.x + d.y * q.y + d.z * q.z;
  if (v < 0.f || u + v > det) return false;
  t = (e2.x * q.x + e2.y * q.y + e2.z * q.z) / det;
  return t > 0.f;
}

struct Tri {
  V3 v[3];
};

// ---------------------------------------------------------------- renderer
// ---------------------------------------------------------------- direction-voxel locator
// Every record whose sample() can accept a point with unit direction u is listed in the
// voxel of u in a V^3 grid over [-1,1]^3, in index order; only occupied voxels are stored
// (sorted 64-bit keys + CSR).  A record's accepting directions are its corner triangle's
// geodesic patch (or, for clockwise corners, the antipodal patch; found by probing its own
// float planes), whose points q/|q| (q on the flat triangle) lie in the corners' box
// stretched by 1/d, d = the flat triangle's distance from the origin; the box is padded by
// 1e-5 (> the float error of a sample point's direction).  Records whose planes carve out
// no cone, or whose patch is too wide for the box bound (d < 0.05), and zero-thickness
// records (accepting every direction at one radius) are tested for every sample.
struct DirGrid {
  int V = 0;
  std::vector<uint64_t> keys;   // occupied voxels, ascending
  std::vector<uint32_t> off;    // keys.size() + 1
  std::vector<uint32_t> recs;   // per voxel, ascending record indices
  std::vector<uint32_t> always; // tested for every sample, ascending
};

struct Scene {
  const oc_cell *cells;
  size_t n;
  int fast;
  DirGrid grid;
  std::vector<CellPlanes> planes;  // fast mode only
  std::vector<Wedge> wedges;       // CUBQL_MODE only
  bool useWedges = false;
  std::vector<float> rr;           // fast mode: {height[0], height[numLayers]} per record
  std::vector<Tri> tris;           // TRIANGLE_MODE only
  bool useTriangles = false;
};

void buildTriangles(Scene &S) {
  S.tris.resize(S.n);
  for (size_t i = 0; i < S.n; ++i)
    for (int k = 0; k < 3; ++k)
      S.tris[i].v[k] = toCartesian({S.cells[i].height[0], S.cells[i].lat[k], S.cells[i].lon[k]});
}

inline bool sampleTriangles(const Scene &S, V3 pos, float &value) {
  const V3 d = -normalize(pos);  // ray.direction = -normalize(ray.origin) (deviceCode.cu:67)
  float best = INFINITY;
  size_t hit = (size_t)-1;
  for (size_t i = 0; i < S.n; ++i) {
    float t;
    if (rayTriangle(pos, d, S.tris[i].v[0], S.tris[i].v[1], S.tris[i].v[2], t) && t < best) {
      best = t;
      hit = i;
    }
  }
  if (hit == (size_t)-1) return false;
  const oc_cell &cell = S.cells[hit];
  const float r = length(pos);  // toSpherical(pos).x (deviceCode.cu:70)
  if (r < cell.height[0] || r > cell.height[cell.numLayers]) return false;
  value = getValue(cell, r);
  return true;
}

// Fast mode's per-record tables (the same tests in the same order, read from compact
// arrays), built on nthreads threads.
void buildFast(Scene &S, int nthreads) {
  S.planes.resize(S.n);
  S.rr.resize(2 * S.n);
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  const size_t chunk = (S.n + nthreads - 1) / nthreads;
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t)
    ts.emplace_back([&S, t, chunk] {
      const size_t b = t * chunk, e = std::min(S.n, b + chunk);
      for (size_t i = b; i < e; ++i) {
        S.planes[i] = cellPlanes(S.cells[i]);
        S.rr[2 * i] = S.cells[i].height[0];
        S.rr[2 * i + 1] = S.cells[i].height[S.cells[i].numLayers];
      }
    });
  for (auto &th : ts) th.join();
}

struct ThreadStats {
  uint64_t launched = 0, inBox = 0, locate = 0, found = 0, draws = 0, leaves = 0;
  // analysis only (oracle_trace_pixels): one letter per counted sampleVolume call -- 'm' outside
  // every cell, 'l' located and rejected, 'A' accepted -- 'E' for a call ending past its tmax
  std::string *trace = nullptr;
  std::vector<float> *missPos = nullptr;  // (analysis) each 'm' sample's point, xyz
};

// sampleVolume, CPU branch: first cell index wins (deviceCode.cu:116-123)
inline uint64_t dirKey(const DirGrid &G, double x, double y, double z) {
  auto q = [&](double c) {
    long v = (long)std::floor((c + 1.0) * 0.5 * G.V);
    return (uint64_t)std::max(0L, std::min((long)G.V - 1, v));
  };
  return (q(z) * (uint64_t)G.V + q(y)) * (uint64_t)G.V + q(x);
}

void buildDirGrid(Scene &S, int nthreads) {
  DirGrid &G = S.grid;
  size_t cols = 0;
  for (size_t i = 0; i < S.n; ++i)
    if (i == 0 || memcmp(S.cells[i].lat, S.cells[i - 1].lat, 12) || memcmp(S.cells[i].lon, S.cells[i - 1].lon, 12))
      ++cols;
  // a voxel about one corner triangle wide: edge ~ sqrt(4 * (4 pi / cols) / sqrt(3)) radians
  G.V = (int)std::max(8.0, std::min(2048.0, 2.0 / std::sqrt(29.0 / (double)std::max<size_t>(cols, 1))));
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> parts(nthreads);
  std::vector<std::vector<uint32_t>> alw(nthreads);
  const size_t chunk = (S.n + nthreads - 1) / nthreads;
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t)
    ts.emplace_back([&, t] {
      for (size_t i = t * chunk; i < std::min(S.n, (t + 1) * chunk); ++i) {
        const oc_cell &c = S.cells[i];
        const float h0 = c.height[0], hN = c.height[c.numLayers];
        if (!(h0 <= hN)) continue;  // inverted: the radial test never passes
        if (h0 == hN) {             // zero thickness: any direction at r == h0
          alw[t].push_back((uint32_t)i);
          continue;
        }
        double d[3][3];
        for (int k = 0; k < 3; ++k) {
          const double la = c.lat[k], lo = c.lon[k];
          d[k][0] = std::cos(la) * std::cos(lo), d[k][1] = std::cos(la) * std::sin(lo), d[k][2] = std::sin(la);
        }
        // which cone do the float planes carve out: probe the centroid and its antipode
        double m[3] = {d[0][0] + d[1][0] + d[2][0], d[0][1] + d[1][1] + d[2][1], d[0][2] + d[1][2] + d[2][2]};
        const double ml = std::sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
        const CellPlanes P = S.fast ? S.planes[i] : cellPlanes(c);
        int side = -1;
        const double rm = 0.5 * ((double)h0 + (double)hN);
        for (int sgn = 0; sgn < 2 && side < 0 && ml > 0; ++sgn) {
          const double s = (sgn ? -rm : rm) / ml;
          const V3 p{(float)(m[0] * s), (float)(m[1] * s), (float)(m[2] * s)};
          if (!(evalPlane(P.p[0], p) > 0.f) && !(evalPlane(P.p[1], p) > 0.f) && !(evalPlane(P.p[2], p) > 0.f))
            side = sgn;
        }
        // distance of the flat triangle's plane from the origin
        const double e1[3] = {d[1][0] - d[0][0], d[1][1] - d[0][1], d[1][2] - d[0][2]};
        const double e2[3] = {d[2][0] - d[0][0], d[2][1] - d[0][1], d[2][2] - d[0][2]};
        const double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const double nl = std::sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
        const double dist = nl > 0 ? std::fabs(nv[0] * d[0][0] + nv[1] * d[0][1] + nv[2] * d[0][2]) / nl : 0.0;
        if (side < 0 || !(dist >= 0.05)) {
          alw[t].push_back((uint32_t)i);
          continue;
        }
        const double sg = side ? -1.0 : 1.0;
        double lo3[3], hi3[3];
        for (int a = 0; a < 3; ++a) {
          double mn = 1e9, mx = -1e9;
          for (int k = 0; k < 3; ++k) {
            mn = std::min(mn, sg * d[k][a]);
            mx = std::max(mx, sg * d[k][a]);
          }
          lo3[a] = std::min(mn, mn / dist) - 1e-5;
          hi3[a] = std::max(mx, mx / dist) + 1e-5;
        }
        auto q = [&](double c2) {
          long v = (long)std::floor((c2 + 1.0) * 0.5 * G.V);
          return std::max(0L, std::min((long)G.V - 1, v));
        };
        for (long z = q(lo3[2]); z <= q(hi3[2]); ++z)
          for (long y = q(lo3[1]); y <= q(hi3[1]); ++y)
            for (long x = q(lo3[0]); x <= q(hi3[0]); ++x)
              parts[t].emplace_back(((uint64_t)z * G.V + (uint64_t)y) * G.V + (uint64_t)x, (uint32_t)i);
      }
    });
  for (auto &th : ts) th.join();
  std::vector<std::pair<uint64_t, uint32_t>> all;
  size_t total = 0;
  for (auto &p : parts) total += p.size();
  all.reserve(total);
  for (auto &p : parts) {
    all.insert(all.end(), p.begin(), p.end());
    std::vector<std::pair<uint64_t, uint32_t>>().swap(p);
  }
  std::sort(all.begin(), all.end());  // by voxel, then record index
  G.recs.resize(all.size());
  G.off.assign(1, 0u);
  for (size_t k = 0; k < all.size(); ++k) {
    if (k == 0 || all[k].first != all[k - 1].first) {
      if (k) G.off.push_back((uint32_t)k);
      G.keys.push_back(all[k].first);
    }
    G.recs[k] = all[k].second;
  }
  G.off.push_back((uint32_t)all.size());
  for (auto &a : alw) G.always.insert(G.always.end(), a.begin(), a.end());
  std::sort(G.always.begin(), G.always.end());
}

// fast == 2: the voxel's records and the always-tested ones, merged in index order
inline bool sampleGrid(const Scene &S, V3 pos, float &value) {
  const DirGrid &G = S.grid;
  const double l = std::sqrt((double)pos.x * pos.x + (double)pos.y * pos.y + (double)pos.z * pos.z);
  const uint32_t *a = nullptr, *ae = nullptr;
  if (l > 0) {
    const uint64_t key = dirKey(G, pos.x / l, pos.y / l, pos.z / l);
    const auto it = std::lower_bound(G.keys.begin(), G.keys.end(), key);
    if (it != G.keys.end() && *it == key) {
      const size_t k = it - G.keys.begin();
      a = G.recs.data() + G.off[k];
      ae = G.recs.data() + G.off[k + 1];
    }
  }
  const uint32_t *b = G.always.data(), *be = b + G.always.size();
  if (l == 0) b = G.always.data(), be = b;  // unreachable for a sample in the shell
  const float r = length(pos);
  while (a != ae || b != be) {
    uint32_t i;
    if (b == be || (a != ae && *a < *b)) i = *a++;
    else i = *b++;
    if (r < S.rr[2 * i] || r > S.rr[2 * i + 1]) continue;
    if (sampleFast(S.cells[i], S.planes[i], pos, value)) return true;
  }
  if (l == 0) {  // direction undefined: the reference's scan, literally
    for (size_t i = 0; i < S.n; ++i)
      if (sampleFast(S.cells[i], S.planes[i], pos, value)) return true;
  }
  return false;
}

inline bool sampleVolume(const Scene &S, V3 pos, float &value) {
  if (S.useTriangles) return sampleTriangles(S, pos, value);  // TRIANGLE_MODE
  if (S.useWedges) {  // CUBQL_MODE (deviceCode.cu:90-115)
    for (const Wedge &wd : S.wedges)
      if (boxContains(wd.box, pos) && intersectWedgeEXT(value, pos, wd.v)) return true;
    return false;
  }
  if (S.fast == 2) return sampleGrid(S, pos, value);
  if (S.fast) {
    const float r = length(pos);
    for (size_t i = 0; i < S.n; ++i) {
      if (r < S.rr[2 * i] || r > S.rr[2 * i + 1]) continue;  // sampleFast's first test
      if (sampleFast(S.cells[i], S.planes[i], pos, value)) return true;
    }
  } else {
    for (size_t i = 0; i < S.n; ++i)
      if (sampleLiteral(S.cells[i], pos, value)) return true;
  }
  return false;
}

// woodcockTracking (deviceCode.cu:149-186)
inline float woodcockTracking(const Scene &S, const oc_params &p, const Ray &ray, LCG &rnd,
                              float majorant, V3 &albedo, float &extinction, ThreadStats &ts) {
  float t = ray.tmin;
  while (1) {
    if (majorant <= 0.f) break;
    t -= (logf(1.f - rnd()) / (majorant / p.unitDistance));
    if (t > ray.tmax) {
      if (ts.trace) ts.trace->push_back('E');
      break;
    }
    V3 P = ray.org + ray.dir * t;
    float value{0.f};
    ++ts.locate;
    if (!sampleVolume(S, P, value)) {
      if (ts.trace) ts.trace->push_back('m');
      if (ts.missPos) ts.missPos->insert(ts.missPos->end(), {P.x, P.y, P.z});
      continue;
    }
    ++ts.found;
    V4 sample = postClassify(p, value);
    float u = rnd();
    if (ts.trace) ts.trace->push_back(sample.w >= u * majorant ? 'A' : 'l');
    if (sample.w >= u * majorant) {
      albedo = {sample.x, sample.y, sample.z};
      extinction = sample.w;
      break;
    }
  }
  return fminf(t, ray.tmax);
}

// generateRay (deviceCode.cu:36-49).  The reference's expression
//   dir_00 + (screen.u+rnd())*dir_du + (screen.v+rnd())*dir_dv
// leaves the two rnd() calls unsequenced; g++ (the reference's CPU compiler)
// evaluates the dir_dv operand's rnd() first.  oracle/ref_harness.cpp pins this.
inline Ray generateRay(const oc_params &p, float su, float sv, LCG &rnd) {
  const float jv = rnd();
  const float ju = rnd();
  V3 dir = toV3(p.dir_00) + v3(su + ju) * toV3(p.dir_du) + v3(sv + jv) * toV3(p.dir_dv);
  dir = normalize(dir);
  if (fabsf(dir.x) < 1e-5f) dir.x = 1e-5f;
  if (fabsf(dir.y) < 1e-5f) dir.y = 1e-5f;
  if (fabsf(dir.z) < 1e-5f) dir.z = 1e-5f;
  return Ray{toV3(p.org), 0.f, dir, 1e10f};
}

// lerp (vecmath.h:1333-1336): x*a + (1-x)*b, then srgb + RGBA8 (deviceCode.cu:333-340)
inline void accumulate(const oc_params &p, V3 color, float alpha, float *acc, uint32_t *fbp) {
  const float a = 1.f / (p.accumID + 1);
  V4 old{acc[0], acc[1], acc[2], acc[3]};
  V4 nv{color.x, color.y, color.z, alpha};
  V4 r{a * nv.x + (1.f - a) * old.x, a * nv.y + (1.f - a) * old.y, a * nv.z + (1.f - a) * old.z,
       a * nv.w + (1.f - a) * old.w};
  acc[0] = r.x; acc[1] = r.y; acc[2] = r.z; acc[3] = r.w;
  V4 c = r;
  c.x = linear_to_srgb(c.x);
  c.y = linear_to_srgb(c.y);
  c.z = linear_to_srgb(c.z);
  *fbp = make_rgba(c);
}

// RAYGEN woodcockTrackingWithAccel (deviceCode.cu:281-341) and
// woodcockTrackingAE (deviceCode.cu:239-275) for one pixel.
void raygen(const Scene &S, const oc_params &p, int x, int y, int W, int H, float *accum,
            uint32_t *fb, ThreadStats &ts) {
  const int pixelID = x + W * y;
  ++ts.launched;
  LCG rnd((uint32_t)p.accumID * (uint32_t)W * (uint32_t)H + (uint32_t)x, (uint32_t)y);
  Ray ray = generateRay(p, (float)x + .5f, (float)y + .5f, rnd);
  float t0, t1;
  const B3 bounds = toB3(p.bounds);
  if (!boxTest(ray, bounds, t0, t1)) {
    ts.draws += rnd.draws;
    return;
  }
  ++ts.inBox;
  ray.tmin = t0;
  ray.tmax = t1;
  V3 color = v3(0.f);
  float alpha = 0.f;
  const V3 amb = toV3(p.ambientColor);
  if (p.raygen == 1) {
    V3 albedo = v3(0.f);
    float extinction = 0.f;
    woodcockTracking(S, p, ray, rnd, 1.f, albedo, extinction, ts);
    color = albedo * amb * p.ambientRadiance;
    alpha = extinction > 0.f ? 1.f : 0.f;
  } else {
    const B3 sb = toB3(p.sphericalBounds);
    auto woodcockFunc = [&](const int leafID, float tt0, float tt1) {
      ++ts.leaves;
      V3 albedo = v3(0.f);
      float extinction = 0.f;
      const float majorant = p.maxOpacities[leafID];
      ray.tmin = tt0;
      ray.tmax = tt1;
      // sampleVolume calls inside zero-length leaves (every leaf after a range's first,
      // since the reference's lat/lon planes are degenerate) can never change the pixel and
      // are not counted; the GPU kernel skips those it does not need for the RNG state.
      ThreadStats uncounted;
      if (ts.trace && tt0 != tt1) ts.trace->push_back('|');
      float t = woodcockTracking(S, p, ray, rnd, majorant, albedo, extinction,
                                 tt0 == tt1 ? uncounted : ts);
      if (t > tt0 && t < tt1) {
        color = albedo * amb * p.ambientRadiance;
        alpha = extinction > 0.f ? 1.f : 0.f;
        return false;
      }
      return true;
    };
    if (p.accelMode == 1) {  // GRID_ACCEL_MODE (deviceCode.cu:326-328)
      const float *gridMaxOp = p.gridMaxOpacities;
      auto gridFunc = [&](const int leafID, float tt0, float tt1) {
        ++ts.leaves;
        V3 albedo = v3(0.f);
        float extinction = 0.f;
        const float majorant = gridMaxOp[leafID];
        ray.tmin = tt0;
        ray.tmax = tt1;
        ThreadStats uncounted;
        float t = woodcockTracking(S, p, ray, rnd, majorant, albedo, extinction,
                                   tt0 == tt1 ? uncounted : ts);
        if (t > tt0 && t < tt1) {
          color = albedo * amb * p.ambientRadiance;
          alpha = extinction > 0.f ? 1.f : 0.f;
          return false;
        }
        return true;
      };
      dda3(ray, p.gridDims, toB3(p.gridBounds), gridFunc);
    } else {
      sdda(ray, p.dims, sb, woodcockFunc);
    }
  }
  accumulate(p, color, alpha, accum + 4 * (size_t)pixelID, fb + pixelID);
  ts.draws += rnd.draws;
}

}  // namespace

// ======================================================================== C API

extern "C" {

size_t oracle_filter_cells(oc_cell *cells, size_t n, float latLo, float latHi, float lonLo,
                           float lonHi) {
  // deg2rad (ICONGrid.h:26-29): d*float(M_PI)/180.f
  auto d2r = [](float d) { return d * float(M_PI) / 180.f; };
  const float la0 = d2r(latLo), la1 = d2r(latHi), lo0 = d2r(lonLo), lo1 = d2r(lonHi);
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    const oc_cell &c = cells[i];
    bool drop = (c.lat[0] < la0 || c.lat[1] < la0 || c.lat[2] < la0) ||
                (c.lat[0] > la1 || c.lat[1] > la1 || c.lat[2] > la1) ||
                (c.lon[0] < lo0 || c.lon[1] < lo0 || c.lon[2] < lo0) ||
                (c.lon[0] > lo1 || c.lon[1] > lo1 || c.lon[2] > lo1);
    if (!drop) {
      if (k != i) cells[k] = cells[i];
      ++k;
    }
  }
  return k;
}

void oracle_compute_bounds(const oc_cell *cells, size_t n, oc_box3 *sphericalBounds,
                           oc_box3 *volbounds, float *dataRange) {
  B3 vb{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
  B3 sb{v3(INFINITY), v3(-INFINITY)};
  B1 dr{INFINITY, -INFINITY};
  for (size_t i = 0; i < n; ++i) {
    const oc_cell &cell = cells[i];
    float minLat = fminf(cell.lat[0], fminf(cell.lat[1], cell.lat[2]));
    float maxLat = fmaxf(cell.lat[0], fmaxf(cell.lat[1], cell.lat[2]));
    float minLon = fminf(cell.lon[0], fminf(cell.lon[1], cell.lon[2]));
    float maxLon = fmaxf(cell.lon[0], fmaxf(cell.lon[1], cell.lon[2]));
    sb.lower.x = fminf(sb.lower.x, cell.height[0]);
    sb.upper.x = fmaxf(sb.upper.x, cell.height[cell.numLayers]);
    sb.lower.y = fminf(sb.lower.y, minLat);
    sb.upper.y = fmaxf(sb.upper.y, maxLat);
    sb.lower.z = fminf(sb.lower.z, minLon);
    sb.upper.z = fmaxf(sb.upper.z, maxLon);
    B3 b = getBounds(cell);
    vb.lower = vmin(vb.lower, b.lower);
    vb.upper = vmax(vb.upper, b.upper);
    for (int j = 0; j < cell.numLayers; ++j) {
      dr.lower = fminf(dr.lower, cell.value[j]);
      dr.upper = fmaxf(dr.upper, cell.value[j]);
    }
  }
  *sphericalBounds = {toOc(sb.lower), toOc(sb.upper)};
  *volbounds = {toOc(vb.lower), toOc(vb.upper)};
  dataRange[0] = dr.lower;
  dataRange[1] = dr.upper;
}

float oracle_unit_distance(float innerRadius) {
  float magnitude = floorf(log10f(innerRadius));
  float scale = powf(10.f, magnitude - 3);
  return 1.0f * scale;
}

void oracle_default_lut5(float *out) {
  static const float lut[20] = {0.149f, 0.015f, 0.705f, 1.0f,  0.486f, 0.603f, 0.956f,
                                0.75f,  0.866f, 0.866f, 0.866f, 0.5f, 0.996f, 0.690f,
                                0.552f, 0.25f,  0.752f, 0.298f, 0.231f, 0.0f};
  memcpy(out, lut, sizeof(lut));
}

void oracle_resample_lut(const float *src, int nsrc, float *dst, int ndst) {
  for (int i = 0; i < ndst; ++i) {
    float indexf = i / (float)(ndst) * (nsrc - 1);
    int indexa = (int)indexf;
    int indexb = std::min(indexa + 1, nsrc - 1);
    float frac = indexf - indexa;
    float x = 1.f - frac;
    for (int c = 0; c < 4; ++c)
      dst[4 * i + c] = x * src[4 * indexa + c] + (1.f - x) * src[4 * indexb + c];
  }
}

static void cameraFrame(V3 origin, V3 poi, V3 up, float fovy, float aspect, oc_vec3 *out4) {
  // Camera::setOrientation (camera.h:34-54) + forceUpFrame (56-64) + getScreen (86-96)
  V3 vz = (poi.x == origin.x && poi.y == origin.y && poi.z == origin.z)
              ? V3{0, 0, 1}
              : -normalize(poi - origin);
  V3 vx = cross(up, vz);
  if (dot(vx, vx) < 1e-8f)
    vx = {0, 1, 0};
  else
    vx = normalize(vx);
  V3 vy = normalize(cross(vz, vx));
  if (!(fabsf(dot(vz, up)) < 1e-6f)) {
    vx = normalize(cross(up, vz));
    vy = normalize(cross(vz, vx));
  }
  float screen_height = 2.f * tanf(0.5f * fovy);
  V3 vertical = v3(screen_height) * vy;
  V3 horizontal = v3(screen_height * aspect) * vx;
  V3 lower_left = -vz - v3(0.5f) * vertical - v3(0.5f) * horizontal;
  out4[0] = toOc(origin);
  out4[1] = toOc(lower_left);
  out4[2] = toOc(horizontal);
  out4[3] = toOc(vertical);
}

void oracle_camera_view_all(oc_box3 box, float fovy_deg, float aspect, oc_vec3 *out4) {
  // camera.h:108 (member default) / pipeline.cu:451 conversion
  const float fovy = fovy_deg * M_PI / 180.f;
  B3 b = toB3(box);
  V3 up{0, 1, 0};
  float diagonal = length(b.upper - b.lower);
  float r = diagonal * 0.5f;
  V3 center = (b.lower + b.upper) / 2.f;
  V3 eye = center + V3{0, 0, r + r / std::atan(fovy)};
  cameraFrame(eye, center, up, fovy, aspect, out4);
}

void oracle_camera_orient(oc_vec3 vp, oc_vec3 vi, oc_vec3 vu, float fovy_deg, float aspect,
                          oc_vec3 *out4) {
  // Pipeline::Impl::setCamera (pipeline.cu:444-454)
  float f = fovy_deg;
  if (f < 1e-3f) f = 90.f;
  const float fovy = f * M_PI / 180.f;
  cameraFrame(toV3(vp), toV3(vi), toV3(vu), fovy, aspect, out4);
}

void oracle_build_shell(const oc_cell *cells, size_t n, const int32_t dims[3],
                        oc_box3 sphericalBounds, float *valueRanges) {
  const int d[3] = {dims[0], dims[1], dims[2]};
  const size_t numMCs = (size_t)d[0] * d[1] * d[2];
  // initGrid(ShellAccel) (hostCode.cu:216-225)
  for (size_t i = 0; i < numMCs; ++i) {
    valueRanges[2 * i] = FLT_MAX;
    valueRanges[2 * i + 1] = -FLT_MAX;
  }
  const B3 sb = toB3(sphericalBounds);
  // buildShell_ICON (hostCode.cu:299-336); float atomicMin/Max (36-56) only store when
  // strictly smaller/larger -- an order-independent min/max (up to the sign of a zero,
  // which depends on atomic arrival order in the reference too), so cells are split over
  // threads with private grids, merged the same way.
  int nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  if (n < 100000) nthreads = 1;
  std::vector<std::vector<float>> priv(nthreads - 1);
  auto rasterize = [&](size_t c0, size_t c1, float *vrBase) {
  for (size_t ci = c0; ci < c1; ++ci) {
    const oc_cell &cell = cells[ci];
    for (int i = 0; i < cell.numLayers; ++i) {
      I3 c1 = projectToSphericalGrid({cell.height[i], cell.lat[0], cell.lon[0]}, d, sb);
      I3 c2 = projectToSphericalGrid({cell.height[i], cell.lat[1], cell.lon[1]}, d, sb);
      I3 c3 = projectToSphericalGrid({cell.height[i], cell.lat[2], cell.lon[2]}, d, sb);
      I3 c4 = projectToSphericalGrid({cell.height[i + 1], cell.lat[0], cell.lon[0]}, d, sb);
      I3 c5 = projectToSphericalGrid({cell.height[i + 1], cell.lat[1], cell.lon[1]}, d, sb);
      I3 c6 = projectToSphericalGrid({cell.height[i + 1], cell.lat[2], cell.lon[2]}, d, sb);
      I3 lo{imin(c1.x, imin(c2.x, c3.x)), imin(c1.y, imin(c2.y, c3.y)),
            imin(c1.z, imin(c2.z, c3.z))};
      I3 up{imax(c4.x, imax(c5.x, c6.x)), imax(c4.y, imax(c5.y, c6.y)),
            imax(c4.z, imax(c5.z, c6.z))};
      B1 range{getValue(cell, cell.height[i]), getValue(cell, cell.height[i + 1])};
      for (int mcz = lo.z; mcz <= up.z; ++mcz)
        for (int mcy = lo.y; mcy <= up.y; ++mcy)
          for (int mcx = lo.x; mcx <= up.x; ++mcx) {
            size_t id = linearIndex({mcx, mcy, mcz}, d);
            float *vr = vrBase + 2 * id;
            if (range.lower < vr[0]) vr[0] = range.lower;
            if (range.upper > vr[1]) vr[1] = range.upper;
          }
    }
  }
  };
  const size_t chunk = (n + nthreads - 1) / nthreads;
  std::vector<std::thread> ts;
  for (int t = 1; t < nthreads; ++t) {
    priv[t - 1].resize(2 * numMCs);
    float *p = priv[t - 1].data();
    for (size_t i = 0; i < numMCs; ++i) {
      p[2 * i] = FLT_MAX;
      p[2 * i + 1] = -FLT_MAX;
    }
    ts.emplace_back(rasterize, std::min(n, t * chunk), std::min(n, (t + 1) * chunk), p);
  }
  rasterize(0, std::min(n, chunk), valueRanges);
  for (auto &th : ts) th.join();
  for (auto &p : priv)
    for (size_t i = 0; i < numMCs; ++i) {
      if (p[2 * i] < valueRanges[2 * i]) valueRanges[2 * i] = p[2 * i];
      if (p[2 * i + 1] > valueRanges[2 * i + 1]) valueRanges[2 * i + 1] = p[2 * i + 1];
    }
}

void oracle_build_grid(const oc_cell *cells, size_t n, const int32_t dims[3], oc_box3 worldBounds,
                       float *valueRanges) {
  const int d[3] = {dims[0], dims[1], dims[2]};
  const size_t numMCs = (size_t)d[0] * d[1] * d[2];
  for (size_t i = 0; i < numMCs; ++i) {  // initGrid(Grid) (hostCode.cu:205-214)
    valueRanges[2 * i] = FLT_MAX;
    valueRanges[2 * i + 1] = -FLT_MAX;
  }
  const B3 wb = toB3(worldBounds);
  for (size_t ci = 0; ci < n; ++ci) {  // buildGrid_ICON (hostCode.cu:245-297)
    const oc_cell &cell = cells[ci];
    for (int i = 0; i < cell.numLayers; ++i) {
      B3 bounds{v3(INFINITY), v3(-INFINITY)};
      V3 bv[3], tv[3];
      for (int k = 0; k < 3; ++k) {
        bv[k] = toCartesian({cell.height[i], cell.lat[k], cell.lon[k]});
        tv[k] = toCartesian({cell.height[i + 1], cell.lat[k], cell.lon[k]});
      }
      for (int k = 0; k < 3; ++k) {
        bounds.lower = vmin(bounds.lower, bv[k]);
        bounds.upper = vmax(bounds.upper, bv[k]);
      }
      const V3 bary = (tv[0] + tv[1] + tv[2]) / 3.f;
      const float R = cell.height[i + 1];
      const float D = R - length(bary);
      const float off = D / R;
      for (int k = 0; k < 3; ++k) {
        tv[k] = tv[k] + tv[k] * off;
        bounds.lower = vmin(bounds.lower, tv[k]);
        bounds.upper = vmax(bounds.upper, tv[k]);
      }
      B1 range{INFINITY, -INFINITY};  // box1f::extend (vecmath.h:1001-1004)
      const float g0 = getValue(cell, cell.height[i]), g1 = getValue(cell, cell.height[i + 1]);
      range.lower = fminf(range.lower, g0);
      range.upper = fmaxf(range.upper, g0);
      range.lower = fminf(range.lower, g1);
      range.upper = fmaxf(range.upper, g1);
      // rasterizeBox (hostCode.cu:227-243)
      const I3 lo = projectOnGrid(bounds.lower, d, wb), up = projectOnGrid(bounds.upper, d, wb);
      for (int mcz = lo.z; mcz <= up.z; ++mcz)
        for (int mcy = lo.y; mcy <= up.y; ++mcy)
          for (int mcx = lo.x; mcx <= up.x; ++mcx) {
            float *vr = valueRanges + 2 * linearIndex({mcx, mcy, mcz}, d);
            if (range.lower < vr[0]) vr[0] = range.lower;
            if (range.upper > vr[1]) vr[1] = range.upper;
          }
    }
  }
}

void oracle_max_opacities(const float *valueRanges, size_t numMCs, const float *lut, int size,
                          float tfLo, float tfHi, float *maxOpacities) {
  for (size_t mc = 0; mc < numMCs; ++mc) {
    B1 vr{valueRanges[2 * mc], valueRanges[2 * mc + 1]};
    if (vr.upper < vr.lower) {
      maxOpacities[mc] = 0.f;
      continue;
    }
    vr.lower -= tfLo;
    vr.lower /= tfHi - tfLo;
    vr.upper -= tfLo;
    vr.upper /= tfHi - tfLo;
    int lo = iclamp(f2i(vr.lower * (size - 1)), 0, size - 1);
    int hi = iclamp(f2i(vr.upper * (size - 1)) + 1, 0, size - 1);
    float maxOpacity = 0.f;
    for (int i = lo; i <= hi; ++i) maxOpacity = fmaxf(maxOpacity, lut[4 * i + 3]);
    maxOpacities[mc] = maxOpacity;
  }
}

void oracle_clear(uint32_t *fb, float *accum, size_t numPixels) {
  V4 zero{0.f, 0.f, 0.f, 0.f};
  uint32_t c = make_rgba(zero);
  for (size_t i = 0; i < numPixels; ++i) {
    if (fb) fb[i] = c;
    if (accum) accum[4 * i] = accum[4 * i + 1] = accum[4 * i + 2] = accum[4 * i + 3] = 0.f;
  }
}

namespace {
// the frame over 64x64 tiles pulled from an atomic counter (parallel::for_each,
// common/for_each.h:70-85, parallel_for.h:62-82, thread_pool.h:146-161)
int render_tiles(const Scene &S, const oc_params *p, int W, int H, int x0, int y0, int x1, int y1,
                 float *accum, uint32_t *fb, int nthreads, oc_stats *stats) {
  const int tw = 64, th = 64;
  const int ntx = (x1 - x0 + tw - 1) / tw, nty = (y1 - y0 + th - 1) / th;
  const long numTiles = (long)ntx * nty;
  std::atomic<long> counter{0};
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  std::vector<ThreadStats> tstats(nthreads);
  auto worker = [&](int tid) {
    ThreadStats &ts = tstats[tid];
    for (;;) {
      long tile = counter.fetch_add(1);
      if (tile >= numTiles) break;
      int fx = (int)(tile % ntx) * tw + x0, lx = std::min(fx + tw, x1);
      int fy = (int)(tile / ntx) * th + y0, ly = std::min(fy + th, y1);
      for (int y = fy; y < ly; ++y)
        for (int x = fx; x < lx; ++x) raygen(S, *p, x, y, W, H, accum, fb, ts);
    }
  };
  std::vector<std::thread> threads;
  for (int t = 1; t < nthreads; ++t) threads.emplace_back(worker, t);
  worker(0);
  for (auto &t : threads) t.join();
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    for (auto &ts : tstats) {
      stats->rays_launched += ts.launched;
      stats->rays_in_box += ts.inBox;
      stats->locate_calls += ts.locate;
      stats->samples_found += ts.found;
      stats->rng_draws += ts.draws;
      stats->leaves += ts.leaves;
    }
  }
  return 0;
}

void prepare(Scene &S, const oc_params *p, int nthreads) {
  if (S.fast && S.planes.empty() && S.n) buildFast(S, nthreads);
  if (S.fast == 2 && S.grid.V == 0) buildDirGrid(S, nthreads);
  if (p && p->mode == 2 && !S.useWedges) {
    S.useWedges = true;
    buildWedges(S.cells, S.n, S.wedges);
  }
  if (p && p->mode == 1 && !S.useTriangles) {
    S.useTriangles = true;
    buildTriangles(S);
  }
}
}  // namespace

struct oc_scene {
  Scene S;
};

oc_scene *oracle_scene_new(const oc_cell *cells, size_t n, int fast, int nthreads) {
  oc_scene *s = new oc_scene{Scene{cells, n, fast, {}, {}, {}, false, {}, {}, false}};
  prepare(s->S, nullptr, nthreads);
  return s;
}

int oracle_scene_render(oc_scene *s, const oc_params *p, int W, int H, int x0, int y0, int x1,
                        int y1, float *accum, uint32_t *fb, int nthreads, oc_stats *stats) {
  if (!s || !p || W <= 0 || H <= 0 || x0 < 0 || y0 < 0 || x1 > W || y1 > H) return -1;
  if (x1 <= x0 || y1 <= y0) return 0;
  prepare(s->S, p, nthreads);
  return render_tiles(s->S, p, W, H, x0, y0, x1, y1, accum, fb, nthreads, stats);
}

void oracle_scene_free(oc_scene *s) { delete s; }

int oracle_render(const oc_cell *cells, size_t n, const oc_params *p, int W, int H, int x0,
                  int y0, int x1, int y1, float *accum, uint32_t *fb, int nthreads, int fast,
                  oc_stats *stats) {
  if (!p || W <= 0 || H <= 0 || x0 < 0 || y0 < 0 || x1 > W || y1 > H) return -1;
  if (x1 <= x0 || y1 <= y0) return 0;
  Scene S{cells, n, fast, {}, {}, {}, false, {}, {}, false};
  prepare(S, p, nthreads);
  return render_tiles(S, p, W, H, x0, y0, x1, y1, accum, fb, nthreads, stats);
}

int oracle_render_pixels(const oc_cell *cells, size_t n, const oc_params *p, int W, int H,
                         const int32_t *xy, int numPixels, float *accum, uint32_t *fb,
                         int nthreads, int fast, oc_stats *stats) {
  if (!p || W <= 0 || H <= 0 || numPixels < 0) return -1;
  for (int i = 0; i < numPixels; ++i)
    if (xy[2 * i] < 0 || xy[2 * i] >= W || xy[2 * i + 1] < 0 || xy[2 * i + 1] >= H) return -1;
  Scene S{cells, n, fast, {}, {}, {}, false, {}, {}, false};
  prepare(S, p, nthreads);
  std::atomic<int> counter{0};
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  std::vector<ThreadStats> tstats(nthreads);
  auto worker = [&](int tid) {
    for (;;) {
      int i = counter.fetch_add(1);
      if (i >= numPixels) break;
      raygen(S, *p, xy[2 * i], xy[2 * i + 1], W, H, accum, fb, tstats[tid]);
    }
  };
  std::vector<std::thread> threads;
  for (int t = 1; t < nthreads; ++t) threads.emplace_back(worker, t);
  worker(0);
  for (auto &t : threads) t.join();
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    for (auto &ts : tstats) {
      stats->rays_launched += ts.launched;
      stats->rays_in_box += ts.inBox;
      stats->locate_calls += ts.locate;
      stats->samples_found += ts.found;
      stats->rng_draws += ts.draws;
      stats->leaves += ts.leaves;
    }
  }
  return 0;
}

// Analysis only (profiles/sample_pattern.py): the sample outcomes of each pixel's ray, as
// letters (ThreadStats::trace) with '|' before each counted woodcockFunc call; pixel i's string
// at out + i * stride, NUL-terminated, cut at stride - 1 letters.
int oracle_trace_pixels(const oc_cell *cells, size_t n, const oc_params *p, int W, int H,
                        const int32_t *xy, int numPixels, char *out, int stride, int nthreads) {
  if (!p || W <= 0 || H <= 0 || numPixels < 0 || stride < 1) return -1;
  Scene S{cells, n, 2, {}, {}, {}, false, {}, {}, false};
  prepare(S, p, nthreads);
  std::atomic<int> counter{0};
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  std::vector<float> acc(4 * (size_t)W * H);
  std::vector<uint32_t> fb((size_t)W * H);
  auto worker = [&]() {
    ThreadStats ts;
    std::string tr;
    ts.trace = &tr;
    for (;;) {
      int i = counter.fetch_add(1);
      if (i >= numPixels) break;
      tr.clear();
      raygen(S, *p, xy[2 * i], xy[2 * i + 1], W, H, acc.data(), fb.data(), ts);
      const size_t m = std::min(tr.size(), (size_t)stride - 1);
      memcpy(out + (size_t)i * stride, tr.data(), m);
      out[(size_t)i * stride + m] = 0;
    }
  };
  std::vector<std::thread> threads;
  for (int t = 1; t < nthreads; ++t) threads.emplace_back(worker);
  worker();
  for (auto &t : threads) t.join();
  return 0;
}

// Analysis only: the points of the counted samples outside every cell of the listed pixels'
// rays (xyz floats into out, at most cap points); returns the number of points (all of them,
// even past cap), -1 on bad arguments.
long oracle_trace_misses(const oc_cell *cells, size_t n, const oc_params *p, int W, int H,
                         const int32_t *xy, int numPixels, float *out, long cap, int nthreads) {
  if (!p || W <= 0 || H <= 0 || numPixels < 0) return -1;
  Scene S{cells, n, 2, {}, {}, {}, false, {}, {}, false};
  prepare(S, p, nthreads);
  std::atomic<int> counter{0};
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  std::vector<float> acc(4 * (size_t)W * H);
  std::vector<uint32_t> fb((size_t)W * H);
  std::vector<std::vector<float>> pts(nthreads);
  auto worker = [&](int tid) {
    ThreadStats ts;
    ts.missPos = &pts[tid];
    for (;;) {
      int i = counter.fetch_add(1);
      if (i >= numPixels) break;
      raygen(S, *p, xy[2 * i], xy[2 * i + 1], W, H, acc.data(), fb.data(), ts);
    }
  };
  std::vector<std::thread> threads;
  for (int t = 1; t < nthreads; ++t) threads.emplace_back(worker, t);
  worker(0);
  for (auto &t : threads) t.join();
  long k = 0;
  for (auto &v : pts)
    for (size_t j = 0; j + 2 < v.size(); j += 3, ++k)
      if (k < cap) memcpy(out + 3 * k, &v[j], 3 * sizeof(float));
  return k;
}

// ------------------------------------------------------------------ KATs
void oracle_lcg(uint32_t seed0, uint32_t seed1, int n, float *out) {
  LCG r(seed0, seed1);
  for (int i = 0; i < n; ++i) out[i] = r();
}

int oracle_sample(const oc_cell *cell, oc_vec3 pos, float *value) {
  float v = 0.f;
  bool ok = sampleLiteral(*cell, toV3(pos), v);
  if (ok) *value = v;
  return ok ? 1 : 0;
}

int oracle_find_height(const oc_cell *cell, float h) { return findHeight(*cell, h); }

int oracle_intersect_sphere(oc_vec3 org, oc_vec3 dir, float radius, float *tn, float *tf) {
  Ray r{toV3(org), 0.f, toV3(dir), 1e10f};
  return intersectSphere(r, radius, *tn, *tf) ? 1 : 0;
}

int oracle_box_test(oc_vec3 org, oc_vec3 dir, float tmin, float tmax, oc_box3 box, float *t0,
                    float *t1) {
  Ray r{toV3(org), tmin, toV3(dir), tmax};
  return boxTest(r, toB3(box), *t0, *t1) ? 1 : 0;
}

int oracle_sdda_trace(oc_vec3 org, oc_vec3 dir, float tmin, float tmax, const int32_t dims[3],
                      oc_box3 sphericalBounds, int maxOut, int32_t *leaf, float *t0, float *t1) {
  Ray r{toV3(org), tmin, toV3(dir), tmax};
  const int d[3] = {dims[0], dims[1], dims[2]};
  int count = 0;
  sdda(r, d, toB3(sphericalBounds), [&](int l, float a, float b) {
    if (count < maxOut) {
      leaf[count] = l;
      t0[count] = a;
      t1[count] = b;
    }
    ++count;
    return count < 100000;
  });
  return count;
}

int oracle_dda3_trace(oc_vec3 org, oc_vec3 dir, float tmin, float tmax, const int32_t dims[3],
                      oc_box3 worldBounds, int maxOut, int32_t *leaf, float *t0, float *t1) {
  Ray r{toV3(org), tmin, toV3(dir), tmax};
  const int d[3] = {dims[0], dims[1], dims[2]};
  int count = 0;
  dda3(r, d, toB3(worldBounds), [&](int l, float a, float b) {
    if (count < maxOut) {
      leaf[count] = l;
      t0[count] = a;
      t1[count] = b;
    }
    ++count;
    return count < 100000;
  });
  return count;
}

int oracle_intersect_wedge(const float *v24, oc_vec3 p, float *value) {
  V4 V[6];
  for (int i = 0; i < 6; ++i) V[i] = {v24[4 * i], v24[4 * i + 1], v24[4 * i + 2], v24[4 * i + 3]};
  float v = 0.f;
  const bool hit = intersectWedgeEXT(v, toV3(p), V);
  if (hit) *value = v;
  return hit;
}

int oracle_wedge_sample(const oc_cell *cells, size_t n, oc_vec3 p, float *value) {
  Scene S{cells, n, 0, {}, {}, {}, true, {}, {}, false};
  buildWedges(cells, n, S.wedges);
  return sampleVolume(S, toV3(p), *value);
}

int oracle_triangle_sample(const oc_cell *cells, size_t n, oc_vec3 p, float *value) {
  Scene S{cells, n, 0, {}, {}, {}, false, {}, {}, true};
  buildTriangles(S);
  return sampleVolume(S, toV3(p), *value);
}

float oracle_linear_to_srgb(float x) { return linear_to_srgb(x); }

uint32_t oracle_make_rgba(const float *c) { return make_rgba({c[0], c[1], c[2], c[3]}); }

void oracle_to_spherical(oc_vec3 c, oc_vec3 *out) { *out = toOc(toSpherical(toV3(c))); }
void oracle_to_cartesian(oc_vec3 s, oc_vec3 *out) { *out = toOc(toCartesian(toV3(s))); }

void oracle_get_bounds(const oc_cell *cell, oc_box3 *out) {
  B3 b = getBounds(*cell);
  *out = {toOc(b.lower), toOc(b.upper)};
}

void oracle_post_classify(const float *lut, int size, float lo, float hi, float opacityScale,
                          float v, float *out4) {
  oc_params p{};
  p.lut = lut;
  p.lut_size = size;
  p.tf_lower = lo;
  p.tf_upper = hi;
  p.opacityScale = opacityScale;
  V4 r = postClassify(p, v);
  out4[0] = r.x; out4[1] = r.y; out4[2] = r.z; out4[3] = r.w;
}

}  // extern "C"
