// ref_harness.cpp -- builds oracle/_ref/libiconref.so from the REFERENCE's own
// headers under /root/reference (TEST INFRASTRUCTURE ONLY; see oracle/Makefile).
//
// Compiled as-is from /root/reference (no stand-in headers): common/vecmath.h,
// common/dvr_course-common-both.h (LCG, linear_to_srgb, make_rgba),
// common/dvr_course-common.h (resampleLUT), common/camera.h (Camera),
// common/thread_pool.h + common/for_each.h (the CPU parallel_for),
// icon_rt/ICONGrid.h (ICONCell, sample, toSpherical/toCartesian),
// icon_rt/ShellAccel.h (intersectSphere, sdda), icon_rt/DDA.h (linearIndex, projectOnGrid,
// dda3), icon_rt/UElems.h (intersectWedgeEXT).
//
// icon_rt/deviceCode.cu itself cannot be compiled here: it includes Params.h,
// which includes cuBQL/traversal/fixedBoxQuery.h from the un-vendored cuBQL
// submodule (empty in the snapshot).  So the ~60 lines of raygen glue from
// deviceCode.cu (generateRay 36-49, the CPU sampleVolume loop 116-123,
// postClassify 127-135, woodcockTracking 149-186, the two raygens 239-341) and
// the host setup / shell build from hostCode.cu (CUDA-only) are restated below
// with the reference's own vector types and operators -- in particular the
// unsequenced `dir_00 + (u+rnd())*dir_du + (v+rnd())*dir_dv` expression is kept
// verbatim so the draw order is whatever g++ does for the reference.
//
// oracle/icon_oracle.cpp is an independent restatement; tests compare the two.

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include <dvr_course-common.h>
#include <dvr_course-common.cuh>
#include <for_each.h>
#include <thread_pool.h>

#include "DDA.h"
#include "ICONGrid.h"
#include "ShellAccel.h"
#include "UElems.h"

using namespace dvr_course;
using namespace icon_rt;

static_assert(sizeof(ICONCell) == 284, "ICONCell layout");

namespace {

struct RefParams {
  vec3f org, dir_00, dir_du, dir_dv;
  int accumID;
  vec3f ambientColor;
  float ambientRadiance;
  float unitDistance;
  int raygen;
  box3f bounds;
  ShellAccel accel;
  box1f tfRange;
  float opacityScale;
  const vec4f *lut;
  int lutSize;
  const ICONCell *cells;
  int numCells;
};

struct Counters {
  unsigned long long locate = 0, found = 0;
};

// volume.gridAccel + volume.accelMode (Params.h:44-49, 74), set by ref_set_accel
struct GridAccel {
  int accelMode = 0;  // SPHERE_ACCEL_MODE
  vec3i dims;
  box3f worldBounds;
  const float *maxOpacities = nullptr;
} g_grid;

// CUBQL_MODE (Params.h:31, 60): the wedge UMesh of buildCuBQLAccel (hostCode.cu:557-600)
// with its primBounds (computeBounds, 534-552), sampled as deviceCode.cu:90-115 does; the
// cuBQL BVH's traversal order is replaced by wedge index order (cuBQL is not vendored).
struct WedgeMesh {
  int mode = 0;
  std::vector<vec3f> vertices;
  std::vector<float> scalars;
  std::vector<int> indices;
  std::vector<box3f> primBounds;
} g_wedges;

void buildWedgeMesh(const ICONCell *cells, int numCells) {
  auto &W = g_wedges;
  W.vertices.clear();
  W.scalars.clear();
  W.indices.clear();
  W.primBounds.clear();
  for (int i = 0; i < numCells; ++i) {
    const ICONCell &cell = cells[i];
    for (int h = 0; h < cell.numLayers; ++h) {
      vec3f bv1 = toCartesian({cell.height[h], cell.lat.x, cell.lon.x});
      vec3f bv2 = toCartesian({cell.height[h], cell.lat.y, cell.lon.y});
      vec3f bv3 = toCartesian({cell.height[h], cell.lat.z, cell.lon.z});
      vec3f tv1 = toCartesian({cell.height[h + 1], cell.lat.x, cell.lon.x});
      vec3f tv2 = toCartesian({cell.height[h + 1], cell.lat.y, cell.lon.y});
      vec3f tv3 = toCartesian({cell.height[h + 1], cell.lat.z, cell.lon.z});
      float bv = h == 0 ? cell.getValue(cell.height[h])
                        : (cell.getValue(cell.height[h - 1]) + cell.getValue(cell.height[h])) * 0.5f;
      int idx0 = (int)W.vertices.size();
      for (const vec3f &v : {bv1, bv2, bv3, tv1, tv2, tv3}) {
        W.vertices.push_back(v);
        W.scalars.push_back(bv);
      }
      for (int k = 0; k < 6; ++k) W.indices.push_back(idx0 + k);
      box3f b(vec3f(1e31f), vec3f(-1e31f));
      for (int k = 0; k < 6; ++k) b.extend(W.vertices[idx0 + k]);
      W.primBounds.push_back(b);
    }
  }
}

inline bool sampleWedges(vec3f pos, float &value) {
  const auto &W = g_wedges;
  for (size_t primID = 0; primID < W.primBounds.size(); ++primID) {
    if (!W.primBounds[primID].contains(pos)) continue;
    const int *I = W.indices.data() + primID * 6;
    const vec4f v0(W.vertices[I[0]], W.scalars[I[0]]);
    const vec4f v1(W.vertices[I[1]], W.scalars[I[1]]);
    const vec4f v2(W.vertices[I[2]], W.scalars[I[2]]);
    const vec4f v3(W.vertices[I[3]], W.scalars[I[3]]);
    const vec4f v4(W.vertices[I[4]], W.scalars[I[4]]);
    const vec4f v5(W.vertices[I[5]], W.scalars[I[5]]);
    float v;
    if (intersectWedgeEXT(v, pos, v0, v1, v2, v3, v4, v5)) {
      value = v;
      return true;
    }
  }
  return false;
}

// deviceCode.cu:36-49 (expression kept as in the reference)
inline Ray generateRay(const RefParams &lp, const vec2f screen, Random &rnd) {
  vec3f org = lp.org;
  vec3f dir = lp.dir_00 + (screen.u + rnd()) * lp.dir_du + (screen.v + rnd()) * lp.dir_dv;
  dir = normalize(dir);
  if (fabsf(dir.x) < 1e-5f) dir.x = 1e-5f;
  if (fabsf(dir.y) < 1e-5f) dir.y = 1e-5f;
  if (fabsf(dir.z) < 1e-5f) dir.z = 1e-5f;
  return Ray(org, dir, 0.f, 1e10f);
}

// deviceCode.cu:116-123 (non-RTCORE branch)
inline bool sampleVolume(const RefParams &lp, vec3f pos, float &value) {
  if (g_wedges.mode == 2) return sampleWedges(pos, value);
  for (unsigned i = 0; i < (unsigned)lp.numCells; ++i) {
    if (sample(lp.cells[i], pos, value)) return true;
  }
  return false;
}

// deviceCode.cu:127-135
inline vec4f postClassify(const RefParams &lp, float v) {
  v = (v - lp.tfRange.lower) / (lp.tfRange.upper - lp.tfRange.lower);
  int idx = v * (lp.lutSize);
  float frac = (v * lp.lutSize) - idx;
  vec4f v1 = lp.lut[clamp(idx, 0, lp.lutSize - 1)];
  vec4f v2 = lp.lut[clamp(idx + 1, 0, lp.lutSize - 1)];
  return v1 * frac + v2 * (1.f - frac) * vec4f(1, 1, 1, lp.opacityScale);
}

// deviceCode.cu:149-186
inline float woodcockTracking(const RefParams &lp, const Ray &ray, Random &rnd, float majorant,
                              vec3f &albedo, float &extinction, Counters &cnt) {
  float t = ray.tmin;
  while (1) {
    if (majorant <= 0.f) break;
    t -= (logf(1.f - rnd()) / (majorant / lp.unitDistance));
    if (t > ray.tmax) break;
    vec3f P = ray.org + ray.dir * t;
    float value{0.f};
    ++cnt.locate;
    if (!sampleVolume(lp, P, value)) continue;
    ++cnt.found;
    vec4f s = postClassify(lp, value);
    float u = rnd();
    if (s.w >= u * majorant) {
      albedo = vec3f(s.x, s.y, s.z);
      extinction = s.w;
      break;
    }
  }
  return fminf(t, ray.tmax);
}

// deviceCode.cu:239-275 and 281-341, one pixel
void raygen(const RefParams &lp, int x, int y, int W, int H, vec4f *accumBuffer,
            uint32_t *fbPointer, Counters &cnt) {
  const vec2i threadIndex(x, y);
  const vec2i launchDim(W, H);
  const int pixelID = threadIndex.x + launchDim.x * threadIndex.y;
  Random rnd(lp.accumID * launchDim.x * launchDim.y + (unsigned)threadIndex.x,
             (unsigned)threadIndex.y);
  Ray ray = generateRay(lp, vec2f(threadIndex) + vec2f(.5f), rnd);
  float t0, t1;
  if (!boxTest(ray, lp.bounds, t0, t1)) return;
  ray.tmin = t0, ray.tmax = t1;
  vec3f color{0.f};
  float alpha{0.f};
  if (lp.raygen == 1) {
    vec3f albedo = 0.f;
    float extinction = 0.f;
    woodcockTracking(lp, ray, rnd, 1.f, albedo, extinction, cnt);
    color = albedo * lp.ambientColor * lp.ambientRadiance;
    alpha = extinction > 0.f ? 1.f : 0.f;
  } else {
    const float *maxOpacities = lp.accel.maxOpacities;  // deviceCode.cu:302, 326
    auto woodcockFunc = [&](const int leafID, float t0, float t1) {
      vec3f albedo = 0.f;
      float extinction = 0.f;
      const float majorant = maxOpacities[leafID];
      ray.tmin = t0;
      ray.tmax = t1;
      // zero-length leaves are not counted (same rule as oracle/icon_oracle.cpp)
      Counters uncounted;
      float t = woodcockTracking(lp, ray, rnd, majorant, albedo, extinction,
                                 t0 == t1 ? uncounted : cnt);
      if (t > t0 && t < t1) {
        color = albedo * lp.ambientColor * lp.ambientRadiance;
        alpha = extinction > 0.f ? 1.f : 0.f;
        return false;
      }
      return true;
    };
    if (g_grid.accelMode == 0) {  // deviceCode.cu:325-331
      sdda(ray, lp.accel, woodcockFunc, false);
    } else {
      maxOpacities = g_grid.maxOpacities;
      dda3(ray, g_grid.dims, g_grid.worldBounds, woodcockFunc);
    }
  }
  float accum = 1.f / (lp.accumID + 1);
  accumBuffer[pixelID] = lerp(vec4f(color, alpha), accumBuffer[pixelID], accum);
  vec4f accumColor = accumBuffer[pixelID];
  accumColor.r = linear_to_srgb(accumColor.r);
  accumColor.g = linear_to_srgb(accumColor.g);
  accumColor.b = linear_to_srgb(accumColor.b);
  fbPointer[pixelID] = make_rgba(accumColor);
}

// float atomicMin/Max semantics of hostCode.cu:36-56 (store only when strictly
// smaller / larger), sequential.
inline void fmin_store(float *a, float v) { if (v < *a) *a = v; }
inline void fmax_store(float *a, float v) { if (v > *a) *a = v; }

}  // namespace

extern "C" {

static RefParams make_params(const void *cells, int numCells, const float *camera12, int accumID,
                      const float *ambient4, float unitDistance, int raygenKind,
                      const float *bounds6, const int *dims, const float *sphericalBounds6,
                      const float *maxOpacities, const float *tf3, const float *lut, int lutSize);

// ---- full frame on the reference's CPU parallel_for (64x64 tiles, thread_pool)
int ref_render(const void *cells, int numCells, const float *camera12, int accumID,
               const float *ambient4, float unitDistance, int raygenKind,
               const float *bounds6, const int *dims, const float *sphericalBounds6,
               const float *maxOpacities, const float *tf3, const float *lut, int lutSize,
               int W, int H, int x0, int y0, int x1, int y1, float *accum, uint32_t *fb,
               int nthreads, unsigned long long *counters2) {
  const RefParams lp = make_params(cells, numCells, camera12, accumID, ambient4, unitDistance,
                                   raygenKind, bounds6, dims, sphericalBounds6, maxOpacities,
                                   tf3, lut, lutSize);
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  std::mutex mtx;
  Counters total;
  auto pixel = [&](int x, int y) {
    Counters c;
    raygen(lp, x, y, W, H, (vec4f *)accum, fb, c);
    std::lock_guard<std::mutex> g(mtx);
    total.locate += c.locate;
    total.found += c.found;
  };
  if (nthreads == 1) {
    // serial::for_each (common/for_each.h:18-37).  The reference's thread_pool publishes
    // `start_threads` and notify_all()s without holding its mutex (thread_pool.h:88-107,
    // 129-139), a lost-wakeup window that deadlocked golden generation here once; the
    // schedule never changes a pixel, so fixtures are made serially.
    serial::for_each(x0, x1, y0, y1, pixel);
  } else {
    thread_pool pool((unsigned)nthreads);
    parallel::for_each(pool, x0, x1, y0, y1, pixel);
  }
  if (counters2) {
    counters2[0] = total.locate;
    counters2[1] = total.found;
  }
  return 0;
}

// ---- the reference raygen over an explicit pixel list, serially (the caller may run
// several calls on disjoint pixel lists concurrently: each only reads the scene)
int ref_render_pixels(const void *cells, int numCells, const float *camera12, int accumID,
                      const float *ambient4, float unitDistance, int raygenKind,
                      const float *bounds6, const int *dims, const float *sphericalBounds6,
                      const float *maxOpacities, const float *tf3, const float *lut, int lutSize,
                      int W, int H, const int *xy, int numPixels, float *accum, uint32_t *fb,
                      unsigned long long *counters2) {
  const RefParams lp = make_params(cells, numCells, camera12, accumID, ambient4, unitDistance,
                                   raygenKind, bounds6, dims, sphericalBounds6, maxOpacities,
                                   tf3, lut, lutSize);
  Counters total;
  for (int i = 0; i < numPixels; ++i) raygen(lp, xy[2 * i], xy[2 * i + 1], W, H, (vec4f *)accum, fb, total);
  if (counters2) {
    counters2[0] = total.locate;
    counters2[1] = total.found;
  }
  return 0;
}

static RefParams make_params(const void *cells, int numCells, const float *camera12, int accumID,
                      const float *ambient4, float unitDistance, int raygenKind,
                      const float *bounds6, const int *dims, const float *sphericalBounds6,
                      const float *maxOpacities, const float *tf3, const float *lut, int lutSize) {
  RefParams lp;
  lp.org = vec3f(camera12[0], camera12[1], camera12[2]);
  lp.dir_00 = vec3f(camera12[3], camera12[4], camera12[5]);
  lp.dir_du = vec3f(camera12[6], camera12[7], camera12[8]);
  lp.dir_dv = vec3f(camera12[9], camera12[10], camera12[11]);
  lp.accumID = accumID;
  lp.ambientColor = vec3f(ambient4[0], ambient4[1], ambient4[2]);
  lp.ambientRadiance = ambient4[3];
  lp.unitDistance = unitDistance;
  lp.raygen = raygenKind;
  lp.bounds = box3f(vec3f(bounds6[0], bounds6[1], bounds6[2]),
                    vec3f(bounds6[3], bounds6[4], bounds6[5]));
  lp.accel.dims = vec3i(dims[0], dims[1], dims[2]);
  lp.accel.sphericalBounds =
      box3f(vec3f(sphericalBounds6[0], sphericalBounds6[1], sphericalBounds6[2]),
            vec3f(sphericalBounds6[3], sphericalBounds6[4], sphericalBounds6[5]));
  lp.accel.valueRanges = nullptr;
  lp.accel.maxOpacities = const_cast<float *>(maxOpacities);
  lp.tfRange = box1f(tf3[0], tf3[1]);
  lp.opacityScale = tf3[2];
  lp.lut = (const vec4f *)lut;
  lp.lutSize = lutSize;
  lp.cells = (const ICONCell *)cells;
  lp.numCells = numCells;
  return lp;
}

// ---- host setup restated from hostCode.cu:792-808 with the reference's types
void ref_compute_bounds(const void *cellsv, int n, float *sb6, float *vb6, float *dr2) {
  const ICONCell *cells = (const ICONCell *)cellsv;
  box3f volbounds({INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY});
  box1f dataRange(INFINITY, -INFINITY);
  box3f sphericalBounds{vec3f(INFINITY), vec3f(-INFINITY)};
  for (int i = 0; i < n; ++i) {
    const ICONCell &cell = cells[i];
    float minLat = fminf(cells[i].lat.x, fminf(cells[i].lat.y, cells[i].lat.z));
    float maxLat = fmaxf(cells[i].lat.x, fmaxf(cells[i].lat.y, cells[i].lat.z));
    float minLon = fminf(cells[i].lon.x, fminf(cells[i].lon.y, cells[i].lon.z));
    float maxLon = fmaxf(cells[i].lon.x, fmaxf(cells[i].lon.y, cells[i].lon.z));
    sphericalBounds.lower.x = fminf(sphericalBounds.lower.x, cell.height[0]);
    sphericalBounds.upper.x = fmaxf(sphericalBounds.upper.x, cell.height[cell.numLayers]);
    sphericalBounds.lower.y = fminf(sphericalBounds.lower.y, minLat);
    sphericalBounds.upper.y = fmaxf(sphericalBounds.upper.y, maxLat);
    sphericalBounds.lower.z = fminf(sphericalBounds.lower.z, minLon);
    sphericalBounds.upper.z = fmaxf(sphericalBounds.upper.z, maxLon);
    volbounds.extend(cell.getBounds());
    for (int j = 0; j < cell.numLayers; ++j) dataRange.extend(cell.value[j]);
  }
  const float s[6] = {sphericalBounds.lower.x, sphericalBounds.lower.y, sphericalBounds.lower.z,
                      sphericalBounds.upper.x, sphericalBounds.upper.y, sphericalBounds.upper.z};
  const float v[6] = {volbounds.lower.x, volbounds.lower.y, volbounds.lower.z,
                      volbounds.upper.x, volbounds.upper.y, volbounds.upper.z};
  memcpy(sb6, s, sizeof(s));
  memcpy(vb6, v, sizeof(v));
  dr2[0] = dataRange.lower;
  dr2[1] = dataRange.upper;
}

// ---- initGrid + buildShell_ICON (hostCode.cu:216-225, 299-336), sequential
void ref_build_shell(const void *cellsv, int n, const int *dimsi, const float *sb6,
                     float *valueRanges) {
  const ICONCell *cells = (const ICONCell *)cellsv;
  ShellAccel shell;
  shell.dims = vec3i(dimsi[0], dimsi[1], dimsi[2]);
  shell.sphericalBounds = box3f(vec3f(sb6[0], sb6[1], sb6[2]), vec3f(sb6[3], sb6[4], sb6[5]));
  shell.valueRanges = (box1f *)valueRanges;
  size_t numMCs = shell.dims.x * size_t(shell.dims.y) * shell.dims.z;
  for (size_t mcID = 0; mcID < numMCs; ++mcID) shell.valueRanges[mcID] = box1f(FLT_MAX, -FLT_MAX);
  for (int cellID = 0; cellID < n; ++cellID) {
    const ICONCell &cell = cells[cellID];
    for (int i = 0; i < cell.numLayers; ++i) {
      vec3i c1 = projectToSphericalGrid(vec3f(cell.height[i], cell.lat.x, cell.lon.x), shell.dims, shell.sphericalBounds);
      vec3i c2 = projectToSphericalGrid(vec3f(cell.height[i], cell.lat.y, cell.lon.y), shell.dims, shell.sphericalBounds);
      vec3i c3 = projectToSphericalGrid(vec3f(cell.height[i], cell.lat.z, cell.lon.z), shell.dims, shell.sphericalBounds);
      vec3i c4 = projectToSphericalGrid(vec3f(cell.height[i + 1], cell.lat.x, cell.lon.x), shell.dims, shell.sphericalBounds);
      vec3i c5 = projectToSphericalGrid(vec3f(cell.height[i + 1], cell.lat.y, cell.lon.y), shell.dims, shell.sphericalBounds);
      vec3i c6 = projectToSphericalGrid(vec3f(cell.height[i + 1], cell.lat.z, cell.lon.z), shell.dims, shell.sphericalBounds);
      vec3i loMC = min(c1, min(c2, c3));
      vec3i upMC = max(c4, max(c5, c6));
      box1f range(cell.getValue(cell.height[i]), cell.getValue(cell.height[i + 1]));
      for (int mcz = loMC.z; mcz <= upMC.z; ++mcz)
        for (int mcy = loMC.y; mcy <= upMC.y; ++mcy)
          for (int mcx = loMC.x; mcx <= upMC.x; ++mcx) {
            const size_t linearID = linearIndex(vec3i(mcx, mcy, mcz), shell.dims);
            box1f &vrange = shell.valueRanges[linearID];
            fmin_store(&vrange.lower, range.lower);
            fmax_store(&vrange.upper, range.upper);
          }
    }
  }
}

// ---- Volume::mode for ref_render: 0 the CPU cell scan, 2 CUBQL_MODE wedges
void ref_set_sampler(int mode, const void *cells, int numCells) {
  g_wedges.mode = mode;
  if (mode == 2) buildWedgeMesh((const ICONCell *)cells, numCells);
}

int ref_intersect_wedge(const float *v24, const float *p3, float *value) {
  const vec4f *V = (const vec4f *)v24;
  float v = 0.f;
  const bool hit = intersectWedgeEXT(v, vec3f(p3[0], p3[1], p3[2]), V[0], V[1], V[2], V[3], V[4], V[5]);
  if (hit) *value = v;
  return hit;
}

int ref_wedge_sample(const void *cells, int numCells, const float *p3, float *value) {
  buildWedgeMesh((const ICONCell *)cells, numCells);
  return sampleWedges(vec3f(p3[0], p3[1], p3[2]), *value);
}

// ---- GRID_ACCEL_MODE selection for ref_render (toggleAccelMode, hostCode.cu:170-199)
void ref_set_accel(int accelMode, const int *dimsi, const float *wb6, const float *maxOpacities) {
  g_grid.accelMode = accelMode;
  if (dimsi) g_grid.dims = vec3i(dimsi[0], dimsi[1], dimsi[2]);
  if (wb6) g_grid.worldBounds = box3f(vec3f(wb6[0], wb6[1], wb6[2]), vec3f(wb6[3], wb6[4], wb6[5]));
  g_grid.maxOpacities = maxOpacities;
}

// ---- initGrid(Grid) + buildGrid_ICON + rasterizeBox (hostCode.cu:205-214, 227-297),
// sequential, with projectOnGrid/linearIndex from the reference's DDA.h
void ref_build_grid(const void *cellsv, int n, const int *dimsi, const float *wb6,
                    float *valueRanges) {
  const ICONCell *cells = (const ICONCell *)cellsv;
  const vec3i dims(dimsi[0], dimsi[1], dimsi[2]);
  const box3f worldBounds(vec3f(wb6[0], wb6[1], wb6[2]), vec3f(wb6[3], wb6[4], wb6[5]));
  box1f *vr = (box1f *)valueRanges;
  const size_t numMCs = dims.x * size_t(dims.y) * dims.z;
  for (size_t mcID = 0; mcID < numMCs; ++mcID) vr[mcID] = box1f(FLT_MAX, -FLT_MAX);
  for (int cellID = 0; cellID < n; ++cellID) {
    const ICONCell &cell = cells[cellID];
    for (int i = 0; i < cell.numLayers; ++i) {
      box3f bounds({INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY});
      vec3f bv1 = toCartesian({cell.height[i], cell.lat.x, cell.lon.x});
      vec3f bv2 = toCartesian({cell.height[i], cell.lat.y, cell.lon.y});
      vec3f bv3 = toCartesian({cell.height[i], cell.lat.z, cell.lon.z});
      bounds.extend(bv1);
      bounds.extend(bv2);
      bounds.extend(bv3);
      vec3f tv1 = toCartesian({cell.height[i + 1], cell.lat.x, cell.lon.x});
      vec3f tv2 = toCartesian({cell.height[i + 1], cell.lat.y, cell.lon.y});
      vec3f tv3 = toCartesian({cell.height[i + 1], cell.lat.z, cell.lon.z});
      vec3f bary = (tv1 + tv2 + tv3) / 3.f;
      float R = cell.height[i + 1];
      float D = R - length(bary);
      float off = D / R;
      tv1 += tv1 * off;
      tv2 += tv2 * off;
      tv3 += tv3 * off;
      bounds.extend(tv1);
      bounds.extend(tv2);
      bounds.extend(tv3);
      box1f valueRange(INFINITY, -INFINITY);
      valueRange.extend(cell.getValue(cell.height[i]));
      valueRange.extend(cell.getValue(cell.height[i + 1]));
      const vec3i loMC = projectOnGrid(bounds.lower, dims, worldBounds);
      const vec3i upMC = projectOnGrid(bounds.upper, dims, worldBounds);
      for (int mcz = loMC.z; mcz <= upMC.z; ++mcz)
        for (int mcy = loMC.y; mcy <= upMC.y; ++mcy)
          for (int mcx = loMC.x; mcx <= upMC.x; ++mcx) {
            box1f &vrange = vr[linearIndex(vec3i(mcx, mcy, mcz), dims)];
            fmin_store(&vrange.lower, valueRange.lower);
            fmax_store(&vrange.upper, valueRange.upper);
          }
    }
  }
}

// ---- computeMaxOpacities(ShellAccel) (hostCode.cu:362-397), sequential
void ref_max_opacities(const float *valueRangesf, long numMCs, const float *lutf, int size,
                       float tfLo, float tfHi, float *maxOpacities) {
  const box1f *valueRanges = (const box1f *)valueRangesf;
  const vec4f *rgbaLUT = (const vec4f *)lutf;
  box1f tf_valueRange(tfLo, tfHi);
  for (long mcID = 0; mcID < numMCs; ++mcID) {
    box1f valueRange = valueRanges[mcID];
    if (valueRange.upper < valueRange.lower) {
      maxOpacities[mcID] = 0.f;
      continue;
    }
    valueRange.lower -= tf_valueRange.lower;
    valueRange.lower /= tf_valueRange.upper - tf_valueRange.lower;
    valueRange.upper -= tf_valueRange.lower;
    valueRange.upper /= tf_valueRange.upper - tf_valueRange.lower;
    int lo = clamp(int(valueRange.lower * (size - 1)), 0, size - 1);
    int hi = clamp(int(valueRange.upper * (size - 1)) + 1, 0, size - 1);
    float maxOpacity = 0.f;
    for (int i = lo; i <= hi; ++i) maxOpacity = fmaxf(maxOpacity, rgbaLUT[i].w);
    maxOpacities[mcID] = maxOpacity;
  }
}

// ---- resampleLUT (dvr_course-common.h:44-70) exactly as the reference
void ref_resample_lut(const float *src, int nsrc, float *dst, int ndst) {
  std::vector<vec4f> s(nsrc), d(ndst);
  memcpy(s.data(), src, sizeof(vec4f) * nsrc);
  resampleLUT(d, s);
  memcpy(dst, d.data(), sizeof(vec4f) * ndst);
}

// ---- Camera (camera.h) as hostCode.cu:819-821,939-945 + pipeline.cu:444-454 use it
void ref_camera(int useViewAll, const float *box6, const float *vp_vi_vu9, float fovyDeg,
                float *out12) {
  Camera cam;
  if (useViewAll) {
    cam.viewAll(box3f(vec3f(box6[0], box6[1], box6[2]), vec3f(box6[3], box6[4], box6[5])));
  } else {
    float fovy = fovyDeg;
    if (fovy < 1e-3f) fovy = 90.f;
    fovy = fovy * M_PI / 180.f;
    cam.setOrientation(vec3f(vp_vi_vu9[0], vp_vi_vu9[1], vp_vi_vu9[2]),
                       vec3f(vp_vi_vu9[3], vp_vi_vu9[4], vp_vi_vu9[5]),
                       vec3f(vp_vi_vu9[6], vp_vi_vu9[7], vp_vi_vu9[8]), fovy);
  }
  vec3f ll, h, v;
  cam.getScreen(ll, h, v);
  vec3f o = cam.getPosition();
  const float r[12] = {o.x, o.y, o.z, ll.x, ll.y, ll.z, h.x, h.y, h.z, v.x, v.y, v.z};
  memcpy(out12, r, sizeof(r));
}

// ---- single-function known answers from the reference's own code
void ref_lcg(unsigned s0, unsigned s1, int n, float *out) {
  Random r(s0, s1);
  for (int i = 0; i < n; ++i) out[i] = r();
}
int ref_sample(const void *cell, const float *pos3, float *value) {
  float v = 0.f;
  bool ok = sample(*(const ICONCell *)cell, vec3f(pos3[0], pos3[1], pos3[2]), v);
  if (ok) *value = v;
  return ok;
}
int ref_find_height(const void *cell, float h) { return ((const ICONCell *)cell)->findHeight(h); }
int ref_intersect_sphere(const float *org3, const float *dir3, float radius, float *tn, float *tf) {
  Ray r(vec3f(org3[0], org3[1], org3[2]), vec3f(dir3[0], dir3[1], dir3[2]), 0.f, 1e10f);
  return intersectSphere(r, radius, *tn, *tf);
}
int ref_box_test(const float *org3, const float *dir3, float tmin, float tmax, const float *box6,
                 float *t0, float *t1) {
  Ray r(vec3f(org3[0], org3[1], org3[2]), vec3f(dir3[0], dir3[1], dir3[2]), tmin, tmax);
  return boxTest(r, box3f(vec3f(box6[0], box6[1], box6[2]), vec3f(box6[3], box6[4], box6[5])), *t0, *t1);
}
int ref_sdda_trace(const float *org3, const float *dir3, float tmin, float tmax, const int *dimsi,
                   const float *sb6, int maxOut, int *leaf, float *t0, float *t1) {
  Ray r(vec3f(org3[0], org3[1], org3[2]), vec3f(dir3[0], dir3[1], dir3[2]), tmin, tmax);
  ShellAccel a;
  a.dims = vec3i(dimsi[0], dimsi[1], dimsi[2]);
  a.sphericalBounds = box3f(vec3f(sb6[0], sb6[1], sb6[2]), vec3f(sb6[3], sb6[4], sb6[5]));
  int count = 0;
  sdda(r, a, [&](const int l, float a0, float a1) {
    if (count < maxOut) { leaf[count] = l; t0[count] = a0; t1[count] = a1; }
    ++count;
    return count < 100000;
  });
  return count;
}
// dda3 (DDA.h:35-136) itself, compiled from the reference header
int ref_dda3_trace(const float *org3, const float *dir3, float tmin, float tmax, const int *dimsi,
                   const float *wb6, int maxOut, int *leaf, float *t0, float *t1) {
  Ray r(vec3f(org3[0], org3[1], org3[2]), vec3f(dir3[0], dir3[1], dir3[2]), tmin, tmax);
  int count = 0;
  dda3(r, vec3i(dimsi[0], dimsi[1], dimsi[2]),
       box3f(vec3f(wb6[0], wb6[1], wb6[2]), vec3f(wb6[3], wb6[4], wb6[5])),
       [&](const int l, float a0, float a1) {
         if (count < maxOut) { leaf[count] = l; t0[count] = a0; t1[count] = a1; }
         ++count;
         return count < 100000;
       });
  return count;
}
float ref_linear_to_srgb(float x) { return linear_to_srgb(x); }
unsigned ref_make_rgba(const float *c) { return make_rgba(vec4f(c[0], c[1], c[2], c[3])); }
void ref_to_spherical(const float *c, float *out) {
  vec3f s = toSpherical(vec3f(c[0], c[1], c[2]));
  out[0] = s.x; out[1] = s.y; out[2] = s.z;
}
void ref_to_cartesian(const float *s, float *out) {
  vec3f c = toCartesian(vec3f(s[0], s[1], s[2]));
  out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
void ref_get_bounds(const void *cell, float *out6) {
  box3f b = ((const ICONCell *)cell)->getBounds();
  const float r[6] = {b.lower.x, b.lower.y, b.lower.z, b.upper.x, b.upper.y, b.upper.z};
  memcpy(out6, r, sizeof(r));
}
// The unsequenced generateRay expression on its own: returns the two LCG draws in
// the order they were consumed (draw #1 multiplies dir_du iff out[2] == 0).
void ref_generate_ray(const float *camera12, int x, int y, unsigned s0, unsigned s1, float *dir3) {
  RefParams lp;
  lp.org = vec3f(camera12[0], camera12[1], camera12[2]);
  lp.dir_00 = vec3f(camera12[3], camera12[4], camera12[5]);
  lp.dir_du = vec3f(camera12[6], camera12[7], camera12[8]);
  lp.dir_dv = vec3f(camera12[9], camera12[10], camera12[11]);
  Random rnd(s0, s1);
  Ray r = generateRay(lp, vec2f(vec2i(x, y)) + vec2f(.5f), rnd);
  dir3[0] = r.dir.x; dir3[1] = r.dir.y; dir3[2] = r.dir.z;
}

}  // extern "C"
