// irt_host.cpp -- host-side setup of the icon_rt frame (no GPU): .ic I/O, lat/lon filter,
// volume facts, default transfer function, camera, synthetic grids, and the libm tables
// the kernels need.  Compiled with g++ -ffp-contract=off (x86-64 SSE), like the
// reference's CPU build, so every float below rounds exactly as the reference's host
// code does.  References are to szellmann/icon-ray-tracing.

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <mutex>
#include <sched.h>
#include <thread>
#include <vector>

#include "irt_internal.h"

namespace irt {

static thread_local std::string g_error;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_error = buf;
}
void clear_error() { g_error.clear(); }

// Host worker threads: the CPUs this process may run on (affinity mask), within
// OMP_NUM_THREADS when set (the GPU box sets it to the job's share) and at most 32.
int default_threads() {
  static const int n = [] {
    int h = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) h = CPU_COUNT(&set);
    if (const char *e = getenv("OMP_NUM_THREADS")) {
      const int v = atoi(e);
      if (v > 0 && v < h) h = v;
    }
    return std::max(1, std::min(h, 32));
  }();
  return n;
}

template <typename F>
static void parallel_for(size_t n, int threads, F &&f) {
  if (threads <= 1 || n < 4096) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  size_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    size_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    ts.emplace_back([&, b, e] { f(b, e); });
  }
  for (auto &t : ts) t.join();
}

// ------------------------------------------------------------------ vector helpers
namespace {
struct V3 {
  float x, y, z;
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 splat(float s) { return {s, s, s}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 u, V3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
inline V3 normalize(V3 u) { return u / sqrtf(dot(u, u)); }
inline float length(V3 u) { return sqrtf(dot(u, u)); }
inline V3 vmin(V3 a, V3 b) { return {fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)}; }
inline V3 vmax(V3 a, V3 b) { return {fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)}; }
inline irt_vec3f iv(V3 v) { return {v.x, v.y, v.z}; }
inline V3 vi(irt_vec3f v) { return {v.x, v.y, v.z}; }

// toCartesian (ICONGrid.h:44-54)
inline V3 toCartesian(float r, float lat, float lon) {
  float x = r * cosf(lat) * cosf(lon);
  float y = r * cosf(lat) * sinf(lon);
  float z = r * sinf(lat);
  return {x, y, z};
}
}  // namespace

// corner trig {cosf lat, sinf lat, cosf lon, sinf lon} x 3 (host glibc)
void corner_trig(const irt_icon_cell &c, float *t12) {
  for (int k = 0; k < 3; ++k) {
    t12[4 * k + 0] = cosf(c.lat[k]);
    t12[4 * k + 1] = sinf(c.lat[k]);
    t12[4 * k + 2] = cosf(c.lon[k]);
    t12[4 * k + 3] = sinf(c.lon[k]);
  }
}

// ICONCell::getBounds (ICONGrid.h:78-115); toCartesian from the corner trig is the same
// float expression as r * cosf(lat) * cosf(lon) etc.
void cell_bounds(const irt_icon_cell &c, const float *t12, float lo3[3], float hi3[3]) {
  auto tc = [&](float r, int k) {
    const float *t = t12 + 4 * k;
    return V3{(r * t[0]) * t[2], (r * t[0]) * t[3], r * t[1]};
  };
  V3 lo = splat(INFINITY), hi = splat(-INFINITY);
  const float h0 = c.height[0], hN = c.height[c.numLayers];
  V3 tv[3];
  for (int k = 0; k < 3; ++k) {
    V3 b = tc(h0, k);
    lo = vmin(lo, b);
    hi = vmax(hi, b);
  }
  for (int k = 0; k < 3; ++k) tv[k] = tc(hN, k);
  V3 bary = (tv[0] + tv[1] + tv[2]) / 3.f;
  float R = hN;
  float D = R - length(bary);
  float off = D / R;
  for (int k = 0; k < 3; ++k) {
    tv[k] = tv[k] + tv[k] * off;
    lo = vmin(lo, tv[k]);
    hi = vmax(hi, tv[k]);
  }
  lo3[0] = lo.x, lo3[1] = lo.y, lo3[2] = lo.z;
  hi3[0] = hi.x, hi3[1] = hi.y, hi3[2] = hi.z;
}

// hostCode.cu:792-808 (bounds, dataRange) and 838-840 (unitDistance), as a fold over the
// records in order (so chunked input gives the same result)
void volume_acc_init(VolumeAcc &a) {
  for (int k = 0; k < 3; ++k) {
    a.vlo[k] = a.slo[k] = INFINITY;
    a.vhi[k] = a.shi[k] = -INFINITY;
  }
  a.dlo = INFINITY;
  a.dhi = -INFINITY;
  a.n = 0;
}

void volume_acc_add(VolumeAcc &a, const irt_icon_cell &c, const float blo[3], const float bhi[3]) {
  float minLat = fminf(c.lat[0], fminf(c.lat[1], c.lat[2]));
  float maxLat = fmaxf(c.lat[0], fmaxf(c.lat[1], c.lat[2]));
  float minLon = fminf(c.lon[0], fminf(c.lon[1], c.lon[2]));
  float maxLon = fmaxf(c.lon[0], fmaxf(c.lon[1], c.lon[2]));
  a.slo[0] = fminf(a.slo[0], c.height[0]);
  a.shi[0] = fmaxf(a.shi[0], c.height[c.numLayers]);
  a.slo[1] = fminf(a.slo[1], minLat);
  a.shi[1] = fmaxf(a.shi[1], maxLat);
  a.slo[2] = fminf(a.slo[2], minLon);
  a.shi[2] = fmaxf(a.shi[2], maxLon);
  for (int k = 0; k < 3; ++k) {
    a.vlo[k] = fminf(a.vlo[k], blo[k]);
    a.vhi[k] = fmaxf(a.vhi[k], bhi[k]);
  }
  for (int j = 0; j < c.numLayers; ++j) {
    a.dlo = fminf(a.dlo, c.value[j]);
    a.dhi = fmaxf(a.dhi, c.value[j]);
  }
  ++a.n;
}

// a's records, then b's: fminf/fmaxf select one of their arguments, ties to the second, so
// folding per-chunk partials in chunk order selects the element the sequential fold selects
// (signed zeros included)
void volume_acc_merge(VolumeAcc &a, const VolumeAcc &b) {
  for (int k = 0; k < 3; ++k) {
    a.vlo[k] = fminf(a.vlo[k], b.vlo[k]);
    a.vhi[k] = fmaxf(a.vhi[k], b.vhi[k]);
    a.slo[k] = fminf(a.slo[k], b.slo[k]);
    a.shi[k] = fmaxf(a.shi[k], b.shi[k]);
  }
  a.dlo = fminf(a.dlo, b.dlo);
  a.dhi = fmaxf(a.dhi, b.dhi);
  a.n += b.n;
}

void volume_acc_finish(const VolumeAcc &a, irt_volume_info &info) {
  memset(&info, 0, sizeof(info));
  info.numCells = a.n;
  info.bounds = {{a.vlo[0], a.vlo[1], a.vlo[2]}, {a.vhi[0], a.vhi[1], a.vhi[2]}};
  info.sphericalBounds = {{a.slo[0], a.slo[1], a.slo[2]}, {a.shi[0], a.shi[1], a.shi[2]}};
  info.dataRange = {a.dlo, a.dhi};
  float magnitude = floorf(log10f(a.slo[0]));
  float scale = powf(10.f, magnitude - 3);
  info.unitDistance = 1.0f * scale;
  info.shellDims[0] = 1;
  info.shellDims[1] = 1024;
  info.shellDims[2] = 1024;
}

void compute_volume_info(const irt_icon_cell *cells, size_t n, irt_volume_info &info) {
  VolumeAcc a;
  volume_acc_init(a);
  for (size_t i = 0; i < n; ++i) {
    float t[12], lo[3], hi[3];
    corner_trig(cells[i], t);
    cell_bounds(cells[i], t, lo, hi);
    volume_acc_add(a, cells[i], lo, hi);
  }
  volume_acc_finish(a, info);
}

const std::vector<float> &logf_table() {
  static std::vector<float> tab;
  static std::once_flag once;
  std::call_once(once, [] {
    tab.resize(size_t(1) << 24);
    parallel_for(tab.size(), default_threads(), [](size_t b, size_t e) {
      for (size_t k = b; k < e; ++k) {
        // exactly the argument deviceCode.cu:165 passes: 1.f - (k / 2^24)
        const float xi = (float)(uint32_t)k / (float)0x01000000;
        tab[k] = logf(1.f - xi);
      }
    });
  });
  return tab;
}

// linear_to_srgb + make_8bit (dvr_course-common-both.h:30-35, 89-92) on the host libm.
static uint32_t srgb_byte(float x) {
  float s = x <= 0.0031308f ? 12.92f * x : 1.055f * powf(x, 1.f / 2.4f) - 0.055f;
  return (uint32_t)fminf(255, fmaxf(0, (float)f2i_x86(s * 256.f)));
}

void srgb_thresholds(float th[256]) {
  th[0] = -INFINITY;
  // byte(x) is monotone non-decreasing in x (tests/test_host_tables.py sweeps every
  // float in [0,1] to confirm under this libm); binary-search each step on the ordered
  // bit patterns of non-negative floats.
  for (int b = 1; b < 256; ++b) {
    uint32_t lo = 0, hi = 0x3f800000u;  // byte(1.0f) == 255
    while (lo < hi) {
      uint32_t mid = lo + (hi - lo) / 2;
      if (srgb_byte(u2f(mid)) >= (uint32_t)b)
        hi = mid;
      else
        lo = mid + 1;
    }
    th[b] = u2f(lo);
  }
}

}  // namespace irt

using namespace irt;

// ====================================================================== C ABI (host)
extern "C" {

const char *irt_last_error(void) { return g_error.c_str(); }

int irt_load_ic(const char *path, long maxNumCells, irt_icon_cell *out, size_t capacity,
                size_t *count) {
  if (!path || !count) {
    set_error("irt_load_ic: null argument");
    return IRT_E_INVALID;
  }
  FILE *f = fopen(path, "rb");
  if (!f) {
    set_error("irt_load_ic: cannot open %s", path);
    return IRT_E_IO;
  }
  fseek(f, 0, SEEK_END);
  long size = ftell(f);
  fseek(f, 0, SEEK_SET);
  size_t n = (size_t)size / sizeof(irt_icon_cell);  // hostCode.cu:725
  if (maxNumCells >= 0) n = std::min(n, (size_t)maxNumCells);  // hostCode.cu:728-730
  *count = n;
  if (!out) {
    fclose(f);
    return IRT_OK;
  }
  if (capacity < n) {
    fclose(f);
    set_error("irt_load_ic: capacity %zu < %zu", capacity, n);
    return IRT_E_INVALID;
  }
  size_t got = fread(out, sizeof(irt_icon_cell), n, f);
  fclose(f);
  if (got != n) {
    set_error("irt_load_ic: short read (%zu of %zu)", got, n);
    return IRT_E_IO;
  }
  return IRT_OK;
}

int irt_save_ic(const char *path, const irt_icon_cell *cells, size_t count) {
  FILE *f = fopen(path, "wb");
  if (!f) {
    set_error("irt_save_ic: cannot open %s", path);
    return IRT_E_IO;
  }
  size_t put = fwrite(cells, sizeof(irt_icon_cell), count, f);
  fclose(f);
  if (put != count) {
    set_error("irt_save_ic: short write");
    return IRT_E_IO;
  }
  return IRT_OK;
}

int irt_filter_cells(irt_icon_cell *cells, size_t n, irt_box1f latDeg, irt_box1f lonDeg,
                     size_t *count) {
  if (!count || (n && !cells)) {
    set_error("irt_filter_cells: null argument");
    return IRT_E_INVALID;
  }
  // deg2rad (ICONGrid.h:26-29)
  auto d2r = [](float d) { return d * float(M_PI) / 180.f; };
  const float la0 = d2r(latDeg.lower), la1 = d2r(latDeg.upper);
  const float lo0 = d2r(lonDeg.lower), lo1 = d2r(lonDeg.upper);
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {  // std::remove_if, hostCode.cu:741-757
    const irt_icon_cell &c = cells[i];
    bool drop = (c.lat[0] < la0 || c.lat[1] < la0 || c.lat[2] < la0) ||
                (c.lat[0] > la1 || c.lat[1] > la1 || c.lat[2] > la1) ||
                (c.lon[0] < lo0 || c.lon[1] < lo0 || c.lon[2] < lo0) ||
                (c.lon[0] > lo1 || c.lon[1] > lo1 || c.lon[2] > lo1);
    if (!drop) {
      if (k != i) cells[k] = cells[i];
      ++k;
    }
  }
  *count = k;
  return IRT_OK;
}

int irt_compute_volume_info(const irt_icon_cell *cells, size_t n, irt_volume_info *info) {
  if (!info || (n && !cells)) {
    set_error("irt_compute_volume_info: null argument");
    return IRT_E_INVALID;
  }
  for (size_t i = 0; i < n; ++i)
    if (cells[i].numLayers < 0 || cells[i].numLayers > 31) {
      set_error("cell %zu: numLayers %d outside [0,31]", i, cells[i].numLayers);
      return IRT_E_DATA;
    }
  compute_volume_info(cells, n, *info);
  return IRT_OK;
}

int irt_resample_lut(const irt_vec4f *src, int nsrc, irt_vec4f *dst, int ndst) {
  if (!src || !dst || nsrc <= 0 || ndst <= 0) {
    set_error("irt_resample_lut: bad argument");
    return IRT_E_INVALID;
  }
  // resampleLUT (common/dvr_course-common.h:44-70)
  for (int i = 0; i < ndst; ++i) {
    float indexf = i / (float)(ndst) * (nsrc - 1);
    int indexa = (int)indexf;
    int indexb = std::min(indexa + 1, nsrc - 1);
    float frac = indexf - indexa;
    float x = 1.f - frac;  // lerp(a, b, x) = x*a + (1-x)*b (vecmath.h:56-59)
    const irt_vec4f &a = src[indexa], &b = src[indexb];
    dst[i] = {x * a.x + (1.f - x) * b.x, x * a.y + (1.f - x) * b.y, x * a.z + (1.f - x) * b.z,
              x * a.w + (1.f - x) * b.w};
  }
  return IRT_OK;
}

int irt_default_transfunc(irt_box1f dataRange, irt_vec4f *out300, irt_box1f *valueRange) {
  if (!out300 || !valueRange) {
    set_error("irt_default_transfunc: null argument");
    return IRT_E_INVALID;
  }
  // hostCode.cu:824-834
  irt_box1f vr = dataRange;
  if (vr.upper <= vr.lower) vr = {0.f, 1.f};
  static const irt_vec4f lut5[5] = {{0.149f, 0.015f, 0.705f, 1.0f},
                                    {0.486f, 0.603f, 0.956f, 0.75f},
                                    {0.866f, 0.866f, 0.866f, 0.5f},
                                    {0.996f, 0.690f, 0.552f, 0.25f},
                                    {0.752f, 0.298f, 0.231f, 0.0f}};
  *valueRange = vr;
  // Pipeline::setTransfunc resamples LUTs with < 300 entries (pipeline.cu:469-473)
  return irt_resample_lut(lut5, 5, out300, 300);
}

static void camera_to_lp(V3 origin, V3 poi, V3 up, float fovy, int imgW, int imgH,
                         irt_launch_params *lp) {
  // Camera::setOrientation + forceUpFrame (camera.h:34-64)
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
  // Camera::getScreen (camera.h:86-96), aspect 1 (never set by icon_rt)
  const float aspect = 1.f;
  float screen_height = 2.f * tanf(0.5f * fovy);
  V3 vertical = splat(screen_height) * vy;
  V3 horizontal = splat(screen_height * aspect) * vx;
  V3 lower_left = -vz - splat(0.5f) * vertical - splat(0.5f) * horizontal;
  // hostCode.cu:942-945
  lp->org = iv(origin);
  lp->dir_00 = iv(lower_left);
  lp->dir_du = iv(horizontal / (float)imgW);
  lp->dir_dv = iv(vertical / (float)imgH);
}

int irt_camera_view_all(irt_box3f bounds, float fovyDeg, int imgW, int imgH,
                        irt_launch_params *lp) {
  if (!lp || imgW <= 0 || imgH <= 0) {
    set_error("irt_camera_view_all: bad argument");
    return IRT_E_INVALID;
  }
  const float fovy = fovyDeg * M_PI / 180.f;  // camera.h:108
  V3 lo = vi(bounds.lower), hi = vi(bounds.upper);
  // Camera::viewAll (camera.h:98-104)
  V3 up{0, 1, 0};
  float diagonal = length(hi - lo);
  float r = diagonal * 0.5f;
  V3 center = (lo + hi) / 2.f;
  V3 eye = center + V3{0, 0, r + r / atanf(fovy)};
  camera_to_lp(eye, center, up, fovy, imgW, imgH, lp);
  return IRT_OK;
}

int irt_camera_look_at(irt_vec3f vp, irt_vec3f vi_, irt_vec3f vu, float fovyDeg, int imgW,
                       int imgH, irt_launch_params *lp) {
  if (!lp || imgW <= 0 || imgH <= 0) {
    set_error("irt_camera_look_at: bad argument");
    return IRT_E_INVALID;
  }
  float f = fovyDeg;  // pipeline.cu:447-451
  if (f < 1e-3f) f = 90.f;
  const float fovy = f * M_PI / 180.f;
  camera_to_lp(vi(vp), vi(vi_), vi(vu), fovy, imgW, imgH, lp);
  return IRT_OK;
}

int irt_num_tiles(int width, int height) {
  if (width <= 0 || height <= 0) return 0;
  return ((width + 63) / 64) * ((height + 63) / 64);
}

// Estimated render cost of one 64x64 tile: rays (no jitter) through every 8th pixel of it,
// in double.  Per ray: 1 (generation + boxTest), +1 inside the box, +8 reaching the shell (the
// Woodcock rounds: ~5x a ray that misses, profiles/r02b_investigation/), + the chord through
// the shell in units of its thickness, capped at 8 (limb rays sample longer).
static double tile_cost(const irt_launch_params &lp, const irt_volume_info &info, int W, int H,
                        int tx, int ty) {
  const double ox = lp.org.x, oy = lp.org.y, oz = lp.org.z;
  const double R0 = info.sphericalBounds.lower.x, R1 = info.sphericalBounds.upper.x;
  const double thick = R1 > R0 ? R1 - R0 : 1.0;
  double cost = 0.0;
  for (int sy = 0; sy < 8; ++sy)
    for (int sx = 0; sx < 8; ++sx) {
      const int px = tx * 64 + 8 * sx + 4, py = ty * 64 + 8 * sy + 4;
      if (px >= W || py >= H) continue;
      double d[3] = {lp.dir_00.x + (px + 0.5) * lp.dir_du.x + (py + 0.5) * lp.dir_dv.x,
                     lp.dir_00.y + (px + 0.5) * lp.dir_du.y + (py + 0.5) * lp.dir_dv.y,
                     lp.dir_00.z + (px + 0.5) * lp.dir_du.z + (py + 0.5) * lp.dir_dv.z};
      const double l = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
      cost += 1.0;
      if (!(l > 0)) continue;
      for (double &v : d) v /= l;
      // slab test against the volume bounds
      const double o[3] = {ox, oy, oz};
      const double lo[3] = {info.bounds.lower.x, info.bounds.lower.y, info.bounds.lower.z};
      const double hi[3] = {info.bounds.upper.x, info.bounds.upper.y, info.bounds.upper.z};
      double t0 = 0.0, t1 = 1e30;
      for (int a = 0; a < 3; ++a) {
        if (d[a] == 0.0) {
          if (o[a] < lo[a] || o[a] > hi[a]) t1 = -1.0;
          continue;
        }
        double u = (lo[a] - o[a]) / d[a], v = (hi[a] - o[a]) / d[a];
        if (u > v) std::swap(u, v);
        t0 = std::max(t0, u);
        t1 = std::min(t1, v);
      }
      if (!(t0 < t1)) continue;
      cost += 1.0;
      const double b = ox * d[0] + oy * d[1] + oz * d[2], oo = ox * ox + oy * oy + oz * oz;
      const double disc1 = b * b - (oo - R1 * R1);
      if (disc1 < 0) continue;
      const double e1 = -b - sqrt(disc1), x1 = -b + sqrt(disc1);
      if (x1 < 0) continue;
      const double disc0 = b * b - (oo - R0 * R0);
      const double stop = disc0 >= 0 && -b - sqrt(disc0) > 0 ? -b - sqrt(disc0) : x1;
      const double chord = std::max(0.0, stop - std::max(e1, 0.0));
      cost += 8.0 + std::min(chord / thick, 8.0);
    }
  return cost;
}

int irt_deal_tiles(const irt_launch_params *lp, const irt_volume_info *info, int W, int H,
                   int N, float rank0Extra, int32_t *table, size_t capacity,
                   int *maxTilesPerRank) {
  if (!lp || !info || !maxTilesPerRank || W <= 0 || H <= 0 || N <= 0 || !(rank0Extra >= 0.f) ||
      !(rank0Extra < 1.f)) {
    set_error("irt_deal_tiles: bad argument");
    return IRT_E_INVALID;
  }
  const int tilesX = (W + 63) / 64, tilesY = (H + 63) / 64, T = tilesX * tilesY;
  std::vector<std::pair<double, int>> order(T);
  double total = 0.0;
  for (int t = 0; t < T; ++t) {
    const double c = tile_cost(*lp, *info, W, H, t % tilesX, t / tilesX);
    order[t] = {-c, t};
    total += c;
  }
  std::sort(order.begin(), order.end());  // heaviest first, ties by tile id
  // longest-processing-time first: each tile to the least-loaded rank (ties: lowest rank);
  // rank 0 starts with the unpack's share
  std::vector<double> load(N, 0.0);
  load[0] = (double)rank0Extra * total;
  std::vector<std::vector<int32_t>> rows(N);
  for (int i = 0; i < T; ++i) {
    int r = 0;
    for (int q = 1; q < N; ++q)
      if (load[q] < load[r]) r = q;
    load[r] += -order[i].first;
    rows[r].push_back(order[i].second);
  }
  int maxT = 0;
  for (auto &row : rows) maxT = std::max(maxT, (int)row.size());
  *maxTilesPerRank = maxT;
  if (!table) return IRT_OK;  // size query
  if (capacity < (size_t)N * (size_t)maxT) {
    set_error("irt_deal_tiles: capacity %zu < %d ranks x %d tiles", capacity, N, maxT);
    return IRT_E_INVALID;
  }
  for (int r = 0; r < N; ++r)
    for (int k = 0; k < maxT; ++k)
      table[(size_t)r * maxT + k] = k < (int)rows[r].size() ? rows[r][k] : -1;
  return IRT_OK;
}

}  // extern "C"
