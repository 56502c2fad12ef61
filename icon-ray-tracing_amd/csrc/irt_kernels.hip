// irt_kernels.hip -- gfx950 kernels of the ICON Woodcock-tracking renderer.
//
// Hot path: k_render = the raygen woodcockTrackingWithAccel / woodcockTrackingAE of
// icon_rt/deviceCode.cu:239-341, one lane per pixel, one wave64 per 8x8 pixel packet,
// a 256-thread workgroup per 16x16 block, 16 workgroups per 64x64 frame tile (the unit
// the reference's CPU parallel_for hands out, common/for_each.h:70-85, and the unit of
// the multi-GPU frame split).  Cell location uses the cube-map candidate lists built in
// host/irt_scene.cpp instead of OptiX/cuBQL/linear scan.
//
// Bit-exactness vs. the reference CPU build (g++, x86-64 SSE): compile with
// -ffp-contract=off (no FMA contraction), keep hipcc's correctly rounded f32 div/sqrt,
// keep every expression's evaluation order, use irt_common.h's x86 float->int and glibc
// asinf/atan2f restatements, and take logf / sRGB from host-built tables.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "irt_common.h"
#include "irt_kernels.h"

#define IRT_FLT_MAX 3.402823466e+38f

namespace irt {

// ------------------------------------------------------------------ small helpers
struct Ray {
  float ox, oy, oz, tmin, dx, dy, dz, tmax;
};

struct Counts {
  uint32_t inBox, locate, found, cand;
};

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
  return ax * bx + ay * by + az * bz;  // vecmath.h:536-538 order
}

// boxTest (vecmath.h:1926-1937)
__device__ __forceinline__ bool box_test(const Ray &r, const RenderArgs &A, float &t0, float &t1) {
  const float lx = (A.bmin.x - r.ox) / r.dx, ly = (A.bmin.y - r.oy) / r.dy, lz = (A.bmin.z - r.oz) / r.dz;
  const float hx = (A.bmax.x - r.ox) / r.dx, hy = (A.bmax.y - r.oy) / r.dy, hz = (A.bmax.z - r.oz) / r.dz;
  const float nx = fminf(lx, hx), ny = fminf(ly, hy), nz = fminf(lz, hz);
  const float fx = fmaxf(lx, hx), fy = fmaxf(ly, hy), fz = fmaxf(lz, hz);
  t0 = fmaxf(r.tmin, fmaxf(fmaxf(nx, ny), nz));
  t1 = fminf(r.tmax, fminf(fminf(fx, fy), fz));
  return t0 < t1;
}

// intersectSphere (ShellAccel.h:34-53)
__device__ __forceinline__ bool intersect_sphere(const Ray &r, float radius, float &tnear, float &tfar) {
  const float A = dot3(r.dx, r.dy, r.dz, r.dx, r.dy, r.dz);
  const float B = dot3(r.dx, r.dy, r.dz, r.ox, r.oy, r.oz) * 2.f;
  const float C = dot3(r.ox, r.oy, r.oz, r.ox, r.oy, r.oz) - radius * radius;
  float d = B * B - 4.f * A * C;
  if (d < 0.f) return false;
  d = sqrtf(d);
  const float q = B < 0.f ? -0.5f * (B - d) : -0.5f * (B + d);
  const float t1 = q / A;
  const float t2 = C / q;
  tnear = fminf(t1, t2);
  tfar = fmaxf(t1, t2);
  return true;
}

// projectToSphericalGrid (ShellAccel.h:57-68) for the lat/lon axes; the radial axis is
// handled by the caller.
__device__ __forceinline__ int project_axis(float s, float lo, float hi, int dim) {
  return f2i_x86((s - lo) / (hi - lo) * (float)(dim - 1));
}

// normalizeGridCoord (ShellAccel.h:71-80): the while-loops compute c mod d in [0,d).
__device__ __forceinline__ int wrap_coord(int c, int d) {
  int m = c % d;
  return m < 0 ? m + d : m;
}

// sampleVolume (deviceCode.cu:58-125) over the cube-map candidate lists: the first entry
// (lists are sorted by record index) passing sample() (ICONGrid.h:181-208) wins.
__device__ __forceinline__ bool locate(const RenderArgs &A, float px, float py, float pz,
                                       float &value, Counts &cnt) {
  if (A.numCells == 0) return false;
  const float r = sqrtf(dot3(px, py, pz, px, py, pz));  // toSpherical(pos).x
  const uint32_t cell = cubemap_cell(px, py, pz, A.G);
  const uint32_t beg = A.offsets[cell], end = A.offsets[cell + 1];
  for (uint32_t e = beg; e < end; ++e) {
    const uint4 E = A.entries[e];
    ++cnt.cand;
    if (r < __uint_as_float(E.x) || r > __uint_as_float(E.y)) continue;  // ICONGrid.h:184
    const float4 *P = A.planes + 3 * (size_t)E.z;
    const float4 p0 = P[0];
    if (dot3(px, py, pz, p0.x, p0.y, p0.z) - p0.w > 0.f) continue;  // ICONGrid.h:201-203
    const float4 p1 = P[1];
    if (dot3(px, py, pz, p1.x, p1.y, p1.z) - p1.w > 0.f) continue;
    const float4 p2 = P[2];
    if (dot3(px, py, pz, p2.x, p2.y, p2.z) - p2.w > 0.f) continue;
    const float *hv = A.hv + (size_t)E.z * kHV;
    const int nl = __float_as_int(hv[63]);
    value = hv[32 + find_height(hv, nl, r)];  // getValue (ICONGrid.h:147-164)
    return true;
  }
  return false;
}

// postClassify (deviceCode.cu:127-135): weights reversed, opacityScale on 2nd term only.
__device__ __forceinline__ float4 post_classify(const RenderArgs &A, float v) {
  v = (v - A.tfLo) / (A.tfHi - A.tfLo);
  const int size = A.lutSize;
  const int idx = f2i_x86(v * (float)size);
  const float frac = (v * (float)size) - (float)idx;
  const int i1 = idx < 0 ? 0 : (idx > size - 1 ? size - 1 : idx);
  const int idx2 = (int)((uint32_t)idx + 1u);
  const int i2 = idx2 < 0 ? 0 : (idx2 > size - 1 ? size - 1 : idx2);
  const float4 a = A.lut[i1], b = A.lut[i2];
  const float om = 1.f - frac;
  float4 o;
  o.x = a.x * frac + b.x * om * 1.f;
  o.y = a.y * frac + b.y * om * 1.f;
  o.z = a.z * frac + b.z * om * 1.f;
  o.w = a.w * frac + b.w * om * A.opacityScale;
  return o;
}

// woodcockTracking (deviceCode.cu:149-186).  logf(1.f - rnd()) == logtab[state & 0xFFFFFF].
__device__ __forceinline__ float woodcock(const RenderArgs &A, const Ray &ray, uint32_t &st,
                                          float majorant, float4 &sampleOut, bool &hit,
                                          Counts &cnt) {
  float t = ray.tmin;
  while (true) {
    if (majorant <= 0.f) break;
    st = lcg_next(st);
    const float lg = A.logtab[st & 0x00FFFFFFu];
    t -= (lg / (majorant / A.unitDistance));
    if (t > ray.tmax) break;
    const float px = ray.ox + ray.dx * t, py = ray.oy + ray.dy * t, pz = ray.oz + ray.dz * t;
    float value = 0.f;
    ++cnt.locate;
    if (!locate(A, px, py, pz, value, cnt)) continue;
    ++cnt.found;
    const float4 s = post_classify(A, value);
    st = lcg_next(st);
    const float u = lcg_float(st);
    if (s.w >= u * majorant) {
      sampleOut = s;
      hit = true;
      break;
    }
  }
  return fminf(t, ray.tmax);
}

// toSpherical (ICONGrid.h:36-42) with glibc-exact asinf / atan2f.
__device__ __forceinline__ void to_spherical(float x, float y, float z, float &r, float &lat, float &lon) {
  r = sqrtf(dot3(x, y, z, x, y, z));
  lat = glibc_asinf(z / r);
  lon = glibc_atan2f(y, x);
}

// make_8bit (dvr_course-common-both.h:89-92)
__device__ __forceinline__ uint32_t make_8bit(float f) {
  return (uint32_t)fminf(255.f, fmaxf(0.f, (float)f2i_x86(f * 256.f)));
}

// make_8bit(linear_to_srgb(x)) via the host-built monotone thresholds (255 in LDS).
__device__ __forceinline__ uint32_t srgb_byte(const float *th, float x) {
  // number of b in [1,255] with th[b] <= x
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = 128; step > 0; step >>= 1) {
    const uint32_t probe = lo + step;
    if (probe <= 255 && th[probe] <= x) lo = probe;
  }
  return lo;
}

// ------------------------------------------------------------------ the raygen kernel
__global__ void __launch_bounds__(256) k_render(RenderArgs A) {
  __shared__ float s_th[256];
  __shared__ uint32_t s_cnt[4];
  const int tid = threadIdx.x;
  s_th[tid] = A.srgbTh[tid];
  if (tid < 4) s_cnt[tid] = 0;
  __syncthreads();

  // block -> (tile k of this launch, 16x16 sub-block); wave -> 8x8 packet; lane -> pixel
  const int k = blockIdx.x >> 4, sub = blockIdx.x & 15;
  const int wave = tid >> 6, lane = tid & 63;
  const int lx = ((sub & 3) << 4) | ((wave & 1) << 3) | (lane & 7);
  const int ly = ((sub >> 2) << 4) | ((wave >> 1) << 3) | (lane >> 3);
  const int tileId = A.tileBegin + k * A.tileStride;
  const int tx = tileId % A.tilesX, ty = tileId / A.tilesX;
  const int x = tx * 64 + lx, y = ty * 64 + ly;
  Counts cnt = {0, 0, 0, 0};
  if (k < A.numTiles && x < A.W && y < A.H) {
    const size_t outIdx = A.packed ? (size_t)k * 4096 + ly * 64 + lx : (size_t)x + (size_t)A.W * y;
    // Random rnd(accumID*W*H + x, y) (deviceCode.cu:288-289)
    uint32_t st = lcg_seed((uint32_t)A.accumID * (uint32_t)A.W * (uint32_t)A.H + (uint32_t)x, (uint32_t)y);
    // generateRay (deviceCode.cu:36-49): g++ draws the dir_dv jitter first
    st = lcg_next(st);
    const float jv = lcg_float(st);
    st = lcg_next(st);
    const float ju = lcg_float(st);
    const float su = (float)x + .5f, sv = (float)y + .5f;
    const float a = su + ju, b = sv + jv;
    float dx = (A.dir00.x + a * A.du.x) + b * A.dv.x;
    float dy = (A.dir00.y + a * A.du.y) + b * A.dv.y;
    float dz = (A.dir00.z + a * A.du.z) + b * A.dv.z;
    const float inv = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
    dx = dx / inv;
    dy = dy / inv;
    dz = dz / inv;
    if (fabsf(dx) < 1e-5f) dx = 1e-5f;
    if (fabsf(dy) < 1e-5f) dy = 1e-5f;
    if (fabsf(dz) < 1e-5f) dz = 1e-5f;
    Ray ray = {A.org.x, A.org.y, A.org.z, 0.f, dx, dy, dz, 1e10f};
    float t0, t1;
    if (box_test(ray, A, t0, t1)) {
      ++cnt.inBox;
      ray.tmin = t0;
      ray.tmax = t1;
      float cr = 0.f, cg = 0.f, cb = 0.f, alpha = 0.f;
      if (A.raygen == 1) {
        // woodcockTrackingAE (deviceCode.cu:239-275): majorant 1 over the box interval
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        bool hit = false;
        woodcock(A, ray, st, 1.f, s, hit, cnt);
        cr = s.x * A.amb.x * A.ambRad;
        cg = s.y * A.amb.y * A.ambRad;
        cb = s.z * A.amb.z * A.ambRad;
        alpha = s.w > 0.f ? 1.f : 0.f;
      } else {
        // sdda (ShellAccel.h:82-229) + the woodcockFunc lambda (deviceCode.cu:304-323)
        const float sbLoR = A.sbLo.x, sbHiR = A.sbHi.x;
        const float sceneEPS = sbLoR * 1e-6f;
        float st1 = 0.f, st2 = 0.f, st3 = 0.f, st4 = 0.f;
        const bool s1 = intersect_sphere(ray, sbHiR, st1, st4);
        const bool s2 = intersect_sphere(ray, sbLoR, st2, st3);
        if ((s1 || s2) && !(st4 < ray.tmin)) {
          float rlo[2] = {__builtin_inff(), __builtin_inff()}, rhi[2] = {-__builtin_inff(), -__builtin_inff()};
          if (s1 && !s2) {
            rlo[0] = st1; rhi[0] = st4;
          } else if (ray.tmin < st2) {
            rlo[0] = st1; rhi[0] = st2;
            rlo[1] = st3; rhi[1] = st4;
          } else {
            rlo[0] = st3; rhi[0] = st4;
          }
          bool done = false;
          for (int i = 0; i < 2 && !done; ++i) {
            const float lower = rlo[i], upper = rhi[i];
            if (upper <= lower) break;  // box1f::empty
            const float e1 = lower + sceneEPS, e2 = upper - sceneEPS;
            float r1, la1, lo1, r2, la2, lo2;
            to_spherical(ray.ox + ray.dx * e1, ray.oy + ray.dy * e1, ray.oz + ray.dz * e1, r1, la1, lo1);
            to_spherical(ray.ox + ray.dx * e2, ray.oy + ray.dy * e2, ray.oz + ray.dz * e2, r2, la2, lo2);
            // cell / step / stop (ShellAccel.h:121-132); x uses dims.x - 1 like y and z
            int cx = f2i_x86((r1 - A.sbLo.x) / (A.sbHi.x - A.sbLo.x) * (float)(A.dims.x - 1));
            int cy = project_axis(la1, A.sbLo.y, A.sbHi.y, A.dims.y);
            int cz = project_axis(lo1, A.sbLo.z, A.sbHi.z, A.dims.z);
            const int sx = r1 < r2 ? 1 : -1, sy = la1 < la2 ? 1 : -1, sz = lo1 < lo2 ? 1 : -1;
            const int ex = (int)((uint32_t)f2i_x86((r2 - A.sbLo.x) / (A.sbHi.x - A.sbLo.x) * (float)(A.dims.x - 1)) + (uint32_t)sx);
            const int ey = (int)((uint32_t)project_axis(la2, A.sbLo.y, A.sbHi.y, A.dims.y) + (uint32_t)sy);
            const int ez = (int)((uint32_t)project_axis(lo2, A.sbLo.z, A.sbHi.z, A.dims.z) + (uint32_t)sz);
            // The lat/lon "planes" of ShellAccel.h:147-160,183-200 are built from
            // toCartesian(vec3f(0.f, ...)) -- radius 0 -- so N = 0, w = 0 and every
            // evalPlane(...) is exactly +-0: tnext = {upper, 0, 0} throughout, and the
            // sign of those zeros never changes a comparison.  (radius/sphereT1 of
            // 136-146 is dead.)
            float tnx = upper;
            const float tny = 0.f, tnz = 0.f;
            float t = lower;
            for (int iter = 0; iter < (1 << 22); ++iter) {
              float tt1 = IRT_FLT_MAX;
              if (tnx < tt1 && tnx >= t) tt1 = tnx;
              if (tny < tt1 && tny >= t) tt1 = tny;
              if (tnz < tt1 && tnz >= t) tt1 = tnz;
              const uint32_t leaf = (uint32_t)wrap_coord(cz, A.dims.z) * (uint32_t)A.dims.x * (uint32_t)A.dims.y +
                                    (uint32_t)wrap_coord(cy, A.dims.y) * (uint32_t)A.dims.x +
                                    (uint32_t)wrap_coord(cx, A.dims.x);
              // woodcockFunc(leafID, t, tt1)
              {
                Ray wr = ray;
                wr.tmin = t;
                wr.tmax = tt1;
                float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
                bool hit = false;
                const float tw = woodcock(A, wr, st, A.maxOp[leaf], s, hit, cnt);
                if (tw > t && tw < tt1) {
                  cr = s.x * A.amb.x * A.ambRad;
                  cg = s.y * A.amb.y * A.ambRad;
                  cb = s.z * A.amb.z * A.ambRad;
                  alpha = s.w > 0.f ? 1.f : 0.f;
                  done = true;
                  break;
                }
              }
              const float t_closest = fminf(fminf(tnx, tny), tnz);
              if (tnx == t_closest) {
                cx += sx;
                if (cx == ex) break;
              }
              if (tny == t_closest) {
                cy += sy;
                if (cy == ey) break;
              }
              if (tnz == t_closest) {
                cz += sz;
                if (cz == ez) break;
              }
              t = t_closest;
            }
          }
        }
      }
      // accumulate: lerp(vec4f(color,alpha), old, 1/(accumID+1)) (deviceCode.cu:333-334)
      const float w = 1.f / (float)(A.accumID + 1);
      float4 old = A.accum[outIdx];
      float4 nv;
      nv.x = w * cr + (1.f - w) * old.x;
      nv.y = w * cg + (1.f - w) * old.y;
      nv.z = w * cb + (1.f - w) * old.z;
      nv.w = w * alpha + (1.f - w) * old.w;
      A.accum[outIdx] = nv;
      // linear_to_srgb + make_rgba (deviceCode.cu:336-340)
      A.fb[outIdx] = srgb_byte(s_th, nv.x) + (srgb_byte(s_th, nv.y) << 8) +
                     (srgb_byte(s_th, nv.z) << 16) + (make_8bit(nv.w) << 24);
    }
  }
  if (A.counters) {
    // per-workgroup reduction, one 64-bit atomic per counter per workgroup
    const int inRange = (k < A.numTiles && x < A.W && y < A.H) ? 1 : 0;
    atomicAdd(&s_cnt[0], (uint32_t)inRange);
    if (cnt.inBox) atomicAdd(&s_cnt[1], cnt.inBox);
    if (cnt.locate) atomicAdd(&s_cnt[2], cnt.locate);
    if (cnt.found) atomicAdd(&s_cnt[3], cnt.found);
    __syncthreads();
    if (tid < 4) atomicAdd(&A.counters[tid], (unsigned long long)s_cnt[tid]);
    // candidate-list entries examined (wave-reduced)
    uint32_t c = cnt.cand;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if (lane == 0 && c) atomicAdd(&A.counters[4], (unsigned long long)c);
  }
}

// ------------------------------------------------------------------ shell accelerator
// initGrid(ShellAccel) (hostCode.cu:216-225)
__global__ void k_shell_init(float2 *valueRanges, size_t numMCs) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < numMCs) valueRanges[i] = make_float2(IRT_FLT_MAX, -IRT_FLT_MAX);
}

// float atomicMin/atomicMax of hostCode.cu:36-56: store only when strictly smaller/larger
__device__ __forceinline__ void atomic_min_f(float *addr, float val) {
  int ret = __float_as_int(*addr);
  while (val < __int_as_float(ret)) {
    const int old = ret;
    if ((ret = atomicCAS((int *)addr, old, __float_as_int(val))) == old) break;
  }
}
__device__ __forceinline__ void atomic_max_f(float *addr, float val) {
  int ret = __float_as_int(*addr);
  while (val > __int_as_float(ret)) {
    const int old = ret;
    if ((ret = atomicCAS((int *)addr, old, __float_as_int(val))) == old) break;
  }
}

// buildShell_ICON (hostCode.cu:299-336).  Per cell and layer i the reference rasterises
// the rectangle [min(proj(bottom corners)), max(proj(top corners))] with the range
// (getValue(h[i]), getValue(h[i+1])).  The lat/lon projections do not depend on the
// height and dims.x = 1 makes the radial index 0 (times dims.x-1 = 0), so every layer of
// a cell hits the same rectangle: rasterising min/max over the layers once is the same
// min/max.  One workgroup-stride loop per cell row keeps seam cells (spanning all 1024
// longitudes) from serialising a single lane.
__global__ void k_shell_build(const irt_icon_cell *cells, size_t n, int3 dims, float3 sbLo,
                              float3 sbHi, float *valueRanges) {
  const size_t ci = blockIdx.x;
  if (ci >= n) return;
  const irt_icon_cell &c = cells[ci];
  const int nl = c.numLayers;
  if (nl <= 0) return;
  // min/max over the layers with the CAS loops' "store only if strictly smaller/larger"
  // semantics (NaN never stores; +-inf and IRT_FLT_MAX behave as in the reference)
  float lo = IRT_FLT_MAX, hi = -IRT_FLT_MAX;
  for (int i = 0; i < nl; ++i) {
    const float v0 = c.value[find_height(c.height, nl, c.height[i])];      // getValue(h[i])
    const float v1 = c.value[find_height(c.height, nl, c.height[i + 1])];  // getValue(h[i+1])
    if (v0 < lo) lo = v0;
    if (v1 > hi) hi = v1;
  }
  int ylo = 0x7fffffff, yhi = (int)0x80000000u, zlo = 0x7fffffff, zhi = (int)0x80000000u;
  int xlo = 0x7fffffff, xhi = (int)0x80000000u;
  for (int k = 0; k < 3; ++k) {
    const int py = project_axis(c.lat[k], sbLo.y, sbHi.y, dims.y);
    const int pz = project_axis(c.lon[k], sbLo.z, sbHi.z, dims.z);
    const int pxb = f2i_x86((c.height[0] - sbLo.x) / (sbHi.x - sbLo.x) * (float)(dims.x - 1));
    const int pxt = f2i_x86((c.height[nl] - sbLo.x) / (sbHi.x - sbLo.x) * (float)(dims.x - 1));
    ylo = min(ylo, py); yhi = max(yhi, py);
    zlo = min(zlo, pz); zhi = max(zhi, pz);
    xlo = min(xlo, pxb); xhi = max(xhi, pxt);
  }
  // Out-of-grid rectangles only arise from degenerate bounds (zero-size or non-finite
  // sphericalBounds), where the reference writes out of bounds; clamp instead.
  xlo = max(xlo, 0); ylo = max(ylo, 0); zlo = max(zlo, 0);
  xhi = min(xhi, dims.x - 1); yhi = min(yhi, dims.y - 1); zhi = min(zhi, dims.z - 1);
  if (xlo > xhi || ylo > yhi || zlo > zhi) return;
  const int nx = xhi - xlo + 1, ny = yhi - ylo + 1, nz = zhi - zlo + 1;
  const long total = (long)nx * ny * nz;
  for (long q = threadIdx.x; q < total; q += blockDim.x) {
    const int mx = xlo + (int)(q % nx);
    const int my = ylo + (int)((q / nx) % ny);
    const int mz = zlo + (int)(q / ((long)nx * ny));
    const size_t id = (size_t)mz * dims.x * dims.y + (size_t)my * dims.x + mx;
    float *vr = valueRanges + 2 * id;
    atomic_min_f(vr, lo);
    atomic_max_f(vr + 1, hi);
  }
}

// computeMaxOpacities(ShellAccel) (hostCode.cu:362-397)
__global__ void k_max_opacities(const float2 *valueRanges, size_t numMCs, const float4 *lut,
                                int size, float tfLo, float tfHi, float *maxOp) {
  const size_t mc = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (mc >= numMCs) return;
  float2 vr = valueRanges[mc];
  if (vr.y < vr.x) {
    maxOp[mc] = 0.f;
    return;
  }
  vr.x -= tfLo;
  vr.x /= tfHi - tfLo;
  vr.y -= tfLo;
  vr.y /= tfHi - tfLo;
  int lo = f2i_x86(vr.x * (float)(size - 1));
  int hi = (int)((uint32_t)f2i_x86(vr.y * (float)(size - 1)) + 1u);
  lo = lo < 0 ? 0 : (lo > size - 1 ? size - 1 : lo);
  hi = hi < 0 ? 0 : (hi > size - 1 ? size - 1 : hi);
  float m = 0.f;
  for (int i = lo; i <= hi; ++i) m = fmaxf(m, lut[i].w);
  maxOp[mc] = m;
}

// clearFramebuffer (common/pipeline.cu:171-199)
__global__ void k_clear(uint32_t *fb, float4 *accum, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (fb) fb[i] = 0u;  // make_rgba(vec4f(0)) == 0
  if (accum) accum[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Scatter rank-major packed tiles into a linear framebuffer (multi-GPU gather epilogue).
__global__ void k_unpack(const uint32_t *gathered, int numRanks, int maxTiles, int W, int H,
                         int tilesX, int numTilesTotal, uint32_t *fb) {
  const int k = blockIdx.x;  // tile slot
  const int rank = blockIdx.y;
  const int tileId = rank + k * numRanks;
  if (k >= maxTiles || tileId >= numTilesTotal) return;
  const int tx = tileId % tilesX, ty = tileId / tilesX;
  const uint32_t *src = gathered + ((size_t)rank * maxTiles + k) * 4096;
  for (int p = threadIdx.x; p < 4096; p += blockDim.x) {
    const int x = tx * 64 + (p & 63), y = ty * 64 + (p >> 6);
    if (x < W && y < H) fb[(size_t)x + (size_t)W * y] = src[p];
  }
}

// ------------------------------------------------------------------ launchers
void launch_render(const RenderArgs &A, int numBlocks, hipStream_t s) {
  hipLaunchKernelGGL(k_render, dim3(numBlocks), dim3(256), 0, s, A);
}
void launch_shell_init(float *vr, size_t numMCs, hipStream_t s) {
  hipLaunchKernelGGL(k_shell_init, dim3((unsigned)((numMCs + 255) / 256)), dim3(256), 0, s,
                     (float2 *)vr, numMCs);
}
void launch_shell_build(const irt_icon_cell *cells, size_t n, int3 dims, float3 lo, float3 hi,
                        float *vr, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_shell_build, dim3((unsigned)n), dim3(64), 0, s, cells, n, dims, lo, hi, vr);
}
void launch_max_opacities(const float *vr, size_t numMCs, const float4 *lut, int size, float lo,
                          float hi, float *maxOp, hipStream_t s) {
  hipLaunchKernelGGL(k_max_opacities, dim3((unsigned)((numMCs + 255) / 256)), dim3(256), 0, s,
                     (const float2 *)vr, numMCs, lut, size, lo, hi, maxOp);
}
void launch_clear(uint32_t *fb, float4 *accum, size_t n, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_clear, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, fb, accum, n);
}
void launch_unpack(const uint32_t *g, int numRanks, int maxTiles, int W, int H, uint32_t *fb,
                   hipStream_t s) {
  const int tilesX = (W + 63) / 64, tilesY = (H + 63) / 64;
  hipLaunchKernelGGL(k_unpack, dim3(maxTiles, numRanks), dim3(256), 0, s, g, numRanks, maxTiles,
                     W, H, tilesX, tilesX * tilesY, fb);
}

}  // namespace irt
