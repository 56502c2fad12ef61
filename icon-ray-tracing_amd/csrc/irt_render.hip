// irt_render.hip -- the hot path: the raygen woodcockTrackingWithAccel /
// woodcockTrackingAE (icon_rt/deviceCode.cu:239-341) as a gfx950 kernel.
//
// One lane per pixel, one wave64 per 8x8 pixel packet (neighbouring rays walk the same
// cube-map cells and records), a 256-thread workgroup per 16x16 block, 16 workgroups per
// 64x64 frame tile -- the unit the reference's CPU parallel_for hands out
// (common/for_each.h:70-85) and the unit of the multi-GPU frame split.
//
// The kernel is a chain of dependent gathers (logf table -> cube-map cell -> candidate
// entries -> side planes -> heights -> value -> LUT), so its speed is the number of
// dependent memory round trips per sample.  The OPT bits below remove round trips without
// changing a single result; each combination is a separate instantiation so variants can
// be A/B-timed in one process (irt_debug_set_variant) and checked for parity.
//
// Bit-exactness: see irt_common.h / irt_device.h and DESIGN.md section 3.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "irt_device.h"

namespace irt {

enum : int {
  OPT_BATCH = 1,    // load candidate entries 4 at a time (one round trip per 4)
  OPT_PLANES = 2,   // issue the 3 side-plane loads together
  OPT_HVEC = 4,     // sorted columns: findHeight from one 128-B line held in registers
  OPT_SPEC = 8,     // issue that line together with the planes (speculative)
  OPT_LUTLDS = 32,  // transfer-function LUT in LDS
  OPT_ACCPF = 64,   // read the old accum value at ray start
  OPT_REC = 8192    // render-record layout (irt_common.h): planes + coarse keys in one
                    // gather, findHeight's block + value in a second
};

constexpr int kLutLds = 1024;

template <int OPT>
struct Tracer {
  const RenderArgs &A;
  const float4 *s_lut;
  bool lutLds;
  const LogfTab *s_logf;
  Counts &cnt;

  __device__ Tracer(const RenderArgs &a, const float4 *sl, bool ll, const LogfTab *lt, Counts &c)
      : A(a), s_lut(sl), lutLds(ll), s_logf(lt), cnt(c) {}

  // logf(1.f - rnd()) for the draw that produced state s (deviceCode.cu:165): glibc's
  // algorithm in registers (irt_common.h), no table gather
  __device__ __forceinline__ float log_at(uint32_t s) { return woodcock_log(s, s_logf); }

  // getValue (ICONGrid.h:147-164) of record E.z at radius r
  __device__ __forceinline__ float get_value(const uint4 &E, float r, const float4 *h, bool haveH) {
    const uint32_t idx = E.z, nl = E.w & 0x7fffffffu;
    const float *hv = A.hv + (size_t)idx * kHV;
    if constexpr ((OPT & OPT_HVEC) != 0) {
      if (E.w >> 31) {
        float4 hh[8];
        const float4 *H = reinterpret_cast<const float4 *>(hv);
#pragma unroll
        for (int q = 0; q < 8; ++q) hh[q] = haveH ? h[q] : H[q];
        // sorted height[1..nl]: lower_bound == #{ j in [1,nl] : height[j] < r }
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float hq[4] = {hh[q].x, hh[q].y, hh[q].z, hh[q].w};
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const uint32_t j = 4 * q + s;
            if (j >= 1) c += (j <= nl && hq[s] < r) ? 1u : 0u;
          }
        }
        return hv[32 + c];
      }
    }
    return hv[32 + find_height(hv, (int)nl, r)];
  }

  // sample(cell, pos, value) (ICONGrid.h:181-208) for one candidate that passed the radial
  // test: the three ccw side planes, then getValue.
  __device__ __forceinline__ bool test_record(const uint4 &E, float px, float py, float pz,
                                              float r, float &value) {
    const float4 *P = A.planes + 3 * (size_t)E.z;
    float4 h[8];
    bool haveH = false;
    if constexpr ((OPT & OPT_SPEC) != 0 && (OPT & OPT_HVEC) != 0) {
      if (E.w >> 31) {
        const float4 *H = reinterpret_cast<const float4 *>(A.hv + (size_t)E.z * kHV);
#pragma unroll
        for (int q = 0; q < 8; ++q) h[q] = H[q];
        haveH = true;
      }
    }
    if constexpr ((OPT & OPT_PLANES) != 0) {
      const float4 p0 = P[0], p1 = P[1], p2 = P[2];
      if (dot3(px, py, pz, p0.x, p0.y, p0.z) - p0.w > 0.f) return false;  // ICONGrid.h:201
      if (dot3(px, py, pz, p1.x, p1.y, p1.z) - p1.w > 0.f) return false;  // 202
      if (dot3(px, py, pz, p2.x, p2.y, p2.z) - p2.w > 0.f) return false;  // 203
    } else {
      const float4 p0 = P[0];
      if (dot3(px, py, pz, p0.x, p0.y, p0.z) - p0.w > 0.f) return false;
      const float4 p1 = P[1];
      if (dot3(px, py, pz, p1.x, p1.y, p1.z) - p1.w > 0.f) return false;
      const float4 p2 = P[2];
      if (dot3(px, py, pz, p2.x, p2.y, p2.z) - p2.w > 0.f) return false;
    }
    value = get_value(E, r, h, haveH);
    return true;
  }

  // sample() on the render record (OPT_REC): two gathers for a hit
  __device__ __forceinline__ bool test_rec(const uint4 &E, float px, float py, float pz, float r,
                                           float &value) {
    const float4 *R = A.arena + A.aRec + (size_t)E.z * kRec4;
    const float4 p0 = R[0], p1 = R[1], p2 = R[2], ck = R[3];
    if (dot3(px, py, pz, p0.x, p0.y, p0.z) - p0.w > 0.f) return false;  // ICONGrid.h:201
    if (dot3(px, py, pz, p1.x, p1.y, p1.z) - p1.w > 0.f) return false;  // 202
    if (dot3(px, py, pz, p2.x, p2.y, p2.z) - p2.w > 0.f) return false;  // 203
    const int nl = (int)(E.w & 0x7fffffffu);
    if (E.w >> 31) {
      const int b = rec_coarse_block(ck.x, ck.y, ck.z, ck.w, nl, r);
      const float4 *B = R + 4 + 4 * b;
      const float4 h0 = B[0], h1 = B[1], v0 = B[2], v1 = B[3];
      const int m = rec_block_index(h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, b, nl, r);
      value = select8(m, v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w);
    } else {
      const float *Rf = reinterpret_cast<const float *>(R);
      int first = 0, count = nl;  // findHeight, literally (ICONGrid.h:117-145)
      while (count > 0) {
        const int stp = count / 2, it = first + stp;
        if (!(r <= Rf[rec_height_pos(it + 1)])) {
          first = it + 1;
          count -= stp + 1;
        } else {
          count = stp;
        }
      }
      value = Rf[rec_value_pos(first)];
    }
    return true;
  }

  __device__ __forceinline__ bool try_entry(const uint4 &E, float px, float py, float pz, float r,
                                            float &value) {
    ++cnt.cand;
    if (r < __uint_as_float(E.x) || r > __uint_as_float(E.y)) return false;  // ICONGrid.h:184
    if constexpr ((OPT & OPT_REC) != 0) return test_rec(E, px, py, pz, r, value);
    return test_record(E, px, py, pz, r, value);
  }

  // sampleVolume (deviceCode.cu:58-125) over the cube-map candidate lists: lists are
  // sorted by record index, so the first entry passing sample() is the reference's
  // lowest-index answer (116-123).
  __device__ __forceinline__ bool locate(float px, float py, float pz, float &value) {
    if (A.numCells == 0) return false;
    const float r = sqrtf(dot3(px, py, pz, px, py, pz));  // toSpherical(pos).x
    const uint32_t cell = cubemap_cell(px, py, pz, A.G);
    const uint32_t beg = A.offsets[cell], end = A.offsets[cell + 1];
    if constexpr ((OPT & OPT_BATCH) != 0) {
      for (uint32_t e = beg; e < end; e += 4) {
        const uint32_t last = end - 1;
        const uint4 E0 = A.entries[e];
        const uint4 E1 = A.entries[min(e + 1, last)];
        const uint4 E2 = A.entries[min(e + 2, last)];
        const uint4 E3 = A.entries[min(e + 3, last)];
        if (try_entry(E0, px, py, pz, r, value)) return true;
        if (e + 1 < end && try_entry(E1, px, py, pz, r, value)) return true;
        if (e + 2 < end && try_entry(E2, px, py, pz, r, value)) return true;
        if (e + 3 < end && try_entry(E3, px, py, pz, r, value)) return true;
      }
    } else {
      for (uint32_t e = beg; e < end; ++e)
        if (try_entry(A.entries[e], px, py, pz, r, value)) return true;
    }
    return false;
  }

  // postClassify (deviceCode.cu:127-135): weights reversed, opacityScale on 2nd term only
  __device__ __forceinline__ float4 post_classify(float v) {
    v = (v - A.tfLo) / (A.tfHi - A.tfLo);
    const int size = A.lutSize;
    const int idx = f2i_x86(v * (float)size);
    const float frac = (v * (float)size) - (float)idx;
    const int i1 = idx < 0 ? 0 : (idx > size - 1 ? size - 1 : idx);
    const int idx2 = (int)((uint32_t)idx + 1u);
    const int i2 = idx2 < 0 ? 0 : (idx2 > size - 1 ? size - 1 : idx2);
    float4 a, b;
    if ((OPT & OPT_LUTLDS) != 0 && lutLds) {
      a = s_lut[i1];
      b = s_lut[i2];
    } else {
      a = A.lut[i1];
      b = A.lut[i2];
    }
    const float om = 1.f - frac;
    float4 o;
    o.x = a.x * frac + b.x * om * 1.f;
    o.y = a.y * frac + b.y * om * 1.f;
    o.z = a.z * frac + b.z * om * 1.f;
    o.w = a.w * frac + b.w * om * A.opacityScale;
    return o;
  }

  // woodcockTracking (deviceCode.cu:149-186).  `count` is false inside zero-length sdda
  // leaves, whose sampleVolume calls are not counted (see the sdda loop below).
  __device__ __forceinline__ float woodcock(const Ray &ray, uint32_t &st, float majorant,
                                            float4 &sampleOut, bool count = true) {
    float t = ray.tmin;
    while (true) {
      if (majorant <= 0.f) break;
      st = lcg_next(st);
      const float lg = log_at(st);
      t -= (lg / (majorant / A.unitDistance));
      if (t > ray.tmax) break;
      const float px = ray.ox + ray.dx * t, py = ray.oy + ray.dy * t, pz = ray.oz + ray.dz * t;
      float value = 0.f;
      if (count) ++cnt.locate;
      if (!locate(px, py, pz, value)) continue;
      if (count) ++cnt.found;
      const float4 s = post_classify(value);
      st = lcg_next(st);
      const float u = lcg_float(st);
      if (s.w >= u * majorant) {
        sampleOut = s;
        break;
      }
    }
    return fminf(t, ray.tmax);
  }
};

// Variant bits 8-11: minimum waves per SIMD asked of the register allocator (0: none).
template <int OPT>
__global__ void __launch_bounds__(256, ((OPT >> 8) & 15) ? ((OPT >> 8) & 15) : 1) k_render(RenderArgs A) {
  __shared__ float s_th[256];
  __shared__ uint32_t s_cnt[4];
  __shared__ float4 s_lut[(OPT & OPT_LUTLDS) != 0 ? kLutLds : 1];
  __shared__ LogfTab s_logf[16];
  const int tid = threadIdx.x;
  s_th[tid] = A.srgbTh[tid];
  if (tid < 16) s_logf[tid] = kLogfTab[tid];
  if (tid < 4) s_cnt[tid] = 0;
  const bool lutLds = (OPT & OPT_LUTLDS) != 0 && A.lutSize <= kLutLds;
  if ((OPT & OPT_LUTLDS) != 0 && lutLds)
    for (int i = tid; i < A.lutSize; i += 256) s_lut[i] = A.lut[i];
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
  Tracer<OPT> T(A, s_lut, lutLds, s_logf, cnt);
  const bool active = k < A.numTiles && x < A.W && y < A.H;
  if (active) {
    const size_t outIdx = A.packed ? (size_t)k * 4096 + ly * 64 + lx : (size_t)x + (size_t)A.W * y;
    float4 old = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr ((OPT & OPT_ACCPF) != 0) old = A.accum[outIdx];
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
    const float len = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
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
        // woodcockTrackingAE (deviceCode.cu:239-275): majorant 1 over the box interval,
        // color/alpha from the last accepted sample (zero if none)
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        T.woodcock(ray, st, 1.f, s);
        cr = s.x * A.amb.x * A.ambRad;
        cg = s.y * A.amb.y * A.ambRad;
        cb = s.z * A.amb.z * A.ambRad;
        alpha = s.w > 0.f ? 1.f : 0.f;
      } else {
        // sdda (ShellAccel.h:82-229) driving the woodcockFunc lambda (deviceCode.cu:304-323)
        const float sceneEPS = A.sbLo.x * 1e-6f;
        float st1 = 0.f, st2 = 0.f, st3 = 0.f, st4 = 0.f;
        const bool s1 = intersect_sphere(ray, A.sbHi.x, st1, st4);
        const bool s2 = intersect_sphere(ray, A.sbLo.x, st2, st3);
        if ((s1 || s2) && !(st4 < ray.tmin)) {
          float rlo[2] = {__builtin_inff(), __builtin_inff()};
          float rhi[2] = {-__builtin_inff(), -__builtin_inff()};
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
            if (upper <= lower) break;  // box1f::empty (vecmath.h:981)
            const float e1 = lower + sceneEPS, e2 = upper - sceneEPS;
            float r1, la1, lo1, r2, la2, lo2;
            to_spherical(ray.ox + ray.dx * e1, ray.oy + ray.dy * e1, ray.oz + ray.dz * e1, r1, la1, lo1);
            to_spherical(ray.ox + ray.dx * e2, ray.oy + ray.dy * e2, ray.oz + ray.dz * e2, r2, la2, lo2);
            // cellID / step / stop (ShellAccel.h:121-132)
            int cx = project_axis(r1, A.sbLo.x, A.sbHi.x, A.dims.x);
            int cy = project_axis(la1, A.sbLo.y, A.sbHi.y, A.dims.y);
            int cz = project_axis(lo1, A.sbLo.z, A.sbHi.z, A.dims.z);
            const int sx = r1 < r2 ? 1 : -1, sy = la1 < la2 ? 1 : -1, sz = lo1 < lo2 ? 1 : -1;
            const int ex = (int)((uint32_t)project_axis(r2, A.sbLo.x, A.sbHi.x, A.dims.x) + (uint32_t)sx);
            const int ey = (int)((uint32_t)project_axis(la2, A.sbLo.y, A.sbHi.y, A.dims.y) + (uint32_t)sy);
            const int ez = (int)((uint32_t)project_axis(lo2, A.sbLo.z, A.sbHi.z, A.dims.z) + (uint32_t)sz);
            // The lat/lon "planes" (ShellAccel.h:147-160, 183-200) are built from
            // toCartesian(vec3f(0.f, ...)) -- radius 0 -- so N = 0, w = 0 and every
            // evalPlane(...) is exactly +-0: tnext = {upper, 0, 0} throughout, and the sign
            // of those zeros never changes a comparison.  (radius/sphereT1, 136-146, is dead.)
            const float tnx = upper, tny = 0.f, tnz = 0.f;
            // Since tnext never changes, every leaf after the first sees the same interval
            // [t_closest, t_closest] (t_closest = min(upper, 0)): a zero-length leaf, where
            // woodcockTracking can only draw (its tw <= tmax == tmin never passes
            // deviceCode.cu:316).  Such leaves matter only through the RNG state they
            // advance, i.e. only when another range follows.
            const bool lastRange = i == 1 || rhi[1] <= rlo[1];
            float t = lower;
            for (int iter = 0; iter < (1 << 22); ++iter) {
              float tt1 = IRT_FLT_MAX;
              if (tnx < tt1 && tnx >= t) tt1 = tnx;
              if (tny < tt1 && tny >= t) tt1 = tny;
              if (tnz < tt1 && tnz >= t) tt1 = tnz;
              const uint32_t leaf = (uint32_t)wrap_coord(cz, A.dims.z) * (uint32_t)A.dims.x * (uint32_t)A.dims.y +
                                    (uint32_t)wrap_coord(cy, A.dims.y) * (uint32_t)A.dims.x +
                                    (uint32_t)wrap_coord(cx, A.dims.x);
              if (tt1 == t) {
                // zero-length leaf: nothing later reads the RNG state in the last range
                if (lastRange) break;
                const float maj = A.maxOp[leaf];
                const float q = maj / A.unitDistance;
                const uint32_t nx = lcg_next(st);
                if (maj > 0.f && q > 0.f && q <= 1e30f && (nx & 0x00FFFFFFu) != 0u) {
                  // one draw: logf(1-xi) < 0 puts t past tmax (deviceCode.cu:165-166)
                  st = nx;
                } else {
                  Ray wr = ray;
                  wr.tmin = t;
                  wr.tmax = tt1;
                  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
                  T.woodcock(wr, st, maj, s, false);
                }
              } else {  // woodcockFunc(leafID, t, tt1)
                Ray wr = ray;
                wr.tmin = t;
                wr.tmax = tt1;
                float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
                const float tw = T.woodcock(wr, st, A.maxOp[leaf], s);
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
      if constexpr ((OPT & OPT_ACCPF) == 0) old = A.accum[outIdx];
      const float w = 1.f / (float)(A.accumID + 1);
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
    atomicAdd(&s_cnt[0], active ? 1u : 0u);
    if (cnt.inBox) atomicAdd(&s_cnt[1], cnt.inBox);
    if (cnt.locate) atomicAdd(&s_cnt[2], cnt.locate);
    if (cnt.found) atomicAdd(&s_cnt[3], cnt.found);
    __syncthreads();
    if (tid < 4) atomicAdd(&A.counters[tid], (unsigned long long)s_cnt[tid]);
    uint32_t c = cnt.cand;  // candidate-list entries examined (wave-reduced)
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if (lane == 0 && c) atomicAdd(&A.counters[4], (unsigned long long)c);
  }
}

// ------------------------------------------------------------------ variants / launcher
#define IRT_VARIANTS(X) \
  X(0) X(1536) X(8192) X(8224) X(9728) X(9760) X(10240) X(10272) X(9729) X(9731)

bool render_variant_available(int v) {
#define IRT_CASE(N) if (v == N) return true;
  IRT_VARIANTS(IRT_CASE)
#undef IRT_CASE
  return false;
}

void launch_render(const RenderArgs &A, int numBlocks, hipStream_t s, int variant) {
  switch (variant) {
#define IRT_CASE(N) \
  case N:           \
    hipLaunchKernelGGL(k_render<N>, dim3(numBlocks), dim3(256), 0, s, A); \
    return;
    IRT_VARIANTS(IRT_CASE)
#undef IRT_CASE
    default:
      hipLaunchKernelGGL(k_render<0>, dim3(numBlocks), dim3(256), 0, s, A);
  }
}

}  // namespace irt
