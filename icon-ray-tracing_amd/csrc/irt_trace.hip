// irt_trace.hip -- the raygen woodcockTrackingWithAccel / woodcockTrackingAE
// (icon_rt/deviceCode.cu:239-341) as a per-lane state machine for gfx950.
//
// The raygen is a chain of dependent gathers: logf table -> cube-map cell -> candidate
// entries -> side planes -> heights -> value (-> LUT).  Written as nested loops (sdda leaves
// > Woodcock draws > candidates > binary search, irt_render.hip) a wave64 executes the
// UNION of its lanes' control paths, so its dependent round trips add up across lanes
// (measured: ~130 vector loads per wave at ~750-cycle latency, 81% of wave time waiting).
// Here every lane carries an explicit state, and one loop iteration
//   1. issues exactly four 16-B gathers per lane, all off one base (the render arena), with
//      addresses the previous iteration prepared, then waits once;
//   2. advances every lane by one step on the data it received.
// A wave's dependent round trips are then the MAXIMUM of its lanes' step counts instead of
// the sum over diverging paths.  The state-specific address choice costs nothing at issue
// time: each transition writes the slot indices for its successor.
//
// Steps (one gather each):
//   LEAF  maxOpacities[leaf]                                        (deviceCode.cu:307)
//   OFFS  cube-map CSR offsets of the sample's cell
// (logf(1-rnd()) itself is computed, glibc's algorithm in registers: irt_common.h)
//   ENT   four candidate entries; the radial test (ICONGrid.h:184) picks the first
//   PLN   that record's three side planes (ICONGrid.h:197-203) + its coarse height keys
//   BLK   the height/value block that holds findHeight's answer (ICONGrid.h:117-164)
//   HS/VAL  literal binary search, for records whose heights are not sorted
//   DEG   up to four zero-length sdda leaves (see below)
// The LUT (postClassify, deviceCode.cu:127-135) is read from LDS.
//
// Zero-length leaves: the reference's lat/lon "planes" are degenerate (irt_render.hip),
// so tnext never changes and every sdda leaf after a range's first one has the interval
// [t_c, t_c].  Woodcock tracking there can only consume draws (its tw <= tmax == tmin never
// passes deviceCode.cu:316), which matter only if another range follows: in the last range
// the walk ends at once, otherwise DEG consumes one draw per leaf with a positive majorant
// (logf(1-xi) < 0 moves t past tmax), falling back to the general path for xi == 0.
// sampleVolume calls in zero-length leaves are not counted (the oracle uses the same rule).
//
// Mapping: one lane per pixel, wave64 = 8x8 packet, 256-thread workgroup = 16x16 block,
// 16 workgroups per 64x64 frame tile (the reference's CPU tile, common/for_each.h:70-85,
// and the unit of the multi-GPU frame split).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "irt_device.h"

namespace irt {
namespace {

enum : uint32_t { S_LEAF, S_OFFS, S_ENT, S_PLN, S_BLK, S_HS, S_VAL, S_DEG, S_DONE };
enum : uint32_t { EV_NONE, EV_VALUE, EV_DRAW, EV_EXIT, EV_RANGE, EV_LEAF };

constexpr int kTraceLut = 1024;         // LUT entries held in LDS (16 KB)
constexpr int kMaxSteps = 1 << 24;      // bound on iterations (the reference has none)

template <int MINW>
__global__ void __launch_bounds__(256, MINW) k_trace(RenderArgs A) {
  __shared__ float s_th[256];
  __shared__ float4 s_lut[kTraceLut];
  __shared__ uint32_t s_cnt[4];
  __shared__ LogfTab s_logf[16];
  const int tid = threadIdx.x;
  s_th[tid] = A.srgbTh[tid];
  if (tid < 16) s_logf[tid] = kLogfTab[tid];
  if (tid < 4) s_cnt[tid] = 0;
  const bool lutLds = A.lutSize <= kTraceLut;
  if (lutLds)
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
  const bool active = k < A.numTiles && x < A.W && y < A.H;
  const bool ae = A.raygen == 1;
  const float4 *__restrict__ ar = A.arena;

  // postClassify (deviceCode.cu:127-135): weights reversed, opacityScale on the 2nd term
  auto classify = [&](float v) {
    v = (v - A.tfLo) / (A.tfHi - A.tfLo);
    const int size = A.lutSize;
    const int idx = f2i_x86(v * (float)size);
    const float frac = (v * (float)size) - (float)idx;
    const int i1 = idx < 0 ? 0 : (idx > size - 1 ? size - 1 : idx);
    const int idx2 = (int)((uint32_t)idx + 1u);
    const int i2 = idx2 < 0 ? 0 : (idx2 > size - 1 ? size - 1 : idx2);
    const float4 a = lutLds ? s_lut[i1] : A.lut[i1];
    const float4 b = lutLds ? s_lut[i2] : A.lut[i2];
    const float om = 1.f - frac;
    float4 o;
    o.x = a.x * frac + b.x * om * 1.f;
    o.y = a.y * frac + b.y * om * 1.f;
    o.z = a.z * frac + b.z * om * 1.f;
    o.w = a.w * frac + b.w * om * A.opacityScale;
    return o;
  };

  Counts cnt = {0, 0, 0, 0};
  uint32_t state = S_DONE, ev = EV_NONE;
  bool write = false, hit = false;
  float value = 0.f;
  // ray
  float dx = 0.f, dy = 0.f, dz = 0.f;
  uint32_t st = 0;
  // Woodcock: sample distance tw, leaf interval [tlo, tmax], majorant, majorant/unitDistance
  float tw = 0.f, tlo = 0.f, tmax = 0.f, maj = 0.f, q = 1.f;
  // sdda (ShellAccel.h:82-229)
  int rIdx = -1;
  float upper = 0.f;
  uint32_t rcase = 0;  // 1: [t1,t4]  2: [t1,t2] then [t3,t4]  3: [t3,t4] (ShellAccel.h:106-117)
  int cx = 0, cy = 0, cz = 0, ex = 0, ey = 0, ez = 0, sx = 1, sy = 1, sz = 1;
  // sample point / locator walk
  float r = 0.f;  // |sample point| (the point itself is recomputed from tw)
  uint32_t e = 0, eend = 0, rec = 0, meta = 0, blk = 0;
  // gather slots (float4 indices into the arena) and their component selectors
  uint32_t sl0 = 0, sl1 = 0, sl2 = 0, sl3 = 0, sel = 0;

  if (active) {
    // Random rnd(accumID*W*H + x, y) (deviceCode.cu:288-289)
    st = lcg_seed((uint32_t)A.accumID * (uint32_t)A.W * (uint32_t)A.H + (uint32_t)x, (uint32_t)y);
    // generateRay (deviceCode.cu:36-49): g++ draws the dir_dv jitter first
    st = lcg_next(st);
    const float jv = lcg_float(st);
    st = lcg_next(st);
    const float ju = lcg_float(st);
    const float a = ((float)x + .5f) + ju, b = ((float)y + .5f) + jv;
    dx = (A.dir00.x + a * A.du.x) + b * A.dv.x;
    dy = (A.dir00.y + a * A.du.y) + b * A.dv.y;
    dz = (A.dir00.z + a * A.du.z) + b * A.dv.z;
    const float len = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
    if (fabsf(dx) < 1e-5f) dx = 1e-5f;
    if (fabsf(dy) < 1e-5f) dy = 1e-5f;
    if (fabsf(dz) < 1e-5f) dz = 1e-5f;
    Ray ray = {A.org.x, A.org.y, A.org.z, 0.f, dx, dy, dz, 1e10f};
    float t0, t1;
    if (box_test(ray, A, t0, t1)) {  // deviceCode.cu:294
      ++cnt.inBox;
      write = true;
      ray.tmin = t0;
      ray.tmax = t1;
      if (ae) {
        // woodcockTrackingAE (deviceCode.cu:239-275): majorant 1 over the box interval
        tlo = t0;
        tmax = t1;
        tw = t0;
        state = S_LEAF;
        sl0 = sl1 = sl2 = sl3 = 0;
        sel = 0;
      } else {
        // sdda ranges (ShellAccel.h:86-117)
        float st1 = 0.f, st2 = 0.f, st3 = 0.f, st4 = 0.f;
        const bool s1 = intersect_sphere(ray, A.sbHi.x, st1, st4);
        const bool s2 = intersect_sphere(ray, A.sbLo.x, st2, st3);
        if ((s1 || s2) && !(st4 < ray.tmin)) {
          rcase = (s1 && !s2) ? 1u : (ray.tmin < st2 ? 2u : 3u);
          ev = EV_RANGE;
        }
      }
    }
  }

  const float sceneEPS = A.sbLo.x * 1e-6f;
  for (int step = 0; step < kMaxSteps; ++step) {
    if (state == S_DONE && ev == EV_NONE) break;
    if (ev == EV_NONE) {
      // ---- 1. one gather step: four 16-B loads, one wait
      // Vector slots feed ENT/PLN/BLK; the scalar view of the same slots (component in
      // `sel`, folded into the address) feeds LEAF/OFFS/HS/VAL/DEG.  Same lines, so the
      // unused half costs issue slots, not HBM traffic.
      const float4 d0 = ar[sl0], d1 = ar[sl1], d2 = ar[sl2], d3 = ar[sl3];
      const float *af = reinterpret_cast<const float *>(ar);
      const float s0 = af[(size_t)sl0 * 4 + (sel & 3u)], s1 = af[(size_t)sl1 * 4 + ((sel >> 2) & 3u)],
                  s2 = af[(size_t)sl2 * 4 + ((sel >> 4) & 3u)], s3 = af[(size_t)sl3 * 4 + ((sel >> 6) & 3u)];
      // ---- 2. consume
      if (state == S_LEAF) {
        maj = ae ? 1.f : s0;
        if (maj <= 0.f) {  // deviceCode.cu:164
          ev = EV_EXIT;
        } else {
          q = maj / A.unitDistance;
          ev = EV_DRAW;
        }
      } else if (state == S_OFFS) {
        const uint32_t beg = __float_as_uint(s0), end = __float_as_uint(s1);
        if (A.numCells == 0 || beg >= end) {
          ev = EV_DRAW;  // not found: next draw
        } else {
          e = beg;
          eend = end;
          state = S_ENT;
        }
      } else if (state == S_ENT) {
        bool found = false;
        uint32_t ne = e + 4;
        const float4 E[4] = {d0, d1, d2, d3};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!found && e + j < eend) {
            ++cnt.cand;
            const float4 Ej = E[j];
            if (!(r < Ej.x || r > Ej.y)) {  // ICONGrid.h:184
              found = true;
              rec = __float_as_uint(Ej.z);
              meta = __float_as_uint(Ej.w);
              ne = e + j + 1;
            }
          }
        }
        e = ne;
        if (found) {
          state = S_PLN;
        } else if (e >= eend) {
          ev = EV_DRAW;
        }
      } else if (state == S_PLN) {
        // ICONGrid.h:201-203 (evaluated in order; no side effects)
        const float px = A.org.x + dx * tw, py = A.org.y + dy * tw, pz = A.org.z + dz * tw;
        const bool out = (dot3(px, py, pz, d0.x, d0.y, d0.z) - d0.w > 0.f) ||
                         (dot3(px, py, pz, d1.x, d1.y, d1.z) - d1.w > 0.f) ||
                         (dot3(px, py, pz, d2.x, d2.y, d2.z) - d2.w > 0.f);
        const int nl = (int)(meta & 0x7fffffffu);
        if (out) {
          if (e < eend) {
            state = S_ENT;
          } else {
            ev = EV_DRAW;
          }
        } else if (meta >> 31) {
          blk = (uint32_t)rec_coarse_block(d3.x, d3.y, d3.z, d3.w, nl, r);
          state = S_BLK;
        } else {
          // findHeight's binary search, literally (ICONGrid.h:117-145): e = first, eend = count
          e = 0;
          eend = (uint32_t)nl;
          state = eend > 0 ? S_HS : S_VAL;
        }
      } else if (state == S_BLK) {
        const int m = rec_block_index(d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, (int)blk,
                                      (int)(meta & 0x7fffffffu), r);
        value = select8(m, d2.x, d2.y, d2.z, d2.w, d3.x, d3.y, d3.z, d3.w);
        ev = EV_VALUE;
      } else if (state == S_HS) {
        const uint32_t stp = eend / 2, it = e + stp;
        if (!(r <= s0)) {  // height[it+1]
          e = it + 1;
          eend -= stp + 1;
        } else {
          eend = stp;
        }
        if (eend == 0) state = S_VAL;
      } else if (state == S_VAL) {
        value = s0;
        ev = EV_VALUE;
      } else if (state == S_DEG) {
        const float M[4] = {s0, s1, s2, s3};
        bool stay = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (stay) {
            const float mj = M[j];
            const float qj = mj / A.unitDistance;
            const uint32_t nx = lcg_next(st);
            if (mj > 0.f && qj > 0.f && qj <= 1e30f && (nx & 0x00FFFFFFu) != 0u) {
              st = nx;  // one draw, t jumps past tmax (deviceCode.cu:165-166)
            } else if (!(mj <= 0.f)) {
              ev = EV_LEAF;  // xi == 0 or an odd majorant: run this leaf literally
              stay = false;
            }
            if (stay) {
              // sdda step (ShellAccel.h:208-227) with tnext = {upper, 0, 0}
              const float tc = fminf(fminf(upper, 0.f), 0.f);
              bool end = false;
              if (upper == tc) { cx += sx; end = cx == ex; }
              if (!end && 0.f == tc) { cy += sy; end = cy == ey; }
              if (!end && 0.f == tc) { cz += sz; end = cz == ez; }
              tlo = tc;
              if (end) {
                ev = EV_RANGE;
                stay = false;
              } else {
                float tt1 = IRT_FLT_MAX;
                if (upper < tt1 && upper >= tlo) tt1 = upper;
                if (0.f < tt1 && 0.f >= tlo) tt1 = 0.f;
                if (tt1 != tlo) {  // cannot happen with a constant tnext; stay literal
                  ev = EV_LEAF;
                  stay = false;
                }
              }
            }
          }
        }
        if (stay) {  // next four leaves
          const float tc = fminf(fminf(upper, 0.f), 0.f);
          const int ix = upper == tc ? sx : 0, iy = 0.f == tc ? sy : 0, iz = 0.f == tc ? sz : 0;
          uint32_t lf[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            lf[j] = (uint32_t)wrap_coord(cz + j * iz, A.dims.z) * (uint32_t)A.dims.x * (uint32_t)A.dims.y +
                    (uint32_t)wrap_coord(cy + j * iy, A.dims.y) * (uint32_t)A.dims.x +
                    (uint32_t)wrap_coord(cx + j * ix, A.dims.x);
          sl0 = A.aMaxOp + (lf[0] >> 2);
          sl1 = A.aMaxOp + (lf[1] >> 2);
          sl2 = A.aMaxOp + (lf[2] >> 2);
          sl3 = A.aMaxOp + (lf[3] >> 2);
          sel = (lf[0] & 3u) | ((lf[1] & 3u) << 2) | ((lf[2] & 3u) << 4) | ((lf[3] & 3u) << 6);
        }
      }
    }

    // ---- a sample value was found: sampleVolume returned true (deviceCode.cu:173-181)
    if (ev == EV_VALUE) {
      if (tlo != tmax) ++cnt.found;
      const float4 s = classify(value);
      st = lcg_next(st);
      const float u = lcg_float(st);
      if (s.w >= u * maj) {
        // accepted; the sdda functor tests t in (t0, t1) (deviceCode.cu:316)
        if (ae || (tw > tlo && tw < tmax)) {
          hit = true;
          state = S_DONE;
          ev = EV_NONE;
        } else {
          ev = EV_EXIT;
        }
      } else {
        ev = EV_DRAW;  // rejected: next draw
      }
    }
    // ---- a distance draw: t -= logf(1-rnd()) / (majorant/unitDistance) (deviceCode.cu:165)
    if (ev == EV_DRAW) {
      st = lcg_next(st);
      tw -= (woodcock_log(st, s_logf) / q);
      if (tw > tmax) {
        ev = EV_EXIT;
      } else {
        if (tlo != tmax) ++cnt.locate;
        const float px = A.org.x + dx * tw, py = A.org.y + dy * tw, pz = A.org.z + dz * tw;
        r = sqrtf(dot3(px, py, pz, px, py, pz));  // toSpherical(pos).x
        const uint32_t cell = A.numCells ? cubemap_cell(px, py, pz, A.G) : 0u;
        sl0 = A.aOffs + (cell >> 2);
        sl1 = A.aOffs + ((cell + 1) >> 2);
        sl2 = sl3 = 0;
        sel = (cell & 3u) | (((cell + 1) & 3u) << 2);
        state = S_OFFS;
        ev = EV_NONE;
      }
    }
    // ---- the Woodcock loop of this leaf ended without a hit
    if (ev == EV_EXIT) {
      if (ae) {
        state = S_DONE;
        ev = EV_NONE;
      } else {
        // sdda step (ShellAccel.h:208-227) with tnext = {upper, 0, 0}
        const float tc = fminf(fminf(upper, 0.f), 0.f);
        bool end = false;
        if (upper == tc) { cx += sx; end = cx == ex; }
        if (!end && 0.f == tc) { cy += sy; end = cy == ey; }
        if (!end && 0.f == tc) { cz += sz; end = cz == ez; }
        tlo = tc;
        ev = end ? EV_RANGE : EV_LEAF;
      }
    }
    // ---- next range (ShellAccel.h:119-135)
    if (ev == EV_RANGE) {
      ++rIdx;
      // the ranges again from the two sphere hits (deterministic; two range switches per ray)
      float lower = __builtin_inff(), up = -__builtin_inff();
      if (rIdx <= 1) {
        const Ray ray = {A.org.x, A.org.y, A.org.z, 0.f, dx, dy, dz, 1e10f};
        float st1 = 0.f, st2 = 0.f, st3 = 0.f, st4 = 0.f;
        intersect_sphere(ray, A.sbHi.x, st1, st4);
        intersect_sphere(ray, A.sbLo.x, st2, st3);
        if (rIdx == 0) {
          lower = rcase == 3u ? st3 : st1;
          up = rcase == 2u ? st2 : st4;
        } else if (rcase == 2u) {
          lower = st3;
          up = st4;
        }
      }
      if (rIdx > 1 || up <= lower) {  // box1f::empty (vecmath.h:981) ends the loop
        state = S_DONE;
        ev = EV_NONE;
      } else {
        upper = up;
        const float e1 = lower + sceneEPS, e2 = up - sceneEPS;
        float r1, la1, lo1, r2, la2, lo2;
        to_spherical(A.org.x + dx * e1, A.org.y + dy * e1, A.org.z + dz * e1, r1, la1, lo1);
        to_spherical(A.org.x + dx * e2, A.org.y + dy * e2, A.org.z + dz * e2, r2, la2, lo2);
        cx = project_axis(r1, A.sbLo.x, A.sbHi.x, A.dims.x);
        cy = project_axis(la1, A.sbLo.y, A.sbHi.y, A.dims.y);
        cz = project_axis(lo1, A.sbLo.z, A.sbHi.z, A.dims.z);
        sx = r1 < r2 ? 1 : -1;
        sy = la1 < la2 ? 1 : -1;
        sz = lo1 < lo2 ? 1 : -1;
        ex = (int)((uint32_t)project_axis(r2, A.sbLo.x, A.sbHi.x, A.dims.x) + (uint32_t)sx);
        ey = (int)((uint32_t)project_axis(la2, A.sbLo.y, A.sbHi.y, A.dims.y) + (uint32_t)sy);
        ez = (int)((uint32_t)project_axis(lo2, A.sbLo.z, A.sbHi.z, A.dims.z) + (uint32_t)sz);
        tlo = lower;
        ev = EV_LEAF;
      }
    }
    // ---- enter the leaf at cellID with t = tlo (ShellAccel.h:201-207)
    if (ev == EV_LEAF) {
      float tt1 = IRT_FLT_MAX;
      if (upper < tt1 && upper >= tlo) tt1 = upper;
      if (0.f < tt1 && 0.f >= tlo) tt1 = 0.f;
      const uint32_t leaf = (uint32_t)wrap_coord(cz, A.dims.z) * (uint32_t)A.dims.x * (uint32_t)A.dims.y +
                            (uint32_t)wrap_coord(cy, A.dims.y) * (uint32_t)A.dims.x +
                            (uint32_t)wrap_coord(cx, A.dims.x);
      ev = EV_NONE;
      // range 1 exists only in case 2 (t3 < t4 there unless the hits are degenerate --
      // then the literal walk of range 0 just runs to its end)
      const bool lastRange = rIdx == 1 || rcase != 2u;
      if (tt1 == tlo && state != S_DEG) {
        // zero-length leaf: only the RNG state can matter, and only if a range follows
        if (lastRange) {
          state = S_DONE;
        } else {
          state = S_DEG;
          const float tc = fminf(fminf(upper, 0.f), 0.f);
          const int ix = upper == tc ? sx : 0, iy = 0.f == tc ? sy : 0, iz = 0.f == tc ? sz : 0;
          uint32_t lf[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            lf[j] = j == 0 ? leaf
                           : (uint32_t)wrap_coord(cz + j * iz, A.dims.z) * (uint32_t)A.dims.x * (uint32_t)A.dims.y +
                                 (uint32_t)wrap_coord(cy + j * iy, A.dims.y) * (uint32_t)A.dims.x +
                                 (uint32_t)wrap_coord(cx + j * ix, A.dims.x);
          sl0 = A.aMaxOp + (lf[0] >> 2);
          sl1 = A.aMaxOp + (lf[1] >> 2);
          sl2 = A.aMaxOp + (lf[2] >> 2);
          sl3 = A.aMaxOp + (lf[3] >> 2);
          sel = (lf[0] & 3u) | ((lf[1] & 3u) << 2) | ((lf[2] & 3u) << 4) | ((lf[3] & 3u) << 6);
        }
      } else {
        // woodcockFunc(leafID, t, tt1) (deviceCode.cu:304-323)
        tmax = tt1;
        tw = tlo;
        state = S_LEAF;
        sl0 = A.aMaxOp + (leaf >> 2);
        sl1 = sl2 = sl3 = 0;
        sel = leaf & 3u;
      }
    }

    // ---- gather addresses of the locator steps
    if (ev == EV_NONE) {
      if (state == S_ENT) {
        const uint32_t last = eend - 1;
        sl0 = A.aEnt + e;
        sl1 = A.aEnt + min(e + 1, last);
        sl2 = A.aEnt + min(e + 2, last);
        sl3 = A.aEnt + min(e + 3, last);
      } else if (state == S_PLN) {
        const uint32_t base = A.aRec + rec * (uint32_t)kRec4;
        sl0 = base;
        sl1 = base + 1;
        sl2 = base + 2;
        sl3 = base + 3;
      } else if (state == S_BLK) {
        const uint32_t base = A.aRec + rec * (uint32_t)kRec4 + 4 + 4 * blk;
        sl0 = base;
        sl1 = base + 1;
        sl2 = base + 2;
        sl3 = base + 3;
      } else if (state == S_HS || state == S_VAL) {
        // S_HS probes height[e + eend/2 + 1]; S_VAL reads value[e]
        const int pos = state == S_HS ? rec_height_pos((int)(e + eend / 2 + 1)) : rec_value_pos((int)e);
        sl0 = sl1 = sl2 = sl3 = A.aRec + rec * (uint32_t)kRec4 + (uint32_t)(pos >> 2);
        sel = (uint32_t)(pos & 3);
      }
    }
  }

  if (write) {
    // color/alpha of the accepted sample (deviceCode.cu:270-274, 317-320), then
    // lerp(vec4f(color,alpha), old, 1/(accumID+1)) and sRGB (deviceCode.cu:333-340)
    float cr = 0.f, cg = 0.f, cb = 0.f, alpha = 0.f;
    if (hit) {
      const float4 s = classify(value);
      cr = s.x * A.amb.x * A.ambRad;
      cg = s.y * A.amb.y * A.ambRad;
      cb = s.z * A.amb.z * A.ambRad;
      alpha = s.w > 0.f ? 1.f : 0.f;
    }
    const size_t outIdx = A.packed ? (size_t)k * 4096 + ly * 64 + lx : (size_t)x + (size_t)A.W * y;
    const float4 old = A.accum[outIdx];
    const float w = 1.f / (float)(A.accumID + 1);
    float4 nv;
    nv.x = w * cr + (1.f - w) * old.x;
    nv.y = w * cg + (1.f - w) * old.y;
    nv.z = w * cb + (1.f - w) * old.z;
    nv.w = w * alpha + (1.f - w) * old.w;
    A.accum[outIdx] = nv;
    A.fb[outIdx] = srgb_byte(s_th, nv.x) + (srgb_byte(s_th, nv.y) << 8) +
                   (srgb_byte(s_th, nv.z) << 16) + (make_8bit(nv.w) << 24);
  }
  if (A.counters) {
    atomicAdd(&s_cnt[0], active ? 1u : 0u);
    if (cnt.inBox) atomicAdd(&s_cnt[1], cnt.inBox);
    if (cnt.locate) atomicAdd(&s_cnt[2], cnt.locate);
    if (cnt.found) atomicAdd(&s_cnt[3], cnt.found);
    __syncthreads();
    if (tid < 4) atomicAdd(&A.counters[tid], (unsigned long long)s_cnt[tid]);
    uint32_t c = cnt.cand;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if (lane == 0 && c) atomicAdd(&A.counters[4], (unsigned long long)c);
  }
}

}  // namespace

#define IRT_TRACE_VARIANTS(X) X(0) X(5) X(6) X(8)

bool trace_variant_available(int v) {
  if ((v & kTraceBit) == 0) return false;
  const int w = (v >> 8) & 15;
#define IRT_CASE(N) if (w == N) return (v & ~(kTraceBit | 0xF00)) == 0;
  IRT_TRACE_VARIANTS(IRT_CASE)
#undef IRT_CASE
  return false;
}

void launch_trace(const RenderArgs &A, int numBlocks, hipStream_t s, int variant) {
  switch ((variant >> 8) & 15) {
#define IRT_CASE(N) \
  case N:           \
    hipLaunchKernelGGL(k_trace<(N) ? (N) : 1>, dim3(numBlocks), dim3(256), 0, s, A); \
    return;
    IRT_TRACE_VARIANTS(IRT_CASE)
#undef IRT_CASE
    default:
      hipLaunchKernelGGL(k_trace<1>, dim3(numBlocks), dim3(256), 0, s, A);
  }
}

}  // namespace irt
