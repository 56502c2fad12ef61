// irt_common.h -- numerics shared by the host build (g++) and the gfx950 kernels (hipcc).
//
// Everything here is pure IEEE-754 single-precision arithmetic (+ - * / sqrt, compares,
// integer ops), which gfx950 and x86-64 SSE evaluate identically when compiled with
// -ffp-contract=off and correctly rounded f32 divide/sqrt (hipcc's default).  That is what
// makes the MI355X path bit-exact against the reference's CPU build: the reference calls
// glibc's asinf/atan2f/logf/powf, so this header restates glibc's (fdlibm-derived)
// algorithms where a device version is needed, and the host tabulates the rest
// (logf over the 2^24 values 1-k/2^24 it can ever see; the sRGB byte thresholds).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define IRT_HD __host__ __device__ __forceinline__
#else
#include <string.h>
#define IRT_HD inline
#endif

namespace irt {

// Bit casts.
IRT_HD uint32_t f2u(float f) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(uint32_t, f);
#else
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
#endif
}
IRT_HD float u2f(uint32_t u) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(float, u);
#else
  float f;
  memcpy(&f, &u, 4);
  return f;
#endif
}

// float -> int with x86-64 cvttss2si semantics (the reference's g++ build): truncate
// toward zero; NaN or out of int range -> INT_MIN.  (gfx950 v_cvt_i32_f32 saturates and
// maps NaN to 0, so the conversion must be spelled out.)
IRT_HD int f2i_x86(float f) {
  if (!(f > -2147483904.0f && f < 2147483648.0f)) return (int)0x80000000u;
  return (int)f;
}

// LCG<4> of common/dvr_course-common-both.h:41-86: 4 TEA-like seeding rounds, then
// state = 1664525*state + 1013904223, sample = (state & 0xFFFFFF) / 2^24.
IRT_HD uint32_t lcg_seed(uint32_t v0, uint32_t v1) {
  uint32_t s0 = 0;
  for (int n = 0; n < 4; n++) {
    s0 += 0x9e3779b9u;
    v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
    v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
  }
  return v0;
}
IRT_HD uint32_t lcg_next(uint32_t s) { return 1664525u * s + 1013904223u; }
IRT_HD float lcg_float(uint32_t s) { return (float)(s & 0x00FFFFFFu) / (float)0x01000000; }

// n LCG steps at once: state_n = mul * state + add (mod 2^32), composed from the one-step
// map by binary powers (the maps commute).  The wave-cooperative Woodcock loop
// (irt_render.hip) evaluates sample k of a ray from the state 2k+1 (its step draw) and 2k+2
// (its acceptance draw) draws ahead; it tabulates n < kLcgJumps in LDS.
constexpr int kLcgJumps = 130;  // < 256 (lcg_jump's 8 bits)
IRT_HD void lcg_jump(uint32_t n, uint32_t &mul, uint32_t &add) {
  uint32_t m = 1u, c = 0u, bm = 1664525u, bc = 1013904223u;
  for (int bit = 0; bit < 8; ++bit) {  // n < 256; selects, no divergent branches
    const bool on = (n >> bit) & 1u;
    c = on ? bm * c + bc : c;
    m = on ? bm * m : m;
    bc = bm * bc + bc;
    bm = bm * bm;
  }
  mul = m;
  add = c;
}
// lcg_jump for n < kLcgJumps, tabulated at compile time as {mul, add} pairs: the kernels
// copy it into LDS with one load per lane instead of running lcg_jump's eight rounds of
// 32-bit multiplies (quarter-rate on the SIMD) in every workgroup's prologue.
struct LcgJumpTab {
  uint32_t ma[kLcgJumps][2];
};
constexpr LcgJumpTab make_lcg_jump_tab() {
  LcgJumpTab t{};
  for (int n = 0; n < kLcgJumps; ++n) {
    uint32_t m = 1u, c = 0u, bm = 1664525u, bc = 1013904223u;
    for (int bit = 0; bit < 8; ++bit) {
      if ((n >> bit) & 1) {
        c = bm * c + bc;
        m = bm * m;
      }
      bc = bm * bc + bc;
      bm = bm * bm;
    }
    t.ma[n][0] = m;
    t.ma[n][1] = c;
  }
  return t;
}
constexpr LcgJumpTab kLcgJumpTab = make_lcg_jump_tab();

// ---------------------------------------------------------------------------------
// glibc 2.35 flt-32 asinf / atanf / atan2f (fdlibm lineage: Sun Microsystems 1993,
// float conversion by Ian Lance Taylor, Cygnus; asinf polynomial by Naohiko Shimizu).
// Restated for the device so toSpherical() (icon_rt/ICONGrid.h:36-42), which sdda()
// evaluates per ray segment (ShellAccel.h:134-135), rounds exactly as the reference's
// glibc calls do.  Verified bit-exact against the host glibc: asinf and atanf over every
// float, atan2f over 2e8 samples (tests/test_math_restatement.py re-checks a sample).

IRT_HD float glibc_asinf(float x) {
  const float one = 1.0f, huge = 1.0e30f;
  const float pio2_hi = 1.57079637050628662109375f;
  const float pio2_lo = -4.37113900018624283e-8f;
  const float pio4_hi = 0.785398185253143310546875f;
  const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f,
              p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
  float t, w, p, q, c, r, s;
  const int32_t hx = (int32_t)f2u(x);
  const int32_t ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {
    if (ix < 0x32000000) {
      if (huge + x > one) return x;
    } else {
      t = x * x;
      w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
      return x + x * w;
    }
  }
  w = one - __builtin_fabsf(x);
  t = w * 0.5f;
  p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
  s = __builtin_sqrtf(t);
  if (ix >= 0x3F79999A) {
    t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
  } else {
    w = u2f(f2u(s) & 0xfffff000u);
    c = (t - w * w) / (s + w);
    r = p;
    p = 2.0f * s * r - (pio2_lo - 2.0f * c);
    q = pio4_hi - 2.0f * w;
    t = pio4_hi - (p - q);
  }
  return hx > 0 ? t : -t;
}

IRT_HD float glibc_atanf(float x) {
  const float one = 1.0f, huge = 1.0e30f;
  const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f,
              atanhi2 = 9.8279368877e-01f, atanhi3 = 1.5707962513e+00f;
  const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f,
              atanlo2 = 3.4473217170e-08f, atanlo3 = 7.5497894159e-08f;
  const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
              aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
              aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
              aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
  float w, s1, s2, z, hi, lo;
  const int32_t hx = (int32_t)f2u(x);
  const int32_t ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {
    if (ix > 0x7f800000) return x + x;
    return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
  }
  if (ix < 0x31000000) {
    if (huge + x > one) return x;
  }
  // the argument reduction of the four intervals -- (2x-1)/(2+x), (x-1)/(x+1),
  // (x-1.5)/(1+1.5x), -1/x on |x| -- as ONE division of selected operands, each operand
  // the same expression as fdlibm's (so the same roundings); below 7/16 x is kept, as x/1.
  // Lanes of a wave in different intervals then share one division instead of running
  // up to four divergent ones.
  {
    const float xa = __builtin_fabsf(x);
    id = ix < 0x3ee00000 ? -1 : ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
    const float num = id < 0 ? x : id == 0 ? 2.0f * xa - one : id == 1 ? xa - one : id == 2 ? xa - 1.5f : -1.0f;
    const float den = id < 0 ? one : id == 0 ? 2.0f + xa : id == 1 ? xa + one : id == 2 ? one + 1.5f * xa : xa;
    x = num / den;
  }
  z = x * x;
  w = z * z;
  s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return hx < 0 ? -z : z;
}

IRT_HD float glibc_atan2f(float y, float x) {
  const float tiny = 1.0e-30f, zero = 0.0f;
  const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
              pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
  float z;
  const int32_t hx = (int32_t)f2u(x), ix = hx & 0x7fffffff;
  const int32_t hy = (int32_t)f2u(y), iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  // (fdlibm's x == 1.0 shortcut, atanf(y), is left out: the general path below gives the same
  // float for x = 1 -- atanf is odd bit for bit, y/1 == y, and for |y| > 2^60 both round to
  // 0x3fc90fdb -- and a second inlined atanf costs the kernel code size)
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    }
    switch (m) {
      case 0: return zero;
      case 1: return -zero;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int32_t k = (iy - ix) >> 23;
  if (k > 60)
    z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60)
    z = 0.0f;
  else
    z = glibc_atanf(__builtin_fabsf(y / x));
  switch (m) {
    case 0: return z;
    case 1: return u2f(f2u(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// ---------------------------------------------------------------------------------
// glibc 2.35 logf (sysdeps/ieee754/flt-32/e_logf.c, from ARM's optimized-routines; the
// table and polynomial of e_logf_data.c): x = 2^k z, log(x) = log1p(z/c-1) + log(c) + k ln2
// in double, one rounding to float at the end.  The Woodcock step evaluates
// logf(1.f - rnd()) (deviceCode.cu:165) only on x = 1 - j/2^24, j in [0, 2^24): all
// positive normal floats <= 1, so the subnormal/zero/inf/NaN branches are not restated.
// Verified against the host glibc on that whole domain (both of glibc's x86-64 builds,
// plain and FMA, agree there) by tests/test_host_logic.py and, for the device, by
// tests/test_gpu_parity.py.
struct LogfTab {
  double invc, logc;
};
constexpr LogfTab kLogfTab[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};
// `tab` is kLogfTab or a copy of it (the kernels keep one in LDS).
IRT_HD float glibc_logf_unit(float x, const LogfTab *tab) {
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  const uint32_t ix = f2u(x);
  if (ix == 0x3f800000u) return 0.f;
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> (23 - 4)) % 16u);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & (0x1ffu << 23));
  const double invc = tab[i].invc, logc = tab[i].logc;
  const double z = (double)u2f(iz);
  const double r = z * invc - 1;
  const double y0 = logc + (double)k * Ln2;
  const double r2 = r * r;
  double y = A1 * r + A2;
  y = A0 * r2 + y;
  y = y * r2 + (y0 + r);
  return (float)y;
}
// logf(1.f - rnd()) for the LCG state s that rnd() just produced
IRT_HD float woodcock_log(uint32_t s, const LogfTab *tab) {
  return glibc_logf_unit(1.f - lcg_float(s), tab);
}

// ---------------------------------------------------------------------------------
// Cube-map point locator: the MI355X replacement for the OptiX / cuBQL cell location
// (icon_rt/deviceCode.cu:58-125).  A direction is mapped to one of 6*G*G cells of a
// gnomonic cube map; each cell lists (conservatively, see host/irt_scene.cpp) every
// record that can contain a point in that direction, sorted by record index, so the first
// record passing sample() is the reference's "lowest index wins" answer.
IRT_HD uint32_t cubemap_cell(float px, float py, float pz, int G) {
  const float ax = __builtin_fabsf(px), ay = __builtin_fabsf(py), az = __builtin_fabsf(pz);
  int face;
  float u, v;
  if (ax >= ay && ax >= az) {
    face = px >= 0.f ? 0 : 1;
    u = py / ax;
    v = pz / ax;
  } else if (ay >= az) {
    face = py >= 0.f ? 2 : 3;
    u = px / ay;
    v = pz / ay;
  } else {
    face = pz >= 0.f ? 4 : 5;
    u = px / az;
    v = py / az;
  }
  const float fg = (float)G;
  int i = (int)((u + 1.f) * 0.5f * fg);
  int j = (int)((v + 1.f) * 0.5f * fg);
  // NaN / non-finite directions fall into cell 0 of face 0 after clamping; callers
  // reject them earlier (a sample point is always finite).
  i = i < 0 ? 0 : (i >= G ? G - 1 : i);
  j = j < 0 ? 0 : (j >= G ? G - 1 : j);
  return (uint32_t)face * (uint32_t)G * (uint32_t)G + (uint32_t)j * (uint32_t)G + (uint32_t)i;
}

#ifndef IRT_SUBCELLS
#define IRT_SUBCELLS 4  // (measurement builds may set 2: 64-B cell headers, coarser masks)
#endif
constexpr int kSubCells = IRT_SUBCELLS;  // sub-cells per cell edge (irt_build.h kSub)
constexpr int kMaskCand = 8;  // candidates per radial bin with a sub-cell mask (irt_build.h)

// cubemap_cell on the kSubCells-times finer grid: the same cell (the scaling by a power of
// two is exact) and the sub-cell s = sj * kSubCells + si within it.
IRT_HD uint32_t cubemap_cell_sub(float px, float py, float pz, int G, uint32_t &sub) {
  const float ax = __builtin_fabsf(px), ay = __builtin_fabsf(py), az = __builtin_fabsf(pz);
  int face;
  float u, v;
  if (ax >= ay && ax >= az) {
    face = px >= 0.f ? 0 : 1;
    u = py / ax;
    v = pz / ax;
  } else if (ay >= az) {
    face = py >= 0.f ? 2 : 3;
    u = px / ay;
    v = pz / ay;
  } else {
    face = pz >= 0.f ? 4 : 5;
    u = px / az;
    v = py / az;
  }
  const int GS = G * kSubCells;
  const float fg = (float)G;
  int i = (int)((u + 1.f) * 0.5f * fg * (float)kSubCells);
  int j = (int)((v + 1.f) * 0.5f * fg * (float)kSubCells);
  i = i < 0 ? 0 : (i >= GS ? GS - 1 : i);
  j = j < 0 ? 0 : (j >= GS ? GS - 1 : j);
  sub = (uint32_t)((j % kSubCells) * kSubCells + (i % kSubCells));
  return (uint32_t)face * (uint32_t)G * (uint32_t)G + (uint32_t)(j / kSubCells) * (uint32_t)G +
         (uint32_t)(i / kSubCells);
}

// Per-record height/value block: 64 floats = 256 B, two 128-B lines.
//   [0..31]  height[0..31]   (ICONCell::height)
//   [32..62] value[0..30]    (ICONCell::value; value[31] is never read by the render
//                             path -- findHeight() < numLayers <= 31 after the radial test)
//   [63]     numLayers (int bits)
constexpr int kHV = 64;

// ---------------------------------------------------------------------------------
// Radially binned candidate lists (the product locator).  Each cube-map cell splits the
// radius axis at up to kMaxEdges edges e0 < e1 < e2 (unused edges = +inf) into open bins
//   bin k = (e_{k-1}, e_k)   (e_{-1} = -inf, e_E = +inf)
// and lists, per bin and in record-index order, every record of the cell whose radial
// extent can contain such an r:  h0 < e_k && hN > e_{k-1}  (plus zero-thickness records
// h0 == hN == e_k, assigned to the bin below their edge).  A radius strictly inside bin k
// therefore scans only bin k; a radius exactly on edge e_k scans bins k and k+1 and keeps
// the lower first hit.  Either way the first record passing sample() is the reference's
// lowest-index answer (deviceCode.cu:119-122).
constexpr int kMaxEdges = 3;
// Cell header (irt_build.h): {e0, e1, e2, base} {end0, end1, end2, end3}, then the sub-cell
// candidate masks: 128 B per cell (64 B with 2 x 2 sub-cells)
constexpr int kBinHdrWords = 8 + kSubCells * kSubCells <= 16 ? 16 : 32;
// the header's per-quad radial bounds (irt_build.h cell_header): quads of 2 x 2 sub-cells
constexpr int kQuadEdge = kSubCells > 1 ? kSubCells / 2 : 1;  // quads per cell edge
constexpr int kQuads = kQuadEdge * kQuadEdge;
constexpr int kBoundWord = 8 + kSubCells * kSubCells;  // after the masks (24 with 4 x 4 sub-cells)
static_assert(kBoundWord + 2 * kQuads <= kBinHdrWords, "the quads' bounds fit the header line");
IRT_HD int quad_of(uint32_t s) {  // sub-cell s = sj * kSubCells + si -> its 2 x 2 quad
  return kSubCells > 1 ? (int)((s / kSubCells / 2) * kQuadEdge + (s % kSubCells) / 2) : 0;
}
IRT_HD int bin_of(float r, float e0, float e1, float e2) {
  return (e0 < r ? 1 : 0) + (e1 < r ? 1 : 0) + (e2 < r ? 1 : 0);
}

// Zero-thickness records are spheres (host/irt_scene.cpp); a 2^14-bit hash bitmap of
// their radii (2 KB of LDS) says "certainly not a sphere radius" for almost every sample.
constexpr int kSphBitWords = 512;
IRT_HD uint32_t sph_hash(float r) {
  uint32_t h = f2u(r) * 0x9E3779B1u;
  return h >> 18;
}

// Fat entry: everything one candidate test of sample() reads, kFat4 float4 = 64 B, packed
// two to a 128-B line (a cell's bin lists are contiguous, so a list's next candidate usually
// shares its first's line):
//   [0..2]  the record's three side planes (n.xyz, w)              ICONGrid.h:197-203
//   [3]     {height[0], height[numLayers], record index, meta}     ICONGrid.h:184
//           meta: see record_meta (irt_build.h) and record_path below
constexpr int kFat4 = 4;
constexpr int kFatStride4 = 4;

// Slot table (round 5): for scenes whose cube-map cells' radial edges, all together, are at most
// kMaxEdges distinct values U0 < U1 < U2 (every column with the same levels, as in C3/C4/C5;
// cells with fewer entries may have fewer of them), the bin of a sample in the table's terms
// follows from r alone, and per (cell, slot unit, table bin) one 128-B line holds what the
// cell's header and the list's first candidate give a sample there, so that a located
// sample's scan usually starts with one gather instead of two dependent ones (header, then entry).
// A slot unit is `subs` sub-cells of the cell: 1 (round 5: 129 GB at C5), 2 (the pairs s, s + 1 of a
// sub-cell row) or 4 (the 2 x 2 quads of quad_of; the default since round 6: 32 GB at C5):
//   [0..3]  in the cell's own bin k that holds the table bin (U_{b-1}, U_b], the candidate that
//           is the first admitted one of the most of the unit's sub-cells, the lowest list
//           position on a tie (its fat entry; zero when no sub-cell admits one).  Quads: 79 % of
//           (sub-cell, bin) pairs find their own first candidate there, 72 % with the unit's
//           lowest admitted one (R2B05)
//   [4]     {the bin's unmasked candidates (list length less kMaskCand, at least 0) | that first
//           candidate's list position j_U << 24, bin k's list start (base + bin begin), the unit's
//           sub-cells' 8-bit masks (masked to the list's length; sub-cell i of the unit in bits
//           8i..8i+7, slot_sub), U_b if it is also the cell's edge e_k (a sample exactly there
//           scans bin k + 1 too), else +inf}
//   [5..7]  0
// A sample in sub-cell i of the unit admits c = popc(m8_i) + unmasked candidates, the first at
// list position j = ctz(m8_i) (kMaskCand when m8_i = 0): when j == j_U the slot's copy is that
// candidate, otherwise the scan gathers it from the list (one line, as from the header).
// Slot (cell, u, b) sits at ((cell * kSubCells^2 / subs + u) * bins + b) * kSlot4.  The rest of the
// scan (the dealt-out candidates, the second pass on a bin edge) reads the header and the
// lists as before.
constexpr int kSlot4 = 8;
constexpr uint32_t kSlotNoFirst = 15u;  // j_U when no sub-cell of the unit admits a candidate
// sub-cell s = sj * kSubCells + si -> its slot unit and its index within the unit
IRT_HD uint32_t slot_unit(uint32_t s, int subs) {
  return subs == 4 ? (uint32_t)quad_of(s) : (subs == 2 ? s >> 1 : s);
}
IRT_HD uint32_t slot_sub(uint32_t s, int subs) {
  return subs == 4 ? (((s / kSubCells) & 1u) << 1) | (s & 1u) : (subs == 2 ? s & 1u : 0u);
}
// sub-cell i of unit u
IRT_HD uint32_t slot_member(uint32_t u, uint32_t i, int subs) {
  if (subs == 4) {
    const uint32_t qe = (uint32_t)kSubCells / 2;
    return (2u * (u / qe) + (i >> 1)) * (uint32_t)kSubCells + 2u * (u % qe) + (i & 1u);
  }
  return subs == 2 ? 2u * u + i : u;
}
// Fills slot (u, b) of a cell from its header H (kBinHdrWords) and the fat entries; U: the
// table's ne edges (ascending); subs: sub-cells per unit.
IRT_HD void slot_fill(const uint32_t *H, const float *fat, int u, int b, const float *U, int ne, int subs, float *S) {
  for (int k = 0; k < 4 * kSlot4; ++k) S[k] = 0.f;
  // the cell's bin holding (U_{b-1}, U_b]: its edges <= U_{b-1} (each is one of the U)
  int k = 0;
  if (b > 0)
    for (int j = 0; j < kMaxEdges; ++j) k += u2f(H[j]) <= U[b - 1] ? 1 : 0;
  const float up = b < ne ? U[b] : __builtin_inff();
  const bool own = b < ne && k < kMaxEdges && u2f(H[k]) == up;
  const uint32_t beg = k ? H[4 + k - 1] : 0u, end = H[4 + k], n = end - beg;
  const uint32_t nx = n > (uint32_t)kMaskCand ? n - (uint32_t)kMaskCand : 0u;
  // the unit's masks, and the list position that is the first admitted candidate of the most of
  // its sub-cells (the lowest such position on a tie): the slot's copy
  uint32_t masks = 0u, firstOf = 0u;  // firstOf: 4 bits per sub-cell, kSlotNoFirst when none
  for (int i = 0; i < subs; ++i) {
    const uint32_t s = slot_member((uint32_t)u, (uint32_t)i, subs);
    const uint32_t m8 = (H[8 + s] >> (8 * k)) & 0xFFu & (n < 8u ? (1u << n) - 1u : 0xFFu);
    masks |= m8 << (8 * i);
    const uint32_t j = m8 ? (uint32_t)__builtin_ctz(m8) : (nx ? (uint32_t)kMaskCand : kSlotNoFirst);
    firstOf |= j << (4 * i);
  }
  uint32_t jU = kSlotNoFirst;
  int most = 0;
  for (uint32_t j = 0; j <= (uint32_t)kMaskCand; ++j) {
    int cnt = 0;
    for (int i = 0; i < subs; ++i) cnt += ((firstOf >> (4 * i)) & 15u) == j ? 1 : 0;
    if (cnt > most) {
      most = cnt;
      jU = j;
    }
  }
  if (jU != kSlotNoFirst) {
    const uint32_t first = H[3] + beg + jU;
    for (int q = 0; q < 4 * kFat4; ++q) S[q] = fat[(size_t)first * 4 * kFatStride4 + q];
  }
  S[16] = u2f((nx < 0xFFFFFFu ? nx : 0xFFFFFFu) | (jU << 24));  // 0xFFFFFF: too long (k_slot_fill drops the table)
  S[17] = u2f(H[3] + beg);
  S[18] = u2f(masks);
  S[19] = own ? up : __builtin_inff();
}
// Per-record height/value blocks (the render record without its planes/keys), kBlk4
// float4 = 256 B: block b (4 float4) = {height[8b..8b+3]}, {height[8b+4..8b+7]},
// {value[8b-1..8b+2]}, {value[8b+3..8b+6]}.  Block 0's value[-1] slot holds value[31]: the
// block path (rec_block_index) never selects that slot, and findHeight returns 31 only for
// heights the radial test rules out in the raygen -- but the grid build (k_grid_build) and
// the wedge scalars take getValue at a record's own heights, where unsorted heights can reach
// index numLayers = 31 (getValue then reads value[31], as the reference does).
constexpr int kBlk4 = 16;
IRT_HD int blk_height_pos(int j) { return 16 * (j >> 3) + (j & 7); }
IRT_HD int blk_value_pos(int c) { return 16 * (((c + 1) >> 3) & 3) + 8 + ((c + 1) & 7); }

// Total order on floats (sort keys, quantised heights): -0 before +0.
IRT_HD uint32_t float_key(float v) {
  const uint32_t b = f2u(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// The meta word of a record (its fat entry's last word; irt_build.h record_meta):
//   bits 0-4   numLayers
//   bit 5      coarse: height[1..numLayers] non-decreasing and height[0] <= height[numLayers],
//              so findHeight's 8-height block follows from the keys height[7], height[15],
//              height[23] (irt_common.h rec_coarse_block; height[31] never counts).
//              height[0] may exceed height[1] (convert_icon's inverted first layer over land):
//              findHeight never reads it
//   bits 6-29  q_j, j = 0,1,2: float_key(height[8j+7]) - float_key(height[0]), in units of
//              meta_quantum, floored (8 bits each): key j lies in [q_j S, q_j S + S - 1]
//              above height[0]'s key
//   bits 30-31 the number of keys below height[0] (a prefix of the sorted keys; their q_j are
//              0): with r >= height[0] they always count
constexpr uint32_t kMetaCoarse = 32u;
constexpr int kMetaBelowShift = 30;
IRT_HD uint32_t meta_quantum(uint32_t k0, uint32_t kN) { return ((kN - k0) >> 8) + 1u; }
// rec_coarse_block from the quantised keys, for r in [h0, hN] (the radial test passed):
// exact wherever r's key is more than one unit outside every key's interval (one unit: the
// -0/+0 pair, equal as floats, sits one key apart); -1 when r is that close to a key
// (about 1 % of samples): the exact keys decide (record_value).
IRT_HD int rec_coarse_block_q(uint32_t meta, float h0, float hN, float r) {
  const int nl = (int)(meta & 31u);
  const uint32_t k0 = float_key(h0), S = meta_quantum(k0, float_key(hN));
  const uint32_t d = float_key(r) - k0;
  const int below = (int)(meta >> kMetaBelowShift);
  int b = 0;
  bool amb = false;
  for (int j = 0; j < 3; ++j) {
    if (8 * j + 7 > nl) break;
    const uint32_t lo = ((meta >> (6 + 8 * j)) & 255u) * S, hi = lo + (S - 1u);
    if (j < below)
      ++b;  // key < height[0] <= r
    else if (d > hi + 1u)
      ++b;  // r > key: !(r <= key) counts
    else if (d + 1u >= lo)
      amb = true;
  }
  return amb ? -1 : b;
}
// The getValue path of a record found at radius r (the kernel's Found::path): bits 0-4
// numLayers; bit 7: one 64-B block (coarse records), bits 5-6 its index b; bit 8: b must be
// settled on the exact keys first; neither: the literal findHeight over the blocks.
constexpr uint32_t kPathBlock = 128u, kPathExactKeys = 256u;
IRT_HD uint32_t record_path(uint32_t meta, float h0, float hN, float r) {
  const uint32_t nl = meta & 31u;
  if (!(meta & kMetaCoarse)) return nl;
  const int b = rec_coarse_block_q(meta, h0, hN, r);
  return nl | kPathBlock | (b < 0 ? kPathExactKeys : ((uint32_t)b << 5));
}

// findHeight for non-decreasing height[1..nl], from the record layout in two gathers.
// lower_bound's answer is #{ j in [1,nl] : !(hpos <= height[j]) } (a monotone predicate on
// sorted data, NaN hpos included).  Step 1: the block b = number of coarse keys
// height[8k+7] (8k+7 <= nl) satisfying the predicate; the answer lies in
// [8b-1, 8b+6] (b = 0: [0, 6]).
IRT_HD int rec_coarse_block(float k0, float k1, float k2, float k3, int nl, float hpos) {
  int b = 0;
  b += (7 <= nl && !(hpos <= k0)) ? 1 : 0;
  b += (15 <= nl && !(hpos <= k1)) ? 1 : 0;
  b += (23 <= nl && !(hpos <= k2)) ? 1 : 0;
  b += (31 <= nl && !(hpos <= k3)) ? 1 : 0;
  return b > 3 ? 3 : b;  // b == 4 needs NaN hpos (the radial test bounds hpos by height[nl])
}
// Step 2: h[m] = height[8b+m] (m = 0..6) -> index m of the answer in the block's value
// quad pair {value[8b-1..8b+6]}.  (Scalars, not an array: keeps the kernel's registers
// out of scratch.)
IRT_HD int rec_block_index(float h0, float h1, float h2, float h3, float h4, float h5,
                           float h6, int b, int nl, float hpos) {
  const int j0 = 8 * b;
  int c = b > 0 ? j0 - 1 : 0;
  c += (j0 >= 1 && j0 <= nl && !(hpos <= h0)) ? 1 : 0;
  c += (j0 + 1 <= nl && !(hpos <= h1)) ? 1 : 0;
  c += (j0 + 2 <= nl && !(hpos <= h2)) ? 1 : 0;
  c += (j0 + 3 <= nl && !(hpos <= h3)) ? 1 : 0;
  c += (j0 + 4 <= nl && !(hpos <= h4)) ? 1 : 0;
  c += (j0 + 5 <= nl && !(hpos <= h5)) ? 1 : 0;
  c += (j0 + 6 <= nl && !(hpos <= h6)) ? 1 : 0;
  return c - j0 + 1;  // in [0, 7]
}
// v[m] of the eight values {a0..a3, b0..b3} as a select tree
IRT_HD float select8(int m, float a0, float a1, float a2, float a3, float b0, float b1, float b2,
                     float b3) {
  const bool o = (m & 1) != 0, t = (m & 2) != 0;
  const float x0 = o ? a1 : a0, x1 = o ? a3 : a2, x2 = o ? b1 : b0, x3 = o ? b3 : b2;
  const float y0 = t ? x1 : x0, y1 = t ? x3 : x2;
  return (m & 4) ? y1 : y0;
}

// ---------------------------------------------------------------------------------
// GRID_ACCEL_MODE (Params.h:34): the 256^3 Cartesian macrocell grid over the volume
// bounds (hostCode.cu:668-682) and its traversal dda3 (DDA.h:35-136).
constexpr int kGridDim = 256;  // Grid{nullptr, vec3i(256), volbounds} (hostCode.cu:670)
constexpr int kGridBlock = 8;  // GRID_ACCEL_MODE empty-space blocks: 32^3 of 8^3 cells, 4 KB of bits
constexpr int kGridBitWords = (kGridDim / kGridBlock) * (kGridDim / kGridBlock) * (kGridDim / kGridBlock) / 32;

// projectOnGrid (DDA.h:23-31), one axis: clamp(int((V-lo)/(hi-lo)*dims), 0, dims-1)
IRT_HD int project_on_grid(float v, float lo, float hi, int dim) {
  const int c = f2i_x86(((v - lo) / (hi - lo)) * (float)dim);
  return c < 0 ? 0 : (c > dim - 1 ? dim - 1 : c);  // vecmath clamp(int) = max(a, min(x, b))
}

// `min(reduce_min(tnext), ray.tmax)` (DDA.h:96): vecmath.h has no float min, so the
// reference's g++ (CPU) build resolves it to `int min(int, int)` (vecmath.h:46-49) --
// both operands truncated (cvttss2si), the int converted back to float.
IRT_HD float dda3_min_quirk(float a, float b) {
  const int x = f2i_x86(a), y = f2i_x86(b);
  return (float)(x < y ? x : y);
}

// ICONCell::findHeight (ICONGrid.h:117-145): lower_bound over height[1..numLayers].
IRT_HD int find_height(const float *height, int numLayers, float hpos) {
  int first = 0, count = numLayers;
  while (count > 0) {
    const int step = count / 2;
    const int it = first + step;
    if (!(hpos <= height[it + 1])) {
      first = it + 1;
      count -= step + 1;
    } else {
      count = step;
    }
  }
  return first;
}

}  // namespace irt

// ---------------------------------------------------------------------------------
// CUBQL_MODE wedges: intersectWedgeEXT (UElems.h:176-311, adapted from OpenVKL) on the
// wedges buildCuBQLAccel makes (hostCode.cu:557-600), shared by the kernel and the host
// checks.  A wedge is 6 vertices (x, y, z, scalar): bottom triangle, then top.
namespace irt {
struct WV4 {
  float x, y, z, w;
};

// determinant(mat3f) (vecmath.h:733-748) of the matrix with columns c0, c1, c2
// (make_LinearSpace3f, UElems.h:20-28)
IRT_HD float wedge_det3(const float *c0, const float *c1, const float *c2) {
  const float a00 = c1[1] * c2[2] - c1[2] * c2[1];
  const float a01 = c0[1] * c2[2] - c0[2] * c2[1];
  const float a02 = c0[1] * c1[2] - c0[2] * c1[1];
  return c0[0] * a00 - c1[0] * a01 + c2[0] * a02;
}

IRT_HD float wmin(float a, float b) { return b < a ? b : a; }  // fminf on finite input
IRT_HD float wmax(float a, float b) { return b > a ? b : a; }
IRT_HD float wabs(float a) { return u2f(f2u(a) & 0x7fffffffu); }

// WEDGE_CONVERGED (1e-4, a double) compared against a float |d|: |d| < 1e-4 <=> |d| <= c
// for c = (float)1e-4, which rounds below 1e-4 (the next float is above it).
constexpr float kWedgeConverged = (float)1e-4;
static_assert((double)kWedgeConverged < 1e-4, "float(1e-4) rounds down");
// lowerlimit / upperlimit: `0.f - 1e-6` and `1.f + 1e-6` folded in double, then to float
constexpr float kWedgeLo = (float)(0.0 - 1e-6), kWedgeHi = (float)(1.0 + 1e-6);

IRT_HD bool intersect_wedge(float &value, float px, float py, float pz, const WV4 *V) {
  // bbox (233-236) and the determinant tolerance: norm2(vec3f) binds to norm2(vec2f)
  // (vecmath.h:317, 386-389), x and y only
  float lx = 1e31f, ly = 1e31f, hx = -1e31f, hy = -1e31f;
  for (int i = 0; i < 6; ++i) {
    lx = wmin(lx, V[i].x);
    ly = wmin(ly, V[i].y);
    hx = wmax(hx, V[i].x);
    hy = wmax(hy, V[i].y);
  }
  const float sx = hx - lx, sy = hy - ly;
  const float tol = (sx * sx + sy * sy) * 1e-6f;
  float p0 = .5f, p1 = .5f, p2 = .5f;
  float w[6];
  bool converged = false;
  for (int it = 0; !converged && it < 10; ++it) {
    const float q = 1.f - p0 - p1, m2 = 1.f - p2;
    w[0] = q * m2;  // wedgeInterpolationFunctions (176-184)
    w[1] = p0 * m2;
    w[2] = p1 * m2;
    w[3] = q * p2;
    w[4] = p0 * p2;
    w[5] = p1 * p2;
    // wedgeInterpolationDerivs (187-212): r, s, t rows
    const float dr[6] = {-1.f + p2, 1.f - p2, 0.f, -p2, p2, 0.f};
    const float ds[6] = {-1.f + p2, 0.f, 1.f - p2, -p2, 0.f, p2};
    const float dt[6] = {-1.f + p0 + p1, -p0, -p1, 1.f - p0 - p1, p0, p1};
    float f[3] = {0.f, 0.f, 0.f}, r[3] = {0.f, 0.f, 0.f}, s[3] = {0.f, 0.f, 0.f},
          t[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < 6; ++i) {  // the Newton columns (253-260), in order
      f[0] = f[0] + V[i].x * w[i];
      f[1] = f[1] + V[i].y * w[i];
      f[2] = f[2] + V[i].z * w[i];
      r[0] = r[0] + V[i].x * dr[i];
      r[1] = r[1] + V[i].y * dr[i];
      r[2] = r[2] + V[i].z * dr[i];
      s[0] = s[0] + V[i].x * ds[i];
      s[1] = s[1] + V[i].y * ds[i];
      s[2] = s[2] + V[i].z * ds[i];
      t[0] = t[0] + V[i].x * dt[i];
      t[1] = t[1] + V[i].y * dt[i];
      t[2] = t[2] + V[i].z * dt[i];
    }
    f[0] = f[0] - px;
    f[1] = f[1] - py;
    f[2] = f[2] - pz;
    const float d = wedge_det3(r, s, t);
    if (wabs(d) < tol) return false;
    const float d0 = wedge_det3(f, s, t) / d;
    const float d1 = wedge_det3(r, f, t) / d;
    const float d2 = wedge_det3(r, s, f) / d;
    p0 = p0 - d0;
    p1 = p1 - d1;
    p2 = p2 - d2;
    if (wabs(d0) <= kWedgeConverged && wabs(d1) <= kWedgeConverged && wabs(d2) <= kWedgeConverged)
      converged = true;
    else if (wabs(p0) > 1e6f || wabs(p1) > 1e6f || wabs(p2) > 1e6f)
      return false;
  }
  if (!converged) return false;
  if (p0 >= kWedgeLo && p0 <= kWedgeHi && p1 >= kWedgeLo && p1 <= kWedgeHi && p2 >= kWedgeLo &&
      p2 <= kWedgeHi && p0 + p1 <= kWedgeHi) {
    float val = 0.f;  // 301-305, with the weights of the last iteration
    for (int i = 0; i < 6; ++i) val += w[i] * V[i].w;
    value = val;
    return true;
  }
  return false;
}
}  // namespace irt

// ---------------------------------------------------------------------------------
// TRIANGLE_MODE (deviceCode.cu:61-76): from the sample point, a ray toward the Earth's
// centre (direction -normalize(pos)) against the bottom triangles of buildTriangleAccel
// (hostCode.cu:445-450), back faces culled, the closest hit wins.  OptiX's watertight
// triangle test is not reproducible here; this is the definition both the oracle and the
// kernel use (parity unpinned): Moller-Trumbore without division except for t, front face
// iff det > 0 (counter-clockwise seen from the ray origin), edges inclusive, t > 0.
namespace irt {
IRT_HD bool ray_triangle(float ox, float oy, float oz, float dx, float dy, float dz,
                         const float *v0, const float *v1, const float *v2, float &t) {
  const float e1x = v1[0] - v0[0], e1y = v1[1] - v0[1], e1z = v1[2] - v0[2];
  const float e2x = v2[0] - v0[0], e2y = v2[1] - v0[1], e2z = v2[2] - v0[2];
  const float px = dy * e2z - dz * e2y, py = dz * e2x - dx * e2z, pz = dx * e2y - dy * e2x;
  const float det = e1x * px + e1y * py + e1z * pz;
  if (!(det > 0.f)) return false;  // back face or parallel: culled
  const float tx = ox - v0[0], ty = oy - v0[1], tz = oz - v0[2];
  const float u = tx * px + ty * py + tz * pz;
  if (u < 0.f || u > det) return false;
  const float qx = ty * e1z - tz * e1y, qy = tz * e1x - tx * e1z, qz = tx * e1y - ty * e1x;
  const float v = dx * qx + dy * qy + dz * qz;
  if (v < 0.f || u + v > det) return false;
  t = (e2x * qx + e2y * qy + e2z * qz) / det;
  return t > 0.f;
}
}  // namespace irt
