// irt_device.h -- device-side building blocks of the raygen, each a bit-exact restatement
// of the reference function it cites (compile with -ffp-contract=off, correctly rounded
// f32 div/sqrt).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "irt_common.h"
#include "irt_kernels.h"

#define IRT_FLT_MAX 3.402823466e+38f

namespace irt {

struct Ray {
  float ox, oy, oz, tmin, dx, dy, dz, tmax;
};

struct Counts {
  uint32_t inBox, locate, found, cand;
  uint32_t steps, deg, rounds;  // OPT_STATS only: Woodcock draws, zero-length leaves, cooperative rounds
  // OPT_STATS only, cooperative loop: per round the wave's longest candidate scan (entry
  // hops), rounds with a locate, and per lane the samples by candidates tested (0,1,2,>=3)
  uint32_t hops, locRounds, candHist[4];
};

// A uniform value the compiler must treat as new at this point: the derived values (int ->
// float conversions, integer-division reciprocals, LDS addresses) are then recomputed where
// they are used instead of being hoisted out of the raygen's loops and held in VGPRs for the
// whole kernel -- register pressure is what limits the waves per SIMD.
__device__ __forceinline__ int opaque_u(int v) {
  v = __builtin_amdgcn_readfirstlane(v);  // uniform: any lane's copy; keeps it scalar
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ float opaque_u(float v) { return __builtin_bit_cast(float, opaque_u(__builtin_bit_cast(int, v))); }
__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
  return ax * bx + ay * by + az * bz;  // vecmath.h:536-538 order
}

// Correctly rounded a / b for per-lane divisors through a double reciprocal, cheaper than the
// f32 division sequence (v_div_scale x2, v_rcp, five fmas, v_div_fmas, v_div_fixup) when
// one divisor serves several quotients.  r = the hardware estimate of 1/b (v_rcp_f32, within
// 1 ulp: |e| <= 2^-22 for e = 1 - b r) refined once cubically, r (1 + e + e^2), by double
// fmas: relative error e^3 plus three roundings, below 2^-52.  Then (double)a * r is within
// 2^-51 (relative) of a/b, while a quotient of two floats that is not itself representable
// lies at least 2^-49 from every rounding boundary of the float grid (a - b m, for a boundary
// m, is a nonzero multiple of 2^min(ea, eb+em): the same argument as div_uniform), so the
// double product rounds to the float a / b rounds to -- overflow to inf and float subnormal
// results included.  Valid for 2^-100 <= |b| <= 2^100 (no zero, inf, NaN or subnormal
// divisor, no double overflow); recip_ok(b) tests that and callers divide otherwise.
// tests/test_host_logic.py checks the identity with estimates perturbed by up to 2 ulps.
__device__ __forceinline__ bool recip_ok(float b) {
  const float ab = __builtin_fabsf(b);
  return ab >= 0x1p-100f && ab <= 0x1p100f;
}
__device__ __forceinline__ double recip_d(float b) {
  const double r0 = (double)__builtin_amdgcn_rcpf(b);
  const double e = __builtin_fma(-(double)b, r0, 1.0);
  return __builtin_fma(r0, __builtin_fma(e, e, e), r0);
}
__device__ __forceinline__ float div_recip(float a, double r) { return (float)((double)a * r); }

// boxTest (vecmath.h:1926-1937); the six quotients through one reciprocal per axis
__device__ __forceinline__ bool box_test(const Ray &r, const RenderArgs &A, float &t0, float &t1) {
  float lx, ly, lz, hx, hy, hz;
  if (recip_ok(r.dx) && recip_ok(r.dy) && recip_ok(r.dz)) {
    const double rx = recip_d(r.dx), ry = recip_d(r.dy), rz = recip_d(r.dz);
    lx = div_recip(A.bmin.x - r.ox, rx);
    ly = div_recip(A.bmin.y - r.oy, ry);
    lz = div_recip(A.bmin.z - r.oz, rz);
    hx = div_recip(A.bmax.x - r.ox, rx);
    hy = div_recip(A.bmax.y - r.oy, ry);
    hz = div_recip(A.bmax.z - r.oz, rz);
  } else {
    lx = (A.bmin.x - r.ox) / r.dx, ly = (A.bmin.y - r.oy) / r.dy, lz = (A.bmin.z - r.oz) / r.dz;
    hx = (A.bmax.x - r.ox) / r.dx, hy = (A.bmax.y - r.oy) / r.dy, hz = (A.bmax.z - r.oz) / r.dz;
  }
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
// The raygen's two intersectSphere calls on one ray (the shell's outer and inner sphere,
// ShellAccel.h:94-95): the same expressions, A = dot(dir, dir) shared, each quotient through
// recip_d when its divisor allows.
__device__ __forceinline__ void intersect_spheres(const Ray &r, float radiusA, float radiusB, bool &hitA,
                                                  float &nearA, float &farA, bool &hitB, float &nearB,
                                                  float &farB) {
  const float A = dot3(r.dx, r.dy, r.dz, r.dx, r.dy, r.dz);
  const float B = dot3(r.dx, r.dy, r.dz, r.ox, r.oy, r.oz) * 2.f;
  const float OO = dot3(r.ox, r.oy, r.oz, r.ox, r.oy, r.oz);
  const bool okA = recip_ok(A);
  const double rA = okA ? recip_d(A) : 0.0;
  auto one = [&](float radius, float &tnear, float &tfar) {
    const float C = OO - radius * radius;
    float d = B * B - 4.f * A * C;
    if (d < 0.f) return false;
    d = sqrtf(d);
    const float q = B < 0.f ? -0.5f * (B - d) : -0.5f * (B + d);
    float t1, t2;
    if (okA && recip_ok(q)) {
      t1 = div_recip(q, rA);
      t2 = div_recip(C, recip_d(q));
    } else {
      t1 = q / A;
      t2 = C / q;
    }
    tnear = fminf(t1, t2);
    tfar = fmaxf(t1, t2);
    return true;
  };
  hitA = one(radiusA, nearA, farA);
  hitB = one(radiusB, nearB, farB);
}

// projectToSphericalGrid (ShellAccel.h:57-68), one axis: int((s-lo)/size*(dims-1))
__device__ __forceinline__ int project_axis(float s, float lo, float hi, int dim) {
  return f2i_x86((s - lo) / (hi - lo) * (float)(dim - 1));
}

// a / b, correctly rounded, for a divisor b fixed per launch, given invB = 1 / (double)b:
// one double product rounded to float.  The product is within 2^-52 (relative) of a/b,
// while a quotient of two floats that is not itself a float midpoint lies at least ~2^-49
// (relative) from every midpoint between floats -- and is never exactly one -- so both round
// to the same float.  b = 0, inf, NaN give 0/0 = NaN, a/0 = +-inf, a/inf = +-0 either way.
// Replaces the ~10-instruction correctly rounded f32 division sequence.
__device__ __forceinline__ float div_uniform(float a, double invB) {
  return (float)((double)a * invB);
}
// project_axis with the per-launch 1 / (double)(hi - lo)
__device__ __forceinline__ int project_axis_inv(float s, float lo, double invSize, int dim) {
  return f2i_x86(div_uniform(s - lo, invSize) * (float)(opaque_u(dim) - 1));
}

// normalizeGridCoord (ShellAccel.h:71-80): the while-loops compute c mod d in [0,d).  A
// coordinate already inside the grid (almost every leaf) skips the integer division, ~25
// VALU instructions per axis on gfx950 (no hardware integer divide).
__device__ __forceinline__ int wrap_coord(int c, int d) {
  if ((unsigned)c < (unsigned)d) return c;
  if (c >= -d && c < 2 * d) return c < 0 ? c + d : c - d;  // one step outside: no division
  d = opaque_u(d);
  const int m = c % d;
  return m < 0 ? m + d : m;
}

// toSpherical (ICONGrid.h:36-42) with glibc-exact asinf / atan2f.
__device__ __forceinline__ void to_spherical(float x, float y, float z, float &r, float &lat,
                                             float &lon) {
  r = sqrtf(dot3(x, y, z, x, y, z));
  lat = glibc_asinf(z / r);
  lon = glibc_atan2f(y, x);
}

// ---------------------------------------------------------------------------------
// Certified fast toSpherical for the sdda entry/exit cells.  sdda (ShellAccel.h:113-138)
// uses the lat/lon of a range's entry and exit point only through
//   * the shell-grid cell int((v - lo)/size * (dims-1)) (projectToSphericalGrid, 57-68), and
//   * the signs of la2 - la1, lo2 - lo1 (the step direction, 125-127).
// Both are monotone in v.  So a value known to lie within E of the glibc value certifies the
// cell when both ends v -+ E project to the same cell, and a sign when |la2 - la1| > 2E (+
// the rounding of the difference); only when that fails (about 1e-3 of the values) are the
// glibc-exact asinf / atan2f evaluated.  The fast functions cost ~35 VALU instructions
// against ~110 for the exact pair (and their branches).
//
// The bounds E are proven exhaustively on the device (tests/test_gpu_parity.py
// test_fast_spherical_bounds, irt_debug_fast_math_bounds):
//   * asin: x = z / r is computed exactly (as the reference computes it) in both paths, and
//     |fast_asin(x) - glibc_asinf(x)| is measured over EVERY float x in [-1, 1];
//   * atan2: |fast_atan(q) - atan(q)| and |glibc_atanf(q) - atan(q)| over every float q in
//     [0, 2^58] (atan in double), the hardware reciprocal's relative error over every float;
//     then |fast - glibc atan2f| <= E_fast + E_glibc + |q_fast - y/x| / 2 + |q_glibc - y/x| / 2
//     (atan's slope q/(1+q^2) <= 1/2 in relative terms) + the four roundings of the
//     quadrant step pi - (z - pi_lo) (two per evaluation, <= ulp(pi)/2 each).
// kLatErr / kLonErr include 1.2e-7 for rounding v -+ E itself (ulp(pi)/2).
constexpr float kLatErr = 1.0e-6f;
constexpr float kLonErr = 2.0e-6f;

// asin for |x| <= 1 (glibc's polynomial in t, Horner with fmas; no split-pio2 refinement;
// the hardware square root)
__device__ __forceinline__ float fast_asin(float x) {
  const float a = __builtin_fabsf(x);
  const bool big = a >= 0.5f;
  const float t = big ? (1.f - a) * 0.5f : a * a;
  const float s = big ? __builtin_amdgcn_sqrtf(t) : a;
  const float p = t * __builtin_fmaf(
                          t, __builtin_fmaf(t, __builtin_fmaf(t, __builtin_fmaf(t, 4.216630880e-2f, 2.417951451e-2f),
                                                                4.547037598e-2f),
                                            7.495297643e-2f),
                          1.666675248e-1f);
  const float r = __builtin_fmaf(s, p, s);
  const float v = big ? __builtin_fmaf(-2.f, r, 1.57079637050628662109375f) : r;
  return __builtin_copysignf(v, x);
}
// atan for q >= 0 (Cephes' reduction at tan(pi/8), tan(3pi/8) with the hardware reciprocal,
// its degree-9 odd polynomial)
__device__ __forceinline__ float fast_atan(float q) {
  const bool big = q > 2.414213562373095f, mid = q > 0.4142135623730950f;
  const float num = big ? -1.f : (mid ? q - 1.f : q);
  const float den = big ? q : (mid ? q + 1.f : 1.f);
  const float x = num * __builtin_amdgcn_rcpf(den);
  const float base = big ? 1.57079637050628662109375f : (mid ? 0.785398185253143310546875f : 0.f);
  const float z = x * x;
  const float p = __builtin_fmaf(
      __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z, 1.99777106478e-1f),
                     z, -3.33329491539e-1f),
      z * x, x);
  return base + p;
}
// atan2(y, x) for finite, nonzero x, y with |y/x| in [2^-58, 2^58] (false otherwise: glibc's
// special cases, take the exact path); glibc's quadrant step (glibc_atan2f)
__device__ __forceinline__ bool fast_atan2(float y, float x, float &lon) {
  const float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
  const float q = ay * __builtin_amdgcn_rcpf(ax);
  const bool ok = ax >= 0x1p-100f && ax <= 0x1p100f && ay >= 0x1p-100f && ay <= 0x1p100f && q >= 0x1p-58f &&
                  q <= 0x1p58f;
  const float z = fast_atan(q);
  const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
  lon = y < 0.f ? (x < 0.f ? (z - pi_lo) - pi : -z) : (x < 0.f ? pi - (z - pi_lo) : z);
  return ok;
}
// the shell-grid cell of v (project_axis_inv), certified for every value within err of v
__device__ __forceinline__ bool cell_certified(float v, float err, float lo, double invSize, int dim, int &cell) {
  const int c0 = project_axis_inv(v - err, lo, invSize, dim), c1 = project_axis_inv(v + err, lo, invSize, dim);
  cell = c0;
  return c0 == c1 && v == v;
}
// the sign of b - a (a < b) for values within err of a and b, certified
__device__ __forceinline__ int sign_certified(float a, float b, float err) {
  const float d = b - a, m = 2.f * err + 2.4e-7f;
  return d > m ? 1 : (-d > m ? -1 : 0);  // 0: uncertain
}

// make_8bit (dvr_course-common-both.h:89-92)
__device__ __forceinline__ uint32_t make_8bit(float f) {
  return (uint32_t)fminf(255.f, fmaxf(0.f, (float)f2i_x86(f * 256.f)));
}

// make_8bit(linear_to_srgb(x)) via the host-built monotone thresholds th[1..255] (LDS):
// the number of thresholds <= x.  The hardware log2/exp2 estimate of the expression
// (dvr_course-common-both.h:29-34, 89-92) is within one byte of it; the thresholds then
// settle the exact count (two independent LDS reads instead of an 8-step binary search).
__device__ __forceinline__ uint32_t srgb_byte(const float *th, float x) {
  const float s = x <= 0.0031308f
                      ? 12.92f * x
                      : 1.055f * __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(x) * (1.f / 2.4f)) - 0.055f;
  int b = (int)fminf(255.f, fmaxf(0.f, s * 256.f));  // NaN -> 0
  const float up = th[b < 255 ? b + 1 : 255], at = th[b];
  if (b < 255 && up <= x) {
    ++b;
    while (b < 255 && th[b + 1] <= x) ++b;
  } else if (b > 0 && !(at <= x)) {
    --b;
    while (b > 0 && !(th[b] <= x)) --b;
  }
  return (uint32_t)b;
}

}  // namespace irt
