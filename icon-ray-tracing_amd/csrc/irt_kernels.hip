// irt_kernels.hip -- gfx950 kernels around the hot path: the spherical-shell accelerator
// build (initGrid / buildShell_ICON / computeMaxOpacities of icon_rt/hostCode.cu), the
// framebuffer clear, and the multi-GPU tile unpack.  The raygen itself is irt_render.hip.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "irt_device.h"

namespace irt {
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
// min/max.
//
// One lane per record, the records staged through LDS (round 2 ran a workgroup per record,
// whose redundant scalar binary searches took 493 ms at C5).  getValue(h[i]) = value[findHeight(h[i])]: for heights
// non-decreasing in float_key order (record_meta's coarse records) findHeight(h[i]) is
// #{j >= 1 : h[j] < h[i]}, which a running index gives (0 for i = 0; i-1, or the previous
// answer on a repeated height); other records run the literal binary search.  Rectangles
// wider than kShellSmall macrocells (the antimeridian seam's full rows, polar caps) go to
// k_shell_rects, a workgroup each.
constexpr int kShellSmall = 64;
struct ShellRect {
  int xlo, ylo, zlo, nx, ny, nz;
  float lo, hi;
};

__device__ __forceinline__ void shell_write(const ShellRect &q, long k, int3 dims, float *valueRanges) {
  const int mx = q.xlo + (int)(k % q.nx);
  const int my = q.ylo + (int)((k / q.nx) % q.ny);
  const int mz = q.zlo + (int)(k / ((long)q.nx * q.ny));
  float *vr = valueRanges + 2 * ((size_t)mz * dims.x * dims.y + (size_t)my * dims.x + mx);
  atomic_min_f(vr, q.lo);
  atomic_max_f(vr + 1, q.hi);
}

__global__ void __launch_bounds__(256) k_shell_build(const irt_icon_cell *cells, size_t n, int3 dims,
                                                     float3 sbLo, float3 sbHi, float *valueRanges,
                                                     ShellRect *wide, unsigned long long *numWide,
                                                     size_t wideCap) {
  // 256 records (72,704 B, 16-B aligned) staged through LDS with coalesced 16-B loads: a
  // lane reading its own 284-B record straight from HBM would touch a different line with
  // every load instruction of the wave
  constexpr int kRecs = 256, kVec = kRecs * (int)sizeof(irt_icon_cell) / 16;
  static_assert(kRecs * sizeof(irt_icon_cell) % 16 == 0, "record batches are float4 aligned");
  __shared__ float4 s_rec[kVec];
  for (size_t b0 = (size_t)blockIdx.x * kRecs; b0 < n; b0 += (size_t)gridDim.x * kRecs) {
    const size_t nb = n - b0 < (size_t)kRecs ? n - b0 : (size_t)kRecs;
    const int nv = (int)((nb * sizeof(irt_icon_cell) + 15) / 16);
    const float4 *src = reinterpret_cast<const float4 *>(cells + b0);
    __syncthreads();  // the previous batch is done with s_rec
    for (int v = threadIdx.x; v < nv; v += blockDim.x) s_rec[v] = src[v];
    __syncthreads();
    if (threadIdx.x >= nb) continue;
    const irt_icon_cell &c = reinterpret_cast<const irt_icon_cell *>(s_rec)[threadIdx.x];
    const int nl = c.numLayers;
    if (nl <= 0) continue;
    // min/max over the layers with the CAS loops' "store only if strictly smaller/larger"
    // semantics (NaN never stores; +-inf and IRT_FLT_MAX behave as in the reference)
    float lo = IRT_FLT_MAX, hi = -IRT_FLT_MAX;
    bool sorted = true;
    for (int j = 1; j <= nl; ++j)
      if (!(float_key(c.height[j - 1]) <= float_key(c.height[j]))) sorted = false;
    if (sorted) {
      int f = 0;  // findHeight(h[i])
      float hp = c.height[0];
      for (int i = 0; i < nl; ++i) {
        const float v0 = c.value[f];  // getValue(h[i])
        const float h1 = c.height[i + 1];
        f = h1 == hp ? f : i;  // findHeight(h[i+1])
        hp = h1;
        const float v1 = c.value[f];  // getValue(h[i+1])
        if (v0 < lo) lo = v0;
        if (v1 > hi) hi = v1;
      }
    } else {
      for (int i = 0; i < nl; ++i) {
        const float v0 = c.value[find_height(c.height, nl, c.height[i])];      // getValue(h[i])
        const float v1 = c.value[find_height(c.height, nl, c.height[i + 1])];  // getValue(h[i+1])
        if (v0 < lo) lo = v0;
        if (v1 > hi) hi = v1;
      }
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
    if (xlo > xhi || ylo > yhi || zlo > zhi) continue;
    const ShellRect q = {xlo, ylo, zlo, xhi - xlo + 1, yhi - ylo + 1, zhi - zlo + 1, lo, hi};
    const long total = (long)q.nx * q.ny * q.nz;
    if (total > kShellSmall && numWide) {
      const unsigned long long k = atomicAdd(numWide, 1ull);
      if (k < wideCap) {
        wide[k] = q;
        continue;
      }  // list full: this lane does it
    }
    for (long k = 0; k < total; ++k) shell_write(q, k, dims, valueRanges);
  }
}

// The deferred wide rectangles: one workgroup per rectangle, lanes sharing its macrocells.
__global__ void __launch_bounds__(256) k_shell_rects(const ShellRect *wide, const unsigned long long *numWide,
                                                     size_t wideCap, int3 dims, float *valueRanges) {
  const unsigned long long nw = *numWide < wideCap ? *numWide : wideCap;
  for (size_t b = blockIdx.x; b < nw; b += gridDim.x) {
    const ShellRect q = wide[b];
    const long total = (long)q.nx * q.ny * q.nz;
    for (long k = threadIdx.x; k < total; k += blockDim.x) shell_write(q, k, dims, valueRanges);
  }
}

// buildGrid_ICON + rasterizeBox (hostCode.cu:227-297): per cell and layer the Cartesian
// box of the layer's wedge (top corners pushed out by (R-|bary|)/R, ICONGrid-style),
// rasterised into the 256^3 grid with the layer's value range.  toCartesian's glibc
// cosf/sinf come precomputed from the host (trig = {cos lat, sin lat, cos lon, sin lon}
// per corner, host/irt_scene.cpp), the rest is the same float expressions.  Consecutive
// layers covering the same macrocell box are merged before the CAS-loop min/max (the
// same min/max).
__device__ __forceinline__ float3 to_cartesian_trig(float r, const float4 &t) {
  return make_float3((r * t.x) * t.z, (r * t.x) * t.w, r * t.y);  // ICONGrid.h:44-54
}

// A merged layer box with its value range, deferred to k_grid_boxes when it covers more
// than kSmallBox macrocells (R1B00/R2B00-class columns): one lane would serialise it.
struct GridBox {
  int3 lo, hi;
  float rLo, rHi;
};
constexpr long kSmallBox = 256;

// findHeight (ICONGrid.h:117-145) over a record's height/value block (irt_common.h kBlk4)
__device__ __forceinline__ int find_height_blk(const float *Bf, int nl, float hpos) {
  int first = 0, count = nl;
  while (count > 0) {
    const int step = count / 2, it = first + step;
    if (!(hpos <= Bf[blk_height_pos(it + 1)])) {
      first = it + 1;
      count -= step + 1;
    } else {
      count = step;
    }
  }
  return first;
}

// Built on first use (irt_context.hip ensure_grid), from the scene's per-record blocks,
// meta words (numLayers) and corner trig -- the records themselves are gone by then.
__global__ void __launch_bounds__(128) k_grid_build(const float4 *blocks, const uint32_t *meta,
                                                    const float4 *trig, size_t n, int dim, float3 lo,
                                                    float3 hi, float *valueRanges, GridBox *big,
                                                    unsigned long long *numBig, size_t bigCap) {
  const size_t ci = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (ci >= n) return;
  const float *Bf = reinterpret_cast<const float *>(blocks + (size_t)kBlk4 * ci);
  const int numLayers = (int)(meta[ci] & 31u);
  const float4 t0 = trig[3 * ci], t1 = trig[3 * ci + 1], t2 = trig[3 * ci + 2];
  int3 pLo = make_int3(0, 0, 0), pHi = make_int3(-1, -1, -1);
  float rLo = 0.f, rHi = 0.f;
  bool have = false;
  auto flush = [&]() {
    const long nx = pHi.x - pLo.x + 1, ny = pHi.y - pLo.y + 1, nz = pHi.z - pLo.z + 1;
    if (numBig && nx * ny * nz > kSmallBox) {
      const unsigned long long k = atomicAdd(numBig, 1ull);
      if (k < bigCap) {
        big[k] = {pLo, pHi, rLo, rHi};
        return;
      }  // list full: this lane does it
    }
    for (int mz = pLo.z; mz <= pHi.z; ++mz)
      for (int my = pLo.y; my <= pHi.y; ++my)
        for (int mx = pLo.x; mx <= pHi.x; ++mx) {
          float *vr = valueRanges + 2 * ((size_t)mz * dim * dim + (size_t)my * dim + mx);
          atomic_min_f(vr, rLo);
          atomic_max_f(vr + 1, rHi);
        }
  };
  for (int i = 0; i < numLayers; ++i) {
    const float hb = Bf[blk_height_pos(i)], ht = Bf[blk_height_pos(i + 1)];
    const float3 b1 = to_cartesian_trig(hb, t0), b2 = to_cartesian_trig(hb, t1), b3 = to_cartesian_trig(hb, t2);
    float3 v1 = to_cartesian_trig(ht, t0), v2 = to_cartesian_trig(ht, t1), v3 = to_cartesian_trig(ht, t2);
    float3 bl = make_float3(__builtin_inff(), __builtin_inff(), __builtin_inff());
    float3 bu = make_float3(-__builtin_inff(), -__builtin_inff(), -__builtin_inff());
    auto ext = [&](const float3 &v) {  // box3f::extend (vecmath.h:1096-1100): fminf/fmaxf
      bl = make_float3(fminf(bl.x, v.x), fminf(bl.y, v.y), fminf(bl.z, v.z));
      bu = make_float3(fmaxf(bu.x, v.x), fmaxf(bu.y, v.y), fmaxf(bu.z, v.z));
    };
    ext(b1); ext(b2); ext(b3);
    const float3 bary = make_float3(((v1.x + v2.x) + v3.x) / 3.f, ((v1.y + v2.y) + v3.y) / 3.f,
                                    ((v1.z + v2.z) + v3.z) / 3.f);
    const float R = ht;
    const float D = R - sqrtf(bary.x * bary.x + bary.y * bary.y + bary.z * bary.z);
    const float off = D / R;
    v1 = make_float3(v1.x + v1.x * off, v1.y + v1.y * off, v1.z + v1.z * off);
    v2 = make_float3(v2.x + v2.x * off, v2.y + v2.y * off, v2.z + v2.z * off);
    v3 = make_float3(v3.x + v3.x * off, v3.y + v3.y * off, v3.z + v3.z * off);
    ext(v1); ext(v2); ext(v3);
    // box1f valueRange(INFINITY,-INFINITY).extend(getValue(h[i])).extend(getValue(h[i+1]))
    const float g0 = Bf[blk_value_pos(find_height_blk(Bf, numLayers, hb))];
    const float g1 = Bf[blk_value_pos(find_height_blk(Bf, numLayers, ht))];
    const float vlo = fminf(fminf(__builtin_inff(), g0), g1);
    const float vhi = fmaxf(fmaxf(-__builtin_inff(), g0), g1);
    const int3 a = make_int3(project_on_grid(bl.x, lo.x, hi.x, dim), project_on_grid(bl.y, lo.y, hi.y, dim),
                             project_on_grid(bl.z, lo.z, hi.z, dim));
    const int3 b = make_int3(project_on_grid(bu.x, lo.x, hi.x, dim), project_on_grid(bu.y, lo.y, hi.y, dim),
                             project_on_grid(bu.z, lo.z, hi.z, dim));
    if (have && a.x == pLo.x && a.y == pLo.y && a.z == pLo.z && b.x == pHi.x && b.y == pHi.y &&
        b.z == pHi.z) {
      rLo = (vlo < rLo) ? vlo : rLo;  // the atomics' "store only if strictly smaller/larger"
      rHi = (vhi > rHi) ? vhi : rHi;
      continue;
    }
    if (have) flush();
    pLo = a;
    pHi = b;
    rLo = vlo;
    rHi = vhi;
    have = true;
  }
  if (have) flush();
}


// The deferred boxes: one workgroup per box, lanes sharing its macrocells.
__global__ void __launch_bounds__(256) k_grid_boxes(const GridBox *big, const unsigned long long *numBig,
                                                    size_t bigCap, int dim, float *valueRanges) {
  const unsigned long long nb = *numBig < bigCap ? *numBig : bigCap;
  for (size_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const GridBox q = big[b];
    const long nx = q.hi.x - q.lo.x + 1, ny = q.hi.y - q.lo.y + 1, nz = q.hi.z - q.lo.z + 1;
    for (long k = threadIdx.x; k < nx * ny * nz; k += blockDim.x) {
      const int mx = q.lo.x + (int)(k % nx), my = q.lo.y + (int)((k / nx) % ny),
                mz = q.lo.z + (int)(k / (nx * ny));
      float *vr = valueRanges + 2 * ((size_t)mz * dim * dim + (size_t)my * dim + mx);
      atomic_min_f(vr, q.rLo);
      atomic_max_f(vr + 1, q.rHi);
    }
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

// The transfer function's expected Woodcock samples per acceptance, over the shell's macrocells
// with a positive majorant: per macrocell 1 / p, p = the mean LUT alpha over its value range's
// entries (the range k_max_opacities scans) over the majorant -- postClassify's alpha against the
// majorant, deviceCode.cu:174-176 -- capped at 1000; out[0] += sum, out[1] += count (one atomic
// pair per workgroup).  A dense TF (the reference's default: ~1.3) takes about one located sample
// per ray, a sparse one many (bench.py's comb: ~32), which decides whether launches start their
// candidate scan from the slot table (irt_context.hip).
__global__ void k_accept_stat(const float2 *valueRanges, const float *maxOp, size_t numMCs, const float4 *lut,
                              int size, float tfLo, float tfHi, double *out) {
  __shared__ double s_sum[256];
  __shared__ double s_cnt[256];
  const size_t mc = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  double inv = 0.0, cnt = 0.0;
  if (mc < numMCs && maxOp[mc] > 0.f) {
    float2 vr = valueRanges[mc];
    vr.x = (vr.x - tfLo) / (tfHi - tfLo);
    vr.y = (vr.y - tfLo) / (tfHi - tfLo);
    int lo = f2i_x86(vr.x * (float)(size - 1));
    int hi = (int)((uint32_t)f2i_x86(vr.y * (float)(size - 1)) + 1u);
    lo = lo < 0 ? 0 : (lo > size - 1 ? size - 1 : lo);
    hi = hi < 0 ? 0 : (hi > size - 1 ? size - 1 : hi);
    float a = 0.f;
    for (int i = lo; i <= hi; ++i) a += lut[i].w;
    const float p = a / (float)(hi - lo + 1) / maxOp[mc];
    inv = p > 1e-3f ? 1.0 / (double)p : 1000.0;
    cnt = 1.0;
  }
  s_sum[threadIdx.x] = inv;
  s_cnt[threadIdx.x] = cnt;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + w];
      s_cnt[threadIdx.x] += s_cnt[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && s_cnt[0] > 0.0) {
    atomicAdd(&out[0], s_sum[0]);
    atomicAdd(&out[1], s_cnt[0]);
  }
}

// clearFramebuffer (common/pipeline.cu:171-199)
__global__ void k_clear(uint32_t *fb, float4 *accum, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (fb) fb[i] = 0u;  // make_rgba(vec4f(0)) == 0
  if (accum) accum[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Scatter rank-major packed tiles into a linear framebuffer (multi-GPU gather epilogue).
// Four workgroups per tile slot (16 rows each); a lane moves 4 pixels of a row with one
// 16-byte load and store when the row is 16-byte aligned in the framebuffer (W % 4 == 0)
// and the 4 pixels are inside the frame, pixel by pixel otherwise (ragged right/bottom edge).
// Slot k of rank r holds tile r + k*numRanks, or table[r*maxTiles + k] (irt_deal_tiles; -1
// marks an empty slot).
__global__ void k_unpack(const uint32_t *gathered, int numRanks, int maxTiles, int W, int H,
                         int tilesX, int numTilesTotal, uint32_t *fb, const int32_t *table) {
  const int k = blockIdx.x >> 2;  // tile slot
  const int rank = blockIdx.y;
  if (k >= maxTiles) return;
  const int tileId = table ? table[(size_t)rank * maxTiles + k] : rank + k * numRanks;
  if (tileId < 0 || tileId >= numTilesTotal) return;
  const int tx = tileId % tilesX, ty = tileId / tilesX;
  const int ly = (blockIdx.x & 3) * 16 + (threadIdx.x >> 4), lx = (threadIdx.x & 15) * 4;
  const uint32_t *src = gathered + ((size_t)rank * maxTiles + k) * 4096 + ly * 64 + lx;
  const int x = tx * 64 + lx, y = ty * 64 + ly;
  if (y >= H || x >= W) return;
  uint32_t *dst = fb + (size_t)x + (size_t)W * y;
  const uint4 v = *reinterpret_cast<const uint4 *>(src);
  if ((W & 3) == 0 && x + 4 <= W) {
    *reinterpret_cast<uint4 *>(dst) = v;
  } else {
    dst[0] = v.x;
    if (x + 1 < W) dst[1] = v.y;
    if (x + 2 < W) dst[2] = v.z;
    if (x + 3 < W) dst[3] = v.w;
  }
}

// Per-launch statistics hand-off of the statistics variant and IRT_COUNTERS=atomic
// (irt_context.hip render_impl): this launch's 16-counter block into the pinned host ring
// (vector stores over the mapped pointer, visible to the host at the kernel's end-of-kernel
// release) and the next ring slot zeroed for the next launch.  (The default path needs no
// such kernel: the render kernel's workgroups write their counts to host memory.)
__global__ void k_stats_out(const unsigned long long *cur, unsigned long long *host,
                            unsigned long long *next, unsigned long long *buckets) {
  const int i = threadIdx.x;  // 64 threads: bucket i's 8 counters
  __shared__ unsigned long long s_b[kCounterBuckets][8];
  for (int j = 0; j < 8; ++j) {
    s_b[i][j] = buckets ? buckets[i * 8 + j] : 0ull;
    if (buckets) buckets[i * 8 + j] = 0ull;  // clean for this slot's next launch
  }
  __syncthreads();
  if (i < 16) {
    unsigned long long v = cur[i];
    if (i < 8)
      for (int b = 0; b < kCounterBuckets; ++b) v += s_b[b][i];
    host[i] = v;
    if (next != cur) next[i] = 0ull;
  }
}

void launch_shell_init(float *vr, size_t numMCs, hipStream_t s) {
  hipLaunchKernelGGL(k_shell_init, dim3((unsigned)((numMCs + 255) / 256)), dim3(256), 0, s,
                     (float2 *)vr, numMCs);
}
void launch_shell_build(const irt_icon_cell *cells, size_t n, int3 dims, float3 lo, float3 hi,
                        float *vr, hipStream_t s) {
  if (n == 0) return;
  const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
  // the wide-rectangle list: sized for the seam and polar columns, capped (overflow stays
  // in-lane)
  const size_t cap = std::min<size_t>(n / 8 + 4096, size_t(1) << 22);
  ShellRect *wide = nullptr;
  unsigned long long *numWide = nullptr;
  if (hipMallocAsync((void **)&wide, cap * sizeof(ShellRect), s) != hipSuccess ||
      hipMallocAsync((void **)&numWide, sizeof(unsigned long long), s) != hipSuccess) {
    hipLaunchKernelGGL(k_shell_build, dim3(blocks), dim3(256), 0, s, cells, n, dims, lo, hi, vr,
                       (ShellRect *)nullptr, (unsigned long long *)nullptr, (size_t)0);
    return;
  }
  (void)hipMemsetAsync(numWide, 0, sizeof(unsigned long long), s);
  hipLaunchKernelGGL(k_shell_build, dim3(blocks), dim3(256), 0, s, cells, n, dims, lo, hi, vr, wide,
                     numWide, cap);
  hipLaunchKernelGGL(k_shell_rects, dim3(2048), dim3(256), 0, s, wide, numWide, cap, dims, vr);
  (void)hipFreeAsync(wide, s);
  (void)hipFreeAsync(numWide, s);
}
void launch_grid_build(const float4 *blocks, const uint32_t *meta, const float4 *trig, size_t n,
                       float3 lo, float3 hi, float *vr, hipStream_t s) {
  if (n == 0) return;
  // the deferred-box list: sized for a few boxes per cell, capped (overflow stays in-lane)
  const size_t cap = std::min<size_t>(4 * n + 1024, size_t(1) << 22);
  GridBox *big = nullptr;
  unsigned long long *numBig = nullptr;
  if (hipMallocAsync((void **)&big, cap * sizeof(GridBox), s) != hipSuccess ||
      hipMallocAsync((void **)&numBig, sizeof(unsigned long long), s) != hipSuccess) {
    // no scratch: every box in-lane
    hipLaunchKernelGGL(k_grid_build, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, blocks, meta,
                       trig, n, kGridDim, lo, hi, vr, (GridBox *)nullptr, (unsigned long long *)nullptr,
                       (size_t)0);
    return;
  }
  (void)hipMemsetAsync(numBig, 0, sizeof(unsigned long long), s);
  hipLaunchKernelGGL(k_grid_build, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, blocks, meta, trig,
                     n, kGridDim, lo, hi, vr, big, numBig, cap);
  hipLaunchKernelGGL(k_grid_boxes, dim3(2048), dim3(256), 0, s, big, numBig, cap, kGridDim, vr);
  (void)hipFreeAsync(big, s);
  (void)hipFreeAsync(numBig, s);
}
// GRID_ACCEL_MODE's empty-space bitmap: bit b = block b (kGridBlock^3 cells of the kGridDim^3
// grid, x fastest) holds a cell whose majorant is not <= 0.  woodcockTracking returns at once
// on a majorant <= 0 (deviceCode.cu:161-162: no draw, no sample, tw = t0 fails the hit test),
// so render_grid may step through a block whose bit is clear without reading its majorants.
__global__ void k_grid_bits(const float *maxOp, uint32_t *bits) {
  const int b = (int)(blockIdx.x * 256 + threadIdx.x);
  constexpr int NB = kGridDim / kGridBlock;
  if (b >= NB * NB * NB) return;
  const int bx = b % NB, by = (b / NB) % NB, bz = b / (NB * NB);
  bool any = false;
  for (int z = 0; z < kGridBlock && !any; ++z)
    for (int y = 0; y < kGridBlock && !any; ++y)
      for (int x = 0; x < kGridBlock && !any; ++x) {
        const size_t i = ((size_t)(bz * kGridBlock + z) * kGridDim + (size_t)(by * kGridBlock + y)) * kGridDim +
                         (size_t)(bx * kGridBlock + x);
        any = !(maxOp[i] <= 0.f);
      }
  const unsigned long long m = __ballot(any);  // 64 blocks per wave -> two words
  const int lane = (int)(threadIdx.x & 63);
  if (lane == 0) bits[b / 32] = (uint32_t)m;
  if (lane == 32) bits[b / 32] = (uint32_t)(m >> 32);
}

void launch_grid_bits(const float *maxOp, uint32_t *bits, hipStream_t s) {
  constexpr int NB = kGridDim / kGridBlock;
  hipLaunchKernelGGL(k_grid_bits, dim3((NB * NB * NB + 255) / 256), dim3(256), 0, s, maxOp, bits);
}

void launch_max_opacities(const float *vr, size_t numMCs, const float4 *lut, int size, float lo,
                          float hi, float *maxOp, hipStream_t s) {
  hipLaunchKernelGGL(k_max_opacities, dim3((unsigned)((numMCs + 255) / 256)), dim3(256), 0, s,
                     (const float2 *)vr, numMCs, lut, size, lo, hi, maxOp);
}
void launch_accept_stat(const float *vr, const float *maxOp, size_t numMCs, const float4 *lut, int size, float lo,
                        float hi, double *out, hipStream_t s) {
  hipLaunchKernelGGL(k_accept_stat, dim3((unsigned)((numMCs + 255) / 256)), dim3(256), 0, s,
                     (const float2 *)vr, maxOp, numMCs, lut, size, lo, hi, out);
}
void launch_stats_out(const unsigned long long *cur, unsigned long long *host,
                      unsigned long long *next, unsigned long long *buckets, hipStream_t s) {
  hipLaunchKernelGGL(k_stats_out, dim3(1), dim3(kCounterBuckets), 0, s, cur, host, next, buckets);
}
// a u32 array between device memory and mapped pinned host memory (either direction):
// the scheduling costs and block orders, without an SDMA copy on the render stream
__global__ void k_copy_u32(const uint32_t *src, uint32_t *dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
void launch_copy_u32(const uint32_t *src, uint32_t *dst, size_t n, hipStream_t s) {
  if (n == 0) return;
  const unsigned blocks = (unsigned)std::min<size_t>(64, (n + 255) / 256);
  hipLaunchKernelGGL(k_copy_u32, dim3(blocks), dim3(256), 0, s, src, dst, n);
}
void launch_clear(uint32_t *fb, float4 *accum, size_t n, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_clear, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, fb, accum, n);
}
void launch_unpack(const uint32_t *g, int numRanks, int maxTiles, int W, int H, uint32_t *fb,
                   hipStream_t s, const int32_t *table) {
  const int tilesX = (W + 63) / 64, tilesY = (H + 63) / 64;
  hipLaunchKernelGGL(k_unpack, dim3(maxTiles * 4, numRanks), dim3(256), 0, s, g, numRanks, maxTiles,
                     W, H, tilesX, tilesX * tilesY, fb, table);
}

}  // namespace irt
