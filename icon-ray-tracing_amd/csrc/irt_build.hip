// irt_build.hip -- the scene build on the GPU: per-record planes and height/value blocks,
// and the cube-map point locator (irt_build.h), from the cells and their corner trig
// already in HBM.  Replaces the reference's device-side accelerator builds (the cuBQL
// gpuBuilder over the cells' wedges, hostCode.cu:557-650, and the OWL BLAS/TLAS builds,
// 440-525): one pass per stage, no host round trip of the data.
//
// Stages (every count and order deterministic, so the arrays are byte-identical to the
// host restatement, host/irt_scene.cpp):
//   1. k_prep        per record: planes, radial range, meta (quantised keys), block; column
//                    starts (records with different corners than their predecessor)
//   2. scan          run (column) index of every record, the run start list
//   3. k_run_count   per run: its kind (irt_build.h run_kind) and, for triangles, the
//                    number of (cell, sub-cell mask) items; k_wide_runs for the rare cone
//                    and every-cell runs (one workgroup each)
//   4. k_run_write   the items (k_wide_runs again for the wide ones)
//   5. k_rec_expand  per record with a positive radial extent: (cell, record | mask) pairs
//                    of its run's items, in record order
//   6. radix sort    stable by cell: each cell's records stay in index order
//   7. k_cell_edges  per cell: the radial edges (cells with > kLocalEntries entries: host)
//   8. k_cell_header per cell: bin ends, sub-cell masks, entry count; scan -> bases
//   9. k_cell_fill   the fat entries, bin by bin
//  10. k_slot_fill   (scenes whose cells share their radial edges) the slot table
//                    (irt_common.h kSlot4), from the headers and entries: build_slots_device

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "irt_build.h"
#include "irt_internal.h"
#include "irt_kernels.h"

namespace irt {

namespace {

constexpr int kLocalEntries = 256;  // per-cell entries the edge search keeps in registers

#define BHIP(call)                                                                \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess) {                                                       \
      set_error("scene build: %s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                __FILE__, __LINE__);                                              \
      return IRT_E_HIP;                                                           \
    }                                                                             \
  } while (0)

inline unsigned grid_for(size_t n, int block = 256) {
  return (unsigned)std::max<size_t>(1, std::min<size_t>((n + block - 1) / block, 1u << 20));
}

// ---------------------------------------------------------------- 1. per record
__global__ void k_prep(const irt_icon_cell *cells, const float4 *trig, size_t n, float4 *planes,
                       float2 *rng, uint32_t *meta, float4 *blocks, uint32_t *runFlag) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const irt_icon_cell &c = cells[i];
    const int nl = c.numLayers;
    float t[12];
    for (int k = 0; k < 3; ++k) {
      const float4 q = trig[3 * i + k];
      t[4 * k] = q.x, t[4 * k + 1] = q.y, t[4 * k + 2] = q.z, t[4 * k + 3] = q.w;
    }
    float pl[12];
    const float h0 = c.height[0], hN = c.height[nl];
    record_planes(h0, hN, t, pl);
    for (int k = 0; k < 3; ++k) planes[3 * i + k] = make_float4(pl[4 * k], pl[4 * k + 1], pl[4 * k + 2], pl[4 * k + 3]);
    rng[i] = make_float2(h0, hN);
    meta[i] = record_meta(c.height, nl);
    float blk[64];
    record_block(c.height, c.value, blk);
    for (int k = 0; k < 16; ++k)
      blocks[16 * i + k] = make_float4(blk[4 * k], blk[4 * k + 1], blk[4 * k + 2], blk[4 * k + 3]);
    runFlag[i] = (i == 0 || !same_corners(c.lat, c.lon, cells[i - 1].lat, cells[i - 1].lon)) ? 1u : 0u;
  }
}

// run starts from the inclusive scan of the flags (runOf[i] = run index + 1)
__global__ void k_run_starts(const uint32_t *runFlag, const uint32_t *runOf1, size_t n,
                             size_t numRuns, uint32_t *runStart) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    if (runFlag[i]) runStart[runOf1[i] - 1] = (uint32_t)i;
  if (blockIdx.x == 0 && threadIdx.x == 0) runStart[numRuns] = (uint32_t)n;
}

// ---------------------------------------------------------------- 3./4. per run
struct CountEmit {
  uint64_t count = 0;
  __device__ void operator()(uint32_t, uint32_t) { ++count; }
};
struct WriteEmit {
  uint2 *out;
  __device__ void operator()(uint32_t cell, uint32_t mask) { *out++ = make_uint2(cell, mask); }
};

__device__ __forceinline__ int run_setup(const uint32_t *runStart, size_t r, const float *trig,
                                         const float *planes, const float *rng, BD3 d[3],
                                         double &cosRho, BD3 &centre) {
  const uint32_t i0 = runStart[r], i1 = runStart[r + 1];
  corner_dirs(trig + 12 * (size_t)i0, d);
  cosRho = 1.0;
  centre = bd3(0, 0, 0);
  return run_kind(d, planes, rng, i0, i1, cosRho, centre);
}

__global__ void k_run_count(const uint32_t *runStart, size_t numRuns, const float *trig,
                            const float *planes, const float *rng, int G, uint64_t *itemCount,
                            uint8_t *kind, uint32_t *wideList, unsigned long long *wideCount) {
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < numRuns;
       r += (size_t)gridDim.x * blockDim.x) {
    BD3 d[3], centre;
    double cosRho;
    const int k = run_setup(runStart, r, trig, planes, rng, d, cosRho, centre);
    kind[r] = (uint8_t)k;
    uint64_t cnt = 0;
    if (k == kRunTri) {
      CountEmit e;
      raster_triangle(d, G, e);
      cnt = e.count;
    } else if (k == kRunCap || k == kRunAll) {
      wideList[atomicAdd(wideCount, 1ull)] = (uint32_t)r;  // counted by k_wide_runs
    }
    itemCount[r] = cnt;
  }
}

__global__ void k_run_write(const uint32_t *runStart, size_t numRuns, const float *trig,
                            const float *planes, const float *rng, int G, const uint8_t *kind,
                            const uint64_t *itemOff, uint2 *items) {
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < numRuns;
       r += (size_t)gridDim.x * blockDim.x) {
    if (kind[r] != kRunTri) continue;
    BD3 d[3], centre;
    double cosRho;
    run_setup(runStart, r, trig, planes, rng, d, cosRho, centre);
    WriteEmit e{items + itemOff[r]};
    raster_triangle(d, G, e);
  }
}

// The cone and every-cell runs (R1B00/R2B00-class triangles, degenerate columns): one
// workgroup per run striding over all 6 G^2 cells.  write == false: count into
// itemCount[run]; write == true: items in any order (a run lists a cell at most once, and
// the stable sort by cell only orders records).
template <bool WRITE>
__global__ void __launch_bounds__(256) k_wide_runs(const uint32_t *wideList, const uint32_t *runStart,
                                                   const float *trig, const float *planes,
                                                   const float *rng, int G, const uint8_t *kind,
                                                   uint64_t *itemCount, const uint64_t *itemOff,
                                                   uint2 *items) {
  __shared__ unsigned long long s_n;
  const uint32_t r = wideList[blockIdx.x];
  BD3 d[3], centre;
  double cosRho;
  run_setup(runStart, r, trig, planes, rng, d, cosRho, centre);
  const bool all = kind[r] == kRunAll;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const uint32_t numCells = 6u * (uint32_t)G * (uint32_t)G;
  unsigned long long mine = 0;
  for (uint32_t k = threadIdx.x; k < numCells; k += blockDim.x) {
    if (!all && !cap_hits_cell(centre, cosRho, G, k)) continue;
    if (WRITE)
      items[itemOff[r] + atomicAdd(&s_n, 1ull)] = make_uint2(k, kFullMask);
    else
      ++mine;
  }
  if (!WRITE) {
    atomicAdd(&s_n, mine);
    __syncthreads();
    if (threadIdx.x == 0) itemCount[r] = s_n;
  }
}

// ---------------------------------------------------------------- 5. per record
__global__ void k_rec_count(const uint32_t *runOf1, const float2 *rng, size_t n,
                            const uint64_t *itemCount, uint64_t *recCount) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const float2 h = rng[i];
    // inverted records never pass the radial test; zero-thickness ones are spheres
    recCount[i] = h.x < h.y ? itemCount[runOf1[i] - 1] : 0ull;
  }
}

__global__ void k_rec_expand(const uint32_t *runOf1, const uint64_t *recCount, const uint64_t *pairOff,
                             size_t n, const uint64_t *itemOff, const uint2 *items, uint32_t *keys,
                             unsigned long long *vals) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t cnt = recCount[i];
    if (!cnt) continue;
    const uint2 *it = items + itemOff[runOf1[i] - 1];
    const uint64_t o = pairOff[i];
    for (uint64_t k = 0; k < cnt; ++k) {
      keys[o + k] = it[k].x;
      vals[o + k] = (unsigned long long)i | ((unsigned long long)it[k].y << 32);
    }
  }
}

__global__ void k_cell_hist(const uint32_t *keys, size_t m, uint32_t *cellCount) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < m;
       p += (size_t)gridDim.x * blockDim.x)
    atomicAdd(&cellCount[keys[p]], 1u);
}

// ---------------------------------------------------------------- 7.-9. per cell
// irt_build.h entry accessor over a cell's sorted pairs
struct DevEntries {
  const unsigned long long *v;  // record | mask << 32, from the cell's first pair
  const float2 *rng;
  __device__ float h0(int k) const { return rng[(uint32_t)v[k]].x; }
  __device__ float hN(int k) const { return rng[(uint32_t)v[k]].y; }
  __device__ uint32_t sub(int k) const { return (uint32_t)(v[k] >> 32); }
};

__global__ void k_cell_edges(const uint32_t *offsets, uint32_t numCells, const unsigned long long *vals,
                             const float2 *rng, float4 *edges, uint32_t *bigList,
                             unsigned long long *bigCount) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < numCells; c += gridDim.x * blockDim.x) {
    const uint32_t q0 = offsets[c], n = offsets[c + 1] - q0;
    if (n > (uint32_t)kLocalEntries) {  // edges from the host (build_scene_device)
      bigList[atomicAdd(bigCount, 1ull)] = c;
      continue;
    }
    const DevEntries en{vals + q0, rng};
    float cand[kLocalEntries];
    double rmin, rmax;
    const int nc = cell_candidates(en, (int)n, cand, rmin, rmax);
    float e[kMaxEdges] = {0.f, 0.f, 0.f};
    const int ne = choose_edges(en, (int)n, cand, nc, rmin, rmax, e);
    edges[c] = make_float4(e[0], e[1], e[2], __uint_as_float((uint32_t)ne));
  }
}

__global__ void k_cell_header(const uint32_t *offsets, uint32_t numCells, const unsigned long long *vals,
                              const float2 *rng, const float4 *edges, uint32_t *hdr,
                              uint64_t *cellCount) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < numCells; c += gridDim.x * blockDim.x) {
    const uint32_t q0 = offsets[c], n = offsets[c + 1] - q0;
    const DevEntries en{vals + q0, rng};
    const float4 E = edges[c];
    const float e[kMaxEdges] = {E.x, E.y, E.z};
    uint32_t H[kBinHdrWords];
    cellCount[c] = cell_header(en, (int)n, e, (int)__float_as_uint(E.w), H);
    uint4 *out = reinterpret_cast<uint4 *>(hdr + (size_t)c * kBinHdrWords);
    for (int k = 0; k < kBinHdrWords / 4; ++k) out[k] = make_uint4(H[4 * k], H[4 * k + 1], H[4 * k + 2], H[4 * k + 3]);
  }
}

__global__ void k_cell_fill(const uint32_t *offsets, uint32_t numCells, const unsigned long long *vals,
                            const float2 *rng, const float4 *edges, const uint64_t *cellBase,
                            uint32_t *hdr, const float *planes, const uint32_t *meta, float4 *fat) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < numCells; c += gridDim.x * blockDim.x) {
    const uint32_t q0 = offsets[c], n = offsets[c + 1] - q0;
    const uint64_t base = cellBase[c];
    hdr[(size_t)c * kBinHdrWords + 3] = (uint32_t)base;
    const float4 E = edges[c];
    const float e[kMaxEdges] = {E.x, E.y, E.z};
    const int ne = (int)__float_as_uint(E.w);
    uint64_t at = base;
    for (int k = 0; k <= ne; ++k) {
      const float lo = k ? e[k - 1] : -__builtin_inff(), hi = k < ne ? e[k] : __builtin_inff();
      for (uint32_t q = 0; q < n; ++q) {
        const uint32_t rec = (uint32_t)vals[q0 + q];
        const float2 h = rng[rec];
        if (!in_bin(h.x, h.y, lo, hi)) continue;
        float F[4 * kFat4];
        fat_entry(rec, planes, reinterpret_cast<const float *>(rng), meta, F);
        float4 *o = fat + (size_t)(at++) * kFatStride4;
        for (int j = 0; j < kFat4; ++j) o[j] = make_float4(F[4 * j], F[4 * j + 1], F[4 * j + 2], F[4 * j + 3]);
        for (int j = kFat4; j < kFatStride4; ++j) o[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
}

// ---------------------------------------------------------------- device scratch
struct Scratch {
  std::vector<void *> ptrs;
  ~Scratch() {
    for (void *p : ptrs) (void)hipFree(p);
  }
  template <typename T>
  hipError_t alloc(T **p, size_t count) {
    *p = nullptr;
    hipError_t e = hipMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
  void release(void *p) {
    for (auto &q : ptrs)
      if (q == p) {
        (void)hipFree(q);
        q = nullptr;
      }
  }
};

template <typename T>
int exclusive_sum(const T *in, T *out, size_t n, hipStream_t s, Scratch &S) {
  size_t bytes = 0;
  BHIP(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n, s));
  void *tmp = nullptr;
  BHIP(S.alloc((char **)&tmp, bytes));
  BHIP(hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, n, s));
  S.release(tmp);
  return IRT_OK;
}

template <typename T>
int inclusive_sum(const T *in, T *out, size_t n, hipStream_t s, Scratch &S) {
  size_t bytes = 0;
  BHIP(hipcub::DeviceScan::InclusiveSum(nullptr, bytes, in, out, n, s));
  void *tmp = nullptr;
  BHIP(S.alloc((char **)&tmp, bytes));
  BHIP(hipcub::DeviceScan::InclusiveSum(tmp, bytes, in, out, n, s));
  S.release(tmp);
  return IRT_OK;
}

template <typename T>
int read_back(T *dst, const T *src, size_t count, hipStream_t s) {
  BHIP(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyDeviceToHost, s));
  BHIP(hipStreamSynchronize(s));
  return IRT_OK;
}

// irt_build.h entry accessor over host copies (the big cells' edge search)
struct HostEntries {
  const std::vector<float> &h0v, &hNv;
  float h0(int k) const { return h0v[k]; }
  float hN(int k) const { return hNv[k]; }
  uint32_t sub(int) const { return 0u; }
};

__global__ void k_gather_rng(const unsigned long long *vals, size_t m, const float2 *rng, float2 *out) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < m;
       p += (size_t)gridDim.x * blockDim.x)
    out[p] = rng[(uint32_t)vals[p]];
}

}  // namespace

// IRT_BUILD_VERBOSE=1: stage times on stderr
struct StageClock {
  bool on = getenv("IRT_BUILD_VERBOSE") != nullptr;
  hipStream_t s;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  void mark(const char *what) {
    if (!on) return;
    (void)hipStreamSynchronize(s);
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[irt build] %-22s %8.1f ms\n", what,
            std::chrono::duration<double, std::milli>(t - t0).count());
    t0 = t;
  }
};

int build_scene_device(const irt_icon_cell *d_cells, const float4 *d_trig, size_t n, size_t numRuns,
                       int G, hipStream_t s, DeviceScene &out) {
  out = DeviceScene();
  Scratch S;
  StageClock clk;
  clk.s = s;
  const unsigned nb = grid_for(n);
  // --- 1. per record
  float4 *planes;
  float2 *rng;
  uint32_t *meta, *runFlag, *runOf1, *runStart;
  BHIP(S.alloc(&planes, 3 * n));
  BHIP(S.alloc(&rng, n));
  BHIP(hipMalloc((void **)&out.meta, std::max<size_t>(n, 1) * sizeof(uint32_t)));
  out.bytes += std::max<size_t>(n, 1) * sizeof(uint32_t);
  meta = out.meta;
  BHIP(hipMalloc((void **)&out.blocks, std::max<size_t>(n, 1) * kBlk4 * sizeof(float4)));
  out.bytes += std::max<size_t>(n, 1) * kBlk4 * sizeof(float4);
  BHIP(S.alloc(&runFlag, n));
  BHIP(S.alloc(&runOf1, n));
  BHIP(S.alloc(&runStart, numRuns + 1));
  if (n) hipLaunchKernelGGL(k_prep, dim3(nb), dim3(256), 0, s, d_cells, d_trig, n, planes, rng, meta, out.blocks, runFlag);
  BHIP(hipGetLastError());
  clk.mark("per-record prep");
  // --- 2. runs
  int rc;
  if (n && (rc = inclusive_sum(runFlag, runOf1, n, s, S))) return rc;
  {
    uint32_t last = 0;
    if (n && (rc = read_back(&last, runOf1 + (n - 1), 1, s))) return rc;
    if ((size_t)last != numRuns) {
      set_error("scene build: %u columns on the device, %zu on the host", last, numRuns);
      return IRT_E_INVALID;
    }
  }
  hipLaunchKernelGGL(k_run_starts, dim3(nb), dim3(256), 0, s, runFlag, runOf1, n, numRuns, runStart);
  BHIP(hipGetLastError());
  S.release(runFlag);
  clk.mark("runs");
  // --- 3. item counts per run
  uint64_t *itemCount, *itemOff;
  uint8_t *kind;
  uint32_t *wideList;
  unsigned long long *wideCount;
  BHIP(S.alloc(&itemCount, numRuns + 1));
  BHIP(S.alloc(&itemOff, numRuns + 1));
  BHIP(S.alloc(&kind, numRuns));
  BHIP(S.alloc(&wideList, numRuns));
  BHIP(S.alloc(&wideCount, 1));
  BHIP(hipMemsetAsync(wideCount, 0, sizeof(unsigned long long), s));
  BHIP(hipMemsetAsync(itemCount + numRuns, 0, sizeof(uint64_t), s));
  const float *trigF = reinterpret_cast<const float *>(d_trig);
  const float *planesF = reinterpret_cast<const float *>(planes);
  const float *rngF = reinterpret_cast<const float *>(rng);
  const unsigned nr = grid_for(numRuns, 64);
  if (numRuns)
    hipLaunchKernelGGL(k_run_count, dim3(nr), dim3(64), 0, s, runStart, numRuns, trigF, planesF, rngF, G,
                       itemCount, kind, wideList, wideCount);
  BHIP(hipGetLastError());
  unsigned long long numWide = 0;
  if ((rc = read_back(&numWide, wideCount, 1, s))) return rc;
  if (numWide)
    hipLaunchKernelGGL(k_wide_runs<false>, dim3((unsigned)numWide), dim3(256), 0, s, wideList, runStart,
                       trigF, planesF, rngF, G, kind, itemCount, (const uint64_t *)nullptr, (uint2 *)nullptr);
  BHIP(hipGetLastError());
  if ((rc = exclusive_sum(itemCount, itemOff, numRuns + 1, s, S))) return rc;
  uint64_t numItems = 0;
  if ((rc = read_back(&numItems, itemOff + numRuns, 1, s))) return rc;
  clk.mark("rasterise (count)");
  // --- 4. items
  uint2 *items;
  BHIP(S.alloc(&items, numItems));
  if (numRuns)
    hipLaunchKernelGGL(k_run_write, dim3(nr), dim3(64), 0, s, runStart, numRuns, trigF, planesF, rngF, G,
                       kind, itemOff, items);
  if (numWide)
    hipLaunchKernelGGL(k_wide_runs<true>, dim3((unsigned)numWide), dim3(256), 0, s, wideList, runStart,
                       trigF, planesF, rngF, G, kind, itemCount, itemOff, items);
  BHIP(hipGetLastError());
  // --- 5. (cell, record | mask) pairs in record order
  uint64_t *recCount, *pairOff;
  BHIP(S.alloc(&recCount, n + 1));
  BHIP(S.alloc(&pairOff, n + 1));
  BHIP(hipMemsetAsync(recCount + n, 0, sizeof(uint64_t), s));
  if (n) hipLaunchKernelGGL(k_rec_count, dim3(nb), dim3(256), 0, s, runOf1, rng, n, itemCount, recCount);
  BHIP(hipGetLastError());
  if ((rc = exclusive_sum(recCount, pairOff, n + 1, s, S))) return rc;
  uint64_t numPairs = 0;
  if ((rc = read_back(&numPairs, pairOff + n, 1, s))) return rc;
  if (numPairs > 0xFFFFFFF0ull) {
    set_error("locator too large (%llu entries)", (unsigned long long)numPairs);
    return IRT_E_INVALID;
  }
  uint32_t *pk, *pk2;
  unsigned long long *pv, *pv2;
  BHIP(S.alloc(&pk, numPairs));
  BHIP(S.alloc(&pv, numPairs));
  if (n)
    hipLaunchKernelGGL(k_rec_expand, dim3(nb), dim3(256), 0, s, runOf1, recCount, pairOff, n, itemOff, items,
                       pk, pv);
  BHIP(hipGetLastError());
  S.release(items);
  S.release(recCount);
  S.release(pairOff);
  S.release(runOf1);
  clk.mark("rasterise + expand");
  // --- 6. stable sort by cell
  const uint32_t numCells = 6u * (uint32_t)G * (uint32_t)G;
  int endBit = 1;
  while (endBit < 32 && (1ull << endBit) < numCells) ++endBit;
  BHIP(S.alloc(&pk2, numPairs));
  BHIP(S.alloc(&pv2, numPairs));
  {
    size_t bytes = 0;
    BHIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, pk, pk2, pv, pv2, numPairs, 0, endBit, s));
    char *tmp = nullptr;
    BHIP(S.alloc(&tmp, bytes));
    if (numPairs) BHIP(hipcub::DeviceRadixSort::SortPairs(tmp, bytes, pk, pk2, pv, pv2, numPairs, 0, endBit, s));
    S.release(tmp);
  }
  S.release(pk);
  S.release(pv);
  uint32_t *cellN, *offsets;
  BHIP(S.alloc(&cellN, numCells + 1));
  BHIP(S.alloc(&offsets, numCells + 1));
  BHIP(hipMemsetAsync(cellN, 0, (numCells + 1) * sizeof(uint32_t), s));
  if (numPairs) hipLaunchKernelGGL(k_cell_hist, dim3(grid_for(numPairs)), dim3(256), 0, s, pk2, numPairs, cellN);
  BHIP(hipGetLastError());
  if ((rc = exclusive_sum(cellN, offsets, numCells + 1, s, S))) return rc;
  S.release(cellN);
  S.release(pk2);
  clk.mark("sort + offsets");
  // --- 7. radial edges
  float4 *edges;
  uint32_t *bigList;
  unsigned long long *bigCount;
  BHIP(S.alloc(&edges, numCells));
  BHIP(S.alloc(&bigList, numCells));
  BHIP(S.alloc(&bigCount, 1));
  BHIP(hipMemsetAsync(bigCount, 0, sizeof(unsigned long long), s));
  const unsigned nc = grid_for(numCells, 64);
  hipLaunchKernelGGL(k_cell_edges, dim3(nc), dim3(64), 0, s, offsets, numCells, pv2, rng, edges, bigList, bigCount);
  BHIP(hipGetLastError());
  unsigned long long numBig = 0;
  if ((rc = read_back(&numBig, bigCount, 1, s))) return rc;
  if (numBig) {
    // cells with more entries than the device search keeps in registers: the same search
    // on the host, over their entries' radial extents
    std::vector<uint32_t> big(numBig);
    if ((rc = read_back(big.data(), bigList, numBig, s))) return rc;
    std::sort(big.begin(), big.end());
    for (uint32_t c : big) {
      uint32_t se[2];
      if ((rc = read_back(se, offsets + c, 2, s))) return rc;
      const size_t m = se[1] - se[0];
      float2 *tmp;
      BHIP(S.alloc(&tmp, m));
      hipLaunchKernelGGL(k_gather_rng, dim3(grid_for(m)), dim3(256), 0, s, pv2 + se[0], m, rng, tmp);
      std::vector<float2> h(m);
      if ((rc = read_back(h.data(), tmp, m, s))) return rc;
      S.release(tmp);
      std::vector<float> h0(m), hN(m), cand(m);
      for (size_t k = 0; k < m; ++k) h0[k] = h[k].x, hN[k] = h[k].y;
      const HostEntries en{h0, hN};
      double rmin, rmax;
      const int ncand = cell_candidates(en, (int)m, cand.data(), rmin, rmax);
      float e[kMaxEdges] = {0.f, 0.f, 0.f};
      const int ne = choose_edges(en, (int)m, cand.data(), ncand, rmin, rmax, e);
      const float4 E = make_float4(e[0], e[1], e[2], u2f((uint32_t)ne));
      BHIP(hipMemcpyAsync(edges + c, &E, sizeof(E), hipMemcpyHostToDevice, s));
      BHIP(hipStreamSynchronize(s));
    }
  }
  clk.mark("radial edges");
  // --- 8. headers and entry counts
  uint64_t *cellCount, *cellBase;
  BHIP(S.alloc(&cellCount, numCells + 1));
  BHIP(S.alloc(&cellBase, numCells + 1));
  BHIP(hipMemsetAsync(cellCount + numCells, 0, sizeof(uint64_t), s));
  BHIP(hipMalloc((void **)&out.binHdr, (size_t)numCells * kBinHdrWords * sizeof(uint32_t)));
  out.bytes += (size_t)numCells * kBinHdrWords * sizeof(uint32_t);
  hipLaunchKernelGGL(k_cell_header, dim3(nc), dim3(64), 0, s, offsets, numCells, pv2, rng, edges,
                     reinterpret_cast<uint32_t *>(out.binHdr), cellCount);
  BHIP(hipGetLastError());
  if ((rc = exclusive_sum(cellCount, cellBase, numCells + 1, s, S))) return rc;
  uint64_t numFat = 0;
  if ((rc = read_back(&numFat, cellBase + numCells, 1, s))) return rc;
  if (numFat > 0xFFFFFFF0ull) {
    set_error("binned locator too large (%llu entries)", (unsigned long long)numFat);
    return IRT_E_INVALID;
  }
  clk.mark("headers");
  // --- 9. fat entries
  BHIP(hipMalloc((void **)&out.fat, std::max<uint64_t>(numFat, 1) * kFatStride4 * sizeof(float4)));
  out.bytes += std::max<uint64_t>(numFat, 1) * kFatStride4 * sizeof(float4);
  clk.mark("fat entries allocated");
  hipLaunchKernelGGL(k_cell_fill, dim3(nc), dim3(64), 0, s, offsets, numCells, pv2, rng, edges, cellBase,
                     reinterpret_cast<uint32_t *>(out.binHdr), planesF, meta, out.fat);
  BHIP(hipGetLastError());
  BHIP(hipStreamSynchronize(s));
  clk.mark("fat entries");
  out.entries = numPairs;
  out.binEntries = numFat;
  out.bigCells = numBig;
  return IRT_OK;
}

// ---------------------------------------------------------------- the slot table
// The cells' distinct finite radial edges other than cell 0's (header words 0-2), into a set of
// kSlotSet words (0: empty) by compare-and-swap; *full when more than that
constexpr int kSlotSet = 8;
__global__ void k_slot_edges(const uint32_t *hdr, uint32_t numCells, uint32_t *set, uint32_t *full) {
  const uint32_t r0 = hdr[0], r1 = hdr[1], r2 = hdr[2];
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < numCells; c += gridDim.x * blockDim.x) {
    const uint32_t *H = hdr + (size_t)c * kBinHdrWords;
    for (int j = 0; j < kMaxEdges; ++j) {
      const uint32_t e = H[j];
      if (e == r0 || e == r1 || e == r2 || __builtin_isinf(__uint_as_float(e))) continue;
      bool in = false;
      for (int q = 0; q < kSlotSet && !in; ++q) {
        const uint32_t old = atomicCAS(&set[q], 0u, e);
        in = old == 0u || old == e;
      }
      if (!in) atomicOr(full, 1u);
    }
  }
}

// one thread per slot (cell, slot unit of `subs` sub-cells, table bin); *bad when a bin's unmasked
// candidates do not fit the slot's 24-bit count
__global__ void k_slot_fill(const uint32_t *hdr, const float *fat, uint32_t numCells, float u0, float u1, float u2,
                            int ne, int subs, float4 *slots, uint32_t *bad) {
  const int bins = ne + 1;
  const int units = kSubCells * kSubCells / subs;
  const float U[kMaxEdges] = {u0, u1, u2};
  const uint64_t total = (uint64_t)numCells * units * bins;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i % bins);
    const uint64_t cu = i / bins;
    const int u = (int)(cu % units);
    const uint64_t c = cu / units;
    float S[4 * kSlot4];
    slot_fill(hdr + c * kBinHdrWords, fat, u, b, U, ne, subs, S);
    if ((__float_as_uint(S[16]) & 0xFFFFFFu) == 0xFFFFFFu) atomicOr(bad, 1u);
    float4 *o = slots + i * kSlot4;
    for (int k = 0; k < kSlot4; ++k) o[k] = make_float4(S[4 * k], S[4 * k + 1], S[4 * k + 2], S[4 * k + 3]);
  }
}

int build_slots_device(const uint32_t *hdr, const float4 *fat, uint32_t numCells, size_t maxBytes, int subs,
                       size_t autoBytes, hipStream_t s, SlotTable &out) {
  out = SlotTable{};
  if (numCells == 0) return IRT_OK;
  uint32_t e[3];
  int rc;
  if ((rc = read_back(e, hdr, 3, s))) return rc;
  Scratch S;
  uint32_t *set;
  BHIP(S.alloc(&set, kSlotSet + 1));
  BHIP(hipMemsetAsync(set, 0, (kSlotSet + 1) * sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_slot_edges, dim3(grid_for(numCells)), dim3(256), 0, s, hdr, numCells, set, set + kSlotSet);
  BHIP(hipGetLastError());
  uint32_t h[kSlotSet + 1];
  if ((rc = read_back(h, set, kSlotSet + 1, s))) return rc;
  if (h[kSlotSet]) {  // more distinct edges than the set holds
    out.skipped = "the cells' radial edges are more than three values";
    return IRT_OK;
  }
  // the table's edges: cell 0's and the others', distinct and ascending
  std::vector<float> U;
  for (int j = 0; j < kMaxEdges; ++j)
    if (!__builtin_isinf(u2f(e[j]))) U.push_back(u2f(e[j]));
  for (int q = 0; q < kSlotSet; ++q)
    if (h[q]) U.push_back(u2f(h[q]));
  std::sort(U.begin(), U.end(), [](float a, float b) { return float_key(a) < float_key(b); });
  U.erase(std::unique(U.begin(), U.end(), [](float a, float b) { return f2u(a) == f2u(b); }), U.end());
  if ((int)U.size() > kMaxEdges) {
    out.skipped = "the cells' radial edges are more than three values";
    return IRT_OK;
  }
  const int ne = (int)U.size(), bins = ne + 1;
  while ((int)U.size() < kMaxEdges) U.push_back(__builtin_inff());
  // sub-cells per slot unit: as asked, or (0) the finest unit whose table is at most autoBytes
  auto table_bytes = [&](int u) { return (size_t)numCells * (kSubCells * kSubCells / u) * bins * kSlot4 * sizeof(float4); };
  if (subs != 1 && subs != 2 && subs != 4) {
    subs = 4;
    for (int u : {1, 2})
      if (table_bytes(u) <= autoBytes && table_bytes(u) <= maxBytes) {
        subs = u;
        break;
      }
  }
  const size_t bytes = table_bytes(subs);
  if (bytes > maxBytes) {
    out.skipped = "the table exceeds its memory cap (IRT_SLOTS_MAX_GB; default half the device's memory, and its free memory less 16 GiB)";
    return IRT_OK;
  }
  float4 *slots = nullptr;
  if (hipMalloc((void **)&slots, bytes) != hipSuccess) {
    (void)hipGetLastError();  // not enough memory: the scene renders without the table
    out.skipped = "hipMalloc of the table failed";
    return IRT_OK;
  }
  hipLaunchKernelGGL(k_slot_fill, dim3(std::min<uint64_t>(grid_for(bytes / (kSlot4 * sizeof(float4))), 1u << 20)),
                     dim3(256), 0, s, hdr, reinterpret_cast<const float *>(fat), numCells, U[0], U[1], U[2], ne, subs,
                     slots, set + kSlotSet);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
    (void)hipFree(slots);
    set_error("slot table build failed");
    return IRT_E_HIP;
  }
  if ((rc = read_back(h, set, kSlotSet + 1, s))) {
    (void)hipFree(slots);
    return rc;
  }
  if (h[kSlotSet]) {  // (never at any scene size this library has seen)
    (void)hipFree(slots);
    out.skipped = "a radial bin's list exceeds the slot's 24-bit count";
    return IRT_OK;
  }
  out.slots = slots;
  out.bins = bins;
  out.subs = subs;
  out.bytes = bytes;
  for (int k = 0; k < kMaxEdges; ++k) out.edges[k] = U[k];
  return IRT_OK;
}

}  // namespace irt
