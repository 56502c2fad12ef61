// irt_render.hip -- the hot path: the raygens woodcockTrackingWithAccel and
// woodcockTrackingAE (icon_rt/deviceCode.cu:239-341) as one gfx950 kernel.
//
// Mapping: one lane per pixel, one wave64 per 8x8 pixel packet (neighbouring rays visit
// the same cube-map cells, fat entries and majorants), a 256-thread workgroup per 16x16
// block, 16 workgroups per 64x64 frame tile -- the unit the reference's CPU parallel_for
// hands out (common/for_each.h:70-85) and the unit of the multi-GPU frame split.
//
// Where the time goes (profiles/): the kernel is a chain of dependent gathers per
// Woodcock sample -- cube-map cell header -> fat candidate entry -> height/value block --
// plus the VALU of the ray setup.  Design choices that follow from that:
//   * the binned locator (irt_common.h): a sample costs ~3 round trips instead of ~10;
//   * one Woodcock call site (the locate code is inlined once), counters aggregated per
//     wave in LDS, coarse height keys fetched only after the plane tests pass: fewer live
//     VGPRs, so more waves per SIMD hide the gathers;
//   * the sdda exit-point toSpherical (two glibc-exact asinf/atan2f) is evaluated only
//     when a later range can still read the RNG state it drives (see below).
//
// Bit-exactness: irt_common.h / irt_device.h and DESIGN.md section 3.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "irt_device.h"

namespace irt {

enum : int {
  OPT_WEDGE = 16384,  // CUBQL / TRIANGLE samplers (locate_wedge, locate_tri); kept out of
                      // the default kernels
  OPT_GRID = 8192,    // GRID_ACCEL_MODE traversal (render_grid); likewise
  OPT_STATS = 32768,  // per-wave statistics into counters[5..15] (measurement only; with the
                      // cooperative loop [7] entry hops, [8] locate rounds, [12..15] samples by
                      // candidates tested 0/1/2/>=3)
  OPT_SERIAL = 65536, // one lane per ray through the Woodcock loop (render_pixel), for A/B:
                      // the default user-geometry/sphere kernel is render_pixel_coop
  OPT_SCAN1 = 131072, // the cooperative loop with each lane's candidate scan on its own
                      // (locate), for A/B against Tracer::locate_wave
  OPT_TIMING = 524288,  // measurement only: per-wave shader-clock time by region into
                        // counters[5..15] (Tracer::tmark)
  OPT_HDRLDS = 1048576, // (A/B) the wave-wide scan's cube-map cell headers staged through LDS:
                        // each distinct header line of the wave's samples loaded once,
                        // cooperatively, then read from LDS (Tracer::stage_headers)
  OPT_DEALALL = 8388608,  // (A/B) the wave-wide scan deals out every candidate, the lists' first
                          // ones included (Tracer::locate_wave)
  OPT_WAVEWG = 4194304,   // (A/B, with OPT_LEAN) one wave per workgroup: a wave's LDS is freed as
                          // soon as it finishes, instead of when its workgroup's last wave does
  OPT_LEAN = 2097152,   // (A/B) less LDS per workgroup (31.0 -> 24 KB), so that more workgroups
                        // fit a CU while finished waves wait for their workgroup's last one:
                        // the sRGB thresholds and the sphere hash read from global memory
                        // (L1/L2), the accum pixel loaded at the end instead of prefetched
  OPT_QUEUE = 16777216,  // the persistent launch (RenderArgs::queue): every resident wave pulls
                        // 8x8-pixel packets from the launch's counter; its own instantiation
                        // of the default kernel (k_render's grid launch is unchanged)
  OPT_FASTSPH = 33554432,  // (A/B) the sdda entry/exit cells from the certified fast lat/lon
                           // (irt_device.h spherical_fast, glibc-exact fallback near cell edges):
                           // no gain at C3, C5 3 % slower (profiles/r04b/) -- the setup waits on
                           // the majorant gather, not on asinf/atan2f
  OPT_NEXTHDR = 134217728,  // (A/B) solo rounds after a wave's first: each lane also loads the
                            // cube-map header line of its ray's next sample (the one taken if
                            // this sample is located and rejected), in the same batch as this
                            // sample's header, so that the next round's header read hits L2
  OPT_WAVEWG2 = 536870912,  // (A/B, with OPT_LEAN) two-wave workgroups: a block's packets in pairs
                            // (each pair sharing a CU's L1), a slot freed per two waves
  OPT_SPLIT = 8,  // measured-cost work items (RenderArgs::splitList): the launches of a single frame
                  // that split packets run this instantiation of the default kernels (kernel_for)
  OPT_ACCPF = 16,  // (A/B, with OPT_LEAN) a single frame's (or a chain's first frame's) accum pixel
                   // fetched into LDS by LDS-DMA at the wave's start, not loaded at the ray's end
  OPT_DPPSCAN = 32,  // (A/B) groups of 2, 4, 16 and 64 lanes take the round's prefix t0 - d0 - ... - dk
                     // by DPP steps across lanes (woodcock_wave), not each lane from LDS
  OPT_XPAIR = 64,  // (A/B, one-wave workgroups) an XCD's two blocks of a 64x64 tile vertically
                   // adjacent (a 16x32-pixel region) instead of two block rows apart
  OPT_DMATAB = 67108864,  // (A/B) one-wave workgroups: the LCG jump and logf tables loaded into
                          // LDS by LDS-DMA, not waited for in the prologue (k_render)
  OPT_NOMISS = 262144,  // (A/B) the user-geometry cooperative loop without its miss mode:
                        // every sample outside all cells ends its ray's round (round 4's
                        // default); convert_icon terrain leaves voids under land, where such runs
                        // cost one round per miss
  OPT_PAIR = 268435456,  // (A/B) the wave-wide scan's first step tests each lane's first two
                         // candidates (both entries gathered together), so the dealt-out step
                         // runs only for lanes whose first two fail
  OPT_VOIDLOC = 1073741824,  // the solo lanes' void walk also in located mode: a certain miss at
                             // the round's sample switches the ray to miss mode there, not a round
                             // later; scenes with holes run it since round 6 (scene_variant:
                             // profiles/r06zg/ C3t chained -1.7 %, single frames even)
  OPT_FPAIR = 1,  // (A/B) chained launches: a wave renders its packet for two consecutive frames,
                  // one after the other (k_render: workgroup (b, y) frames 2y and 2y + 1): the second
                  // frame's hand-off is the wave's own.  (Until profiles/r06f this bit was OPT_CHAINPF,
                  // a chained frame's accum pixel by LDS-DMA at the box test: +6 % from its 1 KB of
                  // LDS, profiles/r06f/ and r06n/.)
  OPT_NOVOIDRUN = 2,   // (A/B) the miss-mode kernels without the solo lanes' void walk (woodcock_wave)
  OPT_NOHOLESKIP = 4,  // (A/B) the miss-mode kernels without the quad-bound miss test (Tracer::locate_wave:
                       // a sample outside its quad's radial range is outside every cell, no
                       // candidate tested)
  OPT_SLOT = 128,  // the wave-wide scan starts from the slot table (RenderArgs::slots, irt_common.h
                   // kSlot4): the first admitted candidate and the list's position in one gather,
                   // instead of the header, then the entry; launches on a scene with a table run
                   // this instantiation of the default kernels (kernel_for)
  // bits 8-11: minimum waves per SIMD asked of the register allocator (0: none)
};

// cube-map cell of a sample point, and its sub-cell (irt_build.h).  The lists are
// rasterised with 1e-5 padding in face coordinates, so the hardware reciprocal (1 ulp) is
// exact enough: any (sub-)cell it picks lists every record that can contain the point.
// The kSubCells-times finer index is exact scaling by a power of two: its cell is the
// coarse grid's cell.
__device__ __forceinline__ uint32_t cubemap_cell_fast(float px, float py, float pz, int G,
                                                      uint32_t &sub) {
  const float ax = __builtin_fabsf(px), ay = __builtin_fabsf(py), az = __builtin_fabsf(pz);
  uint32_t face;
  float num0, num1, den;
  if (ax >= ay && ax >= az) {
    face = px >= 0.f ? 0u : 1u;
    num0 = py;
    num1 = pz;
    den = ax;
  } else if (ay >= az) {
    face = py >= 0.f ? 2u : 3u;
    num0 = px;
    num1 = pz;
    den = ay;
  } else {
    face = pz >= 0.f ? 4u : 5u;
    num0 = px;
    num1 = py;
    den = az;
  }
  const float inv = __builtin_amdgcn_rcpf(den);
  const int GS = opaque_u(G) * kSubCells;
  const float fg = 0.5f * (float)GS;
  int i = (int)((num0 * inv + 1.f) * fg);
  int j = (int)((num1 * inv + 1.f) * fg);
  i = i < 0 ? 0 : (i >= GS ? GS - 1 : i);
  j = j < 0 ? 0 : (j >= GS ? GS - 1 : j);
  sub = (uint32_t)((j & (kSubCells - 1)) * kSubCells + (i & (kSubCells - 1)));
  return face * (uint32_t)G * (uint32_t)G + (uint32_t)(j / kSubCells) * (uint32_t)G +
         (uint32_t)(i / kSubCells);
}
__device__ __forceinline__ uint32_t cubemap_cell_fast(float px, float py, float pz, int G) {
  uint32_t sub;
  return cubemap_cell_fast(px, py, pz, G, sub);
}

// Per-wave LDS of the cooperative Woodcock loop (Tracer::woodcock_wave).
struct CoopWave {
  float4 req[64];   // the request of the rank-r ray: {t, tmax, q = majorant/unitDistance, majorant}
  float4 ray[64];   // {dx, dy, dz, RNG state bits}
  float step[64];   // lane l's Woodcock step log(1 - xi)/q this round
  uint32_t cnt[64]; // the request is counted (a positive-length leaf)
};
// Per-wave LDS of Tracer::locate_wave's candidate scan
struct ScanWave {
  float4 pt[64];    // lane l's sample {point, r}
  uint4 lst[64];    // its candidate list {first entry, sub-cell mask, next position, record limit}
};
// OPT_HDRLDS: up to kHdrStage distinct header lines of a wave's samples, staged in LDS
constexpr int kHdrStage = 8;
struct HdrStage {
  uint32_t cell[kHdrStage];
  uint32_t w[kHdrStage][kBinHdrWords];
};

// t0 - d[0] - d[1] - ... - d[k], subtracted one at a time as woodcockTracking's `t -=`
// (deviceCode.cu:165) does: the same roundings as k+1 iterations of the serial loop.
typedef float fvec2 __attribute__((ext_vector_type(2)));
typedef float fvec4 __attribute__((ext_vector_type(4)));
// 16-byte LDS slots read and written as one ds_read_b128 / ds_write_b128: HIP's float4 and
// uint4 copy member-wise in IR, and with the IR load/store vectorizer off for this file
// (Makefile RENDER_FLAGS) they would split into b32 pairs.
template <class T>
__device__ __forceinline__ T lds_ld16(const T *p) {
  static_assert(sizeof(T) == 16, "16-byte slot");
  return __builtin_bit_cast(T, *reinterpret_cast<const fvec4 *>(p));
}
typedef uint32_t uvec2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 lds_ld8(const uint2 *p) {
  return __builtin_bit_cast(uint2, *reinterpret_cast<const uvec2 *>(p));
}
template <class T>
__device__ __forceinline__ void lds_st16(T *p, T v) {
  static_assert(sizeof(T) == 16, "16-byte slot");
  *reinterpret_cast<fvec4 *>(p) = __builtin_bit_cast(fvec4, v);
}
// The group's steps are read as explicit 4- / 2-float LDS vectors (the group base is a
// multiple of G floats), independent of the IR load/store vectorizer (off for this file).
template <int G>
__device__ __forceinline__ float coop_prefix(float t0, const float *d, int k) {
  float t = t0;
  if constexpr (G == 2) {
    const fvec2 v = *static_cast<const fvec2 *>(__builtin_assume_aligned(d, 8));
    t = t - v.x;
    t = k >= 1 ? t - v.y : t;
  } else {
#pragma unroll
    for (int c = 0; c < G / 4; ++c) {
      const fvec4 v = static_cast<const fvec4 *>(__builtin_assume_aligned(d, 16))[c];
      t = 4 * c <= k ? t - v.x : t;
      t = 4 * c + 1 <= k ? t - v.y : t;
      t = 4 * c + 2 <= k ? t - v.z : t;
      t = 4 * c + 3 <= k ? t - v.w : t;
    }
  }
  return t;
}

// The same prefix by DPP steps across the lanes of groups of G = 2, 4, 16 or 64 (OPT_DPPSCAN):
// lane k starts at t0 - d_k (final for k = 0), and step s sets y_k = y_{k-1} - d_k, so that after
// step s the lanes k <= s hold ((t0 - d0) - d1) - ... - dk, subtracted in the serial loop's order.
// A group's first lane reads itself (quad_perm) or has no source lane (row_shr / wave_shr with
// bound_ctrl off: the old value) and subtracts +0, which leaves every float as it is.
template <int G>
__device__ __forceinline__ float dpp_prefix(float t0, float dk, int k) {
  static_assert(G == 2 || G == 4 || G == 16 || G == 64, "DPP prefix: groups of 2, 4, 16, 64");
  constexpr int ctrl = G == 2 ? 0xA0 : G == 4 ? 0x90 : G == 16 ? 0x111 : 0x138;  // quad_perm [0,0,2,2] /
                                                                                // [0,0,1,2], row_shr:1,
                                                                                // wave_shr:1
  const float e = k == 0 ? 0.f : dk;
  float y = t0 - dk;
#pragma unroll
  for (int s = 1; s < G; ++s) {
    const float prev = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, y),
                                                                             __builtin_bit_cast(int, y), ctrl, 0xf,
                                                                             0xf, false));
    y = prev - e;
  }
  return y;
}

// Measurement only, the probe build (profiles/build_probe_lib.sh, -DIRT_PROBE_BUILD):
// IRT_PROBE_EXIT 8..13 end the first
// woodcockFunc call inside its first round -- 8 after the samples' positions, 9 after the
// header and bin, 10 after the first candidate test, 11 after the dealt-out candidates, 12 after
// locate_wave (getValue included), 13 at the round's end -- so that the SQ counters of runs
// with each exit give the instructions of every piece of a round (profiles/r06m_gpu.sh)
#ifdef IRT_PROBE_BUILD
#define IRT_ROUND_PROBE(n, ...) \
  if (A.probeExit == (n)) return __VA_ARGS__;
#else
#define IRT_ROUND_PROBE(n, ...)
#endif

// OPT_TIMING's per-wave region clocks (Tracer::tmark); empty in every other kernel
struct TimeAccOff {};
struct TimeAccOn {
  static constexpr int kTimeRegions = 9;
  uint64_t tLast = 0, tAcc[kTimeRegions] = {};
};

// The camera of frame `frame` of a launch: the launch's own, or in a sequence of views
// (RenderArgs::frameCams, irt_render_sequence) that frame's words, read through the constant
// address space (scalar loads: uniform values, written by the host before the launch).
typedef const __attribute__((address_space(4))) fvec4 *CamWords;
// a uniform word of a host-written table (tile lists, block orders) through the scalar unit: a
// vector load's wait would also wait for every vector load before it (the counter retires in
// order), the prologue's LDS-DMA table loads included
typedef const __attribute__((address_space(4))) uint32_t *ScalarWords;
__device__ __forceinline__ uint32_t scalar_word(const void *table, uint32_t i) {
  return ((ScalarWords)table)[i];
}
__device__ __forceinline__ float4 cam_word(const RenderArgs &A, int frame, int k) {
  return __builtin_bit_cast(float4, ((CamWords)A.frameCams)[4 * frame + k]);
}
__device__ __forceinline__ float3 cam_org(const RenderArgs &A, int frame) {
  if (A.frameCams) {
    const float4 w = cam_word(A, frame, 0);
    return make_float3(w.x, w.y, w.z);
  }
  return A.org;
}
// the frame's accumID (deviceCode.cu:288-289): accumID + frame in a progressive batch
__device__ __forceinline__ int cam_accum_id(const RenderArgs &A, int frame) {
  if (A.frameCams) return (int)__float_as_uint(cam_word(A, frame, 0).w);
  return A.accumID + frame;
}

// The ray's per-lane state machine reads RenderArgs through fresh_args(): k_render's only
// argument reached through a pointer the compiler cannot follow, so the fields it uses are
// loaded (scalar loads, scalar-cache hits) where it uses them instead of held in SGPRs -- or
// spilled to VGPR lanes -- through the Woodcock rounds; so does the ray's end (chain wait, pixel
// write).  108 -> 65 spilled SGPRs on flat grids, 120 -> 87 and no scratch over terrain; C3
// -1.5 %, C3t -2.4 % (one launch per frame -4.3 %), C3s -0.6 %, C5 even (profiles/r06s/, r06t/).
// The Tracer's late reads (classify_alpha, record_value, sphere_at, the sphere test) too: 62 and
// 73 spilled SGPRs, C3t -1.2 %, C5 -0.9 %, C3 and C3s even (profiles/r06v/; -DIRT_HELD_LATE
// reads them through Ap).  -DIRT_HELD_ARGS builds the held form for A/B.
#ifndef IRT_HELD_ARGS
__device__ __forceinline__ const RenderArgs &fresh_args() {
  typedef const __attribute__((address_space(4))) RenderArgs *KArgs;
  KArgs kp = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(kp));
  return *(const RenderArgs *)kp;
}
#define IRT_SM_ARGS fresh_args()
#else
#define IRT_SM_ARGS A
#endif
// IRT_FRESH_TRACER (A/B build): each woodcockFunc call re-reads the arguments the Tracer uses
// through fresh_args(), so they are live during the call only, not through the state machine
#if defined(IRT_FRESH_TRACER) && !defined(IRT_HELD_ARGS)
#define IRT_TR_ARGS (&fresh_args())
#else
#define IRT_TR_ARGS (&A)
#endif

template <int OPT>
struct Tracer : std::conditional_t<(OPT & OPT_TIMING) != 0, TimeAccOn, TimeAccOff> {
  const RenderArgs &A;
  const LogfTab *s_logf;
  const uint32_t *s_sph;
  uint32_t *s_cnt;  // [0] launched [1] inBox [2] locate [3] found [4] candidates
  Counts cnt;       // per-lane statistics (OPT_STATS)
  uint32_t specCand = 0;  // candidate tests of this lane's sample in a cooperative round
  const uint32_t *s_gbits = nullptr;  // OPT_GRID: the grid's empty-space bitmap in LDS
  // the cooperative loop's statistics, per lane (samples taken, their locates / found /
  // candidate tests), added into s_cnt at the end by flush_coop
  uint32_t nLocate = 0, nFound = 0, nCand = 0;
  int frame = 0;  // the launch's frame this wave renders (its camera: cam_org)
  const RenderArgs *Ap = &A;  // the arguments its methods read (IRT_TR_ARGS: re-read per call)
  // OPT_TIMING: shader clocks per region (wave-uniform), in the TimeAcc base
  __device__ __forceinline__ void tmark(int region) {
    if constexpr ((OPT & OPT_TIMING) != 0) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      this->tAcc[region] += now - this->tLast;
      this->tLast = now;
    }
  }

  // wave sum of a per-lane count: the DPP prefix sum's last lane (wave_incl_sum)
  __device__ __forceinline__ static uint32_t wave_sum(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(v), 63);
  }
  // inclusive prefix sum over the wave's 64 lanes in six DPP adds (row shifts within rows of
  // 16, then the row broadcasts), no LDS round trips
  __device__ __forceinline__ static uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
  }
  __device__ __forceinline__ void flush_coop() {
    const uint32_t a = wave_sum(nLocate), b = wave_sum(nFound), c = wave_sum(nCand);
    if (__lane_id() == 0) {
      if (a) atomicAdd(&s_cnt[2], a);
      if (b) atomicAdd(&s_cnt[3], b);
      if (c) atomicAdd(&s_cnt[4], c);
    }
  }

  // the cooperative Woodcock loop (woodcock_wave) runs in every kernel (any sampler, either
  // accelerator) but the OPT_SERIAL comparison one
  static constexpr bool kCoop = (OPT & OPT_SERIAL) == 0;
  // the miss mode of woodcock_wave: after a sample outside every cell, a ray's next round
  // places its samples as if none were located, until one is.  Misses come in runs wherever
  // the volume has holes: the unstructured samplers' gaps, the grid accel's empty cells, and
  // in the user-geometry sampler the voids convert_icon leaves under land (a column's first
  // record starts at R + HSURF, convert_icon.cpp:361: nothing covers [R, R + HSURF)) -- at C3t a
  // third of the samples miss, in runs of up to ~280 draws, and without the miss mode every
  // miss cost its ray a round (single-frame launches 1.07 ms against 0.09 ms at C3, a few
  // waves running ~1 ms: profiles/r05d_missmode/).  Flat grids almost never miss (C3: 707 of 1.01 M
  // samples).  The kernels with misses everywhere (wedges, grid) start with whole-wave groups.
  static constexpr bool kMiss = kCoop && (OPT & OPT_NOMISS) == 0;
  // the void walk of woodcock_wave's solo miss-mode lanes (the user-geometry sampler from headers)
  static constexpr bool kVoidRun =
      kMiss && (OPT & (OPT_WEDGE | OPT_GRID | OPT_SCAN1 | OPT_SLOT | OPT_HDRLDS | OPT_NOHOLESKIP | OPT_NOVOIDRUN)) == 0;
#ifndef IRT_VOID_RUN_MAX
#define IRT_VOID_RUN_MAX 32  // (A/B builds may set it)
#endif
  static constexpr int kVoidRunMax = IRT_VOID_RUN_MAX;  // samples one lane walks before the round goes on
  static constexpr bool kWideStart = (OPT & (OPT_WEDGE | OPT_GRID)) != 0;

  // one wave-aggregated LDS add per event site
  __device__ __forceinline__ void count(int k) {
    const unsigned long long m = __ballot(1);
    if (__lane_id() == (unsigned)(__ffsll((long long)m) - 1)) atomicAdd(&s_cnt[k], (uint32_t)__popcll(m));
  }

  // findHeight (ICONGrid.h:117-145) literally, over a record's blocks; getValue (147-164)
  __device__ __forceinline__ float find_value_literal(const float4 *B, int nl, float r) {
    const float *Bf = reinterpret_cast<const float *>(B);
    int first = 0, count = nl;
    while (count > 0) {
      const int stp = count / 2, it = first + stp;
      if (!(r <= Bf[blk_height_pos(it + 1)])) {
        first = it + 1;
        count -= stp + 1;
      } else {
        count = stp;
      }
    }
    return Bf[blk_value_pos(first)];
  }

  // sample()'s point test (ICONGrid.h:184, 197-203) on one fat entry {p0, p1, p2, m}:
  // the radial range and the three ccw side planes
  __device__ __forceinline__ bool pass_fat(const float4 &p0, const float4 &p1, const float4 &p2,
                                           const float4 &m, float px, float py, float pz, float r) {
    if constexpr (kCoop)
      ++specCand;  // counted only if the sample is one the reference takes (woodcock_wave)
    else
      count(4);
    if (r < m.x || r > m.y) return false;                                 // ICONGrid.h:184
    if (dot3(px, py, pz, p0.x, p0.y, p0.z) - p0.w > 0.f) return false;  // ICONGrid.h:201
    if (dot3(px, py, pz, p1.x, p1.y, p1.z) - p1.w > 0.f) return false;  // 202
    if (dot3(px, py, pz, p2.x, p2.y, p2.z) - p2.w > 0.f) return false;  // 203
    return true;
  }

  // The record a point test found: index and its getValue path at the sample's radius
  // (irt_common.h record_path: numLayers, which 64-B block, or the literal search).
  struct Found {
    uint32_t rec, path;
  };

  // First entry of fat entries [q, qe) whose point test passes, among records < limit:
  // of the first kMaskCand entries only those whose bit is set in `mask` (the candidates
  // that can reach the sample's sub-cell, irt_build.h), then every later one.  Only the
  // point test runs in the (lane-divergent) loop; getValue's gathers come after.
  __device__ __forceinline__ bool scan_fat(uint32_t q, uint32_t qe, uint32_t mask, uint32_t limit,
                                           float px, float py, float pz, float r, Found &f) {
    const uint32_t n = qe - q;
    for (uint32_t j = 0;; ++j) {
      if (j < (uint32_t)kMaskCand) {
        const uint32_t m = mask >> j;
        j = m ? j + (uint32_t)__builtin_ctz(m) : (uint32_t)kMaskCand;
      }
      if (j >= n) break;
      const float4 *F = (*Ap).fat + (size_t)(q + j) * kFatStride4;
      const float4 a0 = F[0], a1 = F[1], a2 = F[2], am = F[3];
      if (__float_as_uint(am.z) >= limit) return false;
      if (pass_fat(a0, a1, a2, am, px, py, pz, r)) {
        f = {__float_as_uint(am.z), record_path(__float_as_uint(am.w), am.x, am.y, r)};
        return true;
      }
    }
    return false;
  }

  // getValue (ICONGrid.h:147-164) of the found record at radius r: sorted heights take the
  // 64-B height/value block the quantised keys pick (one gather; r within a unit of a key:
  // the exact keys from the record's lines first), others the literal binary search
  __device__ __forceinline__ float record_value(const Found &f, float r) {
#if !defined(IRT_HELD_ARGS) && !defined(IRT_HELD_LATE)
    const RenderArgs &LA = fresh_args();  // read where used (-DIRT_HELD_LATE: through Ap)
#else
    const RenderArgs &LA = *Ap;
#endif
    const int nl = (int)(f.path & 31u);
    const float4 *B = LA.blocks + (size_t)f.rec * kBlk4;
    if (f.path & kPathBlock) {
      int b = (int)((f.path >> 5) & 3u);
      if (f.path & kPathExactKeys) {
        const float *Bf = reinterpret_cast<const float *>(B);
        b = rec_coarse_block(Bf[blk_height_pos(7)], Bf[blk_height_pos(15)], Bf[blk_height_pos(23)],
                             __builtin_inff(), nl, r);  // height[31] = hN >= r never counts
      }
      const float4 *Q = B + 4 * b;
      const float4 h0 = Q[0], h1 = Q[1], v0 = Q[2], v1 = Q[3];
      const int k = rec_block_index(h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, b, nl, r);
      return select8(k, v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w);
    }
    return find_value_literal(B, nl, r);
  }

  // A zero-thickness record at exactly radius r (a sphere, host/irt_scene.cpp), if any:
  // the lowest such record and its getValue.
  __device__ __forceinline__ bool sphere_at(float r, float &value, uint32_t &rec) {
#if !defined(IRT_HELD_ARGS) && !defined(IRT_HELD_LATE)
    const RenderArgs &LA = fresh_args();  // read where used (-DIRT_HELD_LATE: through Ap)
#else
    const RenderArgs &LA = *Ap;
#endif
    uint32_t lo = 0, hi = LA.numSph;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (LA.sphR[mid] < r) lo = mid + 1;
      else hi = mid;
    }
    if (lo >= LA.numSph || !(LA.sphR[lo] == r)) return false;
    const uint2 q = LA.sphRec[LA.sphOff[lo]];
    value = find_value_literal(LA.blocks + (size_t)q.x * kBlk4, (int)q.y, r);
    rec = q.x;
    return true;
  }

  // sampleVolume (deviceCode.cu:58-125) over the binned lists (irt_common.h): the first
  // record in index order passing sample() -- the reference's linear scan's answer
  // (116-123).
  // CUBQL_MODE sampleVolume (deviceCode.cu:90-115) over the wedge locator: the first wedge
  // in (record, layer) order whose primBounds (hostCode.cu:534-552) contain the point and
  // whose intersectWedgeEXT (UElems.h:214-311) accepts it.  Wedges are rebuilt in
  // registers from the record's corner trig and heights exactly as buildCuBQLAccel makes
  // them (hostCode.cu:557-590); a record's union box rejects it first.
  __device__ __forceinline__ bool locate_wedge(float px, float py, float pz, float &value) {
    const uint32_t cell = cubemap_cell_fast(px, py, pz, (*Ap).wG);
    const uint32_t qe = (*Ap).wOff[cell + 1];
    for (uint32_t q = (*Ap).wOff[cell]; q < qe; ++q) {
      const uint32_t rec = (*Ap).wRec[q];
      const float4 lo = (*Ap).wBox[2 * (size_t)rec], hi = (*Ap).wBox[2 * (size_t)rec + 1];
      if (!(lo.x <= px && px <= hi.x && lo.y <= py && py <= hi.y && lo.z <= pz && pz <= hi.z))
        continue;
      const int nl = (int)__float_as_uint(lo.w);
      const float4 t0 = (*Ap).wTrig[3 * (size_t)rec], t1 = (*Ap).wTrig[3 * (size_t)rec + 1],
                   t2 = (*Ap).wTrig[3 * (size_t)rec + 2];
      const float4 *B = (*Ap).blocks + (size_t)rec * kBlk4;
      const float *Bf = reinterpret_cast<const float *>(B);
      for (int h = 0; h < nl; ++h) {
        const float hb = Bf[blk_height_pos(h)], ht = Bf[blk_height_pos(h + 1)];
        WV4 V[6];
        V[0] = {(hb * t0.x) * t0.z, (hb * t0.x) * t0.w, hb * t0.y, 0.f};
        V[1] = {(hb * t1.x) * t1.z, (hb * t1.x) * t1.w, hb * t1.y, 0.f};
        V[2] = {(hb * t2.x) * t2.z, (hb * t2.x) * t2.w, hb * t2.y, 0.f};
        V[3] = {(ht * t0.x) * t0.z, (ht * t0.x) * t0.w, ht * t0.y, 0.f};
        V[4] = {(ht * t1.x) * t1.z, (ht * t1.x) * t1.w, ht * t1.y, 0.f};
        V[5] = {(ht * t2.x) * t2.z, (ht * t2.x) * t2.w, ht * t2.y, 0.f};
        float bl[3] = {1e31f, 1e31f, 1e31f}, bu[3] = {-1e31f, -1e31f, -1e31f};
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          bl[0] = fminf(bl[0], V[k].x);
          bl[1] = fminf(bl[1], V[k].y);
          bl[2] = fminf(bl[2], V[k].z);
          bu[0] = fmaxf(bu[0], V[k].x);
          bu[1] = fmaxf(bu[1], V[k].y);
          bu[2] = fmaxf(bu[2], V[k].z);
        }
        if (!(bl[0] <= px && px <= bu[0] && bl[1] <= py && py <= bu[1] && bl[2] <= pz && pz <= bu[2]))
          continue;
        // the per-layer scalar (hostCode.cu:571-572) on all six vertices (`#if 1`, 574-577)
        const float bv = h == 0 ? find_value_literal(B, nl, hb)
                                : (find_value_literal(B, nl, Bf[blk_height_pos(h - 1)]) +
                                   find_value_literal(B, nl, hb)) * 0.5f;
#pragma unroll
        for (int k = 0; k < 6; ++k) V[k].w = bv;
        if (intersect_wedge(value, px, py, pz, V)) return true;
      }
    }
    return false;
  }

  // TRIANGLE_MODE sampleVolume (deviceCode.cu:61-76): the ray from the sample toward the
  // Earth's centre against the listed records' bottom triangles (hostCode.cu:445-450),
  // closest front-face hit (ray_triangle, irt_common.h), then its radial range and getValue.
  __device__ __forceinline__ bool locate_tri(float px, float py, float pz, float &value) {
    const float len = sqrtf(dot3(px, py, pz, px, py, pz));
    const float dx = -(px / len), dy = -(py / len), dz = -(pz / len);
    const uint32_t cell = cubemap_cell_fast(px, py, pz, (*Ap).wG);
    const uint32_t qe = (*Ap).wOff[cell + 1];
    float best = __builtin_inff();
    uint32_t hit = 0xFFFFFFFFu;
    for (uint32_t q = (*Ap).wOff[cell]; q < qe; ++q) {
      const uint32_t rec = (*Ap).wRec[q];
      const float4 t0 = (*Ap).wTrig[3 * (size_t)rec], t1 = (*Ap).wTrig[3 * (size_t)rec + 1],
                   t2 = (*Ap).wTrig[3 * (size_t)rec + 2];
      const float h0 = reinterpret_cast<const float *>((*Ap).blocks + (size_t)rec * kBlk4)[blk_height_pos(0)];
      const float v0[3] = {(h0 * t0.x) * t0.z, (h0 * t0.x) * t0.w, h0 * t0.y};
      const float v1[3] = {(h0 * t1.x) * t1.z, (h0 * t1.x) * t1.w, h0 * t1.y};
      const float v2[3] = {(h0 * t2.x) * t2.z, (h0 * t2.x) * t2.w, h0 * t2.y};
      float t;
      if (ray_triangle(px, py, pz, dx, dy, dz, v0, v1, v2, t) && t < best) {
        best = t;
        hit = rec;
      }
    }
    if (hit == 0xFFFFFFFFu) return false;
    const float4 *B = (*Ap).blocks + (size_t)hit * kBlk4;
    const float *Bf = reinterpret_cast<const float *>(B);
    const int nl = (int)__float_as_uint((*Ap).wBox[2 * (size_t)hit].w);
    if (len < Bf[blk_height_pos(0)] || len > Bf[blk_height_pos(nl)]) return false;
    value = find_value_literal(B, nl, len);
    return true;
  }

  __device__ __forceinline__ bool locate(float px, float py, float pz, float &value) {
    if ((*Ap).numCells == 0) return false;
    if constexpr ((OPT & OPT_WEDGE) != 0) {
      if ((*Ap).sampler == IRT_MODE_TRIANGLES) return locate_tri(px, py, pz, value);
      return locate_wedge(px, py, pz, value);
    }
    const float r = sqrtf(dot3(px, py, pz, px, py, pz));  // toSpherical(pos).x
    uint32_t sub;
    const uint32_t cell = cubemap_cell_fast(px, py, pz, (*Ap).G, sub);
    // the cell header's words 0..7 and the sub-cell's mask word: one 128-B line
    const uint4 *Hc = (*Ap).binHdr + (size_t)cell * (kBinHdrWords / 4);
    const uint4 H0 = Hc[0], H1 = Hc[1];
    const uint32_t M = reinterpret_cast<const uint32_t *>(Hc)[8 + sub];
    return locate_hdr(px, py, pz, r, H0, H1, M, value);
  }

  __device__ __forceinline__ bool locate_hdr(float px, float py, float pz, float r, const uint4 &H0,
                                             const uint4 &H1, uint32_t M, float &value) {
    const float e0 = __uint_as_float(H0.x), e1 = __uint_as_float(H0.y), e2 = __uint_as_float(H0.z);
    const int b = bin_of(r, e0, e1, e2);
    // bin b's [beg, end) from the cumulative ends, and its upper edge, selected with masks
    // (a select chain on b becomes a scratch lookup table otherwise)
    const uint32_t m1 = b > 0 ? ~0u : 0u, m2 = b > 1 ? ~0u : 0u, m3 = b > 2 ? ~0u : 0u;
    const uint32_t beg = (m1 & H1.x) + (m2 & (H1.y - H1.x)) + (m3 & (H1.z - H1.y));
    const uint32_t end = H1.x + (m1 & (H1.y - H1.x)) + (m2 & (H1.z - H1.y)) + (m3 & (H1.w - H1.z));
    const uint32_t end2 = H1.y + (m1 & (H1.z - H1.y)) + (m2 & (H1.w - H1.z));
    // r exactly on the bin's upper edge: records starting at that edge sit in the next
    // bin, so a second pass scans it for a lower record (one scan site, two passes)
    const float eb = __uint_as_float(H0.x ^ (m1 & (H0.x ^ H0.y)) ^ (m2 & (H0.y ^ H0.z)));
    const bool onEdge = b < kMaxEdges && r == eb;
    Found f = {0xFFFFFFFFu, 0u};
    bool hit = false;
    uint32_t qb = H0.w + beg, qe = H0.w + end;
    for (int pass = 0; pass < 2; ++pass) {
      Found g;
      if (scan_fat(qb, qe, (M >> (8 * (b + pass))) & 0xFFu, f.rec, px, py, pz, r, g)) {
        f = g;
        hit = true;
      }
      if (!onEdge) break;
      qb = qe;
      qe = H0.w + end2;
    }
    if ((*Ap).numSph) {
      const uint32_t h = sph_hash(r);
      if ((s_sph[h >> 5] >> (h & 31)) & 1u) {
        float v2;
        uint32_t rec2;
        if (sphere_at(r, v2, rec2) && (!hit || rec2 < f.rec)) {
          value = v2;
          return true;
        }
      }
    }
    if (hit) value = record_value(f, r);
    return hit;
  }

  // sampleVolume for every lane of the wave with `want` set (the cooperative loop's locate;
  // all lanes call it).  The same answer as locate: the first candidate of the sample's bin
  // and sub-cell, in record order, passing sample().  But the candidate scan is spread over
  // the wave: every lane first tests its list's first candidate (a quarter of C3's samples
  // fail it: 916,920 / 270,995 / 30,517 samples take 1 / 2 / >=3 tests), then the wave's
  // remaining candidates are dealt out one per lane and tested together, so a round waits
  // for two entry gathers instead of the longest lane's chain (2.96 per round at C3).  The
  // lowest passing candidate of each list wins, as in the serial scan.  Samples exactly on a
  // radial bin edge (the two-bin scan) take locate_hdr's serial path.
  static constexpr bool kWaveScan = kCoop && (OPT & (OPT_WEDGE | OPT_GRID | OPT_SCAN1)) == 0;
  static constexpr bool kPair = kWaveScan && (OPT & OPT_PAIR) != 0;
  __device__ __forceinline__ static bool entry_passes(const float4 &a0, const float4 &a1, const float4 &a2,
                                                     const float4 &am, float px, float py, float pz, float r) {
    return !(r < am.x || r > am.y) && !(dot3(px, py, pz, a0.x, a0.y, a0.z) - a0.w > 0.f) &&
           !(dot3(px, py, pz, a1.x, a1.y, a1.z) - a1.w > 0.f) && !(dot3(px, py, pz, a2.x, a2.y, a2.z) - a2.w > 0.f);
  }
  __device__ __forceinline__ bool pass_entry(const float4 *F, float px, float py, float pz, float r,
                                             Found &f) {
    const float4 a0 = F[0], a1 = F[1], a2 = F[2], am = F[3];
    f = {__float_as_uint(am.z), record_path(__float_as_uint(am.w), am.x, am.y, r)};
    if (r < am.x || r > am.y) return false;                               // ICONGrid.h:184
    if (dot3(px, py, pz, a0.x, a0.y, a0.z) - a0.w > 0.f) return false;  // ICONGrid.h:201
    if (dot3(px, py, pz, a1.x, a1.y, a1.z) - a1.w > 0.f) return false;  // 202
    if (dot3(px, py, pz, a2.x, a2.y, a2.z) - a2.w > 0.f) return false;  // 203
    return true;
  }
  // position p of a candidate list {set bits of m8, ascending} ++ {8, 9, ...} -> entry offset
  __device__ __forceinline__ static uint32_t list_entry(uint32_t m8, uint32_t p) {
    const uint32_t nm = (uint32_t)__popc(m8);
    if (p >= nm) return (uint32_t)kMaskCand + (p - nm);
    for (uint32_t k = 0; k < p; ++k) m8 &= m8 - 1u;
    return (uint32_t)__builtin_ctz(m8);
  }
  // OPT_HDRLDS: the header words 0..7 and word 8+sub of every wanting lane's cube-map cell.
  // The wave's distinct cells (in lane order, at most kHdrStage) get one 128-B line each,
  // loaded by 32 lanes together (a dword per lane) and written to LDS; lanes whose cell is
  // past the kHdrStage-th distinct one load their header directly.
  HdrStage *s_hdr = nullptr;
  __device__ __forceinline__ void stage_headers(bool want, uint32_t cell, uint32_t sub, uint4 &H0, uint4 &H1,
                                                uint32_t &M) {
    const int lane = (int)__lane_id();
    HdrStage &S = s_hdr[0];
    uint64_t todo = __ballot(want);
    int slot = -1, ns = 0;
    while (todo != 0ull && ns < kHdrStage) {
      const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cell, (int)__builtin_ctzll(todo));
      const bool mine = want && cell == c;
      todo &= ~__ballot(mine);
      if (mine) slot = ns;
      if (lane == 0) S.cell[ns] = c;
      ++ns;
    }
    __builtin_amdgcn_wave_barrier();
    // two lines per pass, every pass's loads issued before the LDS writes
    uint32_t v[kHdrStage / 2];
#pragma unroll
    for (int p = 0; p < kHdrStage / 2; ++p) {
      const int k = 2 * p + (lane >> 5);
      v[p] = 0u;
      if (k < ns && (lane & 31) < kBinHdrWords)
        v[p] = reinterpret_cast<const uint32_t *>((*Ap).binHdr)[(size_t)S.cell[k] * kBinHdrWords + (lane & 31)];
    }
#pragma unroll
    for (int p = 0; p < kHdrStage / 2; ++p) {
      const int k = 2 * p + (lane >> 5);
      if (k < ns && (lane & 31) < kBinHdrWords) S.w[k][lane & 31] = v[p];
    }
    __builtin_amdgcn_wave_barrier();
    if (slot >= 0) {
      H0 = lds_ld16(reinterpret_cast<const uint4 *>(&S.w[slot][0]));
      H1 = lds_ld16(reinterpret_cast<const uint4 *>(&S.w[slot][4]));
      M = S.w[slot][8 + sub];
    } else if (want) {
      const uint4 *Hc = (*Ap).binHdr + (size_t)cell * (kBinHdrWords / 4);
      H0 = Hc[0];
      H1 = Hc[1];
      M = reinterpret_cast<const uint32_t *>(Hc)[8 + sub];
    }
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ bool locate_wave(bool want, float px, float py, float pz, float &value,
                                              CoopWave &CW, ScanWave &W, const uint32_t *touch = nullptr) {
    want = want && (*Ap).numCells != 0;
    const int lane = (int)__lane_id();
    // The scan's state lives in the wave's LDS (fewer live VGPRs across it):
    //   W.pt[l]  the sample {point, r} of lane l
    //   W.lst[l] its list {first entry, sub-cell mask, next list position, record limit}
    //   frm[l]   the record found so far: {record, getValue path} (in the round's request
    //            slots CW.ray, free once the round has read them)
    //   W.own[s] the lane whose tasks start at s (W.step, free after the round's prefix)
    uint32_t *own = reinterpret_cast<uint32_t *>(CW.step);
    uint2 *frm = reinterpret_cast<uint2 *>(CW.ray);
    uint32_t c = 0u;
    uint32_t fe = 0u, flim = 0xFFFFFFFFu;  // the pass's first candidate entry, record limit
    float fr = 0.f;                        // the sample's r
    bool hit = false, edge = false;
    uint4 H0 = make_uint4(0u, 0u, 0u, 0u), H1 = H0;
    uint32_t M = 0u, cell = 0u, sub = 0u;
    uint32_t tv = 0u;  // OPT_NEXTHDR's loaded word, consumed after the scan
    uint32_t fe2 = 0u; // OPT_PAIR: the pass's second candidate entry
    constexpr bool kSlot = (OPT & OPT_SLOT) != 0;
    // the quad-bound miss test: scenes with holes (the miss-mode kernels) that start from headers
    constexpr bool kHoleSkip = kMiss && !kSlot && (OPT & (OPT_HDRLDS | OPT_NOHOLESKIP)) == 0;
    static_assert(!kSlot || (OPT & (OPT_HDRLDS | OPT_PAIR | OPT_DEALALL | OPT_NEXTHDR)) == 0, "slot table: the default scan");
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0, s2 = s0, sm = s0;  // OPT_SLOT: the first candidate
    bool slotCopy = false;  // OPT_SLOT: the slot's copy is this sample's first admitted candidate
    if constexpr ((OPT & OPT_HDRLDS) != 0) {
      if (want) cell = cubemap_cell_fast(px, py, pz, (*Ap).G, sub);
      stage_headers(want, cell, sub, H0, H1, M);
    }
    if (kSlot && want) {
      // the slot of the sample's (cell, sub-cell, bin): the bins from the scene's shared edges
      const float r = sqrtf(dot3(px, py, pz, px, py, pz));  // toSpherical(pos).x
      cell = cubemap_cell_fast(px, py, pz, (*Ap).G, sub);
      const float e0 = (*Ap).slotEdge[0], e1 = (*Ap).slotEdge[1], e2 = (*Ap).slotEdge[2];
      const int b = bin_of(r, e0, e1, e2);
      const int subs = (*Ap).slotSubs;
      const uint32_t unit = slot_unit(sub, subs);
      const float4 *S = (*Ap).slots + ((size_t)(cell * ((uint32_t)(kSubCells * kSubCells) >> (subs >> 1)) + unit) * (uint32_t)(*Ap).slotBins + (uint32_t)b) * kSlot4;
      s0 = S[0];
      s1 = S[1];
      s2 = S[2];
      sm = S[3];
      const uint4 info = reinterpret_cast<const uint4 *>(S)[4];
      edge = r == __uint_as_float(info.w);  // the cell's own bin edge (+inf: none)
      // this sub-cell's mask and first admitted candidate; the slot's copy is that candidate when
      // its list position is the unit's first (j_U), otherwise it is gathered from the list
      const uint32_t m8 = (info.z >> (8 * slot_sub(sub, subs))) & 0xFFu;
      const uint32_t j = m8 ? (uint32_t)__builtin_ctz(m8) : (uint32_t)kMaskCand;
      c = (uint32_t)__popc(m8) + (info.x & 0xFFFFFFu);
      slotCopy = j == (info.x >> 24);
      fe = info.y + j;
      lds_st16(&W.pt[lane], make_float4(px, py, pz, r));
      lds_st16(&W.lst[lane], make_uint4(info.y, m8, 0u, 0xFFFFFFFFu));
      fr = r;
    } else if (want) {
      const float r = sqrtf(dot3(px, py, pz, px, py, pz));  // toSpherical(pos).x
      if constexpr ((OPT & OPT_HDRLDS) == 0) {
        cell = cubemap_cell_fast(px, py, pz, (*Ap).G, sub);
        const uint4 *Hc = (*Ap).binHdr + (size_t)cell * (kBinHdrWords / 4);
        H0 = Hc[0];
        H1 = Hc[1];
        M = reinterpret_cast<const uint32_t *>(Hc)[8 + sub];
      }
      if constexpr ((OPT & OPT_NEXTHDR) != 0) {
        // issued after this sample's header words: waiting for them leaves it in flight
        // (unconditional -- this sample's own line when there is none: a load under a branch
        // makes the compiler wait for it before the header words)
        tv = *(touch ? touch : reinterpret_cast<const uint32_t *>((*Ap).binHdr + (size_t)cell * (kBinHdrWords / 4)));
      }
      const int b = bin_of(r, __uint_as_float(H0.x), __uint_as_float(H0.y), __uint_as_float(H0.z));
      const uint32_t m1 = b > 0 ? ~0u : 0u, m2 = b > 1 ? ~0u : 0u, m3 = b > 2 ? ~0u : 0u;
      const uint32_t beg = (m1 & H1.x) + (m2 & (H1.y - H1.x)) + (m3 & (H1.z - H1.y));
      const uint32_t end = H1.x + (m1 & (H1.y - H1.x)) + (m2 & (H1.z - H1.y)) + (m3 & (H1.w - H1.z));
      // r exactly on the bin's upper edge: records starting at that edge sit in the next
      // bin, whose list is scanned in a second pass for a lower record (locate_hdr)
      const float eb = __uint_as_float(H0.x ^ (m1 & (H0.x ^ H0.y)) ^ (m2 & (H0.y ^ H0.z)));
      edge = b < kMaxEdges && r == eb;
      const uint32_t n = end - beg;
      const uint32_t m8 = (M >> (8 * b)) & 0xFFu & (n < 8u ? (1u << n) - 1u : 0xFFu);
      c = (uint32_t)__popc(m8) + (n > (uint32_t)kMaskCand ? n - (uint32_t)kMaskCand : 0u);
      if constexpr (kHoleSkip) {
        // the sample's quad's radial range (header words kBoundWord..): outside it no listed
        // record passes the radial test (ICONGrid.h:184), so the scan would test every candidate
        // and find none -- a void of the volume (convert_icon's land columns), decided from the
        // header line alone
        const uint2 bd = reinterpret_cast<const uint2 *>((*Ap).binHdr + (size_t)cell * (kBinHdrWords / 4))
            [kBoundWord / 2 + quad_of(sub)];
        if (r > __uint_as_float(bd.x) || r < __uint_as_float(bd.y)) {
          c = 0u;
          edge = false;
        }
      }
      lds_st16(&W.pt[lane], make_float4(px, py, pz, r));
      lds_st16(&W.lst[lane], make_uint4(H0.w + beg, m8, 0u, 0xFFFFFFFFu));
      fe = H0.w + beg + (m8 ? (uint32_t)__builtin_ctz(m8) : (uint32_t)kMaskCand);
      if constexpr (kPair) fe2 = H0.w + beg + list_entry(m8, 1u);
      fr = r;
    }
    IRT_ROUND_PROBE(9, false)
    for (int pass = 0;; ++pass) {
      // every lane: its list's first candidate (OPT_DEALALL: none -- every candidate of
      // every lane goes through the deal below, so a round's samples wait for one entry
      // gather instead of two when the wave's lists hold <= 64 candidates in all)
      uint32_t rem = (OPT & OPT_DEALALL) != 0 ? c : 0u;
      if (kPair && c > 0u) {
        // both entries gathered before either is tested; the second counts only if the
        // first fails (the serial scan's order)
        const float4 *F1 = (*Ap).fat + (size_t)fe * kFatStride4;
        const float4 *F2 = (*Ap).fat + (size_t)(c > 1u ? fe2 : fe) * kFatStride4;
        const float4 a0 = F1[0], a1 = F1[1], a2 = F1[2], am = F1[3];
        const float4 b0 = F2[0], b1 = F2[1], b2 = F2[2], bm = F2[3];
        const bool ok1 = entry_passes(a0, a1, a2, am, px, py, pz, fr);
        const bool ok2 = entry_passes(b0, b1, b2, bm, px, py, pz, fr);
        const uint32_t rec1 = __float_as_uint(am.z), rec2 = __float_as_uint(bm.z);
        if (rec1 < flim) {
          ++specCand;
          if (ok1) {
            hit = true;
            frm[lane] = make_uint2(rec1, record_path(__float_as_uint(am.w), am.x, am.y, fr));
          } else if (c > 1u && rec2 < flim) {
            ++specCand;
            if (ok2) {
              hit = true;
              frm[lane] = make_uint2(rec2, record_path(__float_as_uint(bm.w), bm.x, bm.y, fr));
            } else {
              rem = c - 2u;
              W.lst[lane].z = 2u;
            }
          }
        }
      } else if ((OPT & OPT_DEALALL) == 0 && c > 0u) {  // (from registers: no LDS round trip before the gather)
        Found f;
        bool ok;
        if (kSlot && pass == 0) {  // the slot's copy
          f = {__float_as_uint(sm.z), record_path(__float_as_uint(sm.w), sm.x, sm.y, fr)};
          ok = entry_passes(s0, s1, s2, sm, px, py, pz, fr);
        } else {
          ok = pass_entry((*Ap).fat + (size_t)fe * kFatStride4, px, py, pz, fr, f);
        }
        if (kSlot && pass == 0 && !slotCopy) {
          // the unit's first candidate is not one this sub-cell admits (a slot unit of several
          // sub-cells): it cannot hold the sample, and the sample's own candidates, its first
          // included, go to the dealt-out step -- no gather of its own on the round's chain
          rem = c;
        } else if (f.rec < flim) {  // scan_fat stops, uncounted, at the first record >= the limit
          ++specCand;
          if (ok) {
            hit = true;
            frm[lane] = make_uint2(f.rec, f.path);
          } else {
            rem = c - 1u;
            W.lst[lane].z = 1u;
          }
        }
      }
      tmark(3);  // header, first candidate
      IRT_ROUND_PROBE(10, false)
      bool need = rem > 0u;
      for (uint64_t nm = __ballot(need); nm != 0ull; nm = __ballot(need)) {
        // deal the owners' untested candidates out to the lanes: exclusive prefix of rem
        const uint32_t incl = wave_incl_sum(need ? rem : 0u);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t start = incl - (need ? rem : 0u);
        const bool owns = need && start < 64u;
        own[lane] = 0xFFFFFFFFu;
        __builtin_amdgcn_wave_barrier();
        if (owns) own[start] = (uint32_t)lane;
        __builtin_amdgcn_wave_barrier();
        const uint64_t sm = __ballot(own[lane] != 0xFFFFFFFFu);  // bit s: an owner's tasks start at s
        // lane t: task t - s0 of the owner whose tasks start at the highest s0 <= t
        const uint32_t t = (uint32_t)lane;
        const bool task = t < total;
        const uint32_t s0 = task ? 63u - (uint32_t)__builtin_clzll(sm & (~0ull >> (63u - t))) : 0u;
        const uint32_t o = own[s0];
        bool tp = false, tl = false;
        Found g;
        if (task) {
          const float4 po = lds_ld16(&W.pt[o]);
          const uint4 d = lds_ld16(&W.lst[o]);
          tp = pass_entry((*Ap).fat + (size_t)(d.x + list_entry(d.y, d.z + (t - s0))) * kFatStride4, po.x, po.y,
                          po.z, po.w, g);
          tl = g.rec >= d.w;  // past the limit: the serial scan stops there
          tp = tp && !tl;
        }
        const uint64_t pm = __ballot(tp), lm = __ballot(tl);
        // the lowest event of each owner's tasks: a passing record (it hands it over) or the limit
        const uint64_t below = t ? (~0ull >> (64u - t)) : 0ull;  // tasks < t
        if (tp && ((pm | lm) & below & (~0ull << s0)) == 0ull) frm[o] = make_uint2(g.rec, g.path);
        __builtin_amdgcn_wave_barrier();
        if (owns) {
          const uint32_t k = min(rem, 64u - start);  // this owner's tasks in this batch
          const uint64_t ev = (pm | lm) & ((k >= 64u ? ~0ull : ((1ull << k) - 1ull)) << start);
          if (ev) {
            const uint32_t e = (uint32_t)__builtin_ctzll(ev) - start;
            const bool ps = (pm >> (start + e)) & 1ull;
            specCand += e + (ps ? 1u : 0u);
            hit = hit || ps;
            need = false;
          } else {
            specCand += k;
            rem -= k;
            W.lst[lane].z += k;
            need = rem > 0u;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      tmark(4);  // the dealt-out candidates
      IRT_ROUND_PROBE(11, false)
      // the second pass: bin-edge samples, the next bin's list below the record found
      if (pass == 1 || __ballot(edge) == 0ull) break;
      c = 0u;
      if (edge) {
        const float4 p = lds_ld16(&W.pt[lane]);
        uint32_t sub;
        const uint32_t cell = cubemap_cell_fast(p.x, p.y, p.z, (*Ap).G, sub);
        const uint4 *Hc = (*Ap).binHdr + (size_t)cell * (kBinHdrWords / 4);
        const uint4 H0 = Hc[0], H1 = Hc[1];
        const uint32_t M = reinterpret_cast<const uint32_t *>(Hc)[8 + sub];
        const int b = bin_of(p.w, __uint_as_float(H0.x), __uint_as_float(H0.y), __uint_as_float(H0.z)) + 1;
        const uint32_t m1 = b > 0 ? ~0u : 0u, m2 = b > 1 ? ~0u : 0u, m3 = b > 2 ? ~0u : 0u;
        const uint32_t beg = (m1 & H1.x) + (m2 & (H1.y - H1.x)) + (m3 & (H1.z - H1.y));
        const uint32_t end = H1.x + (m1 & (H1.y - H1.x)) + (m2 & (H1.z - H1.y)) + (m3 & (H1.w - H1.z));
        const uint32_t n = end - beg;
        const uint32_t m8 = (M >> (8 * b)) & 0xFFu & (n < 8u ? (1u << n) - 1u : 0xFFu);
        c = (uint32_t)__popc(m8) + (n > (uint32_t)kMaskCand ? n - (uint32_t)kMaskCand : 0u);
        flim = hit ? frm[lane].x : 0xFFFFFFFFu;
        lds_st16(&W.lst[lane], make_uint4(H0.w + beg, m8, 0u, flim));
        fe = H0.w + beg + (m8 ? (uint32_t)__builtin_ctz(m8) : (uint32_t)kMaskCand);
        if constexpr (kPair) fe2 = H0.w + beg + list_entry(m8, 1u);
      }
    }
    if constexpr ((OPT & OPT_NEXTHDR) != 0) asm volatile("" ::"v"(tv));
    if (!want) return false;
    const float r = W.pt[lane].w;
    Found f = {0xFFFFFFFFu, 0u};
    if (hit) {
      const uint2 rm = frm[lane];
      f = {rm.x, rm.y};
    }
    if ((*Ap).numSph) {
      const uint32_t h = sph_hash(r);
      if ((s_sph[h >> 5] >> (h & 31)) & 1u) {
        float v2;
        uint32_t rec2;
        if (sphere_at(r, v2, rec2) && (!hit || rec2 < f.rec)) {
          value = v2;
          return true;
        }
      }
    }
    if (hit) value = record_value(f, r);
    return hit;
  }

  // postClassify's alpha only (the acceptance test needs nothing else); the colour comes
  // from post_classify on acceptance
  __device__ __forceinline__ float classify_alpha(float v) {
#if !defined(IRT_HELD_ARGS) && !defined(IRT_HELD_LATE)
    const RenderArgs &LA = fresh_args();  // read where used (-DIRT_HELD_LATE: through Ap)
#else
    const RenderArgs &LA = *Ap;
#endif
    v = div_uniform(v - LA.tfLo, LA.invTf);  // (v - tfLo) / (tfHi - tfLo), correctly rounded
    const int size = opaque_u(LA.lutSize);
    const int idx = f2i_x86(v * (float)size);
    const float frac = (v * (float)size) - (float)idx;
    const int i1 = idx < 0 ? 0 : (idx > size - 1 ? size - 1 : idx);
    const int idx2 = (int)((uint32_t)idx + 1u);
    const int i2 = idx2 < 0 ? 0 : (idx2 > size - 1 ? size - 1 : idx2);
    const float a = LA.lut[i1].w, b = LA.lut[i2].w;
    return a * frac + b * (1.f - frac) * LA.opacityScale;
  }

  // postClassify (deviceCode.cu:127-135): weights reversed, opacityScale on 2nd term only
  __device__ __forceinline__ float4 post_classify(float v) {
#if !defined(IRT_HELD_ARGS) && !defined(IRT_HELD_LATE)
    const RenderArgs &LA = fresh_args();  // read where used (-DIRT_HELD_LATE: through Ap)
#else
    const RenderArgs &LA = *Ap;
#endif
    v = div_uniform(v - LA.tfLo, LA.invTf);  // (v - tfLo) / (tfHi - tfLo), correctly rounded
    const int size = opaque_u(LA.lutSize);
    const int idx = f2i_x86(v * (float)size);
    const float frac = (v * (float)size) - (float)idx;
    const int i1 = idx < 0 ? 0 : (idx > size - 1 ? size - 1 : idx);
    const int idx2 = (int)((uint32_t)idx + 1u);
    const int i2 = idx2 < 0 ? 0 : (idx2 > size - 1 ? size - 1 : idx2);
    const float4 a = LA.lut[i1], b = LA.lut[i2];
    const float om = 1.f - frac;
    float4 o;
    o.x = a.x * frac + b.x * om * 1.f;
    o.y = a.y * frac + b.y * om * 1.f;
    o.z = a.z * frac + b.z * om * 1.f;
    o.w = a.w * frac + b.w * om * LA.opacityScale;
    return o;
  }

  // woodcockTracking (deviceCode.cu:149-186) over [tmin, tmax].  `counted` is false in
  // zero-length sdda leaves, whose sampleVolume calls the statistics leave out.
  __device__ __forceinline__ float woodcock(float dx, float dy, float dz, float tmin, float tmax,
                                            uint32_t &st, float majorant, float4 &sampleOut,
                                            bool counted) {
    float t = tmin;
    if (majorant <= 0.f) return fminf(t, tmax);
    const float q = majorant / (*Ap).unitDistance;  // the same value every iteration (165)
    while (true) {
      if constexpr ((OPT & OPT_STATS) != 0) ++cnt.steps;
      st = lcg_next(st);
      t -= (woodcock_log(st, s_logf) / q);
      if (t > tmax) break;
      const float3 O = cam_org((*Ap), frame);
      const float px = O.x + dx * t, py = O.y + dy * t, pz = O.z + dz * t;
      float value = 0.f;
      if (counted) count(2);
      if (!locate(px, py, pz, value)) continue;
      if (counted) count(3);
      const float sw = classify_alpha(value);  // postClassify(value).w
      st = lcg_next(st);
      const float u = lcg_float(st);
      if (sw >= u * majorant) {
        sampleOut = post_classify(value);
        break;
      }
    }
    return fminf(t, tmax);
  }

  // woodcockTracking (deviceCode.cu:149-186) for every lane of the wave with `req` set,
  // evaluated together.  A ray's sample positions depend on nothing but its RNG: sample k
  // (k = 0, 1, ...) of a ray whose earlier samples were all located and rejected lies at
  // t - d_0 - ... - d_k with d_j from the state 2j+1 draws ahead, and is accepted against
  // the state 2k+2 draws ahead.  So each round the wave's R undecided rays get G = 64/R
  // (a power of two) lanes each; lane k of a group takes sample k of its ray -- independent
  // gathers in parallel instead of a chain -- and the ray's first event among its G samples
  // (past tmax / not located / accepted) decides it exactly as the serial loop would; the
  // samples after the event are discarded.  A not-located sample consumes only its step
  // draw, so the ray resumes from there next round -- in miss mode: its samples are then
  // placed as if none were located (sample k from the state k+1 draws ahead) until one is,
  // which switches back (samples outside every cell come in runs: grid-accel cells and
  // wedge gaps).  Statistics count only the samples
  // the reference takes.  Returns in t the woodcockTracking return value.
  __device__ __forceinline__ void woodcock_wave(bool req, float dx, float dy, float dz, float &t,
                                                float tmax, uint32_t &st, float majorant,
                                                bool counted, float4 &sampleOut, bool &miss,
                                                CoopWave &W, ScanWave *SW, const uint2 *jmp) {
    Ap = IRT_TR_ARGS;
    const int lane = (int)__lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    const float q = majorant / (*Ap).unitDistance;
    bool active = req && !(majorant <= 0.f);  // majorant <= 0: return at once (161-162)
    // speculation ramps up: a ray gets at most 2^lgCap lanes this round, and lgCap grows
    // each round it stays undecided.  Most chains end within a few samples (default TF:
    // 3 draws), and the lines of samples past the event are wasted gathers; long chains
    // (sparse TFs) reach whole-wave groups after six rounds.  The miss-mode kernels (wedge
    // samplers, grid accel) keep whole-wave groups from the start: their misses come in
    // runs that wide groups cross in one round (2 % faster there, profiles/r02e_coop_cap).
    int lgCap = kWideStart ? 6 : (*Ap).coopMaxLg;
    tmark(6);  // between woodcockFunc calls (sdda leaves, ranges)
    for (int wr = 0;; lgCap = min(lgCap + (*Ap).coopRamp, 6), ++wr) {
      const uint64_t am = __ballot(active);
      if (am == 0ull) break;
      if constexpr ((OPT & OPT_STATS) != 0) ++cnt.rounds;
      const int R = __popcll(am);
      const int lg = min(lgCap, R > 32 ? 0 : R > 16 ? 1 : R > 8 ? 2 : R > 4 ? 3 : R > 2 ? 4 : R > 1 ? 5 : 6);
      const int G = 1 << lg;
      // solo round (G = 1): every ray on its own lane, nothing exchanged
      const bool solo = lg == 0;
      const int rank = __popcll(am & below);
      int grp, k;
      bool used, cntd, mm;
      float4 rq, ry;
      if (solo) {
        grp = lane;
        k = 0;
        used = active;
        cntd = counted;
        mm = kMiss && miss;
        rq = make_float4(t, tmax, q, majorant);
        ry = make_float4(dx, dy, dz, __uint_as_float(st));
      } else {
        if (active) {
          lds_st16(&W.req[rank], make_float4(t, tmax, q, majorant));
          lds_st16(&W.ray[rank], make_float4(dx, dy, dz, __uint_as_float(st)));
          W.cnt[rank] = (counted ? 1u : 0u) | (miss ? 2u : 0u);
        }
        __builtin_amdgcn_wave_barrier();
        grp = lane >> lg;
        k = lane & (G - 1);
        used = grp < R;
        const int g = used ? grp : 0;
        rq = lds_ld16(&W.req[g]);
        ry = lds_ld16(&W.ray[g]);
        const uint32_t cf = W.cnt[g];
        cntd = cf & 1u;
        mm = kMiss && (cf & 2u);
      }
      const uint32_t s0 = __float_as_uint(ry.w);
      // sample k's step draw: 2k+1 draws ahead if every earlier sample is located (and
      // rejected), k+1 if none is (miss mode)
      const int jk = mm ? k + 1 : 2 * k + 1;
      uint32_t sk;
      if (solo) {
        sk = lcg_next(s0);
      } else {
        const uint2 j = lds_ld8(&jmp[jk]);  // {mul, add}: one 8-byte LDS read
        sk = j.x * s0 + j.y;
      }
      const float dk = woodcock_log(sk, s_logf) / rq.z;
      float tk;
      constexpr bool dppScan = (OPT & OPT_DPPSCAN) != 0;
      if (solo) {
        tk = rq.x - dk;
      } else if (dppScan && (lg == 1 || lg == 2 || lg == 4 || lg == 6)) {
        tk = lg == 1 ? dpp_prefix<2>(rq.x, dk, k)
                     : lg == 2 ? dpp_prefix<4>(rq.x, dk, k) : lg == 4 ? dpp_prefix<16>(rq.x, dk, k) : dpp_prefix<64>(rq.x, dk, k);
      } else {
        W.step[lane] = dk;
        __builtin_amdgcn_wave_barrier();
        const float *dg = &W.step[grp << lg];
        switch (lg) {
          case 1: tk = coop_prefix<2>(rq.x, dg, k); break;
          case 2: tk = coop_prefix<4>(rq.x, dg, k); break;
          case 3: tk = coop_prefix<8>(rq.x, dg, k); break;
          case 4: tk = coop_prefix<16>(rq.x, dg, k); break;
          case 5: tk = coop_prefix<32>(rq.x, dg, k); break;
          default: tk = coop_prefix<64>(rq.x, dg, k); break;
        }
      }
      bool past = used && tk > rq.y;
      if constexpr (kVoidRun) {
        // A solo lane in miss mode walks the void its ray is in on its own: while its sample lies
        // outside the radial range of every record that can reach the sample's quad (the cell
        // header's bounds, the quad-bound test of locate_wave), the sample is outside every cell
        // -- sampleVolume finds nothing and woodcockTracking takes its next step after one draw
        // (deviceCode.cu:165-173) -- so the lane takes that step here, with no candidate test (the
        // header's bound word, an L1 hit while the walk stays in one cell).  The round then scans the first sample
        // that may be located.  convert_icon's voids (over and under every land column) are
        // crossed in one round instead of one round per sample.
        constexpr bool kVoidLoc = (OPT & OPT_VOIDLOC) != 0;
        if (solo && used && !past && (mm || kVoidLoc)) {
          const float3 O = cam_org((*Ap), frame);
#pragma nounroll
          for (int it = 0; it < kVoidRunMax; ++it) {
            const float px = O.x + ry.x * tk, py = O.y + ry.y * tk, pz = O.z + ry.z * tk;
            const float r = sqrtf(dot3(px, py, pz, px, py, pz));  // toSpherical(pos).x
            uint32_t sub;
            const uint32_t cell = cubemap_cell_fast(px, py, pz, (*Ap).G, sub);
            // (the same header line as the last sample's while the walk stays in one cell: an L1 hit)
            const uint2 bd = reinterpret_cast<const uint2 *>((*Ap).binHdr + (size_t)cell * (kBinHdrWords / 4))
                [kBoundWord / 2 + quad_of(sub)];
            if (!(r > __uint_as_float(bd.x) || r < __uint_as_float(bd.y))) break;  // may be located: the round's scan decides
            if ((*Ap).numSph) {  // a zero-thickness record at exactly r is not in the lists
              const uint32_t h = sph_hash(r);
              if ((s_sph[h >> 5] >> (h & 31)) & 1u) break;
            }
            // outside every cell: the sample is taken (a sampleVolume call), one draw.  In
            // located mode (OPT_VOIDLOC) this miss breaks the round's assumption: a solo lane's
            // sample 0 takes its step draw first in either mode, so the ray switches to miss
            // mode here and walks on
            if (kVoidLoc && !mm) {
              mm = true;
              miss = true;
            }
            if (cntd) ++nLocate;
            if constexpr ((OPT & OPT_STATS) != 0) ++cnt.steps;
            rq.x = tk;
            sk = lcg_next(sk);
            tk = rq.x - woodcock_log(sk, s_logf) / rq.z;
            if (tk > rq.y) {
              past = true;
              break;
            }
          }
        }
      }
      IRT_ROUND_PROBE(8)
      bool found = false, acc = false;
      float value = 0.f;
      tmark(2);  // round start: exchange, jumps, logf, prefix
#ifdef IRT_PROBE_BUILD
      // measurement only (31): 100 extra VALU instructions per Woodcock round
      if ((*Ap).probeExit == 31) {
#pragma nounroll
        for (int k = 0; k < 25; ++k) asm volatile("v_nop\n v_nop\n v_nop\n v_nop" ::: "memory");
      }
#endif
      if constexpr (kWaveScan) {
        const uint32_t *tp = nullptr;
        if constexpr ((OPT & OPT_NEXTHDR) != 0) {
          // the next sample if this one is located and rejected: two draws on (approximate
          // step: only its header line is wanted)
          if (solo && wr > 0 && used && !past) {
            const float t1 = tk - woodcock_log(lcg_next(lcg_next(sk)), s_logf) * __builtin_amdgcn_rcpf(rq.z);
            if (t1 <= rq.y) {
              uint32_t sb;
              const float3 O = cam_org((*Ap), frame);
              const uint32_t c1 = cubemap_cell_fast(O.x + ry.x * t1, O.y + ry.y * t1, O.z + ry.z * t1,
                                                    (*Ap).G, sb);
              tp = reinterpret_cast<const uint32_t *>((*Ap).binHdr + (size_t)c1 * (kBinHdrWords / 4));
            }
          }
        } else {
          (void)wr;
        }
        const float3 O = cam_org((*Ap), frame);
        found = locate_wave(used && !past, O.x + ry.x * tk, O.y + ry.y * tk, O.z + ry.z * tk,
                            value, W, *SW, tp);
      } else if (used && !past) {
        const float3 O = cam_org((*Ap), frame);
        found = locate(O.x + ry.x * tk, O.y + ry.y * tk, O.z + ry.z * tk, value);
      }
      tmark(5);  // locate's tail: sphere, getValue
#ifdef IRT_PROBE_BUILD
      if ((*Ap).probeExit >= 9 && (*Ap).probeExit <= 12) return;
#endif
      if (found) {
        const float sw = classify_alpha(value);  // postClassify(value).w
        acc = sw >= lcg_float(lcg_next(sk)) * rq.w;
      }
      // the first sample that breaks the round's assumption, or ends the ray's leaf
      const bool ev = used && (past || acc || (mm ? found : !found));
      // the lane's group: its first event, G if none; the samples up to it are taken
      int first;
      uint64_t em = 0ull;
      if (solo) {
        first = ev ? 0 : 1;
      } else {
        em = __ballot(ev);
        const uint64_t gm = lg == 6 ? ~0ull : (((1ull << G) - 1ull) << (grp << lg));
        first = (em & gm) ? (int)__builtin_ctzll(em & gm) - (grp << lg) : G;
      }
      if (used && k <= first) {
        if (cntd) {
          nLocate += past ? 0u : 1u;
          nFound += found ? 1u : 0u;
        }
        nCand += specCand;
      }
      if constexpr ((OPT & OPT_STATS) != 0) {
        const bool loc = used && !past;
        uint32_t m = loc ? specCand : 0u;
        for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
        cnt.hops += m;
        cnt.locRounds += __ballot(loc) ? 1u : 0u;
        if (loc) ++cnt.candHist[specCand < 3u ? specCand : 3u];
      }
      specCand = 0u;
      // the rays' owners take their group's outcome
      int of;
      float tsrc, vsrc;
      bool pastS, accS, foundS;
      if (solo) {
        of = first;
        tsrc = tk;
        vsrc = value;
        pastS = past;
        accS = acc;
        foundS = found;
      } else {
        const uint64_t pastM = __ballot(past), accM = __ballot(acc), foundM = kMiss ? __ballot(found) : 0ull;
        const int ob = active ? rank << lg : 0;  // < 64 for an owner
        const uint64_t om = lg == 6 ? ~0ull : (((1ull << G) - 1ull) << ob);
        of = (active && (em & om)) ? (int)__builtin_ctzll(em & om) - ob : G;
        const int src = active ? ob + (of < G ? of : G - 1) : lane;
        tsrc = __shfl(tk, src, 64);
        vsrc = __shfl(value, src, 64);
        pastS = (pastM >> src) & 1ull;
        accS = (accM >> src) & 1ull;
        foundS = (foundM >> src) & 1ull;
      }
      if (active) {
        if constexpr ((OPT & OPT_STATS) != 0) cnt.steps += of < G ? (uint32_t)of + 1u : (uint32_t)G;
        t = tsrc;
        // draws taken: two per located sample, one per miss (and the one past tmax)
        const int n = (kMiss && miss) ? (of == G ? G : (foundS ? of + 2 : of + 1))
                           : (of == G ? 2 * G : (accS ? 2 * of + 2 : 2 * of + 1));
        if (solo) {
          st = n == 1 ? sk : lcg_next(sk);  // the draws this round made
        } else {
          const uint2 j = lds_ld8(&jmp[n]);
          st = j.x * st + j.y;
        }
        if (of < G && (pastS || accS)) {
          active = false;
          if (accS) sampleOut = post_classify(vsrc);
        } else if (kMiss && of < G) {
          miss = !miss;  // the assumption broke: a miss, or (miss mode) a located sample
        }
      }
      IRT_ROUND_PROBE(13)
    }
    if (req) t = fminf(t, tmax);
    tmark(7);  // the rounds' classify, LUT, ballots, outcomes
  }
};

// ------------------------------------------------------------------ per-pixel pieces
// The frame grid: 256-thread workgroup b, thread t -> gid = 256 b + t.  Workgroup b covers
// 16x16 pixels of tile k = b / 16 of this launch (frame tile tileBegin + k*tileStride, or
// tileList[k]),
// wave w an 8x8 packet, lane l one pixel.  The block index is passed on its own so that the
// tile arithmetic (an integer division by tilesX) stays scalar: it is uniform per workgroup.
struct Pixel {
  int x, y;
  size_t outIdx;
  bool active;
};
__device__ __forceinline__ Pixel pixel_of(const RenderArgs &A, uint32_t blkU, int tid) {
  const int blk = (int)__builtin_amdgcn_readfirstlane(blkU);
  const int k = blk >> 4, sub = blk & 15;
  const int wave = tid >> 6, lane = tid & 63;
  const int lx = ((sub & 3) << 4) | ((wave & 1) << 3) | (lane & 7);
  const int ly = ((sub >> 2) << 4) | ((wave >> 1) << 3) | (lane >> 3);
  const int tileId = !A.tileList ? A.tileBegin + k * A.tileStride : (k < A.numTiles ? (int)scalar_word(A.tileList, (uint32_t)k) : 0);
  const int tx = tileId % A.tilesX, ty = tileId / A.tilesX;
  Pixel p;
  p.x = tx * 64 + lx;
  p.y = ty * 64 + ly;
  p.active = k < A.numTiles && p.x < A.W && p.y < A.H;
  p.outIdx = A.packed ? (size_t)k * 4096 + ly * 64 + lx : (size_t)p.x + (size_t)A.W * p.y;
  return p;
}

// Random rnd(accumID*W*H + x, y) (deviceCode.cu:288-289) and generateRay (36-49); g++
// draws the dir_dv jitter first.
__device__ __forceinline__ void gen_ray(const RenderArgs &A, int accumID, int x, int y, uint32_t &st,
                                        float &dx, float &dy, float &dz, int frame = 0) {
  st = lcg_seed((uint32_t)accumID * (uint32_t)A.W * (uint32_t)A.H + (uint32_t)x, (uint32_t)y);
  st = lcg_next(st);
  const float jv = lcg_float(st);
  st = lcg_next(st);
  const float ju = lcg_float(st);
  const float su = (float)x + .5f, sv = (float)y + .5f;
  const float a = su + ju, b = sv + jv;
  float3 d00 = A.dir00, du = A.du, dv = A.dv;
  if (A.frameCams) {  // a sequence of views: this frame's camera
    const float4 w1 = cam_word(A, frame, 1), w2 = cam_word(A, frame, 2), w3 = cam_word(A, frame, 3);
    d00 = make_float3(w1.x, w1.y, w1.z);
    du = make_float3(w2.x, w2.y, w2.z);
    dv = make_float3(w3.x, w3.y, w3.z);
  }
  dx = (d00.x + a * du.x) + b * dv.x;
  dy = (d00.y + a * du.y) + b * dv.y;
  dz = (d00.z + a * du.z) + b * dv.z;
  const float len = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
  if (recip_ok(len)) {  // normalize's three quotients through one reciprocal (irt_device.h)
    const double r = recip_d(len);
    dx = div_recip(dx, r);
    dy = div_recip(dy, r);
    dz = div_recip(dz, r);
  } else {
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
  }
  if (fabsf(dx) < 1e-5f) dx = 1e-5f;
  if (fabsf(dy) < 1e-5f) dy = 1e-5f;
  if (fabsf(dz) < 1e-5f) dz = 1e-5f;
}

// accumulate lerp(vec4f(color,alpha), old, 1/(accumID+1)) and write linear_to_srgb +
// make_rgba (deviceCode.cu:333-340).  Stream (nt = true): the pixel's lines are stored with
// the streaming hint -- nothing in the launch reads them again, so they should not displace
// locator lines in L2 (5-wave builds, the default: C3 -1.6 %, C4 -4.4 % with the accum
// prefetch also nt; the 4-wave A/B build keeps plain stores; profiles/r03za_nt/,
// profiles/r03zb_*).
template <bool nt = false>
__device__ __forceinline__ void write_pixel(const RenderArgs &A, size_t outIdx, float cr, float cg,
                                            float cb, float alpha, const float *s_th, float4 old) {
  const float w = A.accumW;  // 1.f / (float)(accumID + 1), on the host (the same division)
  float4 nv;
  nv.x = w * cr + (1.f - w) * old.x;
  nv.y = w * cg + (1.f - w) * old.y;
  nv.z = w * cb + (1.f - w) * old.z;
  nv.w = w * alpha + (1.f - w) * old.w;
  const uint32_t rgba = srgb_byte(s_th, nv.x) + (srgb_byte(s_th, nv.y) << 8) +
                        (srgb_byte(s_th, nv.z) << 16) + (make_8bit(nv.w) << 24);
  if constexpr (nt) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v t = {nv.x, nv.y, nv.z, nv.w};
    __builtin_nontemporal_store(t, reinterpret_cast<f4v *>(&A.accum[outIdx]));
    __builtin_nontemporal_store(rgba, &A.fb[outIdx]);
  } else {
    A.accum[outIdx] = nv;
    A.fb[outIdx] = rgba;
  }
}
__device__ __forceinline__ void write_pixel(const RenderArgs &A, size_t outIdx, float cr, float cg,
                                            float cb, float alpha, const float *s_th) {
  write_pixel(A, outIdx, cr, cg, cb, alpha, s_th, A.accum[outIdx]);
}

// Chained progressive frames (RenderArgs::chain).  Workgroup (b, f) of a launch renders block
// b of frame accumID + f and lerps into accum/fb directly; the previous frame's colour of the
// same pixel must be in accum first.  The hand-off (cdna_hip_programming.md Guideline 16, R1):
// frame f - 1's wave stores its pixels write-through (sc1), drains them (vmcnt 0) and stores
// chainEpoch + f to its (block, wave) word (an sc1 store); frame f's wave polls that word
// (relaxed, agent scope: sc1 loads), then reads accum with sc1 loads (past this CU's L1).
// Every handed-off byte is stored and loaded sc1, so the hand-off does not depend on the two
// workgroups sharing an XCD (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the
// sc1 table).  Frame f's wave gets there at the end of its rays, tens of microseconds after
// frame f - 1's workgroup -- dispatched numBlocks workgroups earlier -- finished, so the first
// poll normally hits.  A wait gives up after A.chainSpins polls and flags the launch
// (*A.chainFail, pinned host memory; the host returns IRT_E_CHAIN).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t out_pixels(const RenderArgs &A) {
  return A.packed ? (uint32_t)A.numTiles * 4096u : (uint32_t)A.W * (uint32_t)A.H;
}
__device__ __forceinline__ void chain_wait(const RenderArgs &A, uint32_t blk, int pwave, int frame) {
  uint32_t *f = A.chainFlag + (size_t)blk * 4u + (uint32_t)pwave;
  const uint32_t want = A.chainEpoch + (uint32_t)frame;  // frame - 1's publish
  for (uint32_t spins = 0;; ++spins) {
    const uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (v == want) break;
    if (spins >= A.chainSpins) {
      if (__lane_id() == (unsigned)(__ffsll((long long)__ballot(1)) - 1))
        __hip_atomic_store(A.chainFail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: the loads stay below
}
// the previous frame's accum pixel, past this CU's L1
__device__ __forceinline__ float4 chain_load_accum(const RenderArgs &A, size_t outIdx) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)A.accum, 0, (int)(out_pixels(A) * 16u), 0x00020000);
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(outIdx * 16u), 0, 16));
}
// write_pixel's lerp and RGBA8 with the weight of this frame; publish: write-through (sc1)
// stores that the next frame's wave reads, else streaming stores as write_pixel<true>
__device__ __forceinline__ void write_pixel_chain(const RenderArgs &A, size_t outIdx, float cr, float cg, float cb,
                                                  float alpha, float w, const float *s_th, float4 old, bool publish) {
  float4 nv;
  nv.x = w * cr + (1.f - w) * old.x;
  nv.y = w * cg + (1.f - w) * old.y;
  nv.z = w * cb + (1.f - w) * old.z;
  nv.w = w * alpha + (1.f - w) * old.w;
  const uint32_t rgba = srgb_byte(s_th, nv.x) + (srgb_byte(s_th, nv.y) << 8) +
                        (srgb_byte(s_th, nv.z) << 16) + (make_8bit(nv.w) << 24);
#ifdef IRT_PROBE_BUILD
  if (publish && A.probeExit == 17) {  // measurement only (17, probe build): plain stores to publish
    A.accum[outIdx] = nv;
    A.fb[outIdx] = rgba;
    return;
  }
#endif
  if (publish) {
    const uint32_t n = out_pixels(A);
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)A.accum, 0, (int)(n * 16u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc((void *)A.fb, 0, (int)(n * 4u), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, nv), ra, (int)(outIdx * 16u), 0, 16);
    __builtin_amdgcn_raw_buffer_store_b32(rgba, rf, (int)(outIdx * 4u), 0, 16);
  } else {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v t = {nv.x, nv.y, nv.z, nv.w};
    __builtin_nontemporal_store(t, reinterpret_cast<f4v *>(&A.accum[outIdx]));
    __builtin_nontemporal_store(rgba, &A.fb[outIdx]);
  }
}

// The workgroup's event counts (LDS) out to the launch's statistics, by the workgroup's
// last wave to finish (k_render).  Default: one store of the kCnt counts per workgroup into
// wgCounts, pinned host memory the host sums when asked (irt_context.hip finish_slot): no
// statistics kernel, and no two workgroups touch the same line.  Without wgCounts:
// device-scope atomics into the counter block -- 4 096 workgroups x 5 same-line atomics per
// 1024^2 frame, ~35 us of serialised atomics.
__device__ __forceinline__ void flush_counters(const RenderArgs &A, const uint32_t *s_cnt, int lane) {
  if (A.wgCounts) {
    const size_t wg = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    if (lane < kCnt) A.wgCounts[wg * kCnt + lane] = s_cnt[lane];
  } else if (lane < 5 && s_cnt[lane]) {
    const size_t wg = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    unsigned long long *dst = A.counterBuckets ? A.counterBuckets + (wg % kCounterBuckets) * 8 : A.counters;
    atomicAdd(&dst[lane], (unsigned long long)s_cnt[lane]);
  }
}

// sample-buffer marker of a frame whose ray missed the box (alpha is 0 or 1 otherwise)
constexpr float kNoSample = -1.f;

// The woodcockTrackingWithAccel raygen in GRID_ACCEL_MODE (deviceCode.cu:326-328): dda3
// (DDA.h:35-136) over the 256^3 Cartesian grid, each cell handed to the woodcockFunc
// lambda (304-323) with the grid's majorant.  Written exactly as the reference's g++ CPU
// build evaluates it, including `min(reduce_min(tnext), ray.tmax)` going through
// `int min(int, int)` (dda3_min_quirk, irt_common.h).
template <int OPT>
__device__ __forceinline__ void render_grid(const RenderArgs &A, Tracer<OPT> &T, const Ray &ray,
                                            float rtmin, float rtmax, uint32_t &st, float &cr,
                                            float &cg, float &cb, float &alpha) {
  const int D = kGridDim;
  // move ray so tmin becomes 0 (DDA.h:42-46)
  const float ox = ray.ox + rtmin * ray.dx, oy = ray.oy + rtmin * ray.dy, oz = ray.oz + rtmin * ray.dz;
  const float tmax = rtmax - rtmin;
  const float rx = 1.f / ray.dx, ry = 1.f / ray.dy, rz = 1.f / ray.dz;
  const float lx = (A.bmin.x - ox) * rx, ly = (A.bmin.y - oy) * ry, lz = (A.bmin.z - oz) * rz;
  const float hx = (A.bmax.x - ox) * rx, hy = (A.bmax.y - oy) * ry, hz = (A.bmax.z - oz) * rz;
  float nx = fminf(lx, hx), ny = fminf(ly, hy), nz = fminf(lz, hz);
  const float fx = fmaxf(lx, hx), fy = fmaxf(ly, hy), fz = fmaxf(lz, hz);
  if (ray.dx == 0.f) nx = IRT_FLT_MAX;
  if (ray.dy == 0.f) ny = IRT_FLT_MAX;
  if (ray.dz == 0.f) nz = IRT_FLT_MAX;
  int cx = project_on_grid(ox, A.bmin.x, A.bmax.x, D);
  int cy = project_on_grid(oy, A.bmin.y, A.bmax.y, D);
  int cz = project_on_grid(oz, A.bmin.z, A.bmax.z, D);
  const float dx = fmaxf(0.f, (fx - nx) / (float)D), dy = fmaxf(0.f, (fy - ny) / (float)D),
              dz = fmaxf(0.f, (fz - nz) / (float)D);
  const int sx = ray.dx > 0.f ? 1 : -1, sy = ray.dy > 0.f ? 1 : -1, sz = ray.dz > 0.f ? 1 : -1;
  const int ex = ray.dx > 0.f ? D : -1, ey = ray.dy > 0.f ? D : -1, ez = ray.dz > 0.f ? D : -1;
  float tnx = ray.dx > 0.f ? nx + (float)(cx + 1) * dx : nx + (float)(D - cx) * dx;
  float tny = ray.dy > 0.f ? ny + (float)(cy + 1) * dy : ny + (float)(D - cy) * dy;
  float tnz = ray.dz > 0.f ? nz + (float)(cz + 1) * dz : nz + (float)(D - cz) * dz;
  float tc0 = 0.f;
  for (int iter = 0; iter < 4 * D + 16; ++iter) {  // a cell per step, <= 3*D steps
    const float tmn = fminf(fminf(tnx, tny), tnz);  // reduce_min (vecmath.h:512-514)
    const float tc1 = dda3_min_quirk(tmn, tmax);
    const float w0 = rtmin + tc0, w1 = rtmin + tc1;  // func(leaf, ray_tmin+t0, ray_tmin+t1)
    // every majorant of this cell's block <= 0 (k_grid_bits): woodcockTracking would return
    // at once (deviceCode.cu:161-162) -- no draw, no sample, no hit -- so only the walk goes on
    constexpr int NB = kGridDim / kGridBlock;
    const bool inGrid = (unsigned)cx < (unsigned)D && (unsigned)cy < (unsigned)D && (unsigned)cz < (unsigned)D;
    const uint32_t gb = inGrid ? ((uint32_t)(cz / kGridBlock) * NB + (uint32_t)(cy / kGridBlock)) * NB +
                                     (uint32_t)(cx / kGridBlock)
                               : 0u;
    if (!inGrid || ((T.s_gbits[gb >> 5] >> (gb & 31)) & 1u)) {
      const float maj = A.gridMaxOp[(size_t)cz * D * D + (size_t)cy * D + cx];
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      const float tw = T.woodcock(ray.dx, ray.dy, ray.dz, w0, w1, st, maj, s, !(w0 == w1));
      if (tw > w0 && tw < w1) {
        cr = s.x * A.amb.x * A.ambRad;
        cg = s.y * A.amb.y * A.ambRad;
        cb = s.z * A.amb.z * A.ambRad;
        alpha = s.w > 0.f ? 1.f : 0.f;
        return;
      }
    }
    if (tnx == tmn) {
      tnx += dx;
      cx += sx;
      if (cx == ex) return;
    }
    if (tny == tmn) {
      tny += dy;
      cy += sy;
      if (cy == ey) return;
    }
    if (tnz == tmn) {
      tnz += dz;
      cz += sz;
      if (cz == ez) return;
    }
    tc0 = tc1;
  }
}

// ------------------------------------------------------------------ the full raygen
// One pixel of woodcockTrackingWithAccel / woodcockTrackingAE, every range and leaf.
template <int OPT>
__device__ __forceinline__ void render_pixel(const RenderArgs &A, Tracer<OPT> &T, const Pixel &px,
                                             const float *s_th, int4 *s_dda, float4 *s_entry,
                                             int tid, int accumID, float4 *sampleOut) {
  uint32_t st;
  float dx, dy, dz;
  gen_ray(A, accumID, px.x, px.y, st, dx, dy, dz);
  const Ray ray = {A.org.x, A.org.y, A.org.z, 0.f, dx, dy, dz, 1e10f};
  float t0, t1;
  if (!box_test(ray, A, t0, t1)) {  // deviceCode.cu:294-295: pixel untouched
    if (sampleOut) *sampleOut = make_float4(0.f, 0.f, 0.f, kNoSample);
    return;
  }
  T.count(1);
  float cr = 0.f, cg = 0.f, cb = 0.f, alpha = 0.f;
  const bool ae = A.raygen == 1;
  // The ranges the raygen tracks.  woodcockTrackingAE (deviceCode.cu:239-275): the box
  // interval, majorant 1, one leaf.  woodcockTrackingWithAccel: sdda (ShellAccel.h:82-229)
  // over the shell's (at most two) sphere ranges (94-111), each a sequence of macrocell
  // leaves handed to the woodcockFunc lambda (deviceCode.cu:304-323).
  float rlo0 = t0, rhi0 = t1, rlo1 = __builtin_inff(), rhi1 = -__builtin_inff();
  int numRanges = 1;
  if (!ae) {
    float st1 = 0.f, st2 = 0.f, st3 = 0.f, st4 = 0.f;
    const bool s1 = intersect_sphere(ray, A.sbHi.x, st1, st4);
    const bool s2 = intersect_sphere(ray, A.sbLo.x, st2, st3);
    numRanges = 0;
    if ((s1 || s2) && !(st4 < t0)) {  // ray.tmin == t0 here
      numRanges = 2;
      if (s1 && !s2) {
        rlo0 = st1; rhi0 = st4;
      } else if (t0 < st2) {
        rlo0 = st1; rhi0 = st2;
        rlo1 = st3; rhi1 = st4;
      } else {
        rlo0 = st3; rhi0 = st4;
      }
    }
  }
  if constexpr ((OPT & OPT_GRID) != 0) {
    if (!ae) {
      render_grid(A, T, ray, t0, t1, st, cr, cg, cb, alpha);
      numRanges = 0;
    }
  }
  const float sceneEPS = A.sbLo.x * 1e-6f;
  for (int i = 0; i < numRanges; ++i) {
    const float lower = i ? rlo1 : rlo0, upper = i ? rhi1 : rhi0;
    if (upper <= lower) break;  // box1f::empty (vecmath.h:981)
    const bool lastRange = ae || i == 1 || rhi1 <= rlo1;
    // cellID of the entry point (ShellAccel.h:121-124)
    int cx = 0, cy = 0, cz = 0;
    if (!ae) {
      const float e1 = lower + sceneEPS;
      float r1, la1, lo1;
      to_spherical(ray.ox + ray.dx * e1, ray.oy + ray.dy * e1, ray.oz + ray.dz * e1, r1, la1, lo1);
      cx = project_axis(r1, A.sbLo.x, A.sbHi.x, A.dims.x);
      cy = project_axis(la1, A.sbLo.y, A.sbHi.y, A.dims.y);
      cz = project_axis(lo1, A.sbLo.z, A.sbHi.z, A.dims.z);
      if (!lastRange) lds_st16(&s_entry[tid], make_float4(r1, la1, lo1, 0.f));  // for step (125-127)
    }
    // The lat/lon "planes" (ShellAccel.h:147-160, 183-200) are built from
    // toCartesian(vec3f(0.f, ...)) -- radius 0 -- so N = 0, w = 0 and every evalPlane(...)
    // is exactly +-0: tnext = {upper, 0, 0} throughout, and the sign of those zeros never
    // changes a comparison.  (radius/sphereT1, 136-146, is dead.)  So only a range's FIRST
    // leaf can have positive length: every later one is [t_c, t_c] with t_c = min(upper, 0),
    // where woodcockTracking can only consume draws (its tw <= tmax == tmin never passes
    // deviceCode.cu:316).  Those leaves matter only through the RNG state, i.e. only when
    // another range follows -- and only then are the exit point, step and stop needed.
    const float tnx = upper, tny = 0.f, tnz = 0.f;
    float t = lower;
    for (int iter = 0; iter < (1 << 22); ++iter) {
      float tt1 = IRT_FLT_MAX;
      if (ae) {
        tt1 = upper;
      } else {
        if (tnx < tt1 && tnx >= t) tt1 = tnx;
        if (tny < tt1 && tny >= t) tt1 = tny;
        if (tnz < tt1 && tnz >= t) tt1 = tnz;
      }
      const bool zeroLen = tt1 == t;
      if (zeroLen && lastRange) break;
      if constexpr ((OPT & OPT_STATS) != 0) T.cnt.deg += zeroLen ? 1u : 0u;
      float maj = 1.f;
      if (!ae) {
        const uint32_t leaf = (uint32_t)wrap_coord(cz, A.dims.z) * (uint32_t)A.dims.x * (uint32_t)A.dims.y +
                              (uint32_t)wrap_coord(cy, A.dims.y) * (uint32_t)A.dims.x +
                              (uint32_t)wrap_coord(cx, A.dims.x);
        maj = A.maxOp[leaf];
      }
      bool fast = false;
      if (zeroLen) {
        const float q = maj / A.unitDistance;
        const uint32_t nx = lcg_next(st);
        if (!(maj > 0.f)) {
          fast = true;  // woodcockTracking returns at once (deviceCode.cu:161-162)
        } else if (q > 0.f && q <= 1e30f && (nx & 0x00FFFFFFu) != 0u) {
          st = nx;  // one draw: logf(1-xi) < 0 puts t past tmax (165-166)
          fast = true;
        }
      }
      if (!fast) {  // woodcockFunc(leafID, t, tt1)
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool counted = !zeroLen;
        const float tw = T.woodcock(ray.dx, ray.dy, ray.dz, t, tt1, st, maj, s, counted);
        if (!zeroLen && (ae || (tw > t && tw < tt1))) {
          // AE: colour/alpha from the last accepted sample, zero if none (239-275)
          cr = s.x * A.amb.x * A.ambRad;
          cg = s.y * A.amb.y * A.ambRad;
          cb = s.z * A.amb.z * A.ambRad;
          alpha = s.w > 0.f ? 1.f : 0.f;
          i = 2;  // done: no further ranges
          break;
        }
      }
      if (lastRange) break;  // every later leaf of the last range is zero-length
      int4 dd;               // {packed steps, ex, ey, ez}
      if (iter == 0) {
        // exit point, step and stop (ShellAccel.h:125-132), first needed now
        const float e2 = upper - sceneEPS;
        float r2, la2, lo2;
        to_spherical(ray.ox + ray.dx * e2, ray.oy + ray.dy * e2, ray.oz + ray.dz * e2, r2, la2, lo2);
        const float4 en = lds_ld16(&s_entry[tid]);
        const float r1 = en.x, la1 = en.y, lo1 = en.z;
        const int sx = r1 < r2 ? 1 : -1, sy = la1 < la2 ? 1 : -1, sz = lo1 < lo2 ? 1 : -1;
        dd.x = (sx > 0 ? 1 : 0) | (sy > 0 ? 2 : 0) | (sz > 0 ? 4 : 0);
        dd.y = (int)((uint32_t)project_axis(r2, A.sbLo.x, A.sbHi.x, A.dims.x) + (uint32_t)sx);
        dd.z = (int)((uint32_t)project_axis(la2, A.sbLo.y, A.sbHi.y, A.dims.y) + (uint32_t)sy);
        dd.w = (int)((uint32_t)project_axis(lo2, A.sbLo.z, A.sbHi.z, A.dims.z) + (uint32_t)sz);
        s_dda[tid] = dd;
      } else {
        dd = s_dda[tid];
      }
      const float t_closest = fminf(fminf(tnx, tny), tnz);
      if (tnx == t_closest) {
        cx += (dd.x & 1) ? 1 : -1;
        if (cx == dd.y) break;
      }
      if (tny == t_closest) {
        cy += (dd.x & 2) ? 1 : -1;
        if (cy == dd.z) break;
      }
      if (tnz == t_closest) {
        cz += (dd.x & 4) ? 1 : -1;
        if (cz == dd.w) break;
      }
      t = t_closest;
    }
  }
  if (sampleOut)
    *sampleOut = make_float4(cr, cg, cb, alpha);
  else
    write_pixel(A, px.outIdx, cr, cg, cb, alpha, s_th);
}

// toSpherical (ICONGrid.h:36-42) of an sdda entry or exit point with the certified fast
// lat/lon (irt_device.h): r exactly, lat/lon within kLatErr/kLonErr of glibc's, and the
// point's shell-grid cells (ShellAccel.h:121-124, 128-130).  Returns false when a cell is
// not certified (the caller takes the glibc-exact path, to_spherical).
__device__ __forceinline__ bool spherical_fast(const RenderArgs &A, float x, float y, float z, float &r, float &la,
                                               float &lo, int &cy, int &cz) {
  r = sqrtf(dot3(x, y, z, x, y, z));
  la = fast_asin(z / r);  // z / r rounds as toSpherical's
  const bool okLon = fast_atan2(y, x, lo);
  const bool okY = cell_certified(la, kLatErr, A.sbLo.y, A.invSb[1], A.dims.y, cy);
  const bool okZ = cell_certified(lo, kLonErr, A.sbLo.z, A.invSb[2], A.dims.z, cz);
  return okY && okZ && okLon;
}

// render_pixel restated as a per-lane state machine whose one Woodcock call site is reached
// by the whole wave together (Tracer::woodcock_wave): each lane runs its ranges and sdda
// leaves on its own until it needs a woodcockFunc on a leaf (kWait) or is finished
// (kDone); then the wave tracks every waiting lane's leaf at once, and each lane resumes
// with the leaf's outcome.  Every lane of the wave calls it (those without a pixel start
// finished).  Same ranges, leaves, draws and results as render_pixel, step for step.

template <int OPT>
__device__ __forceinline__ void render_pixel_coop(const RenderArgs &A, Tracer<OPT> &T, const Pixel &px,
                                                  const float *s_th, int4 *s_dda, float4 *s_entry,
                                                  float4 *s_acc, CoopWave &W, ScanWave *SW, const uint2 *jmp,
                                                  int tid, int accumID, uint32_t blk, int pwave, int frame,
                                                  int partSel = -1, int pairPos = 0) {
  // At 5+ waves/SIMD the pixel's output addresses are recomputed where they are used (from the
  // workgroup's uniform block index), not held in VGPRs through the rounds: a progressive
  // batch's sample slot (k_accumulate reads it) and the frame index.  (At 4 waves there is
  // room for them, and recomputing costs 1 %: profiles/r03u_waves/.)
  constexpr bool kRecompute = ((OPT >> 8) & 15) >= 5;
  // the pixel's thread index within its 256-pixel block: the packet's wave pwave (uniform) of
  // the block, and the lane (tid is the LDS index within this workgroup: a persistent launch's
  // wave renders any packet; OPT_WAVEWG has four one-wave workgroups per block)
  const int ptid = pwave * 64 + (tid & 63);
  // ... and so is the thread index itself after the rounds: the wave's base (uniform, an SGPR)
  // plus the lane id, instead of tid and the pixel's in-block coordinates held in scratch
  // across the rounds (24 B per lane of spill stores and reloads at 5 waves)
  const int wbase = __builtin_amdgcn_readfirstlane(tid) & ~63;
  auto tid_late = [&]() { return kRecompute ? (opaque_u(wbase) | (int)__lane_id()) : tid; };
  auto ptid_late = [&]() {
    if constexpr (!kRecompute) return ptid;
    int lane = (int)__lane_id();
    asm volatile("" : "+v"(lane));  // not CSE'd with the pixel's coordinates at the ray's start
    if (partSel >= 0) {  // a split packet's part (k_render): pn rays from ray part * pn
      const int ps = opaque_u(partSel), pn = 64 >> (ps & 255);
      lane = ((ps >> 8) * pn) | (lane & (pn - 1));
    }
    return (opaque_u(pwave) << 6) | lane;
  };
  const bool toSample = A.numSamples > 1 && !A.chain;
  // chained frames: frame f > 0 of the launch reads its accum pixel at the end, once frame
  // f - 1's wave has published it (chain_wait); frame 0 prefetches it as a single frame does
  // (pairPos, the OPT_FPAIR kernels: 1 = the first of two consecutive frames this wave
  // renders -- no publish --, 2 = the second -- its previous frame is this wave's own, so no wait,
  // and its accum pixel is read back, past this CU's L1, at the end)
  const bool chainLate = A.chain && frame > 0 && pairPos != 2;
  // ... unless frame f - 1's wave has published by the time this wave's rays are set up (a
  // large frame's previous-frame workgroup ran numBlocks workgroups earlier): its publish word,
  // loaded now, compared after the box test, and then the accum pixel prefetched (sc1) as frame 0
  uint32_t chainSeen = 0u;
  if (chainLate)
    chainSeen = __hip_atomic_load(A.chainFlag + (size_t)blk * 4u + (uint32_t)pwave, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  float4 *const slot0 = kRecompute || !toSample
                            ? nullptr
                            : A.sampleBuf + (size_t)frame * A.numTiles * 4096u + (size_t)blk * 256u + (size_t)ptid;
  auto sample_slot = [&]() {
    if constexpr (!kRecompute) return slot0;
    return A.sampleBuf + (size_t)opaque_u(frame) * opaque_u(A.numTiles) * 4096u + (size_t)opaque_u((int)blk) * 256u +
           (size_t)ptid_late();
  };
  enum : int { kRange, kLeaf, kWait, kDone, kGrid, kGridNext };
  constexpr bool kFastSph = (OPT & OPT_FASTSPH) != 0;
  constexpr bool grid = (OPT & OPT_GRID) != 0;
  const bool ae = A.raygen == 1;
  // OPT_ACCPF: the lerp's accum pixel straight into the wave's LDS slots now (a distinct LDS
  // array: the compiler's LDS-DMA tracking waits for it only where the slots are read, at the end)
  constexpr bool accPf = (OPT & OPT_ACCPF) != 0 && (OPT & OPT_LEAN) != 0;
  const bool accEarly = accPf && !toSample && !chainLate;
  if (accEarly && px.active)
    __builtin_amdgcn_global_load_lds((const void *)(A.accum + px.outIdx),
                                     (__attribute__((address_space(3))) void *)(s_acc + (tid & ~63)), 16, 0, 0);
  uint32_t st = 0;
  float dx = 1.f, dy = 1.f, dz = 1.f;
  float rlo0 = 0.f, rhi0 = 0.f, rlo1 = __builtin_inff(), rhi1 = -__builtin_inff();
  int numRanges = 0, phase = kDone;
  bool inBox = false;
  float t0box = 0.f, t1box = 0.f;
  if (px.active) {
    gen_ray(A, accumID, px.x, px.y, st, dx, dy, dz, frame);
    const float3 O = cam_org(A, frame);
    const Ray ray = {O.x, O.y, O.z, 0.f, dx, dy, dz, 1e10f};
    float t0, t1;
    const bool boxHit = box_test(ray, A, t0, t1);
#ifdef IRT_PROBE_BUILD
    // measurement only (30): 200 extra VALU instructions per wave in the ray setup -- is the
    // frame's time sensitive to VALU work at all?
    if (A.probeExit == 30) {
#pragma nounroll
      for (int k = 0; k < 50; ++k) asm volatile("v_nop\n v_nop\n v_nop\n v_nop" ::: "memory");
    }
#endif
    if (A.probeExit == 3) {  // measurement only: ray generation and boxTest, nothing written
      if (boxHit && t0 == -1.2345f) A.fb[0] = 0u;  // keeps the work live
      return;
    }
    if (boxHit) {
      inBox = true;  // counted at the ray's end: an LDS add here would wait for the prologue's LDS-DMA
      phase = kRange;
      t0box = t0;
      t1box = t1;
      // the accum pixel the lerp reads at the end, fetched now straight into LDS (no VGPRs
      // held through the Woodcock rounds; its latency hides behind them)
      if (!toSample && !chainLate && (OPT & OPT_LEAN) == 0)
        __builtin_amdgcn_global_load_lds((const void *)(A.accum + px.outIdx),
                                         (__attribute__((address_space(3))) void *)(s_acc + (tid & ~63)),
                                         16, 0, kRecompute ? 2 : 0);  // 2: nt (write_pixel)
      rlo0 = t0;
      rhi0 = t1;
      numRanges = 1;
      if (!ae) {  // the shell's sphere ranges, as render_pixel
        float st1 = 0.f, st2 = 0.f, st3 = 0.f, st4 = 0.f;
        bool s1, s2;
        intersect_spheres(ray, A.sbHi.x, A.sbLo.x, s1, st1, st4, s2, st2, st3);
        numRanges = 0;
        if ((s1 || s2) && !(st4 < t0)) {
          numRanges = 2;
          if (s1 && !s2) {
            rlo0 = st1; rhi0 = st4;
          } else if (t0 < st2) {
            rlo0 = st1; rhi0 = st2;
            rlo1 = st3; rhi1 = st4;
          } else {
            rlo0 = st3; rhi0 = st4;
          }
        }
      }
    } else if (toSample) {
      *sample_slot() = make_float4(0.f, 0.f, 0.f, kNoSample);  // deviceCode.cu:294-295
    }
  }
  const bool chainReady = !chainLate || __builtin_amdgcn_readfirstlane(chainSeen) == A.chainEpoch + (uint32_t)frame;
  if ((OPT & OPT_LEAN) == 0 && chainLate && chainReady && inBox)
    __builtin_amdgcn_global_load_lds((const void *)(A.accum + px.outIdx),
                                     (__attribute__((address_space(3))) void *)(s_acc + (tid & ~63)), 16, 0, 16);  // sc1
  // GRID_ACCEL_MODE (deviceCode.cu:326-328): dda3 (DDA.h:35-136) over the 256^3 grid as
  // render_grid walks it, each cell's woodcockFunc one of the wave's cooperative requests
  int gcx = 0, gcy = 0, gcz = 0, gsteps = 0, gdirs = 0;
  float gtnx = 0.f, gtny = 0.f, gtnz = 0.f, gdx = 0.f, gdy = 0.f, gdz = 0.f, gtmax = 0.f, grtmin = 0.f,
        gtc0 = 0.f, gtc1 = 0.f;
  if constexpr (grid) {
    if (phase == kRange && !ae) {
      const float rtmin = t0box, rtmax = t1box;  // the box interval [t0, t1]
      const int D = kGridDim;
      const float3 O = cam_org(A, frame);
      const float ox = O.x + rtmin * dx, oy = O.y + rtmin * dy, oz = O.z + rtmin * dz;
      gtmax = rtmax - rtmin;
      grtmin = rtmin;
      const float rx = 1.f / dx, ry = 1.f / dy, rz = 1.f / dz;
      const float lx = (A.bmin.x - ox) * rx, ly = (A.bmin.y - oy) * ry, lz = (A.bmin.z - oz) * rz;
      const float hx = (A.bmax.x - ox) * rx, hy = (A.bmax.y - oy) * ry, hz = (A.bmax.z - oz) * rz;
      float nx = fminf(lx, hx), ny = fminf(ly, hy), nz = fminf(lz, hz);
      const float fx = fmaxf(lx, hx), fy = fmaxf(ly, hy), fz = fmaxf(lz, hz);
      if (dx == 0.f) nx = IRT_FLT_MAX;
      if (dy == 0.f) ny = IRT_FLT_MAX;
      if (dz == 0.f) nz = IRT_FLT_MAX;
      gcx = project_on_grid(ox, A.bmin.x, A.bmax.x, D);
      gcy = project_on_grid(oy, A.bmin.y, A.bmax.y, D);
      gcz = project_on_grid(oz, A.bmin.z, A.bmax.z, D);
      gdx = fmaxf(0.f, (fx - nx) / (float)D);
      gdy = fmaxf(0.f, (fy - ny) / (float)D);
      gdz = fmaxf(0.f, (fz - nz) / (float)D);
      gdirs = (dx > 0.f ? 1 : 0) | (dy > 0.f ? 2 : 0) | (dz > 0.f ? 4 : 0);
      gtnx = dx > 0.f ? nx + (float)(gcx + 1) * gdx : nx + (float)(D - gcx) * gdx;
      gtny = dy > 0.f ? ny + (float)(gcy + 1) * gdy : ny + (float)(D - gcy) * gdy;
      gtnz = dz > 0.f ? nz + (float)(gcz + 1) * gdz : nz + (float)(D - gcz) * gdz;
      phase = kGrid;
    }
  }
  // sceneEPS (ShellAccel.h:121-127), recomputed where it is used (a VALU product the
  // compiler would otherwise hold in a VGPR through every loop)
  auto sceneEPS = [&]() {
    const RenderArgs &SA = IRT_SM_ARGS;
    return opaque_u(SA.sbLo.x) * 1e-6f;
  };
  int i = 0, iter = 0, cx = 0, cy = 0, cz = 0;
  float t = 0.f, upper = 0.f, tt1 = 0.f, maj = 0.f;
  bool lastRange = true, zeroLen = false, hit = false;
  bool miss = false;  // the cooperative loop's speculation mode, carried from leaf to leaf
  bool first = true;  // OPT_TIMING
  // after a leaf without a hit: the next leaf of the range, or the next range
  // (render_pixel's loop tail, ShellAccel.h:201-226)
  auto next_leaf = [&]() {
    const RenderArgs &SA = IRT_SM_ARGS;
    if (lastRange) {  // every later leaf of the last range is zero-length
      ++i;
      phase = kRange;
      return;
    }
    const float tnx = upper, tny = 0.f, tnz = 0.f;
    int4 dd;
    if (iter == 0) {
      // exit point, step and stop (ShellAccel.h:125-132); the entry's (r1, la1, lo1, lower)
      // wait in s_entry.  OPT_FASTSPH: the certified fast lat/lon (spherical_fast).
      const float e2 = upper - sceneEPS();
      float r2, la2, lo2;
      int cy2 = 0, cz2 = 0;
      bool ok2 = false;
      const float3 O = cam_org(SA, frame);
      if constexpr (kFastSph)
        ok2 = spherical_fast(A, O.x + dx * e2, O.y + dy * e2, O.z + dz * e2, r2, la2, lo2, cy2, cz2);
      else
        to_spherical(O.x + dx * e2, O.y + dy * e2, O.z + dz * e2, r2, la2, lo2);
      const float4 en = lds_ld16(&s_entry[tid_late()]);
      const float r1 = en.x;
      const int sx = r1 < r2 ? 1 : -1;
      int sy, sz;
      if constexpr (!kFastSph) {
        sy = en.y < la2 ? 1 : -1;
        sz = en.z < lo2 ? 1 : -1;
        cy2 = project_axis_inv(la2, SA.sbLo.y, SA.invSb[1], SA.dims.y);
        cz2 = project_axis_inv(lo2, SA.sbLo.z, SA.invSb[2], SA.dims.z);
      } else {
        sy = sign_certified(en.y, la2, kLatErr);
        sz = sign_certified(en.z, lo2, kLonErr);
      }
      if (kFastSph && (!ok2 || sy == 0 || sz == 0)) {  // not certified (rare): both points glibc-exact
        float la1 = 0.f, lo1 = 0.f;
#pragma nounroll
        for (int k = 0; k < 2; ++k) {  // the entry, then the exit point (one inlined copy)
          const float e = k == 0 ? en.w + sceneEPS() : upper - sceneEPS();
          float rr, la, lo;
          to_spherical(O.x + dx * e, O.y + dy * e, O.z + dz * e, rr, la, lo);
          if (k == 0) {
            la1 = la;
            lo1 = lo;
          } else {
            la2 = la;
            lo2 = lo;
          }
        }
        sy = la1 < la2 ? 1 : -1;
        sz = lo1 < lo2 ? 1 : -1;
        cy2 = project_axis_inv(la2, SA.sbLo.y, SA.invSb[1], SA.dims.y);
        cz2 = project_axis_inv(lo2, SA.sbLo.z, SA.invSb[2], SA.dims.z);
      }
      dd.x = (sx > 0 ? 1 : 0) | (sy > 0 ? 2 : 0) | (sz > 0 ? 4 : 0);
      dd.y = (int)((uint32_t)project_axis_inv(r2, SA.sbLo.x, SA.invSb[0], SA.dims.x) + (uint32_t)sx);
      dd.z = (int)((uint32_t)cy2 + (uint32_t)sy);
      dd.w = (int)((uint32_t)cz2 + (uint32_t)sz);
      lds_st16(&s_entry[tid_late()], __builtin_bit_cast(float4, dd));  // the entry point is not needed again
    } else {
      dd = __builtin_bit_cast(int4, lds_ld16(&s_entry[tid_late()]));
    }
    const float t_closest = fminf(fminf(tnx, tny), tnz);
    bool stop = false;
    if (tnx == t_closest) {
      cx += (dd.x & 1) ? 1 : -1;
      stop = cx == dd.y;
    }
    if (!stop && tny == t_closest) {
      cy += (dd.x & 2) ? 1 : -1;
      stop = cy == dd.z;
    }
    if (!stop && tnz == t_closest) {
      cz += (dd.x & 4) ? 1 : -1;
      stop = cz == dd.w;
    }
    t = t_closest;
    if (stop || ++iter >= (1 << 22)) {
      ++i;
      phase = kRange;
    } else {
      phase = kLeaf;
    }
  };
  while (true) {
    if constexpr (grid) {
      // this lane's dda3 cells, on its own: up to the next one whose woodcockFunc can act
      const int D = kGridDim;
      constexpr int NB = kGridDim / kGridBlock;
      while (phase == kGrid || phase == kGridNext) {
        if (phase == kGridNext) {  // the step to the next cell (render_grid)
          const float tmn = fminf(fminf(gtnx, gtny), gtnz);
          bool out = false;
          if (gtnx == tmn) {
            gtnx += gdx;
            gcx += (gdirs & 1) ? 1 : -1;
            out = gcx == ((gdirs & 1) ? D : -1);
          }
          if (!out && gtny == tmn) {
            gtny += gdy;
            gcy += (gdirs & 2) ? 1 : -1;
            out = gcy == ((gdirs & 2) ? D : -1);
          }
          if (!out && gtnz == tmn) {
            gtnz += gdz;
            gcz += (gdirs & 4) ? 1 : -1;
            out = gcz == ((gdirs & 4) ? D : -1);
          }
          gtc0 = gtc1;
          if (out || ++gsteps >= 4 * D + 16) {
            phase = kDone;
            break;
          }
          phase = kGrid;
        }
        const float tmn = fminf(fminf(gtnx, gtny), gtnz);  // reduce_min (vecmath.h:512-514)
        gtc1 = dda3_min_quirk(tmn, gtmax);
        // a cell whose block holds no majorant above 0 (k_grid_bits), or whose own majorant
        // is <= 0: woodcockTracking returns at once (deviceCode.cu:161-162), nothing to do
        const bool inGrid = (unsigned)gcx < (unsigned)D && (unsigned)gcy < (unsigned)D && (unsigned)gcz < (unsigned)D;
        const uint32_t gb = inGrid ? ((uint32_t)(gcz / kGridBlock) * NB + (uint32_t)(gcy / kGridBlock)) * NB +
                                         (uint32_t)(gcx / kGridBlock)
                                   : 0u;
        if (!inGrid || ((T.s_gbits[gb >> 5] >> (gb & 31)) & 1u)) {
          maj = A.gridMaxOp[(size_t)gcz * D * D + (size_t)gcy * D + gcx];
          if (!(maj <= 0.f)) {
            t = grtmin + gtc0;  // woodcockFunc(leaf, ray_tmin + t0, ray_tmin + t1)
            tt1 = grtmin + gtc1;
            zeroLen = t == tt1;  // counted = !(w0 == w1)
            phase = kWait;
            break;
          }
        }
        phase = kGridNext;
      }
    }
    // this lane, on its own: up to its next woodcockFunc, or to the end
    while (phase == kRange || phase == kLeaf) {
      const RenderArgs &SA = IRT_SM_ARGS;
      if (phase == kRange) {
        if (i >= numRanges) {
          phase = kDone;
          break;
        }
        const float lower = i ? rlo1 : rlo0;
        upper = i ? rhi1 : rhi0;
        if (upper <= lower) {  // box1f::empty (vecmath.h:981)
          phase = kDone;
          break;
        }
        lastRange = ae || i == 1 || rhi1 <= rlo1;
        cx = cy = cz = 0;
        if (!ae) {  // cellID of the entry point (ShellAccel.h:121-124)
          const float e1 = lower + sceneEPS();
          const float3 O = cam_org(SA, frame);
          const float x1 = O.x + dx * e1, y1 = O.y + dy * e1, z1 = O.z + dz * e1;
          float r1, la1, lo1;
          // OPT_FASTSPH: the certified fast lat/lon, glibc-exact when not certified
          if (!(kFastSph && spherical_fast(A, x1, y1, z1, r1, la1, lo1, cy, cz))) {
            to_spherical(x1, y1, z1, r1, la1, lo1);
            cy = project_axis_inv(la1, SA.sbLo.y, SA.invSb[1], SA.dims.y);
            cz = project_axis_inv(lo1, SA.sbLo.z, SA.invSb[2], SA.dims.z);
          }
          cx = project_axis_inv(r1, SA.sbLo.x, SA.invSb[0], SA.dims.x);
          // for the exit's step (sign_certified) and its exact fallback (`lower`)
          if (!lastRange) lds_st16(&s_entry[tid_late()], make_float4(r1, la1, lo1, lower));
        }
        t = lower;
        iter = 0;
        phase = kLeaf;
      }
      // the leaf [t, tt1] (tnext = {upper, 0, 0}: render_pixel)
      tt1 = IRT_FLT_MAX;
      if (ae) {
        tt1 = upper;
      } else {
        if (upper < tt1 && upper >= t) tt1 = upper;
        if (0.f < tt1 && 0.f >= t) tt1 = 0.f;
      }
      zeroLen = tt1 == t;
      if (zeroLen && lastRange) {
        ++i;
        phase = kRange;
        continue;
      }
      if (!ae && zeroLen && iter >= 1 && upper > 0.f) {
        // The zero-length leaves after a non-last range's first leaf (see render_pixel): with
        // upper > 0 the walk steps cy and cz together (tnext = {upper, 0, 0}, t = 0) until one reaches its
        // stop, and each leaf only reads its majorant and, if positive, consumes one draw
        // (deviceCode.cu:161-166, the fast path above).  The leaves are known in advance, so
        // their majorants are gathered kWalk at a time (independent loads, one round trip)
        // instead of one dependent gather per leaf; the draws are then applied in order, and
        // a leaf that needs the full woodcockFunc (its draw's low 24 bits zero, or q out of
        // range) is handed to the single-leaf path below.  Same leaves, draws and state.
        const int4 dd = __builtin_bit_cast(int4, lds_ld16(&s_entry[tid_late()]));
        const int sy = (dd.x & 2) ? 1 : -1, sz = (dd.x & 4) ? 1 : -1;
        const int ky = (dd.z - cy) * sy, kz = (dd.w - cz) * sz;  // leaves left: min(ky, kz)
        if (ky >= 1 && kz >= 1 && iter + min(ky, kz) < (1 << 22)) {
          constexpr int kWalk = 8;
          const int n = min(min(ky, kz), kWalk);
          const int dimx = opaque_u(SA.dims.x), dimy = opaque_u(SA.dims.y);
          const uint32_t wx = (uint32_t)wrap_coord(cx, dimx);
          float mj[kWalk];
#pragma unroll
          for (int j = 0; j < kWalk; ++j) {
            mj[j] = 0.f;
            if (j < n) {
              const uint32_t leaf = (uint32_t)wrap_coord(cz + j * sz, SA.dims.z) * (uint32_t)dimx * (uint32_t)dimy +
                                    (uint32_t)wrap_coord(cy + j * sy, dimy) * (uint32_t)dimx + wx;
              mj[j] = SA.maxOp[leaf];
            }
          }
          int done = n;  // leaves taken by the fast path
#pragma unroll
          for (int j = 0; j < kWalk; ++j) {
            if (j < done) {
              const float q = mj[j] / SA.unitDistance;
              const uint32_t nx = lcg_next(st);
              if (!(mj[j] > 0.f)) {
              } else if (q > 0.f && q <= 1e30f && (nx & 0x00FFFFFFu) != 0u) {
                st = nx;
              } else {
                done = j;  // this leaf needs woodcockFunc: the single-leaf path takes it
              }
            }
          }
          if constexpr ((OPT & OPT_STATS) != 0) T.cnt.deg += (uint32_t)done;
          cy += done * sy;
          cz += done * sz;
          iter += done;
          if (done == min(ky, kz)) {  // the walk's stop (render_pixel's loop tail)
            ++i;
            phase = kRange;
            continue;
          }
          if (done == n) continue;  // the next batch
        }
      }
      if constexpr ((OPT & OPT_STATS) != 0) T.cnt.deg += zeroLen ? 1u : 0u;
      maj = 1.f;
      if (!ae) {
        const uint32_t leaf = (uint32_t)wrap_coord(cz, SA.dims.z) * (uint32_t)SA.dims.x * (uint32_t)SA.dims.y +
                              (uint32_t)wrap_coord(cy, SA.dims.y) * (uint32_t)SA.dims.x +
                              (uint32_t)wrap_coord(cx, SA.dims.x);
        maj = SA.maxOp[leaf];
      }
      bool fast = false;
      if (zeroLen) {
        const float q = maj / SA.unitDistance;
        const uint32_t nx = lcg_next(st);
        if (!(maj > 0.f)) {
          fast = true;
        } else if (q > 0.f && q <= 1e30f && (nx & 0x00FFFFFFu) != 0u) {
          st = nx;
          fast = true;
        }
      }
      if (!fast) {
        phase = kWait;
        break;
      }
      next_leaf();
    }
    // the wave, together: woodcockFunc(leafID, t, tt1) of every waiting lane
    const bool req = phase == kWait;
    if (__ballot(req) == 0ull) break;
    if (A.probeExit == 4) break;  // measurement only: ray setup up to the first woodcockFunc
    float tw = t;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr ((OPT & OPT_TIMING) != 0) {
      if (first) {
        T.tmark(1);  // ray setup up to the first woodcockFunc
        first = false;
      }
    }
    T.woodcock_wave(req, dx, dy, dz, tw, tt1, st, maj, !zeroLen, s, miss, W, SW, jmp);
    if (A.probeExit == 5) break;  // measurement only: the first woodcockFunc of every lane
#ifdef IRT_PROBE_BUILD
    if (A.probeExit >= 8 && A.probeExit < 16) break;  // (IRT_ROUND_PROBE)
#endif
    if (grid && req && phase == kWait && !ae) {
      if (tw > t && tw < tt1) {  // render_grid's hit test (deviceCode.cu:316)
        lds_st16(&s_entry[tid_late()], make_float4(s.x * A.amb.x * A.ambRad, s.y * A.amb.y * A.ambRad,
                                   s.z * A.amb.z * A.ambRad, s.w > 0.f ? 1.f : 0.f));
        hit = true;
        phase = kDone;
      } else {
        phase = kGridNext;
      }
    } else if (req) {
      if (!zeroLen && (ae || (tw > t && tw < tt1))) {
        // the colour waits in the lane's s_entry slot (free once it is finished)
        lds_st16(&s_entry[tid_late()], make_float4(s.x * A.amb.x * A.ambRad, s.y * A.amb.y * A.ambRad,
                                   s.z * A.amb.z * A.ambRad, s.w > 0.f ? 1.f : 0.f));
        hit = true;
        phase = kDone;
      } else {
        next_leaf();
      }
    }
  }
  // chained frames: every wave of frame f > 0 waits for frame f - 1's wave of its pixels -- also
  // a wave none of whose rays hit the box, so that the publish words advance in frame order and
  // frame f - 1's word covers every earlier frame's stores
  const RenderArgs &TA = IRT_SM_ARGS;  // the ray's end: chain wait, pixel write
  if (chainLate && !chainReady) chain_wait(TA, blk, pwave, frame);
  {
    const uint64_t ib = __ballot(inBox);  // rays in the box (T.count(1) at the box test)
    if (ib && __lane_id() == (unsigned)__builtin_ctzll(ib)) atomicAdd(&T.s_cnt[1], (uint32_t)__popcll(ib));
  }
  if (!inBox) return;
  const int tl = tid_late();
  const float4 c = hit ? lds_ld16(&s_entry[tl]) : make_float4(0.f, 0.f, 0.f, 0.f);
  if (toSample) {
    *sample_slot() = c;
  } else {
    const size_t outIdx = kRecompute ? pixel_of(TA, (uint32_t)opaque_u((int)blk), ptid_late()).outIdx : px.outIdx;
    if (TA.chain) {
      float4 old;
      if (pairPos == 2 || (chainLate && (!chainReady || (OPT & OPT_LEAN) != 0))) {
        old = chain_load_accum(TA, outIdx);
      } else if constexpr (accPf) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the accum prefetch has landed
        old = lds_ld16(&s_acc[tl]);
      } else if constexpr ((OPT & OPT_LEAN) != 0) {
        old = TA.accum[outIdx];
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the accum prefetch has landed
        old = lds_ld16(&s_acc[tl]);
      }
      // 1.f / (float)(accumID + 1) of this frame, correctly rounded as the host's TA.accumW
      write_pixel_chain(TA, outIdx, c.x, c.y, c.z, c.w, 1.f / (float)(accumID + 1), s_th, old,
                        frame < TA.numSamples - 1 && pairPos != 1);
    } else if constexpr ((OPT & OPT_LEAN) != 0 && !accPf) {
#ifdef IRT_PROBE_BUILD
      if (TA.probeExit == 6) {  // measurement only (probe build): the lerp without its accum read
        write_pixel(TA, outIdx, c.x, c.y, c.z, c.w, s_th, make_float4(0.f, 0.f, 0.f, 0.f));
        return;
      }
      if (TA.probeExit == 7) return;  // measurement only (probe build): no accum read, no pixel stores
#endif
      write_pixel(TA, outIdx, c.x, c.y, c.z, c.w, s_th);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the accum prefetch has landed
      write_pixel<kRecompute>(TA, outIdx, c.x, c.y, c.z, c.w, s_th, lds_ld16(&s_acc[tl]));
    }
  }
}

// The persistent launch's packet queues (RenderArgs::queue, kQueueWords u32 per launch slot):
// one counter per XCD, each on its own 128-B line, and the launch's done count.  XCD x owns
// the 16x16 blocks g (over every frame of the launch) with g % 8 == x -- the grid launch's
// workgroup-to-XCD deal, so each XCD's L2 sees the blocks it would have seen -- and hands out
// their packets in order; a wave on XCD x takes from queue x, and once that is exhausted from
// the others in turn (a plain load first, so finished queues cost no read-modify-write).  (One
// counter for the whole launch, with the next fetch issued at each packet's start: 0.40 ms per
// C3 frame against 0.09, profiles/r04b/.)  The launch's last wave resets every counter (each
// wave's last fetch precedes its done count).
constexpr int kQueueXcds = 8;
struct QueueCursor {
  int cur;        // the queue this wave takes from
  uint32_t dead;  // bit x: queue x is exhausted
};
__device__ __forceinline__ uint32_t queue_take(uint32_t *Q, uint32_t numBlocksAll, QueueCursor &c) {
  while (c.dead != (1u << kQueueXcds) - 1u) {
    const uint32_t x = (uint32_t)c.cur;
    // blocks g < numBlocksAll with g % 8 == x, four packets each
    const uint32_t limit = numBlocksAll > x ? 4u * ((numBlocksAll - x + kQueueXcds - 1) / kQueueXcds) : 0u;
    uint32_t v = 0xFFFFFFFFu;
    if (__lane_id() == 0) {
      uint32_t *q = Q + (size_t)x * kQueueLine;
      if (__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < limit) v = atomicAdd(q, 1u);
    }
    v = __builtin_amdgcn_readfirstlane(v);
    if (v < limit) return ((v >> 2) * kQueueXcds + x) * 4u + (v & 3u);  // block g's packet v & 3
    c.dead |= 1u << x;
    c.cur = (c.cur + 1) & (kQueueXcds - 1);
  }
  return 0xFFFFFFFFu;
}
__device__ __forceinline__ void queue_done(uint32_t *Q) {
  if (__lane_id() == 0) {
    __threadfence();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    if (atomicAdd(&Q[kQueueXcds * kQueueLine], 1u) == waves - 1u) {
      for (int x = 0; x <= kQueueXcds; ++x)
        __hip_atomic_store(&Q[(size_t)x * kQueueLine], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The raygen over the frame grid: one lane per pixel (see pixel_of).
template <int OPT>
__global__ void __launch_bounds__((OPT & OPT_WAVEWG) ? 64 : ((OPT & OPT_WAVEWG2) ? 128 : 256),
                                  ((OPT >> 8) & 15) ? ((OPT >> 8) & 15) : 1)
    k_render(RenderArgs A) {
  constexpr bool lean = (OPT & OPT_LEAN) != 0;
  constexpr bool wavewg = (OPT & OPT_WAVEWG) != 0;
  constexpr int kWpg = wavewg ? 1 : ((OPT & OPT_WAVEWG2) ? 2 : 4);  // waves per workgroup
  constexpr bool split = kWpg < 4;  // several workgroups per 256-pixel block
  static_assert(!split || (lean && Tracer<OPT>::kCoop), "one-/two-wave workgroups: lean, cooperative kernels");
  constexpr int kT = 64 * kWpg;   // threads per workgroup
  constexpr int kW = kT / 64;            // waves per workgroup
  __shared__ float s_th[lean ? 1 : 256];
  __shared__ uint32_t s_cnt[kCnt];
  __shared__ LogfTab s_logf[16];
  __shared__ uint32_t s_sph[lean ? 1 : kSphBitWords];
  __shared__ int4 s_dda[split ? 1 : 256];  // sdda state needed only after a range's first leaf
  __shared__ float4 s_entry[kT];
  __shared__ CoopWave s_coop[kW];   // the cooperative Woodcock loop (kCoop kernels)
  __shared__ ScanWave s_scan[Tracer<OPT>::kWaveScan ? kW : 1];  // its wave-wide candidate scan
  __shared__ HdrStage s_hdrs[(OPT & OPT_HDRLDS) ? kW : 1];       // OPT_HDRLDS: staged header lines
  __shared__ float4 s_acc[lean ? ((OPT & OPT_ACCPF) ? 64 : 1) : 256];  // kCoop: the accum pixels, prefetched
  __shared__ uint2 s_jmp[kLcgJumps];  // lcg_jump's {mul, add} (kLcgJumpTab)
  const int tid = threadIdx.x;
#ifdef IRT_LDS_PAD
  // measurement only (profiles/r06n_gpu.sh): IRT_LDS_PAD unused bytes of LDS per workgroup
  __shared__ float4 s_pad[IRT_LDS_PAD / 16];
  if (A.probeExit == 99) s_pad[tid % (IRT_LDS_PAD / 16)] = make_float4(0.f, 0.f, 0.f, 0.f);
#endif
  if (A.wgTrace && tid == 0) {  // measurement only: the workgroup's start, where it ran
    uint32_t *w = A.wgTrace + 4 * (blockIdx.y * gridDim.x + blockIdx.x);
    w[0] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    w[2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    w[3] = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
  }
  if (A.probeExit == 1) return;  // measurement only
  uint64_t tStart = 0;
  if constexpr ((OPT & OPT_TIMING) != 0) tStart = __builtin_amdgcn_s_memtime();
  // OPT_DMATAB (one-wave workgroups): the LCG jump and logf tables go straight from global
  // memory into LDS (global_load_lds, 16 B per lane: 1,040 + 256 B), and nothing waits for them
  // here -- the compiler's LDS-DMA tracking puts the vmcnt wait before their first read, in the
  // first Woodcock round, so the ray generation and setup overlap the loads (the register path
  // below waits for two round trips before the first ray is generated)
  constexpr bool dmaTab = (OPT & OPT_DMATAB) != 0 && kT == 64 && Tracer<OPT>::kCoop;
  if constexpr (dmaTab) {
    typedef __attribute__((address_space(3))) void *LdsPtr;
    const char *jt = reinterpret_cast<const char *>(&kLcgJumpTab.ma[0][0]);
    static_assert(sizeof(kLcgJumpTab.ma) == kLcgJumps * 8 && kLcgJumps * 8 <= 64 * 16 + 16, "jump table: 65 chunks");
    __builtin_amdgcn_global_load_lds((const void *)(jt + 16 * tid), (LdsPtr)s_jmp, 16, 0, 0);
    if (tid == 0)
      __builtin_amdgcn_global_load_lds((const void *)(jt + 1024), (LdsPtr)(reinterpret_cast<char *>(s_jmp) + 1024), 16, 0, 0);
    static_assert(sizeof(LogfTab) == 16, "logf table: one chunk per entry");
    if (tid < 16) __builtin_amdgcn_global_load_lds((const void *)(kLogfTab + tid), (LdsPtr)s_logf, 16, 0, 0);
  }
  // the prologue's global loads issued together, one wait (not one round trip each)
  const float th = lean ? 0.f : A.srgbTh[tid];
  const LogfTab lt = dmaTab ? LogfTab{0.0, 0.0} : kLogfTab[tid & 15];
  uint32_t sph[kSphBitWords / 256];
  if (!lean && A.numSph) {
#pragma unroll
    for (int k = 0; k < kSphBitWords / 256; ++k) sph[k] = A.sphBits[tid + 256 * k];
  }
  uint2 jmpv[(kLcgJumps + kT - 1) / kT];
#pragma unroll
  for (int k = 0; k < (kLcgJumps + kT - 1) / kT; ++k) {
    const int j = tid + kT * k;
    jmpv[k] = make_uint2(0u, 0u);
    if (!dmaTab && Tracer<OPT>::kCoop && j < kLcgJumps) jmpv[k] = make_uint2(kLcgJumpTab.ma[j][0], kLcgJumpTab.ma[j][1]);
  }
#pragma unroll
  for (int k = 0; k < (kLcgJumps + kT - 1) / kT; ++k) {
    const int j = tid + kT * k;
    if (!dmaTab && Tracer<OPT>::kCoop && j < kLcgJumps) *reinterpret_cast<uvec2 *>(&s_jmp[j]) = __builtin_bit_cast(uvec2, jmpv[k]);
  }
  if constexpr (!lean) s_th[tid] = th;
  if (!dmaTab && tid < 16) s_logf[tid] = lt;
  if (!lean && A.numSph) {
#pragma unroll
    for (int k = 0; k < kSphBitWords / 256; ++k) s_sph[tid + 256 * k] = sph[k];
  }
  if (tid < kCnt) s_cnt[tid] = 0;
  __shared__ uint32_t s_done;  // waves of this workgroup finished (the epilogue)
  if (tid == 0) s_done = 0;
  __shared__ uint32_t s_gbits[(OPT & OPT_GRID) ? kGridBitWords : 1];
  if constexpr ((OPT & OPT_GRID) != 0) {
#pragma unroll
    for (int k = 0; k < kGridBitWords / 256; ++k) s_gbits[tid + 256 * k] = A.gridBits[tid + 256 * k];
  }
  if constexpr (dmaTab)
    __builtin_amdgcn_wave_barrier();  // one wave: its LDS writes are ordered; no wait for the DMA
  else
    __syncthreads();
  if (A.probeExit == 2) return;  // measurement only
  Tracer<OPT> T{{}, A, s_logf, lean ? A.sphBits : s_sph, s_cnt, {0, 0, 0, 0, 0, 0, 0}};
  T.s_gbits = s_gbits;
  const float *th_p = lean ? A.srgbTh : s_th;
  T.s_hdr = &s_hdrs[(OPT & OPT_HDRLDS) ? tid >> 6 : 0];
  // OPT_WAVEWG: four one-wave workgroups per 256-pixel block.  The hardware deals workgroup i
  // to XCD i % 8, so workgroup i renders wave (i >> 3) & 3 of block ((i >> 5) << 3) | (i & 7):
  // a block's four packets share one XCD's L2, as the four waves of a 256-thread workgroup do
  // (numBlocks is a multiple of 16)
  // (OPT_WAVEWG2: two-wave workgroups, workgroup i the waves 2 ((i >> 3) & 1) + {0, 1} of block
  // ((i >> 4) << 3) | (i & 7))
  constexpr uint32_t kNwb = 4 / kWpg;  // workgroups per block
  // A single frame's costliest packets first (A.numSplit, measured-cost scheduling): the
  // launch's first numSplit workgroups render the work items splitList[b] = (packet << 8) | (part
  // << 4) | lg -- part `part` of 2^lg of the packet: its rays part * (64 >> lg) .. on lanes 0 ..
  // (64 >> lg) - 1 (lg = 0: the whole packet) --, ~0u an empty item (numSplit is a multiple of 8);
  // the regular workgroups follow, and those of the listed packets render nothing.
  uint32_t bx = blockIdx.x;
  int partSel = -1;  // (part << 8) | lg for a listed item, -1 for a regular workgroup
  uint32_t splitP = 0u;
  bool emptyItem = false;
  constexpr bool splitOk = wavewg && (OPT & OPT_SPLIT) != 0;
  if constexpr (splitOk) {
    if (bx < A.numSplit) {
      const uint32_t item = scalar_word(A.splitList, bx);
      emptyItem = item == ~0u;
      partSel = emptyItem ? 0 : (int)((((item >> 4) & 15u) << 8) | (item & 15u));
      splitP = emptyItem ? 0u : item >> 8;
    } else {
      bx -= A.numSplit;
    }
  }
  uint32_t wg = split ? (((bx >> 3) / kNwb) << 3) | (bx & 7u) : bx;
  if constexpr ((OPT & OPT_XPAIR) != 0 && wavewg) {
    // tile t's blocks 8 h + x (h = 0, 1: the tile's halves) run on XCD x; here block (x & 3,
    // 2 (x >> 2) + h) of the tile's 4 x 4, so XCD x's two blocks share a block edge
    const uint32_t q = bx >> 5, x = bx & 7u;
    wg = ((q >> 1) << 4) | (x & 3u) | ((x >> 2) << 3) | ((q & 1u) << 2);
  }
  const int wwave = partSel >= 0 ? (int)(splitP & 3u)
                                  : split ? (int)(((bx >> 3) % kNwb) * kWpg) : 0;  // the block's first wave in this workgroup
  const int ptid = split ? wwave * 64 + tid : tid;
  if constexpr ((OPT & OPT_TIMING) != 0) {
    T.tLast = tStart;
    T.tmark(0);  // prologue
  }
  const uint64_t c0 = A.schedCost ? wall_clock64() : 0;
  // grid.y = frame k of a progressive batch (accumID + k), whose colour goes to the sample
  // buffer for k_accumulate; a single frame writes accum/fb directly.  With measured-cost
  // scheduling (irt_context.hip) workgroup b renders block order[b].
  const uint32_t blk = partSel >= 0 ? splitP >> 2 : A.schedOrder ? scalar_word(A.schedOrder, wg) : wg;  // uniform: an SGPR
  // a split packet's regular workgroup: nothing to render (its counts and trace are still written)
  const uint32_t pkt = blk * 4u + (uint32_t)wwave;
  const bool splitAway = splitOk && partSel < 0 && ((scalar_word(A.splitMask, pkt >> 5) >> (pkt & 31u)) & 1u);
  uint32_t launched = 0u;  // rays of this wave's pixels (uniform)
  bool pxActive = false;   // the one-lane-per-ray kernel's pixel
  if constexpr (Tracer<OPT>::kCoop) {
    // One call site for both launch forms.  Grid launch: this workgroup's block, once.
    // Persistent launch (A.queue): the wave pulls packets -- the 8x8-pixel unit a wave renders
    // -- from the launch's counter until none is left, as the reference's thread pool pulls
    // 64x64 tiles (common/thread_pool.h:146-161), each wave on its own (no workgroup
    // barrier: a wave whose packet finishes early takes the next one at once).  Every packet
    // renders exactly as in the grid launch (same block, wave, frame, seeds).  The next index
    // is fetched when a packet starts, so its round trip hides behind the packet's work.
    constexpr bool queued = (OPT & OPT_QUEUE) != 0;
    static_assert(!queued || (!split && (OPT & (OPT_STATS | OPT_TIMING | OPT_HDRLDS)) == 0),
                  "persistent launches: 256-thread workgroups, no per-wave statistics");
    const uint32_t perFrame = (uint32_t)A.numTiles * 16u;  // blocks per frame
    const uint32_t blocksAll = perFrame * (uint32_t)A.numSamples;
    QueueCursor qc = {(int)(blockIdx.x & (kQueueXcds - 1)), 0u};  // workgroup b runs on XCD b % 8
    uint32_t p = queued ? queue_take(A.queue, blocksAll, qc) : 0u;
    bool more = !queued || p != 0xFFFFFFFFu;
    // chained frames two per wave (OPT_FPAIR): workgroup (b, y) renders frames
    // 2y and 2y + 1 of its packet, one after the other
    const int fpw = (OPT & OPT_FPAIR) != 0 && !queued && A.chain ? 2 : 1;
    int fi = 0;
    while (more) {
      uint32_t pblk = blk, nx = 0u;
      int pw = wwave + (tid >> 6), frame = (int)blockIdx.y * fpw + fi;
      if constexpr (queued) {
        const uint32_t g = p >> 2;  // the packet's block over all frames
        frame = A.numSamples > 1 ? (int)(g / perFrame) : 0;
        pblk = g - (uint32_t)frame * perFrame;
        pw = (int)(p & 3u);
      }
      pblk = __builtin_amdgcn_readfirstlane(pblk);
      pw = __builtin_amdgcn_readfirstlane(pw);
      frame = __builtin_amdgcn_readfirstlane(frame);
      // the thread index, new to the compiler in every iteration: what derives from it (the
      // pixel's coordinates, LDS slot addresses) is recomputed per packet, not hoisted out of
      // the loop and held in VGPRs through it
      int ltid = tid;
      if constexpr (queued) {
        asm volatile("" : "+v"(ltid));
        // ... and so are the launch's arguments: the kernel-argument segment (RenderArgs is the
        // kernel's only argument, at offset 0) through a pointer the compiler cannot follow
        // across iterations.  Every value derived from them (the box's corners relative to
        // the eye, |eye|^2, cube-map and LUT scales, ...) is then computed per packet as in
        // the grid launch, instead of once before the loop and held in VGPRs (or scratch)
        // through every packet.
        typedef const __attribute__((address_space(4))) RenderArgs *KArgs;
        KArgs kp = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        const RenderArgs &AL = *(const RenderArgs *)kp;
        Tracer<OPT> TL{{}, AL, s_logf, lean ? AL.sphBits : s_sph, s_cnt, {0, 0, 0, 0, 0, 0, 0}};
        TL.s_gbits = s_gbits;
        const Pixel ppx = pixel_of(AL, pblk, pw * 64 + (ltid & 63));
        launched += (uint32_t)__popcll(__ballot(ppx.active));
        render_pixel_coop<OPT>(AL, TL, ppx, lean ? AL.srgbTh : s_th, s_dda, s_entry, s_acc, s_coop[ltid >> 6],
                               &s_scan[Tracer<OPT>::kWaveScan ? ltid >> 6 : 0], s_jmp, ltid, AL.accumID + frame,
                               pblk, pw, frame);
        TL.flush_coop();  // this packet's counts (nothing carried from packet to packet)
      } else if constexpr ((OPT & OPT_FPAIR) != 0) {
        // two chained frames per wave: as the persistent launch, the thread index and the
        // launch's arguments are new to the compiler in each of the wave's frames, so nothing
        // derived from them is held through both
        asm volatile("" : "+v"(ltid));
        typedef const __attribute__((address_space(4))) RenderArgs *KArgs;
        KArgs kp = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        const RenderArgs &AL = *(const RenderArgs *)kp;
        Tracer<OPT> TL{{}, AL, s_logf, lean ? AL.sphBits : s_sph, s_cnt, {0, 0, 0, 0, 0, 0, 0}};
        TL.s_gbits = s_gbits;
        TL.frame = frame;
        const Pixel ppx = pixel_of(AL, pblk, pw * 64 + (ltid & 63));
        launched += (uint32_t)__popcll(__ballot(ppx.active));
        const bool pairNext = fpw == 2 && fi == 0 && frame + 1 < AL.numSamples;  // this wave renders frame + 1 too
        render_pixel_coop<OPT>(AL, TL, ppx, lean ? AL.srgbTh : s_th, s_dda, s_entry, s_acc, s_coop[ltid >> 6],
                               &s_scan[Tracer<OPT>::kWaveScan ? ltid >> 6 : 0], s_jmp, ltid, cam_accum_id(AL, frame),
                               pblk, pw, frame, -1, pairNext ? 1 : (fi == 1 ? 2 : 0));
        TL.flush_coop();  // this frame's counts
        if (AL.chain && frame < AL.numSamples - 1 && frame != AL.chainWithhold && !pairNext) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (__lane_id() == 0)
            __hip_atomic_store(AL.chainFlag + (size_t)pblk * 4u + (uint32_t)pw, AL.chainEpoch + (uint32_t)frame + 1u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        const int pl = partSel & 255, pn = 64 >> pl;  // a split packet's part: pn rays
        Pixel ppx = pixel_of(A, pblk, pw * 64 + (partSel < 0 ? (ltid & 63) : ((partSel >> 8) * pn) | (ltid & (pn - 1))));
        if (partSel >= 0) ppx.active = ppx.active && (ltid & 63) < pn;
        if (splitAway || emptyItem) ppx.active = false;
        launched += (uint32_t)__popcll(__ballot(ppx.active));
        T.frame = frame;
        render_pixel_coop<OPT>(A, T, ppx, th_p, s_dda, s_entry, s_acc, s_coop[ltid >> 6],
                               &s_scan[Tracer<OPT>::kWaveScan ? ltid >> 6 : 0], s_jmp, ltid, cam_accum_id(A, frame),
                               pblk, pw, frame, partSel);
        if (A.chain && frame < A.numSamples - 1 && frame != A.chainWithhold) {
          // chained frames: this wave's pixels are written through; tell frame + 1's wave
#ifdef IRT_PROBE_BUILD
          if (A.probeExit != 16)  // measurement only (16, probe build): the flag without the drain
#endif
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (__lane_id() == 0)
            __hip_atomic_store(A.chainFlag + (size_t)pblk * 4u + (uint32_t)pw, A.chainEpoch + (uint32_t)frame + 1u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      // the next packet once this one is done: a fetch issued at the packet's start (to
      // hide its round trip) made the packet's first gather wait for it as well (vector
      // memory counts retire in order) -- 0.32 ms per C3 frame against 0.09 (profiles/r04c/)
      if constexpr (queued) nx = queue_take(A.queue, blocksAll, qc);
      p = nx;
      more = queued && p != 0xFFFFFFFFu;
      if ((OPT & OPT_FPAIR) != 0 && !queued && fpw == 2 && fi == 0 && frame + 1 < A.numSamples) {
        fi = 1;
        more = true;
      }
    }
    if constexpr (queued) queue_done(A.queue);
    T.flush_coop();
  }
  else {
    const Pixel px = pixel_of(A, blk, ptid);
    float4 *slot = A.numSamples > 1 ? A.sampleBuf + (size_t)blockIdx.y * gridDim.x * blockDim.x + blk * 256u + ptid
                                    : nullptr;
    if (px.active) render_pixel<OPT>(A, T, px, th_p, s_dda, s_entry, tid, A.accumID + (int)blockIdx.y, slot);
    pxActive = px.active;
    launched = (uint32_t)__popcll(__ballot(px.active));
  }
  if constexpr ((OPT & OPT_TIMING) != 0) {
    T.tmark(8);  // after the last woodcockFunc: pixel write, epilogue
    if ((tid & 63) == 0) {
      for (int k = 0; k < TimeAccOn::kTimeRegions; ++k)
        atomicAdd(&A.counters[5 + k], (unsigned long long)T.tAcc[k]);
      atomicAdd(&A.counters[14], (unsigned long long)(__builtin_amdgcn_s_memtime() - tStart));
      atomicAdd(&A.counters[15], 1ull);
    }
  }
  if constexpr ((OPT & OPT_STATS) != 0) {
    // Woodcock draws and zero-length sdda leaves: sums, per-wave maxima, draws histogram
    uint32_t ss = T.cnt.steps, sm = T.cnt.steps, ds = T.cnt.deg, dm = T.cnt.deg;
    for (int off = 32; off > 0; off >>= 1) {
      ss += __shfl_down(ss, off, 64);
      sm = max(sm, (uint32_t)__shfl_down(sm, off, 64));
      ds += __shfl_down(ds, off, 64);
      dm = max(dm, (uint32_t)__shfl_down(dm, off, 64));
    }
    const uint32_t d = T.cnt.steps;  // draws histogram: 0, 1-2, 3-5, > 5
    const int bkt = d == 0 ? 0 : (d <= 2 ? 1 : (d <= 5 ? 2 : 3));
    uint32_t hist[4];
    for (int k = 0; k < 4; ++k)
      hist[k] = T.kCoop ? Tracer<OPT>::wave_sum(T.cnt.candHist[k])
                        : (uint32_t)__popcll(__ballot(pxActive && bkt == k));
    if ((tid & 63) == 0) {
      atomicAdd(&A.counters[5], (unsigned long long)ss);
      atomicAdd(&A.counters[6], (unsigned long long)sm);
      atomicAdd(&A.counters[7], (unsigned long long)(T.kCoop ? T.cnt.hops : ds));       // uniform per wave
      atomicAdd(&A.counters[8], (unsigned long long)(T.kCoop ? T.cnt.locRounds : dm));  // likewise
      atomicMax(&A.counters[9], (unsigned long long)sm);
      atomicMax(&A.counters[10], (unsigned long long)dm);
      atomicAdd(&A.counters[11], (unsigned long long)T.cnt.rounds);  // uniform per wave
      for (int k = 0; k < 4; ++k)
        if (hist[k]) atomicAdd(&A.counters[12 + k], (unsigned long long)hist[k]);
    }
  }
  if (A.counters || A.schedCost || A.wgTrace) {
    const int lane = (int)__lane_id();
    if (A.counters && lane == 0 && launched) atomicAdd(&s_cnt[0], launched);  // rays launched, once per wave
    // The last wave of the workgroup to get here writes the workgroup's counts and duration.
    // No end-of-workgroup barrier: a wave that finishes early frees its slot at once instead
    // of waiting for the slowest wave of its workgroup.  The acq-rel LDS add orders every
    // wave's count adds before the last wave's reads.
    uint32_t prev = 0;
    if (lane == 0)
      prev = __hip_atomic_fetch_add(&s_done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    prev = (uint32_t)__shfl((int)prev, 0, 64);
    if (prev == (blockDim.x >> 6) - 1u) {
      if (A.counters) flush_counters(A, s_cnt, lane);
      if (A.schedCost && lane == 0 && (wavewg || wwave == 0) && !splitAway && !emptyItem) {  // this workgroup's duration, for the next launches' order
        // per packet (4 per block; a 256-thread workgroup's in its first packet's slot), a split
        // packet's part counted for the whole packet (parts x its duration)
        uint64_t dt = wall_clock64() - c0;
        if (partSel >= 0) dt <<= (partSel & 255);
        A.schedCost[pkt] = dt > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)dt;
      }
      if (A.wgTrace && lane == 0)
        A.wgTrace[4 * (blockIdx.y * gridDim.x + blockIdx.x) + 1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    }
  }
}

// ------------------------------------------------------------------ progressive batch
// The lerp chain of K consecutive frames (deviceCode.cu:333-334, accumID..accumID+K-1) over
// the per-frame samples k_render stored, in frame order: bit-identical to K launches.
// Frames whose ray missed the box leave the pixel untouched (kNoSample), as the
// reference's raygen returns before writing (294-295); fb is written after the last frame.
__global__ void __launch_bounds__(256) k_accumulate(RenderArgs A) {
  __shared__ float s_th[256];
  s_th[threadIdx.x] = A.srgbTh[threadIdx.x];
  __syncthreads();
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  const Pixel px = pixel_of(A, blockIdx.x, (int)threadIdx.x);
  if (!px.active) return;
  const size_t lanes = (size_t)gridDim.x * 256u;
  float4 a = A.accum[px.outIdx];
  bool wrote = false;
  for (int k = 0; k < A.numSamples; ++k) {
    const float4 c = A.sampleBuf[(size_t)k * lanes + gid];
    if (c.w == kNoSample) continue;
    const float w = 1.f / (float)(A.accumID + k + 1);
    a.x = w * c.x + (1.f - w) * a.x;
    a.y = w * c.y + (1.f - w) * a.y;
    a.z = w * c.z + (1.f - w) * a.z;
    a.w = w * c.w + (1.f - w) * a.w;
    wrote = true;
  }
  if (!wrote) return;
  A.accum[px.outIdx] = a;
  A.fb[px.outIdx] = srgb_byte(s_th, a.x) + (srgb_byte(s_th, a.y) << 8) +
                    (srgb_byte(s_th, a.z) << 16) + (make_8bit(a.w) << 24);
}

// ------------------------------------------------------------------ debug: point location
// The default kernel's Tracer::locate (sampleVolume over the binned lists) on given points:
// the device locator pinned point by point (tests/test_gpu_parity.py), e.g. exactly on
// radial bin edges, which frames almost never hit.
__global__ void __launch_bounds__(256) k_debug_locate(RenderArgs A, const float *xyz, int n,
                                                      int *found, float *value) {
  __shared__ uint32_t s_sph[kSphBitWords];
  __shared__ uint32_t s_cnt[kCnt];
  for (int i = threadIdx.x; i < kSphBitWords; i += 256) s_sph[i] = A.numSph ? A.sphBits[i] : 0u;
  if (threadIdx.x < kCnt) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  Tracer<kDefaultVariant & ~4096> T{{}, A, nullptr, s_sph, s_cnt, {0, 0, 0, 0, 0, 0, 0}};
  const int j = (int)(blockIdx.x * 256 + threadIdx.x);
  if (j < n) {
    float v = 0.f;
    found[j] = T.locate(xyz[3 * j], xyz[3 * j + 1], xyz[3 * j + 2], v) ? 1 : 0;
    value[j] = v;
  }
}

// The same points through the cooperative kernel's wave-wide candidate scan
// (Tracer::locate_wave; every lane of a wave calls it, lanes past n with want = false):
// pins its dealt-out candidates and its second pass on radial bin edges to the serial path.
template <int O>
__global__ void __launch_bounds__(256) k_debug_locate_wave(RenderArgs A, const float *xyz, int n,
                                                           int *found, float *value) {
  __shared__ uint32_t s_sph[kSphBitWords];
  __shared__ uint32_t s_cnt[kCnt];
  __shared__ CoopWave s_coop[4];
  __shared__ ScanWave s_scan[4];
  for (int i = threadIdx.x; i < kSphBitWords; i += 256) s_sph[i] = A.numSph ? A.sphBits[i] : 0u;
  if (threadIdx.x < kCnt) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  Tracer<O> T{{}, A, nullptr, s_sph, s_cnt, {0, 0, 0, 0, 0, 0, 0}};
  static_assert(Tracer<O>::kWaveScan, "the default kernel scans wave-wide");
  const int j = (int)(blockIdx.x * 256 + threadIdx.x);
  const bool want = j < n;
  float x = 0.f, y = 0.f, z = 0.f;
  if (want) {
    x = xyz[3 * j];
    y = xyz[3 * j + 1];
    z = xyz[3 * j + 2];
  }
  float v = 0.f;
  const bool f = T.locate_wave(want, x, y, z, v, s_coop[threadIdx.x >> 6], s_scan[threadIdx.x >> 6]);
  if (want) {
    found[j] = f ? 1 : 0;
    value[j] = v;
  }
}

void launch_debug_locate(const RenderArgs &A, const float *xyz, int n, int *found, float *value,
                         hipStream_t s, bool wave) {
  if (n <= 0) return;
  constexpr int D = kDefaultVariant & ~4096;
  if (wave && A.slots)  // the scan from the slot table (OPT_SLOT), as the scene's launches run it
    hipLaunchKernelGGL(k_debug_locate_wave<D | OPT_SLOT>, dim3((n + 255) / 256), dim3(256), 0, s, A, xyz, n, found, value);
  else if (wave)
    hipLaunchKernelGGL(k_debug_locate_wave<D>, dim3((n + 255) / 256), dim3(256), 0, s, A, xyz, n, found, value);
  else
    hipLaunchKernelGGL(k_debug_locate, dim3((n + 255) / 256), dim3(256), 0, s, A, xyz, n, found, value);
}

// ------------------------------------------------------------------ variants / launcher
// Variant bits: irt_render.hip OPT_* (bits 8-11: minimum waves per SIMD asked of the
// register allocator).  OPT_MONO (4096) is kept in the numbering of round 1 (the one-kernel
// raygen; the setup -> march -> continuation pipeline it distinguished from was removed).
// 5376 (the default since r03u): 5 waves/SIMD, 96 VGPRs, the few spills in the prologue and
// epilogue only; 5120: the same kernel at 4 waves/SIMD (117 VGPRs), for A/B.  70656 = 5120 |
// OPT_SERIAL: the one-lane-per-ray Woodcock loop, for A/B against the cooperative loop.
// 1053696 = 5120 | OPT_HDRLDS: the cell headers staged through LDS (profiles/r03s_variants/).
// 2102272 = 5120 | OPT_LEAN (24 KB of LDS per workgroup), 2102528 the same at 5 waves/SIMD;
// 8393728 / 8393984 = 5120 / 5376 | OPT_DEALALL (profiles/r03t_regs/); 6296576 / 6296832 =
// 2102272 / 2102528 | OPT_WAVEWG (one-wave workgroups); 73405696 = 6296832 | OPT_DMATAB,
// 73405728 = 73405696 | OPT_DPPSCAN (the default since round 5), 73667872 its hole-free form (|
// OPT_NOMISS); 73405760 / 73405712 = 73405696 | OPT_XPAIR / OPT_ACCPF (profiles/r05p_ab/).  All
// variants give identical results.  73930016 / 74192160: the default / its hole-free form with
// OPT_TIMING (per-region shader clocks, profiles/probe.py; s_memtime slows them ~17x).
constexpr int OPT_MONO = 4096;
static_assert((kDefaultVariant & OPT_MONO) != 0, "variant numbering");

// The product build instantiates the default (one-wave workgroups), 5376 (four-wave
// workgroups, which also has the persistent-launch kernel) and the statistics variant
// (IRT_COUNTERS, profiles/wave_stats.py); the A/B variants are built only by `make VARIANTS=all`
// (libicon_rt_hip_all.so, loaded through IRT_LIB_PATH by the profiles/ tools and by
// tests/test_gpu_parity.py::test_all_render_variants_identical when present).
#ifdef IRT_ALL_VARIANTS
#define IRT_VARIANTS(X) X(4096) X(5120) X(5376) X(36864) X(70656) X(136192) X(529408) X(1053696) X(2102272) X(2102528) X(8393728) X(8393984) X(6296576) X(6296832) X(529664) X(2102784) X(33559808) X(134223104) X(268440832) X(39851264) X(538973440) X(6297088) X(6558976) X(73405696) X(73667840) X(73405728) X(73667872) X(73405760) X(73667904) X(73405712) X(73667856) X(73930016) X(74192160) X(73405732) X(73405730) X(73405729) X(73667873) X(73405744) X(73667888) X(1147147552) X(107222304) X(106960160) X(73438496) X(73700640)
#else
#define IRT_VARIANTS(X) X(73405728) X(73667872) X(1147147552) X(5376) X(36864)
#endif
static_assert(kDefaultVariant == 73405728 && (kDefaultVariant | kNoMissBit) == 73667872 && kNoMissBit == OPT_NOMISS &&
                  (kDefaultVariant | kVoidLocBit) == 1147147552 && kVoidLocBit == OPT_VOIDLOC,
              "the product build's variant list names the default and its scene forms (scene_variant)");

int render_variants(int *out, int cap) {
  int n = 0;
#define IRT_LIST(N) \
  if (n < cap && out) out[n] = N; \
  ++n;
  IRT_VARIANTS(IRT_LIST)
#undef IRT_LIST
  return n;
}

bool render_variant_available(int v) {
#define IRT_CASE(N) if (v == N) return true;
  IRT_VARIANTS(IRT_CASE)
#undef IRT_CASE
  return false;
}

// chained frames per wave of a launch: 2 for the OPT_FPAIR variants' own user-geometry kernels
// (kernel_for: the grid-accel and wedge kernels carry no variant bits), else 1
int render_frames_per_wave(const RenderArgs &A, int variant) {
  return (variant & OPT_FPAIR) != 0 && A.chain && render_variant_available(variant) &&
                 A.sampler == IRT_MODE_USER_GEOM && A.accelMode != IRT_ACCEL_GRID
             ? 2
             : 1;
}

int render_wg_per_block(const RenderArgs &A, int variant) {
  const int per = (variant & OPT_WAVEWG) ? 4 : ((variant & OPT_WAVEWG2) ? 2 : 1);
  return render_variant_available(variant) && A.sampler == IRT_MODE_USER_GEOM && A.accelMode != IRT_ACCEL_GRID ? per : 1;
}

// variant bits without a persistent form
constexpr int kNoQueue = OPT_WAVEWG | OPT_WAVEWG2 | OPT_SERIAL | OPT_STATS | OPT_TIMING | OPT_HDRLDS;
// Persistent launches (OPT_QUEUE, 3-4x slower: DESIGN.md section 5) are compiled into the A/B
// library only (make VARIANTS=all); the product library has no persistent kernel.
bool render_split_ok(const RenderArgs &A, int variant) {
  return (variant == kDefaultVariant || variant == (kDefaultVariant | kNoMissBit) || variant == (kDefaultVariant | OPT_VOIDLOC)) &&
         render_wg_per_block(A, variant) == 4;
}

bool render_queue_compiled() {
#ifdef IRT_ALL_VARIANTS
  return true;
#else
  return false;
#endif
}
bool render_queue_ok(const RenderArgs &A, int variant) {
  return render_queue_compiled() && render_variant_available(variant) && (variant & kNoQueue) == 0 &&
         A.sampler == IRT_MODE_USER_GEOM && A.accelMode != IRT_ACCEL_GRID;
}

typedef void (*RenderKernel)(RenderArgs);
// The kernel a launch of variant N runs for these arguments, and its workgroup size.  The
// grid accel or the unstructured samplers: their own instantiations of the raygen (kept out
// of the default kernel, whose registers they would cost); the wedge kernels hold a 6-vertex
// Newton state: no waves-per-SIMD floor.  Both run the cooperative Woodcock loop with its
// miss mode (C2: TRIANGLES 3.4x, CUBQL 2.5x faster than one lane per ray;
// profiles/r02b_investigation/).
template <int N>
RenderKernel kernel_for(const RenderArgs &A, int &threads) {
  constexpr int K = N & ~OPT_MONO;
  constexpr int D = kDefaultVariant & ~OPT_MONO;
  constexpr int DB = D & ~(0xF00 | OPT_WAVEWG | OPT_WAVEWG2 | OPT_LEAN);  // 256-thread workgroups, full LDS
  constexpr int DW = DB | OPT_WEDGE | (K & OPT_SERIAL);
  constexpr int DG = DB | 0x400;  // the grid-accel raygen: 4 waves/SIMD as measured in round 2
  const bool g = A.accelMode == IRT_ACCEL_GRID;
  threads = 256;
  if (A.sampler != IRT_MODE_USER_GEOM && g) return k_render<DW | OPT_GRID>;  // CUBQL / TRIANGLES
  if (A.sampler != IRT_MODE_USER_GEOM) return k_render<DW>;
  if (g) return k_render<DG | OPT_GRID | (K & OPT_SERIAL)>;
  if ((K & OPT_WAVEWG) != 0) threads = 64;  // four one-wave workgroups per 256-pixel block
  if ((K & OPT_WAVEWG2) != 0) threads = 128;  // two two-wave workgroups per block
#ifdef IRT_ALL_VARIANTS
  if constexpr ((K & kNoQueue) == 0)
    if (A.queue) return k_render<K | OPT_QUEUE>;
#endif
  // a single frame with measured-cost work items: the default kernels' split-capable form
  // and a scene with a slot table: their OPT_SLOT form
  if constexpr (K == (kDefaultVariant & ~OPT_MONO) || K == ((kDefaultVariant | kNoMissBit) & ~OPT_MONO) ||
                K == ((kDefaultVariant | OPT_VOIDLOC) & ~OPT_MONO)) {
    if (A.slots) return A.numSplit ? k_render<K | OPT_SPLIT | OPT_SLOT> : k_render<K | OPT_SLOT>;
    if (A.numSplit) return k_render<K | OPT_SPLIT>;
  }
  return k_render<K>;
}

template <int N>
void launch_variant(const RenderArgs &A, int numBlocks, hipStream_t s) {
  int threads = 256;
  const RenderKernel k = kernel_for<N>(A, threads);
  if (A.queue) {  // persistent: numBlocks workgroups (render_queue_wgs) pull the packets
    hipLaunchKernelGGL(k, dim3(numBlocks), dim3(256), 0, s, A);
    numBlocks = A.numTiles * 16;
  } else {
    const int split = A.numSplit ? (int)A.numSplit : 0;  // the listed work items first (kernel_for: OPT_SPLIT)
    const int fpw = render_frames_per_wave(A, N);  // chained frames per wave
    hipLaunchKernelGGL(k, dim3(numBlocks * (256 / threads) + split, (A.numSamples + fpw - 1) / fpw), dim3(threads), 0, s, A);
  }
  // progressive batch: the lerp chain over the frames' samples (chained frames lerp in k_render)
  if (A.numSamples > 1 && !A.chain) hipLaunchKernelGGL(k_accumulate, dim3(numBlocks), dim3(256), 0, s, A);
}

template <int N>
int queue_wgs_variant(const RenderArgs &A, int numCU, int numBlocks) {
  int threads = 256;
  const RenderKernel k = kernel_for<N>(A, threads);
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, threads, 0) != hipSuccess || occ < 1) {
    (void)hipGetLastError();
    occ = 1;
  }
  const long long n = (long long)occ * numCU;
  return (int)(n < numBlocks ? n : numBlocks);
}

int render_queue_wgs(const RenderArgs &A, int variant, int numCU, int numBlocks) {
  switch (variant) {
#define IRT_CASE(N) \
  case N:           \
    return queue_wgs_variant<N>(A, numCU, numBlocks);
    IRT_VARIANTS(IRT_CASE)
#undef IRT_CASE
    default:
      return queue_wgs_variant<kDefaultVariant>(A, numCU, numBlocks);
  }
}

// The first launch of a kernel pays the HIP runtime's lazy per-kernel setup on the host
// (~0.6 ms between the launch's start event and the dispatch, against a ~0.1 ms frame): a
// one-workgroup launch that returns at once (probeExit 1) at context creation takes it there.
template <int N>
void prewarm_variant(hipStream_t s) {
  RenderArgs A = {};
  A.probeExit = 1;
  A.numSamples = 1;
  int threads = 256;
  const RenderKernel k = kernel_for<N>(A, threads);  // sets threads (64 for one-wave workgroups)
  hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, s, A);
  A.numSplit = 8;  // the split-capable form of the default kernels (never read: it returns first)
  const RenderKernel ks = kernel_for<N>(A, threads);
  if (ks != k) hipLaunchKernelGGL(ks, dim3(1), dim3(threads), 0, s, A);
  A.slots = reinterpret_cast<const float4 *>(16);  // and the slot-table forms (never dereferenced)
  const RenderKernel kts = kernel_for<N>(A, threads);
  if (kts != ks) hipLaunchKernelGGL(kts, dim3(1), dim3(threads), 0, s, A);
  A.numSplit = 0;
  const RenderKernel kt = kernel_for<N>(A, threads);
  if (kt != k) hipLaunchKernelGGL(kt, dim3(1), dim3(threads), 0, s, A);
  A.slots = nullptr;
  A.queue = reinterpret_cast<uint32_t *>(16);  // never dereferenced: the kernel returns first
  const RenderKernel kq = kernel_for<N>(A, threads);
  if (kq != kernel_for<N>(RenderArgs{}, threads)) hipLaunchKernelGGL(kq, dim3(1), dim3(256), 0, s, A);
}

void prewarm_render(int variant, hipStream_t s) {
  switch (variant) {
#define IRT_CASE(N) \
  case N:           \
    prewarm_variant<N>(s); \
    return;
    IRT_VARIANTS(IRT_CASE)
#undef IRT_CASE
    default:
      prewarm_variant<kDefaultVariant>(s);
  }
}

void launch_render(const RenderArgs &A, int numBlocks, hipStream_t s, int variant) {
  switch (variant) {
#define IRT_CASE(N) \
  case N:           \
    launch_variant<N>(A, numBlocks, s); \
    return;
    IRT_VARIANTS(IRT_CASE)
#undef IRT_CASE
    default:
      launch_variant<kDefaultVariant>(A, numBlocks, s);
  }
}

}  // namespace irt
