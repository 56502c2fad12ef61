// irt_kernels.h -- kernel argument block and launchers (HIP translation units only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icon_rt_hip.h"

namespace irt {

// Everything k_render reads: the per-frame LaunchParams (Params.h:92-119) plus the
// context-owned HBM arrays.  Passed by value (kernarg segment).
struct RenderArgs {
  // camera / frame (Params.h:100-118)
  float3 org, dir00, du, dv;
  int accumID;
  float accumW;          // 1.f / (float)(accumID + 1), the single frame's lerp weight
  float3 amb;
  float ambRad;
  float unitDistance;
  int raygen;
  // volume (Params.h:62-74)
  float3 bmin, bmax;     // Volume::bounds
  int3 dims;             // ShellAccel::dims
  float3 sbLo, sbHi;     // ShellAccel::sphericalBounds
  const float *maxOp;    // ShellAccel::maxOpacities
  int accelMode;         // Volume::accelMode (Params.h:33-34): 0 sphere (sdda), 1 grid (dda3)
  const float *gridMaxOp;  // Grid::maxOpacities, kGridDim^3 over bmin..bmax (Params.h:44-49)
  const uint32_t *gridBits;  // per kGridBlock^3 block: any majorant not <= 0 (k_grid_bits)
  int sampler;           // Volume::mode (Params.h:60): 0 cell sample() scan, 2 CUBQL wedges
  int wG;                // CUBQL_MODE wedge locator (host/irt_scene.cpp build_wedges)
  const uint32_t *wOff, *wRec;
  const float4 *wBox;    // per record: {lo.xyz, numLayers bits}, {hi.xyz, 0}
  const float4 *wTrig;   // per record: 3 corners {cosf lat, sinf lat, cosf lon, sinf lon}
  // transfer function (Params.h:77-82)
  float tfLo, tfHi, opacityScale;
  // 1 / (double)(tfHi - tfLo) and 1 / (double)(sbHi - sbLo) per axis (the float differences):
  // quotients by these per-launch divisors as one double product (div_uniform, irt_device.h)
  double invTf;
  double invSb[3];
  const float4 *lut;
  int lutSize;
  // locator
  uint32_t numCells;
  int G;
  // sRGB byte thresholds (256 entries, host/irt_host.cpp)
  const float *srgbTh;
  // output
  int W, H;
  uint32_t *fb;
  float4 *accum;
  int packed;            // 0: linear x + W*y; 1: packed 64x64 tiles
  int tileBegin, tileStride, numTiles, tilesX;
  const int32_t *tileList;  // explicit tile ids (irt_render_tile_list); null: tileBegin + k*tileStride
  unsigned long long *counters;  // [0] launched [1] inBox [2] locate [3] found [4] candidates
  // the device-atomic fallback of the per-workgroup counts (a launch past wgCountsMax
  // workgroups): kCounterBuckets x 8 counters, workgroup w adding into bucket w % 64 (one line
  // would serialise every workgroup's adds), summed into counters[0..4] by k_stats_out
  unsigned long long *counterBuckets;
  // The binned locator (irt_common.h): per cube-map cell a 32-B header, fat entries,
  // per-record height/value blocks.
  const uint4 *binHdr;
  const float4 *fat;
  const float4 *blocks;
  // zero-thickness records (spheres, host/irt_scene.cpp): sorted distinct radii, CSR into
  // (record, numLayers) pairs, and the radius hash bitmap (kSphBitWords words)
  uint32_t numSph;
  const float *sphR;
  const uint32_t *sphOff;
  const uint2 *sphRec;
  const uint32_t *sphBits;
  // per-workgroup event counts (kCnt u32 per workgroup, in pinned host memory, summed by
  // the host); null: device-scope atomics into `counters`
  uint32_t *wgCounts;
  // progressive batch (irt_render_accumulate): frames accumID .. accumID+numSamples-1;
  // for numSamples > 1 each frame's colour goes to sampleBuf[frame][lane] first
  int numSamples;
  // measured-cost workgroup scheduling of the one-kernel raygen (irt_context.hip): the
  // block order to render (null: identity) and this launch's per-block durations
  const uint32_t *schedOrder;
  uint32_t *schedCost;
  float4 *sampleBuf;
  // cooperative Woodcock loop: at most 2^coopMaxLg lanes (samples) per ray in the first
  // round of a woodcock_wave call, coopRamp powers of two more per later round (any
  // setting gives the same frame)
  int coopMaxLg;
  int coopRamp;
  // measurement only (IRT_PROBE_EXIT, profiles/): 1 = every workgroup returns at once,
  // 2 = after the prologue, 3 = after ray generation and boxTest (no pixel written), 4 = at
  // the first woodcockFunc, 5 = after it
  int probeExit;
  // persistent launch (the thread pool's queue, common/thread_pool.h:146-161, per wave):
  // non-null: kQueueWords u32 of per-XCD packet counters and a done count -- every wave pulls
  // 8x8-pixel packets (packet p: block p >> 2 over the launch's frames, the block's wave p & 3)
  // until none is left; the launch's last wave resets the counters for the next launch
  uint32_t *queue;
  uint32_t numPackets;
  // chained progressive frames (numSamples > 1, irt_render_accumulate & co.): workgroup (b, f)
  // of the launch renders block b of frame accumID + f and lerps straight into accum/fb, after
  // waiting for (b, f - 1)'s wave to publish the same pixels -- chainFlag[4 b + wave] = chainEpoch
  // + f after its write-through (sc1) stores -- instead of the sample buffer + k_accumulate.
  // The hand-off is cdna_hip_programming.md Guideline 16's R1 form (sc1 payload stores drained
  // by the storing wave, an sc1 flag store; sc1 polls and sc1 loads of every handed-off byte),
  // so it holds whichever XCD the two workgroups run on.  A frame's workgroups wait on the
  // previous frame's, which the linear dispatch order starts earlier; a wait gives up after
  // chainSpins polls and sets *chainFail (pinned host memory, one word per launch slot): the
  // frames are then unordered and the host reports IRT_E_CHAIN.
  int chain;
  // a sequence of views (irt_render_sequence; null otherwise): frame f's camera and accumID
  // as 4 float4 {org, accumID bits} {dir_00} {dir_du} {dir_dv}, uploaded before the launch and
  // read by the scalar unit in place of org/dir00/du/dv and accumID + f
  const float4 *frameCams;
  uint32_t chainEpoch;
  uint32_t *chainFlag;
  uint32_t *chainFail;
  uint32_t chainSpins;   // polls before a wait gives up (kChainSpinsDefault; tests lower it)
  int chainWithhold;     // test hook (irt_debug_set_chain_fault): this frame's waves never publish

  // measurement only (irt_debug_set_wg_trace, profiles/wg_trace.py): non-null: workgroup b
  // writes {start, end} (s_memrealtime, 100 MHz, low 32 bits), HW_ID and XCC_ID to
  // wgTrace[4b..4b+3] -- when the machine is idle at a launch's ramp and tail
  uint32_t *wgTrace;
  // a single frame's costliest packets first (one-wave workgroups, measured-cost scheduling:
  // irt_context.hip sched_prepare): numSplit work items (a multiple of 8; 0: none), item i =
  // (packet << 8) | (part << 4) | lg -- part `part` of 2^lg of packet 4 block + wave, 64 >> lg rays
  // -- rendered by the launch's workgroup i (~0u: nothing); splitMask bit p marks the listed
  // packets (their regular workgroups render nothing)
  const uint32_t *splitList;
  const uint32_t *splitMask;
  uint32_t numSplit;
  // the slot table (irt_common.h kSlot4; null: none -- the cells' radial edges are more than
  // three values in all, the headers fit the last-level cache, or IRT_SLOTS=0): slotEdge = the
  // table's edges (+inf past slotBins - 1), slotBins = table bins per slot unit, slotSubs =
  // sub-cells per slot unit (1, 2 or 4).
  // Launches with a table run the default kernels' OPT_SLOT form (kernel_for).
  const float4 *slots;
  float slotEdge[3];
  int slotBins;
  int slotSubs;
};
// a persistent launch's queue words (irt_render.hip queue_take): 8 per-XCD counters and the
// done count, each on its own 128-B line
constexpr int kQueueLine = 32;
// polls of a chained wait (an L2 round trip + s_sleep 2 each: ~1 s in all) before it gives up
constexpr uint32_t kChainSpinsDefault = 1u << 20;
constexpr int kQueueWords = 9 * kQueueLine;

// Event counts kept per workgroup: [0] launched [1] inBox [2] locate [3] found [4] candidates
constexpr int kCnt = 8;

// Render-kernel variants: the bit set of irt_render.hip's OPT_* flags (bits 8-11: minimum
// waves per SIMD).  All give identical results.
// one kernel per frame, 5 waves/SIMD (96 VGPRs; spills only in the prologue/epilogue): against
// 4 waves C3 -1.8 %, C4 -4.9 %, comb TF -9 %, C5 +1.9 % (profiles/r03u_waves/)
// Round 4: one-wave workgroups with the leaner LDS (OPT_WAVEWG | OPT_LEAN, 5 waves/SIMD): a
// finished wave frees its slot at once instead of when its 256-pixel block's slowest wave does;
// against 5376 (four-wave workgroups) with chained frames C3 -1.7 %, C3s -5.8 %, C4 -1.1 %, C5
// -2.3 %, a single C3 frame -1.1 % (profiles/r04p_ab/)
// Round 5: + OPT_DMATAB (67108864: the prologue's LCG-jump and logf tables by LDS-DMA, with no
// wait before the ray generation): against 6296832 C3 -1.2 %, one frame per launch -1.7 %, C5
// -2.5 %, C3t -1.2 %, C3s -0.3 % (profiles/r05k_dmatab/); + OPT_DPPSCAN (32: the round's prefix
// by DPP steps across lanes): C3t -1.1 %, comb TF -1.3 %, C3 -0.3 % (profiles/r05p_ab/)
constexpr int kDefaultVariant = 73405728;
// Round 5: the raygen's miss mode (woodcock_wave) is on in the default variant; a scene
// without holes (every column starting at the same radius, no gaps inside columns) runs it
// without (bit 262144, OPT_NOMISS): C3 -2.3 %, while convert_icon terrain (voids under land)
// runs 2.25x faster with it (profiles/r05d/)
constexpr int kNoMissBit = 262144;
// measured-cost scheduling (irt_context.hip sched_prepare): at most this many work items run first
// in a single frame (RenderArgs::splitList), a multiple of 8
constexpr uint32_t kMaxSplit = 4096;
// Round 6: a scene with holes also walks a certain miss in located mode (bit 1073741824,
// OPT_VOIDLOC: a solo lane whose sample is outside its quad's records switches its ray to the miss
// mode in the same round and walks on): C3t 8 chained frames -1.7 %, one per launch even
// (profiles/r06zg/)
constexpr int kVoidLocBit = 1073741824;
inline int scene_variant(bool holes) { return holes ? kDefaultVariant | kVoidLocBit : kDefaultVariant | kNoMissBit; }
bool render_variant_available(int variant);
int render_variants(int *out, int cap);  // the compiled variants (count; the first cap into out)
// workgroups per 256-pixel block the launch of `variant` uses for these arguments (4 only for
// the one-wave-workgroup A/B variants on the user-geometry sphere path)
int render_wg_per_block(const RenderArgs &A, int variant);
// chained frames per wave (2: the OPT_FPAIR variants, irt_render.hip)
int render_frames_per_wave(const RenderArgs &A, int variant);
// whether `variant` can run as a persistent launch (RenderArgs::queue) with these arguments:
// the cooperative user-geometry sphere-accel kernels with 256-thread workgroups
bool render_queue_ok(const RenderArgs &A, int variant);
bool render_queue_compiled();  // the A/B library (make VARIANTS=all) only
// whether a single frame of `variant` can run measured-cost work items (RenderArgs::splitList):
// the default kernels with one-wave workgroups
bool render_split_ok(const RenderArgs &A, int variant);
// workgroups a persistent launch of `variant` runs on a device with numCU compute units:
// every slot the kernel's occupancy allows (resident at once), at most `numBlocks`
int render_queue_wgs(const RenderArgs &A, int variant, int numCU, int numBlocks);
// numBlocks: the frame's 256-pixel blocks (grid launch), or the workgroups of a persistent
// launch (A.queue, render_queue_wgs)
void launch_render(const RenderArgs &A, int numBlocks, hipStream_t s, int variant);
// one empty launch of the variant's raygen kernels (grid and persistent): the runtime's
// first-launch setup happens at context creation, not in the first frame
void prewarm_render(int variant, hipStream_t s);
void launch_debug_locate(const RenderArgs &A, const float *xyz, int n, int *found, float *value,
                         hipStream_t s, bool wave);
void launch_shell_init(float *valueRanges, size_t numMCs, hipStream_t s);
void launch_shell_build(const irt_icon_cell *cells, size_t n, int3 dims, float3 lo, float3 hi,
                        float *valueRanges, hipStream_t s);
void launch_grid_build(const float4 *blocks, const uint32_t *meta, const float4 *trig, size_t n,
                       float3 lo, float3 hi, float *valueRanges, hipStream_t s);
void launch_grid_bits(const float *maxOp, uint32_t *bits, hipStream_t s);
// the TF's mean Woodcock samples per acceptance over the macrocells: out[0] += sum, out[1] += count
// (k_accept_stat, irt_kernels.hip)
void launch_accept_stat(const float *valueRanges, const float *maxOp, size_t numMCs, const float4 *lut, int size,
                        float lo, float hi, double *out, hipStream_t s);
void launch_max_opacities(const float *valueRanges, size_t numMCs, const float4 *lut, int size,
                          float lo, float hi, float *maxOp, hipStream_t s);
void launch_clear(uint32_t *fb, float4 *accum, size_t n, hipStream_t s);
constexpr int kCounterBuckets = 64;
// copies a launch's 16 counters to the host (plus, with `buckets`, the bucketed fallback
// counts, whose buckets it zeroes again) and zeroes the next launch's block
void launch_stats_out(const unsigned long long *cur, unsigned long long *host,
                      unsigned long long *next, unsigned long long *buckets, hipStream_t s);
void launch_copy_u32(const uint32_t *src, uint32_t *dst, size_t n, hipStream_t s);
// The scene build on the device (irt_build.hip): per-record blocks and the binned cube-map
// locator (irt_build.h) from the cells and their glibc corner trig in HBM.  On success the
// caller owns blocks / binHdr / fat; on failure it frees whatever is non-null.
struct DeviceScene {
  float4 *blocks = nullptr;
  uint32_t *meta = nullptr;  // per record (irt_build.h record_meta), kept for the lazy grid build
  uint4 *binHdr = nullptr;
  float4 *fat = nullptr;
  size_t entries = 0, binEntries = 0, bigCells = 0, bytes = 0;
};
int build_scene_device(const irt_icon_cell *d_cells, const float4 *d_trig, size_t n, size_t numRuns,
                       int G, hipStream_t s, DeviceScene &out);
// The slot table (irt_common.h kSlot4) of a built scene whose cells' radial edges are at most
// three values in all, if it fits in maxBytes (and the device's free memory); otherwise slots
// stays null.
struct SlotTable {
  float4 *slots = nullptr;
  int bins = 0;
  int subs = 0;  // sub-cells per slot unit (irt_common.h slot_unit; IRT_SLOT_SUBS=1|2|4)
  float edges[3] = {0.f, 0.f, 0.f};
  size_t bytes = 0;
  const char *skipped = nullptr;  // why no table was built (nullptr: built, or not asked for)
};
// Round 5: with the table C5 -9 %, C3s -3 %, but C3 +4 %, C4 +3 % (profiles/r05aa/): on by
// default only when the headers exceed the 256-MB last-level cache (C5: 2.7 GB; C3: 167 MB).
// Round 6: slot units of 2 or 4 sub-cells (a half or a quarter of the table): C5 -7.6 % / -6.0 %
// against no table, one sub-cell -7.5 to -9 % (profiles/r06x/); the default unit keeps the
// table within the scene's own bytes (C5: quads, 32 GB)
constexpr size_t kSlotAutoHdrBytes = (size_t)256 << 20;
// subs: sub-cells per slot unit (irt_common.h slot_unit), 1, 2 or 4; any other value: the finest
// unit whose table is at most autoBytes (and maxBytes), else 4
int build_slots_device(const uint32_t *hdr, const float4 *fat, uint32_t numCells, size_t maxBytes, int subs,
                       size_t autoBytes, hipStream_t s, SlotTable &out);
void launch_unpack(const uint32_t *gathered, int numRanks, int maxTiles, int W, int H,
                   uint32_t *fb, hipStream_t s, const int32_t *table = nullptr);

}  // namespace irt
