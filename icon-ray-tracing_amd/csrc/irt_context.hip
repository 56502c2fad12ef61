// irt_context.hip -- the C ABI of include/icon_rt_hip.h on the HIP runtime: context
// lifetime, HBM layout, accelerator builds, and frame launches.  Host-side preparation
// (planes, locator, tables) lives in host/*.cpp (compiled by g++).

#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#include "irt_build.h"
#include "irt_internal.h"
#include "icon_rt_hip_debug.h"
#include "irt_device.h"
#include "irt_kernels.h"

using namespace irt;

#define IRT_HIP(call)                                                             \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess) {                                                       \
      set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__,  \
                __LINE__);                                                        \
      return IRT_E_HIP;                                                           \
    }                                                                             \
  } while (0)

// the split threshold of single frames of scenes with holes (irt_context::splitFactor)
constexpr float kSplitFactorHoles = 0.35f;
// A transfer function whose mean Woodcock samples per acceptance over the shell's macrocells
// (k_accept_stat) is at least this is sparse: launches on a scene whose headers fit the
// last-level cache then start their candidate scan from the slot table (built on the first such
// TF), which the dense default TF does not pay for.  Quads on the C3 grid (2.0 GB): the comb TF
// (32 samples per acceptance) -3.8 %, the default TF (1.3) +3.0 % (profiles/r06zl/).
constexpr double kSparseTfSamples = 8.0;

struct irt_context {
  int device = 0;
  hipStream_t stream = nullptr;
  irt_volume_info info{};
  uint32_t n = 0;
  int G = 0;
  // HBM
  uint4 *d_binHdr = nullptr;   // binned locator (irt_common.h)
  float4 *d_fat = nullptr;
  float4 *d_blocks = nullptr;
  SlotTable slot;              // the slot table (irt_common.h kSlot4; IRT_SLOTS=0: none)
  bool slotAlways = false;     // every launch starts its scan from it (large scenes, IRT_SLOTS=1)
  bool slotLazy = false;       // a smaller scene builds it for a sparse transfer function
  bool slotTried = false;      // a build was attempted (never again)
  bool slotSparse = false;     // the current transfer function is sparse (kSparseTfSamples)
  double tfSamples = 0.0;      // its mean Woodcock samples per acceptance (k_accept_stat)
  double *d_tfStat = nullptr;  // k_accept_stat's sum and count
  size_t binEntries = 0;       // fat entries
  uint32_t numSph = 0;         // zero-thickness records (spheres): distinct radii
  uint32_t numSphRec = 0;      // ... and records
  float *d_sphR = nullptr;
  uint32_t *d_sphOff = nullptr;
  uint2 *d_sphRec = nullptr;
  uint32_t *d_sphBits = nullptr;
  // per-workgroup event counts of the launches in flight, written by the render kernel
  // straight into pinned host memory (kSlots x wgCap x kCnt u32) and summed on the host
  // when a launch's statistics are asked for (finish_slot): no statistics kernel, no
  // same-line atomics per frame.  A slot is rewritten only once its launch is retired.
  uint32_t *h_wgCounts = nullptr, *dh_wgCounts = nullptr;
  size_t wgCap = 0;             // workgroups per slot
  size_t slotWG[32] = {};       // workgroups of the launch in each slot
  bool slotBlock[32] = {};      // whether k_stats_out copied the slot's 16-counter block
  bool lastBlock = false;       // ... for the previous launch (which zeroed this slot's)
  bool wgCountsOn = true;       // IRT_COUNTERS=atomic: device-scope atomics instead
  bool statsOff = false;        // irt_set_statistics(ctx, 0): no counts at all
  int countersProbe = 0;        // measurement only: IRT_COUNTERS=off (no counts), =device
                                // (per-workgroup stores into device memory, never read)
  uint32_t *d_probeCounts = nullptr;
  size_t probeCap = 0;          // workgroups d_probeCounts holds
  float4 *d_samples = nullptr;   // per-frame colours of a progressive batch
  size_t sampleCap = 0;
  float *d_srgb = nullptr;
  float *d_valueRanges = nullptr;
  float *d_maxOp = nullptr;
  // GRID_ACCEL_MODE's 256^3 grid, built on first use (ensure_grid): 201 MB and ~0.16 s at C5
  // that a sphere-mode run never needs
  bool gridBuilt = false;
  uint32_t *d_meta = nullptr;    // per record numLayers (+ quantised keys), for the grid build
  float *d_gridVR = nullptr;     // GRID_ACCEL_MODE: Grid::valueRanges, kGridDim^3 box1f
  float *d_gridMaxOp = nullptr;  // Grid::maxOpacities
  uint32_t *d_gridBits = nullptr;  // its empty-space bitmap (k_grid_bits)
  // CUBQL_MODE wedge locator (irt_build_wedge_accel; irt_internal.h WedgeScene)
  int wG = 0;
  uint32_t *d_wOff = nullptr, *d_wRec = nullptr;
  float4 *d_wBox = nullptr, *d_wTrig = nullptr;
  size_t numMCs = 0;
  float4 *d_lut = nullptr;
  int lutCap = 0;
  int lutSize = 0;
  float tfLo = 0.f, tfHi = 1.f, opScale = 1.f;
  bool tfSet = false;
  // Per-launch statistics, read back without stalling the host: a ring of kSlots
  // counter blocks and event pairs; a slot is finished (synchronised) only when it is
  // reused or its statistics are asked for.  The last finished launch is `stats`; every
  // finished launch also adds into `total`.
  static constexpr int kSlots = 32;
  // launches with more workgroups (x frames) than this count through the device-atomic block
  // (the per-workgroup ring would need 1 KiB of pinned memory per workgroup: 256 MiB here)
  static constexpr size_t kWgCountsMax = size_t(1) << 18;
  size_t wgCountsMax = kWgCountsMax;  // IRT_WG_COUNTS_MAX overrides (tests)
  unsigned long long *d_counters = nullptr;  // kSlots x 16
  unsigned long long *d_counterBuckets = nullptr;  // kSlots x kCounterBuckets x 8 (zeroed)
  unsigned long long *h_counters = nullptr;  // pinned, kSlots x 16
  unsigned long long *dh_counters = nullptr; // h_counters as the device sees it
  hipStream_t lastStream = nullptr;  // stream of the previous launch
  // kernel-timing events on every n-th launch only (irt_set_timing_interval): an event
  // pair around every frame costs ~10 us of stream gaps against a 0.17 ms kernel
  int timingEvery = 8;
  bool timed[kSlots] = {};
  float lastMs = 0.f;          // most recent timed launch
  double timedMs = 0.0;        // sum over the timed launches since the last reset
  long long timedLaunches = 0;
  hipEvent_t ev0[kSlots] = {}, ev1[kSlots] = {};  // kernel timing
  hipEvent_t evDone[kSlots] = {};                  // counters landed in h_counters
  bool pending[kSlots] = {};
  // evDone[i] is recorded after launch i only every kDoneEvery-th launch, at a stream switch,
  // or when asked for (done_event): each marker on the queue costs its launch ~1-2 us, and a
  // later marker on the same stream completes after launch i as well
  static constexpr int kDoneEvery = 8;
  bool evRec[kSlots] = {};
  hipStream_t slotStream[kSlots] = {};
  long long slotLaunch[kSlots] = {};
  long long launches = 0;     // slot of launch i: i % kSlots
  irt_render_stats stats{};
  unsigned long long h_last[16] = {};
  irt_render_stats total{};
  long long totalLaunches = 0;
  size_t bytes = 0;
  int variant = kDefaultVariant;  // render-kernel variant (irt_render.hip OPT_* bits)
  // Measured-cost workgroup scheduling of the one-kernel raygen: every launch records its
  // workgroups' durations (d_schedCost); now and then a launch copies them back
  // (h_schedCost, pinned, in the stats ring), and once that copy has landed the host
  // orders the frame tiles by descending cost (longest-processing-time first) and uploads
  // the order (d_schedOrder) for later launches with the same grid.
  // Per order buffer (2, ping-pong; sched_stride words each): the block order (cap words), the
  // split packets (kMaxSplit words) and their bitmap (4 cap / 32 words); costs per packet
  // (4 cap words per launch slot)
  uint32_t *d_schedOrder = nullptr, *d_schedCost = nullptr;  // 2 x stride, 4 cap
  uint32_t *h_schedCost = nullptr, *h_schedOrder = nullptr;  // pinned: kSlots x 4 cap, 2 x stride
  uint32_t schedSplit[2] = {0, 0};  // split packets in each order buffer
  uint32_t lastNumSplit = 0;        // the last launch's split work items (parts x packets, padded to 8)
  int splitLg = 2;                  // parts per split packet: 2^splitLg (IRT_SPLIT_LG; 0: no splits)
  float splitFactor = 1.f;          // a packet splits when its cost exceeds this x the frame's ideal span
                                    // (IRT_SPLIT_FACTOR; scenes with holes: kSplitFactorHoles)
  bool splitFixed = false;          // IRT_SPLIT_FACTOR given
  int schedBuf = 0;             // the order buffer launches read now
  long long schedSwitch = 0;    // first launch reading it
  size_t schedCap = 0;
  bool schedOn = false;        // IRT_SCHED=1|2|3 enables (neutral on flat grids since the ramped loop;
                               // on by default, policy 1, for scenes with holes: irt_create_end)
  bool schedFixed = false;     // IRT_SCHED given: scenes keep it
  // cooperative Woodcock loop: a ray's lanes per round <= 2^(coopMaxLg + round) with the
  // ramp, 2^coopMaxLg without (IRT_COOP_MAXLG, IRT_COOP_RAMP; profiles/r02e_dist/)
  int coopMaxLg = 0;
  int coopRamp = 1;
  int probeExit = 0;           // IRT_PROBE_EXIT (measurement only, RenderArgs::probeExit)
  uint32_t *wgTrace = nullptr; // irt_debug_set_wg_trace (measurement only, RenderArgs::wgTrace)
  // chained progressive frames (RenderArgs::chain; IRT_CHAIN=0 / irt_debug_set_chain: the
  // sample buffer + k_accumulate instead): per (block, wave) publish words, the next epoch, and
  // the timeout word
  bool chainOn = true;
  uint32_t *d_chainFlag = nullptr;
  size_t chainCap = 0;           // words in d_chainFlag
  uint32_t chainEpoch = 1;
  // per launch slot, in pinned host memory: set by a chained wait of that launch that gave up
  // (RenderArgs::chainFail); finish_slot reports it (IRT_E_CHAIN) and turns chaining off
  uint32_t *h_chainFail = nullptr, *dh_chainFail = nullptr;
  long long chainFailLaunches = 0;  // launches reported so (irt_debug_chain_errors)
  uint32_t chainSpins = 0;          // irt_debug_set_chain_fault: poll cap (0: the kernel's default)
  int chainWithhold = -1;           // ... and the frame whose waves do not publish (-1: none)
  // irt_render_sequence: the frames' camera words on the device, and per launch slot their
  // pinned staging (a slot is reused only after its launch is retired)
  float4 *d_frameCams = nullptr;
  float4 *h_frameCams = nullptr;
  size_t frameCamCap = 0;        // frames per slot
  // persistent launches (RenderArgs::queue, IRT_QUEUE=0|1): every resident wave pulls 8x8
  // packets from per-slot queue counters (kSlots x kQueueWords u32, zero between launches)
  bool queueOn = false;
  uint32_t *d_queue = nullptr;
  int numCU = 0;
  int queuePerCU = 0;   // IRT_QUEUE_WGS: workgroups per CU of a persistent launch (0: occupancy)
  int lastQueueWG = 0;  // workgroups of the last persistent launch (irt_debug_get_queue)
  int schedPolicy = 2;         // IRT_SCHED: 1 tiles, 2 bands of tiles (a tile row; default), 3 reversed
  bool schedOrderValid = false;
  bool schedLastApplied = false;   // the last launch ran in a measured-cost order
  long long schedApplied = 0;      // launches that did
  long long schedKey[8] = {};
  long long schedSrc = -1;      // launch whose costs the current order came from
  long long schedCopied[kSlots] = {};  // launch index whose costs slot i holds (-1: none)
  long long schedLastCopy = -1000;
  // streaming creation (irt_create_begin / _append / _end): the cells and their glibc
  // corner trig go to HBM chunk by chunk; the volume facts, column count and sphere
  // records are folded on the host in record order
  bool building = false;
  size_t expected = 0, received = 0;
  // Holes in the volume, folded in record order (append_chunk): columns that start at
  // different radii (convert_icon's first record of a land column starts at R + HSURF, so
  // nothing covers [R, R + HSURF)), or records that leave a gap in their column.  Samples
  // there are outside every cell and come in runs; the raygen's miss mode takes such a run
  // in one cooperative round (irt_render.hip Tracer::kMiss).  A scene without holes runs
  // the variant without it (OPT_NOMISS: 2-3 % faster where nearly every sample is located).
  float bottomMin = INFINITY, bottomMax = -INFINITY;
  bool voids = false;
  bool variantFixed = false;  // IRT_RENDER_VARIANT chose the variant
  irt_icon_cell *d_cells = nullptr;  // freed once the scene is built
  float4 *d_trig = nullptr;          // corner trig: kept for the lazy grid build
  VolumeAcc vacc{};
  size_t numRuns = 0;
  irt_icon_cell last{};
  struct Sphere {
    float r;
    uint32_t rec;
    int32_t nl;
  };
  std::vector<Sphere> sph;  // zero-thickness records
  // device copies of the explicit tile lists / tables of irt_render_tile_list and
  // irt_unpack_tile_table, keyed by content (a multi-GPU deal is fixed for a run: uploaded
  // once, never rewritten while a launch may read it)
  struct TileTable {
    std::vector<int32_t> ids;
    int32_t *dev;
  };
  std::vector<TileTable> tileTables;
};

namespace {

template <typename T>
int dalloc(irt_context *c, T **p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  IRT_HIP(hipMalloc((void **)p, count * sizeof(T)));
  c->bytes += count * sizeof(T);
  return IRT_OK;
}

template <typename T>
int upload(irt_context *c, T **p, const T *src, size_t count) {
  int rc = dalloc(c, p, count);
  if (rc) return rc;
  if (count) IRT_HIP(hipMemcpyAsync(*p, src, count * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return IRT_OK;
}

void free_all(irt_context *c) {
  if (c->device >= 0) (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void *ptrs[] = {c->d_binHdr, c->d_fat, c->slot.slots, c->d_blocks, c->d_sphR, c->d_sphOff, c->d_sphRec,
                  c->d_sphBits, c->d_samples, c->d_maxOp, c->d_gridVR, c->d_gridMaxOp, c->d_gridBits, c->d_wOff, c->d_wRec, c->d_wBox, c->d_wTrig, c->d_schedOrder, c->d_schedCost, c->d_srgb, c->d_valueRanges,
                  c->d_lut, c->d_counters, c->d_counterBuckets, c->d_meta, c->d_queue, c->d_chainFlag,
                  c->d_frameCams, c->d_tfStat};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  if (c->d_cells) (void)hipFree(c->d_cells);
  if (c->d_trig) (void)hipFree(c->d_trig);
  if (c->h_counters) (void)hipHostFree(c->h_counters);
  if (c->h_wgCounts) (void)hipHostFree(c->h_wgCounts);
  if (c->h_schedCost) (void)hipHostFree(c->h_schedCost);
  if (c->h_schedOrder) (void)hipHostFree(c->h_schedOrder);
  if (c->h_frameCams) (void)hipHostFree(c->h_frameCams);
  if (c->h_chainFail) (void)hipHostFree(c->h_chainFail);
  for (int i = 0; i < irt_context::kSlots; ++i) {
    if (c->ev0[i]) (void)hipEventDestroy(c->ev0[i]);
    if (c->ev1[i]) (void)hipEventDestroy(c->ev1[i]);
    if (c->evDone[i]) (void)hipEventDestroy(c->evDone[i]);
  }
  for (auto &t : c->tileTables) (void)hipFree(t.dev);
  c->tileTables.clear();
  if (c->stream) (void)hipStreamDestroy(c->stream);
}

// The device copy of a tile list / table (see irt_context::tileTables): found by content, or
// uploaded (synchronously: a new allocation no launch in flight can be reading).  Entries
// must be in [lo, total).
int tile_table(irt_context *c, const int32_t *ids, size_t n, int lo, int total, const int32_t **out) {
  for (size_t k = 0; k < n; ++k)
    if (ids[k] < lo || ids[k] >= total) {
      set_error("tile id %d at %zu outside [%d, %d)", ids[k], k, lo, total);
      return IRT_E_INVALID;
    }
  for (auto &t : c->tileTables)
    if (t.ids.size() == n && std::equal(t.ids.begin(), t.ids.end(), ids)) {
      *out = t.dev;
      return IRT_OK;
    }
  if (c->tileTables.size() >= 64) {  // a camera per step would re-deal every frame: bounded
    IRT_HIP(hipDeviceSynchronize());
    for (auto &t : c->tileTables) (void)hipFree(t.dev);
    c->tileTables.clear();
  }
  int32_t *d = nullptr;
  IRT_HIP(hipMalloc((void **)&d, std::max<size_t>(n, 1) * sizeof(int32_t)));
  if (hipMemcpy(d, ids, n * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    set_error("tile table upload failed");
    return IRT_E_HIP;
  }
  c->tileTables.push_back({std::vector<int32_t>(ids, ids + n), d});
  *out = d;
  return IRT_OK;
}

// An event that completes after the launch in slot i (pending): its own marker if recorded,
// else the first later marker of the same stream, else a marker recorded now on that stream.
hipEvent_t done_event(irt_context *c, int i) {
  const long long L = c->slotLaunch[i];
  for (int k = 0; k < irt_context::kSlots; ++k) {
    const int j = (i + k) % irt_context::kSlots;
    if (!c->pending[j] || c->slotLaunch[j] != L + k || c->slotStream[j] != c->slotStream[i]) break;
    if (c->evRec[j]) return c->evDone[j];
  }
  // the newest launch on that stream: mark it now
  int last = i;
  for (int k = 1; k < irt_context::kSlots; ++k) {
    const int j = (i + k) % irt_context::kSlots;
    if (!c->pending[j] || c->slotLaunch[j] != L + k || c->slotStream[j] != c->slotStream[i]) break;
    last = j;
  }
  if (hipEventRecord(c->evDone[last], c->slotStream[last]) == hipSuccess) {
    c->evRec[last] = true;
    return c->evDone[last];
  }
  // that stream is gone (destroyed by the caller after its last launch): wait for the device
  (void)hipGetLastError();
  (void)hipDeviceSynchronize();
  return nullptr;
}
// waits for the launch in slot i (pending)
hipError_t wait_slot(irt_context *c, int i) {
  const hipEvent_t e = done_event(c, i);
  return e ? hipEventSynchronize(e) : hipSuccess;
}

int finish_slot(irt_context *c, int i) {
  if (!c->pending[i]) return IRT_OK;
  IRT_HIP(wait_slot(c, i));
  float ms = 0.f;
  if (c->timed[i]) {
    IRT_HIP(hipEventElapsedTime(&ms, c->ev0[i], c->ev1[i]));
    c->lastMs = ms;
    c->timedMs += ms;
    ++c->timedLaunches;
  }
  unsigned long long h[16] = {};
  if (c->slotBlock[i]) memcpy(h, c->h_counters + 16 * i, sizeof(h));
  if (c->slotWG[i]) {  // the workgroups' counts, from pinned host memory
    const uint32_t *w = c->h_wgCounts + (size_t)i * c->wgCap * kCnt;
    for (size_t b = 0; b < c->slotWG[i]; ++b)
      for (int k = 0; k < 5; ++k) h[k] += w[b * kCnt + k];
  }
  irt_render_stats st;
  st.raysLaunched = h[0];
  st.raysInBox = h[1];
  st.locateCalls = h[2];
  st.samplesFound = h[3];
  st.candidatesTested = h[4];
  st.kernelMs = c->lastMs;
  c->stats = st;
  memcpy(c->h_last, h, sizeof(c->h_last));
  c->total.raysLaunched += st.raysLaunched;
  c->total.raysInBox += st.raysInBox;
  c->total.locateCalls += st.locateCalls;
  c->total.samplesFound += st.samplesFound;
  c->total.candidatesTested += st.candidatesTested;
  ++c->totalLaunches;
  c->pending[i] = false;
  if (c->h_chainFail[i]) {
    // a chained wait of this launch gave up: its frames were lerped out of order.  Report it
    // (once), and render later multi-frame launches unchained (sample buffer + k_accumulate)
    c->h_chainFail[i] = 0;
    ++c->chainFailLaunches;
    c->chainOn = false;
    set_error("chained-frame hand-off timed out in launch %lld: its frames are not the sequential "
              "frames (chaining is now off for this context)", c->slotLaunch[i]);
    return IRT_E_CHAIN;
  }
  return IRT_OK;
}

// finish every pending launch, oldest first (the last one ends up in c->stats)
int finish_stats(irt_context *c) {
  for (long long j = c->launches - irt_context::kSlots; j < c->launches; ++j) {
    if (j < 0) continue;
    int rc = finish_slot(c, (int)(j % irt_context::kSlots));
    if (rc) return rc;
  }
  return IRT_OK;
}

// Measured-cost scheduling, host side (see irt_context::d_schedOrder): (re)allocate for
// the grid, drop the order when the grid changes, and rebuild it from the newest landed
// cost copy of a launch with the same grid.
// words of one order buffer: the block order, the split list, the split bitmap
size_t sched_stride(size_t cap) { return cap + kMaxSplit + (4 * cap + 31) / 32; }

int sched_prepare(irt_context *c, int numBlocks, int W, int H, int packed, int tileBegin,
                  int tileStride, int numTiles, const irt_launch_params *lp, bool wavewg, hipStream_t s) {
  if ((size_t)numBlocks > c->schedCap) {
    IRT_HIP(hipStreamSynchronize(s));
    if (c->d_schedOrder) IRT_HIP(hipFree(c->d_schedOrder));
    if (c->d_schedCost) IRT_HIP(hipFree(c->d_schedCost));
    if (c->h_schedCost) IRT_HIP(hipHostFree(c->h_schedCost));
    if (c->h_schedOrder) IRT_HIP(hipHostFree(c->h_schedOrder));
    c->d_schedOrder = c->d_schedCost = c->h_schedCost = c->h_schedOrder = nullptr;
    c->bytes -= (2 * sched_stride(c->schedCap) + 4 * c->schedCap) * sizeof(uint32_t);
    c->schedCap = 0;
    int rc;
    if ((rc = dalloc(c, &c->d_schedOrder, 2 * sched_stride((size_t)numBlocks))) ||
        (rc = dalloc(c, &c->d_schedCost, 4 * (size_t)numBlocks)))
      return rc;
    IRT_HIP(hipMemsetAsync(c->d_schedCost, 0, 4 * (size_t)numBlocks * sizeof(uint32_t), s));
    IRT_HIP(hipHostMalloc((void **)&c->h_schedCost, (size_t)irt_context::kSlots * 4 * numBlocks * sizeof(uint32_t)));
    memset(c->h_schedCost, 0, (size_t)irt_context::kSlots * 4 * numBlocks * sizeof(uint32_t));
    IRT_HIP(hipHostMalloc((void **)&c->h_schedOrder, 2 * sched_stride((size_t)numBlocks) * sizeof(uint32_t)));
    c->schedCap = numBlocks;
    c->schedSplit[0] = c->schedSplit[1] = 0;
    c->schedOrderValid = false;
    for (auto &v : c->schedCopied) v = -1;
    c->info.deviceBytes = c->bytes;
  }
  const long long key[8] = {numBlocks, W, H, packed, tileBegin, tileStride, numTiles,
                            lp->accelMode * 4 + lp->mode};
  if (memcmp(key, c->schedKey, sizeof(key)) != 0) {
    memcpy(c->schedKey, key, sizeof(key));
    c->schedOrderValid = false;
    c->schedSrc = c->launches;  // costs of launches before this one belong to another grid
    for (auto &v : c->schedCopied) v = -1;
  }
  // the newest cost copy that has landed -- from a launch no older than the first reader
  // of the current order buffer, so every launch reading the other buffer has finished and
  // it (and its pinned staging copy) may be rewritten without a stall
  long long best = -1;
  int bestSlot = -1;
  for (int i = 0; i < irt_context::kSlots; ++i)
    if (c->schedCopied[i] > c->schedSrc && c->schedCopied[i] >= c->schedSwitch &&
        c->schedCopied[i] > best && (!c->pending[i] || (c->evRec[i] && hipEventQuery(c->evDone[i]) == hipSuccess))) {
      best = c->schedCopied[i];
      bestSlot = i;
    }
  if (bestSlot < 0) return IRT_OK;
  // longest-processing-time first over whole 64x64 tiles (16 consecutive workgroups, kept
  // together for the locator's cache locality)
  const uint32_t *cost = c->h_schedCost + (size_t)bestSlot * 4 * c->schedCap;  // per packet
  const int nt = numBlocks / 16;
  // group size in tiles: 1, or a band of consecutive launch tiles (one image row of tiles)
  const int tilesX = (W + 63) / 64;
  const int band = c->schedPolicy == 2 ? std::max(1, tilesX / std::max(1, tileStride)) : 1;
  const int ng = (nt + band - 1) / band;
  std::vector<std::pair<uint64_t, int>> groups(ng);
  for (int g = 0; g < ng; ++g) {
    uint64_t sum = 0;
    for (int t = g * band; t < std::min(nt, (g + 1) * band); ++t)
      for (int j = 0; j < 64; ++j) sum += cost[64 * t + j];
    groups[g] = {c->schedPolicy == 3 ? (uint64_t)g : sum, g};
  }
  std::stable_sort(groups.begin(), groups.end(),
                   [](const std::pair<uint64_t, int> &a, const std::pair<uint64_t, int> &b) {
                     return a.first > b.first;
                   });
  const int nb = c->schedOrderValid ? 1 - c->schedBuf : c->schedBuf;
  const size_t stride = sched_stride(c->schedCap);
  uint32_t *h = c->h_schedOrder + (size_t)nb * stride;
  int p = 0;
  for (const auto &g : groups)
    for (int t = g.second * band; t < std::min(nt, (g.second + 1) * band); ++t, ++p)
      for (int j = 0; j < 16; ++j) h[16 * p + j] = (uint32_t)(16 * t + j);
  // Work items ahead of the regular order (one-wave workgroups only), costliest first: every
  // packet whose measured duration exceeds splitFactor x the frame's ideal span (all packets'
  // durations over the resident slots), in 2^splitLg parts of 64 >> splitLg rays -- such a packet
  // would end the frame after the rest, and it is lane-bound: its parts take about 1/2^splitLg of
  // its time. (Packets shorter than the span are better left whole and in place: listing them
  // first, whole, or splitting them cost C3 +16 to +27 %, profiles/r05s_split/.) A packet's parts
  // are 8 items apart, so they run on one XCD; at most a tenth of the packets, kMaxSplit items.
  uint32_t *list = h + c->schedCap, *mask = list + kMaxSplit;
  memset(mask, 0, (4 * c->schedCap + 31) / 32 * sizeof(uint32_t));
  uint32_t ns = 0;
  // (a work item holds the packet index in 24 bits: no splits past 2^24 packets)
  if (c->splitLg > 0 && c->splitFactor > 0.f && wavewg && 4 * (size_t)numBlocks < ((size_t)1 << 24)) {
    const size_t np = 4 * (size_t)numBlocks;
    double total = 0.0;
    for (size_t k = 0; k < np; ++k) total += cost[k];
    const double span = total / (double)std::max(1, 20 * c->numCU);  // 5 waves x 4 SIMDs per CU
    const size_t cap = np / 10;
    std::vector<uint32_t> byCost(np);
    for (size_t k = 0; k < np; ++k) byCost[k] = (uint32_t)k;
    std::partial_sort(byCost.begin(), byCost.begin() + std::min(cap, np), byCost.end(),
                      [&](uint32_t a, uint32_t b) { return cost[a] > cost[b] || (cost[a] == cost[b] && a < b); });
    const uint32_t parts = 1u << c->splitLg;
    std::vector<uint32_t> heavy;
    for (size_t k = 0; k < cap && (heavy.size() + 8) * parts <= kMaxSplit; ++k) {
      const double v = (double)cost[byCost[k]];
      if (!(v > c->splitFactor * span) || v <= 0.0) break;
      heavy.push_back(byCost[k]);
    }
    while (heavy.size() % 8) heavy.push_back(~0u);  // empty packets: their parts render nothing
    for (size_t g = 0; g < heavy.size(); g += 8)
      for (uint32_t part = 0; part < parts; ++part)
        for (size_t j = 0; j < 8; ++j)
          list[ns++] = heavy[g + j] == ~0u ? ~0u : (heavy[g + j] << 8) | (part << 4) | (uint32_t)c->splitLg;
    while (ns % 8) list[ns++] = ~0u;
    for (size_t k = 0; k < ns; ++k)
      if (list[k] != ~0u) mask[(list[k] >> 8) >> 5] |= 1u << ((list[k] >> 8) & 31);
  }
  c->schedSplit[nb] = ns;
  uint32_t *dh = nullptr;
  IRT_HIP(hipHostGetDevicePointer((void **)&dh, h, 0));
  launch_copy_u32(dh, c->d_schedOrder + (size_t)nb * stride, stride, s);
  IRT_HIP(hipGetLastError());
  c->schedBuf = nb;
  c->schedSwitch = c->launches;
  c->schedOrderValid = true;
  c->schedSrc = best;
  return IRT_OK;
}

// buildICONGrid (hostCode.cu:668-682: initGrid + buildGrid_ICON over volbounds) on first
// use of GRID_ACCEL_MODE (a render with IRT_ACCEL_GRID, irt_get_grid), from the scene's
// blocks, meta words and corner trig, then the grid's majorants for the current transfer
// function.  The reference builds it in main() whatever the accel mode (hostCode.cu:875);
// the grid is the same whenever it is built.
int ensure_grid(irt_context *c) {
  if (c->gridBuilt) return IRT_OK;
  const size_t gridMCs = (size_t)kGridDim * kGridDim * kGridDim;
  int rc;
  if (!c->d_gridVR && (rc = dalloc(c, &c->d_gridVR, 2 * gridMCs))) return rc;
  if (!c->d_gridMaxOp && (rc = dalloc(c, &c->d_gridMaxOp, gridMCs))) return rc;
  if (!c->d_gridBits && (rc = dalloc(c, &c->d_gridBits, (size_t)kGridBitWords))) return rc;
  IRT_HIP(hipMemsetAsync(c->d_gridBits, 0, kGridBitWords * sizeof(uint32_t), c->stream));
  launch_shell_init(c->d_gridVR, gridMCs, c->stream);  // initGrid(Grid) (hostCode.cu:205-214)
  IRT_HIP(hipMemsetAsync(c->d_gridMaxOp, 0, gridMCs * sizeof(float), c->stream));
  if (c->n) {
    const irt_box3f &vb = c->info.bounds;
    launch_grid_build(c->d_blocks, c->d_meta, c->d_trig, c->n, make_float3(vb.lower.x, vb.lower.y, vb.lower.z),
                      make_float3(vb.upper.x, vb.upper.y, vb.upper.z), c->d_gridVR, c->stream);
  }
  if (c->tfSet) {
    launch_max_opacities(c->d_gridVR, gridMCs, c->d_lut, c->lutSize, c->tfLo, c->tfHi, c->d_gridMaxOp,
                         c->stream);
    launch_grid_bits(c->d_gridMaxOp, c->d_gridBits, c->stream);
  }
  IRT_HIP(hipGetLastError());
  IRT_HIP(hipStreamSynchronize(c->stream));
  c->gridBuilt = true;
  c->info.deviceBytes = c->bytes;
  return IRT_OK;
}

int render_impl(irt_context *c, const irt_launch_params *lp, int W, int H, int packed,
                int tileBegin, int tileStride, uint32_t *fb, irt_vec4f *accum, int *numTilesOut,
                void *stream, int numFrames = 1, const int32_t *tileList = nullptr,
                int listCount = 0, const irt_launch_params *seq = nullptr) {
  if (!c || !lp || W <= 0 || H <= 0 || !fb || !accum || tileStride <= 0 || tileBegin < 0 ||
      numFrames < 1 || numFrames > 65535 || listCount < 0 || (listCount > 0 && !tileList)) {
    set_error("irt_render: bad argument");
    return IRT_E_INVALID;
  }
  if (!c->tfSet) {
    set_error("irt_render: no transfer function set (irt_set_transfunc)");
    return IRT_E_INVALID;
  }
  if (lp->raygen != IRT_RAYGEN_WITH_ACCEL && lp->raygen != IRT_RAYGEN_AE) {
    set_error("irt_render: unknown raygen %d", lp->raygen);
    return IRT_E_INVALID;
  }
  if (lp->accelMode != IRT_ACCEL_SPHERE && lp->accelMode != IRT_ACCEL_GRID) {
    set_error("irt_render: unknown accelMode %d", lp->accelMode);
    return IRT_E_INVALID;
  }
  if (lp->mode != IRT_MODE_USER_GEOM && lp->mode != IRT_MODE_CUBQL &&
      lp->mode != IRT_MODE_TRIANGLES) {
    set_error("irt_render: unknown sampler mode %d", lp->mode);
    return IRT_E_INVALID;
  }
  if (lp->mode != IRT_MODE_USER_GEOM && c->wG == 0 && c->n != 0) {
    set_error("irt_render: sampler mode %d needs irt_build_wedge_accel first (buildCuBQLAccel / "
              "buildTriangleAccel, hostCode.cu:557-649, 440-484)", lp->mode);
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  if (lp->accelMode == IRT_ACCEL_GRID) {
    int rc = ensure_grid(c);
    if (rc) return rc;
  }
  // NULL is the null stream itself (ordered with the caller's blocking streams), never the
  // context's private non-blocking stream
  hipStream_t s = (hipStream_t)stream;
  const int tilesX = (W + 63) / 64, tilesY = (H + 63) / 64;
  const int total = tilesX * tilesY;
  int numTiles = tileBegin < total ? (total - tileBegin + tileStride - 1) / tileStride : 0;
  const int32_t *dList = nullptr;
  if (tileList) {  // irt_render_tile_list
    numTiles = listCount;
    if (listCount > 0) {
      int rc = tile_table(c, tileList, (size_t)listCount, 0, total, &dList);
      if (rc) return rc;
    }
  }
  if (numTilesOut) *numTilesOut = numTiles;

  RenderArgs A;
  memset(&A, 0, sizeof(A));
  A.org = make_float3(lp->org.x, lp->org.y, lp->org.z);
  A.dir00 = make_float3(lp->dir_00.x, lp->dir_00.y, lp->dir_00.z);
  A.du = make_float3(lp->dir_du.x, lp->dir_du.y, lp->dir_du.z);
  A.dv = make_float3(lp->dir_dv.x, lp->dir_dv.y, lp->dir_dv.z);
  A.accumID = lp->accumID;
  A.accumW = 1.f / (float)(lp->accumID + 1);  // the lerp weight (deviceCode.cu:333), per launch
  A.amb = make_float3(lp->ambientColor.x, lp->ambientColor.y, lp->ambientColor.z);
  A.ambRad = lp->ambientRadiance;
  A.unitDistance = lp->unitDistance;
  A.raygen = lp->raygen;
  const irt_volume_info &I = c->info;
  A.bmin = make_float3(I.bounds.lower.x, I.bounds.lower.y, I.bounds.lower.z);
  A.bmax = make_float3(I.bounds.upper.x, I.bounds.upper.y, I.bounds.upper.z);
  A.dims = make_int3(I.shellDims[0], I.shellDims[1], I.shellDims[2]);
  A.sbLo = make_float3(I.sphericalBounds.lower.x, I.sphericalBounds.lower.y, I.sphericalBounds.lower.z);
  A.sbHi = make_float3(I.sphericalBounds.upper.x, I.sphericalBounds.upper.y, I.sphericalBounds.upper.z);
  A.maxOp = c->d_maxOp;
  A.accelMode = lp->accelMode;
  A.gridMaxOp = c->d_gridMaxOp;
  A.gridBits = c->d_gridBits;
  A.sampler = lp->mode;
  A.wG = c->wG;
  A.wOff = c->d_wOff;
  A.wRec = c->d_wRec;
  A.wBox = c->d_wBox;
  A.wTrig = c->d_wTrig;
  A.tfLo = c->tfLo;
  A.tfHi = c->tfHi;
  {
    const float tfSize = c->tfHi - c->tfLo;  // float, as the reference subtracts
    A.invTf = 1.0 / (double)tfSize;
    const float sz[3] = {I.sphericalBounds.upper.x - I.sphericalBounds.lower.x,
                         I.sphericalBounds.upper.y - I.sphericalBounds.lower.y,
                         I.sphericalBounds.upper.z - I.sphericalBounds.lower.z};
    for (int k = 0; k < 3; ++k) A.invSb[k] = 1.0 / (double)sz[k];
  }
  A.opacityScale = c->opScale;
  A.lut = c->d_lut;
  A.lutSize = c->lutSize;
  A.coopMaxLg = c->coopMaxLg;
  A.coopRamp = c->coopRamp;
  A.probeExit = c->probeExit;
  A.wgTrace = c->wgTrace;
  A.numCells = c->n;
  A.G = c->G;
  A.srgbTh = c->d_srgb;
  A.W = W;
  A.H = H;
  A.fb = fb;
  A.accum = (float4 *)accum;
  A.packed = packed;
  A.tileBegin = tileBegin;
  A.tileStride = tileStride;
  A.numTiles = numTiles;
  A.tilesX = tilesX;
  A.tileList = dList;
  A.counters = c->d_counters + 16 * (c->launches % irt_context::kSlots);
  A.binHdr = c->d_binHdr;
  A.fat = c->d_fat;
  A.blocks = c->d_blocks;
  A.slots = c->slotAlways || c->slotSparse ? c->slot.slots : nullptr;
  A.slotBins = c->slot.bins;
  A.slotSubs = c->slot.subs;
  for (int k = 0; k < 3; ++k) A.slotEdge[k] = c->slot.edges[k];
  A.numSph = c->numSph;
  A.sphR = c->d_sphR;
  A.sphOff = c->d_sphOff;
  A.sphRec = c->d_sphRec;
  A.sphBits = c->d_sphBits;

  // a launch in flight whose chained wait gave up (its pinned flag is set as it happens):
  // report it now, from the next call, instead of when its slot is retired
  for (int i = 0; i < irt_context::kSlots; ++i)
    if (c->pending[i] && c->h_chainFail[i]) {
      int rc = finish_slot(c, i);
      if (rc) return rc;
    }
  const int slot = (int)(c->launches % irt_context::kSlots);
  if (c->pending[slot]) {  // the ring is full: retire that launch (long done by now)
    int rc = finish_slot(c, slot);
    if (rc) return rc;
  }
  // Launches of a context run in call order, also across streams: a launch on another stream
  // than the previous one waits for it before anything of this call is queued (the chain words,
  // the frame cameras and the counter block below are shared by every launch of the context;
  // two chained launches in flight at once on two streams would overwrite each other's words)
  if (c->launches > 0 && s != c->lastStream) {
    const int prev = (int)((c->launches - 1) % irt_context::kSlots);
    if (c->pending[prev]) {
      const hipEvent_t e = done_event(c, prev);
      if (e) IRT_HIP(hipStreamWaitEvent(s, e, 0));
    }
  }
  c->lastStream = s;
  const size_t lanes = (size_t)numTiles * 4096;
  // persistent launch: the cooperative kernels, not for the measurement-only early exits
  // (every wave must reach the queue's done count)
  const bool queued = c->queueOn && numTiles > 0 && (c->probeExit == 0 || c->probeExit >= 16) && render_queue_ok(A, c->variant);
  int queueWG = 0;
  if (queued) {
    A.queue = c->d_queue + (size_t)kQueueWords * slot;
    A.numPackets = (uint32_t)numTiles * 64u * (uint32_t)numFrames;
    queueWG = c->queuePerCU > 0 ? std::min(c->queuePerCU * c->numCU, numTiles * 16 * numFrames)
                                : render_queue_wgs(A, c->variant, c->numCU, numTiles * 16 * numFrames);
    c->lastQueueWG = queueWG;
  }
  // measured-cost scheduling: single-frame launches of the one-kernel raygen only (before the
  // workgroup count: the split packets' parts are extra workgroups)
  A.schedOrder = nullptr;
  A.schedCost = nullptr;
  A.splitList = A.splitMask = nullptr;
  A.numSplit = 0;
  const int numBlocks = numTiles * 16;
  bool copyCosts = false;
  if (c->schedOn && numFrames == 1 && numBlocks > 0 && !dList && !queued) {
    int rc = sched_prepare(c, numBlocks, W, H, packed, tileBegin, tileStride, numTiles, lp,
                           render_split_ok(A, c->variant), s);
    if (rc) return rc;
    const uint32_t *ob = c->d_schedOrder + (size_t)c->schedBuf * sched_stride(c->schedCap);
    A.schedOrder = c->schedOrderValid ? ob : nullptr;
    if (c->schedOrderValid && c->schedSplit[c->schedBuf] && render_split_ok(A, c->variant) &&
        (c->probeExit == 0 || c->probeExit >= 16)) {
      A.splitList = ob + c->schedCap;
      A.splitMask = ob + c->schedCap + kMaxSplit;
      A.numSplit = c->schedSplit[c->schedBuf];
    }
    // every 8th launch writes its workgroups' durations straight into this slot's pinned
    // host copy; the others into device memory nobody reads
    copyCosts = c->launches - c->schedLastCopy >= 8;
    if (copyCosts) {
      uint32_t *dh = nullptr;
      IRT_HIP(hipHostGetDevicePointer((void **)&dh, c->h_schedCost + (size_t)slot * 4 * c->schedCap, 0));
      A.schedCost = dh;
    } else {
      A.schedCost = c->d_schedCost;
    }
  }
  // chained frames: the cooperative kernels (not the one-lane-per-ray A/B variant), grid
  // launches, no measurement-only early exit
  // The hand-off's buffer resources address accum with 32-bit byte offsets: frames of 2^27
  // pixels or more (11,585^2) go through the sample buffer instead
  const uint64_t outPixels = packed ? (uint64_t)numTiles * 4096u : (uint64_t)W * (uint64_t)H;
  const bool chain = c->chainOn && numFrames > 1 && !queued && (c->probeExit == 0 || c->probeExit >= 16) &&
                     (c->variant & 65536) == 0 && outPixels * 16u <= 0x7FFFFFFFull;
  // two chained frames per wave (the OPT_FPAIR variants, bit 1): half the grid's frame rows
  A.chain = chain ? 1 : 0;
  const int fpw = render_frames_per_wave(A, c->variant);
  // workgroups of this launch: 16 per 64x64 tile, x4 for the one-wave-workgroup variants
  // (irt_render.hip OPT_WAVEWG, bit 4194304), per frame (per pair of frames), + the split
  // packets' parts; a persistent launch's resident ones
  const size_t numWG = queued ? (size_t)queueWG
                              : (size_t)numTiles * 16 * (size_t)render_wg_per_block(A, c->variant) *
                                        (size_t)((numFrames + fpw - 1) / fpw) +
                                    (size_t)A.numSplit;
  // Per-workgroup counts need kSlots x 32 B of pinned host memory per workgroup and frame
  // (1 KiB): a launch past kWgCountsMax workgroups (a large progressive batch) counts through
  // the device-atomic block instead, for that launch only.
  const bool useWG = c->wgCountsOn && numWG <= c->wgCountsMax;
  if (useWG && numWG > c->wgCap) {
    // every slot's launch must be retired before the ring is reallocated
    int rc = finish_stats(c);
    if (rc) return rc;
    if (c->h_wgCounts) IRT_HIP(hipHostFree(c->h_wgCounts));
    c->h_wgCounts = c->dh_wgCounts = nullptr;
    c->wgCap = 0;
    // kSlots x 1 KiB of pinned memory per workgroup and frame: a huge progressive batch may
    // not get it -- then the counters go through the device-atomic block from here on
    // (IRT_COUNTERS=atomic), which needs no per-workgroup memory
    if (hipHostMalloc((void **)&c->h_wgCounts, numWG * irt_context::kSlots * kCnt * sizeof(uint32_t)) !=
            hipSuccess ||
        hipHostGetDevicePointer((void **)&c->dh_wgCounts, c->h_wgCounts, 0) != hipSuccess) {
      (void)hipGetLastError();
      if (c->h_wgCounts) (void)hipHostFree(c->h_wgCounts);
      c->h_wgCounts = c->dh_wgCounts = nullptr;
      c->wgCountsOn = false;
    } else {
      c->wgCap = numWG;
    }
  }
  A.wgCounts = useWG && c->wgCountsOn ? c->dh_wgCounts + (size_t)slot * c->wgCap * kCnt : nullptr;
  const bool statsVariant = (c->variant & (32768 | 524288)) != 0;  // statistics, timing
  if (c->countersProbe == 1 || c->statsOff) {
    // measurement only: no counts -- except that the statistics and timing variants add into
    // the counter block unconditionally, so it stays
    A.wgCounts = nullptr;
    if (!statsVariant) A.counters = nullptr;
  } else if (c->countersProbe == 2) {
    if (numWG > c->probeCap) {  // per-workgroup stores into device memory: one slot per workgroup
      IRT_HIP(hipStreamSynchronize(s));
      if (c->d_probeCounts) IRT_HIP(hipFree(c->d_probeCounts));
      c->d_probeCounts = nullptr;
      c->probeCap = 0;
      IRT_HIP(hipMalloc((void **)&c->d_probeCounts, numWG * kCnt * sizeof(uint32_t)));
      c->probeCap = numWG;
    }
    A.wgCounts = c->d_probeCounts;
  }
  A.numSamples = numFrames;
  A.chain = chain ? 1 : 0;
  if (A.chain) {
    const size_t words = (size_t)numTiles * 16 * 4;  // one per (block, wave)
    if (words > c->chainCap || c->chainEpoch > 0xF0000000u - (uint32_t)numFrames) {
      if (words > c->chainCap) {
        int rc = finish_stats(c);  // every launch that may still read the old words, on any stream
        if (rc) return rc;
        IRT_HIP(hipStreamSynchronize(s));
        if (c->d_chainFlag) IRT_HIP(hipFree(c->d_chainFlag));
        c->d_chainFlag = nullptr;
        c->bytes -= c->chainCap * sizeof(uint32_t);
        c->chainCap = 0;
        if ((rc = dalloc(c, &c->d_chainFlag, words))) return rc;
        c->chainCap = words;
        c->info.deviceBytes = c->bytes;
      }
      IRT_HIP(hipMemsetAsync(c->d_chainFlag, 0, c->chainCap * sizeof(uint32_t), s));
      c->chainEpoch = 1;  // never 0: the zeroed words match no epoch
    }
    A.chainFlag = c->d_chainFlag;
    c->h_chainFail[slot] = 0;
    A.chainFail = c->dh_chainFail + slot;
    A.chainSpins = c->chainSpins ? c->chainSpins : kChainSpinsDefault;
    A.chainWithhold = c->chainWithhold;
    A.chainEpoch = c->chainEpoch;
    c->chainEpoch += (uint32_t)numFrames;
  }
  if (seq) {
    // a sequence of views (irt_render_sequence): frame k's camera and accumID as 4 float4
    if (!A.chain) {
      set_error("irt_render_sequence: needs chained frames (a cooperative variant, IRT_CHAIN on)");
      return IRT_E_INVALID;
    }
    if ((size_t)numFrames > c->frameCamCap) {
      int rc = finish_stats(c);  // every slot's staging retired before it is reallocated
      if (rc) return rc;
      IRT_HIP(hipStreamSynchronize(s));
      if (c->d_frameCams) IRT_HIP(hipFree(c->d_frameCams));
      if (c->h_frameCams) IRT_HIP(hipHostFree(c->h_frameCams));
      c->d_frameCams = c->h_frameCams = nullptr;
      c->bytes -= c->frameCamCap * 4 * sizeof(float4);
      c->frameCamCap = 0;
      if ((rc = dalloc(c, &c->d_frameCams, (size_t)numFrames * 4))) return rc;
      IRT_HIP(hipHostMalloc((void **)&c->h_frameCams, (size_t)irt_context::kSlots * numFrames * 4 * sizeof(float4)));
      c->frameCamCap = (size_t)numFrames;
      c->info.deviceBytes = c->bytes;
    }
    float4 *h = c->h_frameCams + (size_t)slot * c->frameCamCap * 4;
    for (int k = 0; k < numFrames; ++k) {
      const irt_launch_params &q = seq[k];
      h[4 * k + 0] = make_float4(q.org.x, q.org.y, q.org.z, __builtin_bit_cast(float, q.accumID));
      h[4 * k + 1] = make_float4(q.dir_00.x, q.dir_00.y, q.dir_00.z, 0.f);
      h[4 * k + 2] = make_float4(q.dir_du.x, q.dir_du.y, q.dir_du.z, 0.f);
      h[4 * k + 3] = make_float4(q.dir_dv.x, q.dir_dv.y, q.dir_dv.z, 0.f);
    }
    IRT_HIP(hipMemcpyAsync(c->d_frameCams, h, (size_t)numFrames * 4 * sizeof(float4), hipMemcpyHostToDevice, s));
    A.frameCams = c->d_frameCams;
  }
  if (numFrames > 1 && !A.chain) {
    const size_t need = lanes * (size_t)numFrames;
    if (need > c->sampleCap) {
      IRT_HIP(hipStreamSynchronize(s));
      if (c->d_samples) IRT_HIP(hipFree(c->d_samples));
      c->d_samples = nullptr;
      c->bytes -= c->sampleCap * sizeof(float4);
      c->sampleCap = 0;
      int rc = dalloc(c, &c->d_samples, need);
      if (rc) return rc;
      c->sampleCap = need;
      c->info.deviceBytes = c->bytes;
    }
  }
  A.sampleBuf = c->d_samples;
  // measured-cost scheduling: single-frame launches of the one-kernel raygen only
  c->schedLastApplied = A.schedOrder != nullptr;
  c->lastNumSplit = A.numSplit;
  c->schedApplied += c->schedLastApplied ? 1 : 0;
  // the 16-counter block (device atomics) is only needed by the statistics variant and the
  // IRT_COUNTERS=atomic mode; it must start zeroed
  // the atomic fallback of the per-workgroup counts adds into this slot's buckets
  A.counterBuckets = A.counters && !A.wgCounts ? c->d_counterBuckets + (size_t)slot * kCounterBuckets * 8 : nullptr;
  const bool block = A.counters && (!A.wgCounts || statsVariant);
  if (block && !c->lastBlock) IRT_HIP(hipMemsetAsync(A.counters, 0, 16 * sizeof(unsigned long long), s));
  c->timed[slot] = c->launches % c->timingEvery == 0;
  if (c->timed[slot]) IRT_HIP(hipEventRecord(c->ev0[slot], s));
  if (numTiles > 0) {
    launch_render(A, queued ? queueWG : numTiles * 16, s, c->variant);
  }
  IRT_HIP(hipGetLastError());
  if (c->timed[slot]) IRT_HIP(hipEventRecord(c->ev1[slot], s));
  if (block) {
    launch_stats_out(A.counters, c->dh_counters + 16 * slot,
                     c->d_counters + 16 * ((c->launches + 1) % irt_context::kSlots), A.counterBuckets, s);
    IRT_HIP(hipGetLastError());
  }
  c->slotBlock[slot] = block;
  c->lastBlock = block;
  c->slotWG[slot] = (A.wgCounts && c->countersProbe == 0 && !c->statsOff && numTiles > 0) ? numWG : 0;
  c->schedCopied[slot] = -1;
  if (copyCosts) {
    c->schedCopied[slot] = c->launches;
    c->schedLastCopy = c->launches;
  }
  c->slotStream[slot] = s;
  c->slotLaunch[slot] = c->launches;
  c->evRec[slot] = c->launches % irt_context::kDoneEvery == irt_context::kDoneEvery - 1 || copyCosts;
  if (c->evRec[slot]) IRT_HIP(hipEventRecord(c->evDone[slot], s));
  c->pending[slot] = true;
  ++c->launches;
  return IRT_OK;
}

}  // namespace

extern "C" {

int irt_create_begin(size_t numCells, int device, irt_context **out) {
  if (!out) {
    set_error("irt_create: null argument");
    return IRT_E_INVALID;
  }
  *out = nullptr;
  if (numCells > 0xFFFFFFF0ull) {
    set_error("too many cells (%zu)", numCells);
    return IRT_E_INVALID;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_error("irt_create: no HIP device visible (this product has no CPU fallback)");
    return IRT_E_HIP;
  }
  if (device < 0 || device >= ndev) {
    set_error("irt_create: device %d out of range (%d devices)", device, ndev);
    return IRT_E_INVALID;
  }
  irt_context *c = new irt_context();
  c->device = device;
  if (const char *v = getenv("IRT_RENDER_VARIANT")) {
    const int var = atoi(v);
    if (render_variant_available(var)) {
      c->variant = var;
      c->variantFixed = true;
    }
  }
  auto fail = [&](int code) {
    free_all(c);
    delete c;
    return code;
  };
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    set_error("irt_create: cannot initialise device %d", device);
    return fail(IRT_E_HIP);
  }
  if (const char *e = getenv("IRT_SPLIT_LG")) c->splitLg = std::min(3, std::max(0, atoi(e)));
  if (const char *e = getenv("IRT_SPLIT_FACTOR")) {
    c->splitFactor = (float)atof(e);
    c->splitFixed = true;
  }
  if (const char *e = getenv("IRT_SCHED")) {
    c->schedOn = atoi(e) != 0;
    c->schedPolicy = atoi(e);
    c->schedFixed = true;
  }
  if (hipMalloc((void **)&c->d_cells, std::max<size_t>(numCells, 1) * sizeof(irt_icon_cell)) != hipSuccess ||
      hipMalloc((void **)&c->d_trig, std::max<size_t>(numCells, 1) * 3 * sizeof(float4)) != hipSuccess) {
    set_error("irt_create: cannot allocate %zu cells in HBM", numCells);
    return fail(IRT_E_HIP);
  }
  volume_acc_init(c->vacc);
  c->expected = numCells;
  c->building = true;
  *out = c;
  return IRT_OK;
}

namespace {
// One chunk of records: validation, glibc corner trig and getBounds, and the record-order
// folds (volume facts, column count, sphere records), per contiguous slice of records in
// parallel; the slices' partial folds are combined in slice order, which selects the same
// elements as one sequential fold (volume_acc_merge).  Then the cells and their trig go to
// HBM: synchronously from the caller's memory, or, with `trigPinned` (cells already in
// pinned memory, irt_create_synth), asynchronously on the context stream.
int append_chunk(irt_context *c, const irt_icon_cell *cells, size_t n, float *trigPinned) {
  const size_t base = c->received;
  std::vector<float> trigHeap;
  float *trig = trigPinned;
  if (!trig) {
    trigHeap.resize(n * 12);
    trig = trigHeap.data();
  }
  const int threads = n < 4096 ? 1 : default_threads();
  const size_t slice = (n + threads - 1) / threads;
  struct Part {
    VolumeAcc acc;
    size_t runs = 0, bad = SIZE_MAX;
    std::vector<irt_context::Sphere> sph;
    float bottomMin = INFINITY, bottomMax = -INFINITY;  // height[0] of the columns' first records
    bool gap = false;  // a record that does not continue its column (or holds no radius)
  };
  std::vector<Part> part(threads);
  auto work = [&](int t) {
    Part &P = part[t];
    volume_acc_init(P.acc);
    const size_t b = (size_t)t * slice, e = std::min(n, b + slice);
    for (size_t i = b; i < e; ++i) {
      const irt_icon_cell &x = cells[i];
      bool ok = x.numLayers >= 0 && x.numLayers <= 31;
      for (int k = 0; ok && k < 3; ++k) ok = std::isfinite(x.lat[k]) && std::isfinite(x.lon[k]);
      for (int j = 0; ok && j <= x.numLayers; ++j) ok = std::isfinite(x.height[j]);
      if (!ok) {
        P.bad = i;
        return;
      }
      float *tr = &trig[12 * i];
      if (i > b && same_corners(x.lat, x.lon, cells[i - 1].lat, cells[i - 1].lon))
        memcpy(tr, tr - 12, 12 * sizeof(float));  // same column, same corners
      else
        corner_trig(x, tr);
      float lo[3], hi[3];
      cell_bounds(x, tr, lo, hi);
      volume_acc_add(P.acc, x, lo, hi);
      const irt_icon_cell &prev = i ? cells[i - 1] : c->last;
      if (base + i == 0 || !same_corners(x.lat, x.lon, prev.lat, prev.lon)) {
        ++P.runs;
        P.bottomMin = std::min(P.bottomMin, x.height[0]);
        P.bottomMax = std::max(P.bottomMax, x.height[0]);
      } else if (!(x.height[0] == prev.height[prev.numLayers])) {
        P.gap = true;
      }
      if (!(x.height[0] <= x.height[x.numLayers])) P.gap = true;
      if (x.height[0] == x.height[x.numLayers])  // a sphere record
        P.sph.push_back({x.height[0], (uint32_t)(base + i), x.numLayers});
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(work, t);
    for (auto &t : ts) t.join();
  }
  size_t bad = SIZE_MAX;
  for (const Part &P : part) bad = std::min(bad, P.bad);
  if (bad != SIZE_MAX) {  // the first bad record, as a sequential check would report
    const irt_icon_cell &x = cells[bad];
    if (x.numLayers < 0 || x.numLayers > 31)
      set_error("cell %zu: numLayers %d outside [0,31] (MAX_LAYERS 32, ICONGrid.h:57)", base + bad, x.numLayers);
    else
      set_error("cell %zu: non-finite lat/lon/height", base + bad);
    return IRT_E_DATA;
  }
  for (const Part &P : part) {
    volume_acc_merge(c->vacc, P.acc);
    c->numRuns += P.runs;
    c->sph.insert(c->sph.end(), P.sph.begin(), P.sph.end());
    c->bottomMin = std::min(c->bottomMin, P.bottomMin);
    c->bottomMax = std::max(c->bottomMax, P.bottomMax);
    c->voids = c->voids || P.gap;
  }
  IRT_HIP(hipSetDevice(c->device));
  if (trigPinned) {
    IRT_HIP(hipMemcpyAsync(c->d_cells + base, cells, n * sizeof(irt_icon_cell), hipMemcpyHostToDevice, c->stream));
    IRT_HIP(hipMemcpyAsync(c->d_trig + 3 * base, trig, n * 12 * sizeof(float), hipMemcpyHostToDevice, c->stream));
  } else {
    IRT_HIP(hipMemcpy(c->d_cells + base, cells, n * sizeof(irt_icon_cell), hipMemcpyHostToDevice));
    IRT_HIP(hipMemcpy(c->d_trig + 3 * base, trig, n * 12 * sizeof(float), hipMemcpyHostToDevice));
  }
  c->last = cells[n - 1];
  c->received += n;
  return IRT_OK;
}
}  // namespace

int irt_create_append(irt_context *c, const irt_icon_cell *cells, size_t n) {
  if (!c || !c->building || (n && !cells)) {
    set_error("irt_create_append: no context being created, or null cells");
    return IRT_E_INVALID;
  }
  if (n > c->expected - c->received) {
    set_error("irt_create_append: %zu more cells than irt_create_begin announced", n - (c->expected - c->received));
    return IRT_E_INVALID;
  }
  if (n == 0) return IRT_OK;
  return append_chunk(c, cells, n, nullptr);
}

// The slot table of a built scene (irt_kernels.h build_slots_device), if its cells share their
// radial edges and it fits: at most IRT_SLOTS_MAX_GB, half the device's memory and its free memory
// less 16 GiB.  Sub-cells per slot unit (irt_common.h slot_unit): by default the finest unit -- 1
// sub-cell, a pair or a quad -- whose table is at most the scene's own bytes (C5: quads, 32 GB
// beside 38.7 GB of headers, entries and blocks); IRT_SLOT_SUBS=1, 2 or 4 asks for one.
int build_slot_table(irt_context *c, bool forced) {
  c->slotTried = true;
  // the kernel's slot index (cell * kSubCells^2 + sub) is 32-bit
  const bool indexable = (uint64_t)6 * c->G * c->G * kSubCells * kSubCells < ((uint64_t)1 << 32);
  int slotSubs = 0;
  if (const char *v = getenv("IRT_SLOT_SUBS")) slotSubs = atoi(v);
  // the scene's own bytes: the locator and the records it indexes (headers, entries, blocks)
  const size_t hdrBytes = (size_t)6 * c->G * c->G * kBinHdrWords * 4;
  const size_t sceneBytes = hdrBytes + c->binEntries * kFatStride4 * 16 + (size_t)c->n * kBlk4 * 16;
  size_t fr = 0, tot = 0;
  IRT_HIP(hipMemGetInfo(&fr, &tot));
  size_t cap = fr > ((size_t)16 << 30) ? fr - ((size_t)16 << 30) : 0;
  cap = std::min(cap, tot / 2);
  if (const char *g = getenv("IRT_SLOTS_MAX_GB")) cap = std::min(cap, (size_t)(atof(g) * (double)(1ull << 30)));
  if (!indexable) {
    c->slot = SlotTable{};
    c->slot.skipped = "the cube map has 2^28 cells or more (32-bit slot index)";
  } else if (int rc = build_slots_device(reinterpret_cast<const uint32_t *>(c->d_binHdr), c->d_fat, 6u * c->G * c->G,
                                         cap, slotSubs, sceneBytes, c->stream, c->slot)) {
    return rc;
  }
  c->bytes += c->slot.bytes;
  c->info.deviceBytes = c->bytes;
  if (c->slot.bytes)
    fprintf(stderr, "icon_rt_hip: slot table built on device %d: %.1f GB of HBM, %d sub-cells per slot (IRT_SLOTS=0: none)\n",
            c->device, c->slot.bytes / 1e9, c->slot.subs);
  else if (forced)
    fprintf(stderr, "icon_rt_hip: IRT_SLOTS=1 but no slot table was built: %s\n",
            c->slot.skipped ? c->slot.skipped : "unknown reason");
  return IRT_OK;
}

int irt_create_end(irt_context *c) {
  if (!c || !c->building) {
    set_error("irt_create_end: no context being created");
    return IRT_E_INVALID;
  }
  if (c->received != c->expected) {
    set_error("irt_create_end: %zu of %zu cells appended", c->received, c->expected);
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  const size_t numCells = c->expected;
  const bool verbose = getenv("IRT_BUILD_VERBOSE") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto mark = [&](const char *what) {
    if (!verbose) return;
    (void)hipStreamSynchronize(c->stream);
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[irt create] %-20s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
    t0 = t;
  };
  volume_acc_finish(c->vacc, c->info);
  c->n = (uint32_t)numCells;
  const bool holes = c->voids || c->bottomMin < c->bottomMax;
  if (!c->variantFixed && c->variant == kDefaultVariant) c->variant = scene_variant(holes);
  // single frames of a scene with holes: longest 64x64 tiles first, by the durations every 8th
  // launch records (the voids' limb packets run 190-240 us against a 29 us median; C3t -7 %, flat
  // scenes even: profiles/r05r_sched/)
  if (!c->schedFixed && holes) {
    c->schedOn = true;
    c->schedPolicy = 1;
  }
  // ... and their packets longer than 0.35 x the frame's ideal span split (C3t one frame 0.177 ->
  // 0.144 ms against 1.0 x, profiles/r06y/; chained launches never split)
  if (!c->splitFixed && holes) c->splitFactor = kSplitFactorHoles;
  c->G = locator_resolution(c->numRuns);
  // the scene build on the device (irt_build.hip)
  DeviceScene D;
  int rc = build_scene_device(c->d_cells, c->d_trig, numCells, c->numRuns, c->G, c->stream, D);
  c->d_blocks = D.blocks;
  c->d_meta = D.meta;
  c->d_binHdr = D.binHdr;
  c->d_fat = D.fat;
  c->bytes += D.bytes;
  if (rc) return rc;
  c->info.locatorFaceRes = c->G;
  c->info.locatorEntries = D.entries;
  c->binEntries = D.binEntries;
  mark("device scene build");
  // the slot table, when the cells share their radial edges, their headers outgrow the
  // last-level cache (kSlotAutoHdrBytes) and it fits: at most IRT_SLOTS_MAX_GB, by default half
  // the device's memory and never more than its free memory less 16 GiB (a process sharing the
  // GPU keeps the rest); IRT_SLOTS=1: whatever the headers' size, 0: none.  Without IRT_SLOTS a
  // smaller scene gets it when a sparse transfer function is set (irt_set_transfunc).  A built
  // table is announced on stderr with its size; an explicit IRT_SLOTS=1 that builds none says why.
  {
    const char *e = getenv("IRT_SLOTS");
    const bool forced = e && atoi(e) != 0;
    const char *sp = getenv("IRT_SLOTS_SPARSE_TF");  // 0: not for sparse transfer functions either
    c->slotLazy = !e && (!sp || atoi(sp) != 0);
    const size_t hdrBytes = (size_t)6 * c->G * c->G * kBinHdrWords * 4;
    if (e ? forced : hdrBytes > kSlotAutoHdrBytes) {
      if ((rc = build_slot_table(c, forced))) return rc;
      c->slotAlways = c->slot.slots != nullptr;
    }
  }
  mark("slot table");
  // zero-thickness records (spheres): sorted by (radius, record) -- see host/irt_scene.cpp
  {
    std::sort(c->sph.begin(), c->sph.end(), [](const irt_context::Sphere &a, const irt_context::Sphere &b) {
      return a.r < b.r || (a.r == b.r && a.rec < b.rec);
    });
    std::vector<float> R;
    std::vector<uint32_t> off(1, 0u), bits(kSphBitWords, 0u);
    std::vector<uint2> rec;
    for (size_t k = 0; k < c->sph.size(); ++k) {
      if (k == 0 || c->sph[k].r != c->sph[k - 1].r) {
        if (k) off.push_back((uint32_t)rec.size());
        R.push_back(c->sph[k].r);
      }
      rec.push_back(make_uint2(c->sph[k].rec, (uint32_t)c->sph[k].nl));
    }
    if (!c->sph.empty()) off.push_back((uint32_t)rec.size());
    for (float r : R) {
      const uint32_t h = sph_hash(r);
      bits[h >> 5] |= 1u << (h & 31);
    }
    c->numSph = (uint32_t)R.size();
    c->numSphRec = (uint32_t)rec.size();
    if ((rc = upload(c, &c->d_sphR, R.data(), R.size())) || (rc = upload(c, &c->d_sphOff, off.data(), off.size())) ||
        (rc = upload(c, &c->d_sphRec, rec.data(), rec.size())) ||
        (rc = upload(c, &c->d_sphBits, bits.data(), bits.size())))
      return rc;
    IRT_HIP(hipStreamSynchronize(c->stream));
    std::vector<irt_context::Sphere>().swap(c->sph);
  }
  mark("sphere table");
  float th[256];
  srgb_thresholds(th);
  mark("sRGB thresholds");
  const int dims[3] = {c->info.shellDims[0], c->info.shellDims[1], c->info.shellDims[2]};
  c->numMCs = (size_t)dims[0] * dims[1] * dims[2];
  if ((rc = dalloc(c, &c->d_maxOp, c->numMCs))) return rc;
  IRT_HIP(hipMemsetAsync(c->d_maxOp, 0, c->numMCs * sizeof(float), c->stream));
  if ((rc = upload(c, &c->d_srgb, th, 256))) return rc;
  if ((rc = dalloc(c, &c->d_counters, 16 * irt_context::kSlots))) return rc;
  if ((rc = dalloc(c, &c->d_counterBuckets, (size_t)kCounterBuckets * 8 * irt_context::kSlots))) return rc;
  IRT_HIP(hipMemsetAsync(c->d_counterBuckets, 0, (size_t)kCounterBuckets * 8 * irt_context::kSlots * sizeof(unsigned long long),
                         c->stream));
  IRT_HIP(hipHostMalloc((void **)&c->h_counters, 16 * irt_context::kSlots * sizeof(unsigned long long)));
  for (int i = 0; i < irt_context::kSlots; ++i) {
    IRT_HIP(hipEventCreate(&c->ev0[i]));
    IRT_HIP(hipEventCreate(&c->ev1[i]));
    // no timestamps: this event only orders the slot's reuse (a timing event's marker costs more)
    IRT_HIP(hipEventCreateWithFlags(&c->evDone[i], hipEventDisableTiming));
  }
  memset(c->h_counters, 0, 16 * irt_context::kSlots * sizeof(unsigned long long));
  if (const char *e = getenv("IRT_COUNTERS")) {
    c->wgCountsOn = strcmp(e, "atomic") != 0;
    c->countersProbe = strcmp(e, "off") == 0 ? 1 : (strcmp(e, "device") == 0 ? 2 : 0);
  }
  if (const char *e = getenv("IRT_TIMING_EVERY")) c->timingEvery = std::max(1, atoi(e));
  if (const char *e = getenv("IRT_WG_COUNTS_MAX")) c->wgCountsMax = (size_t)std::max(0LL, atoll(e));
  if (const char *e = getenv("IRT_COOP_MAXLG")) c->coopMaxLg = std::min(6, std::max(0, atoi(e)));
  if (const char *e = getenv("IRT_COOP_RAMP")) c->coopRamp = std::min(6, std::max(0, atoi(e)));
  if (const char *e = getenv("IRT_PROBE_EXIT")) c->probeExit = atoi(e);
  if (const char *e = getenv("IRT_QUEUE")) c->queueOn = atoi(e) != 0 && render_queue_compiled();
  if (const char *e = getenv("IRT_QUEUE_WGS")) c->queuePerCU = std::max(0, atoi(e));
  if (const char *e = getenv("IRT_CHAIN")) c->chainOn = atoi(e) != 0;
  IRT_HIP(hipHostMalloc((void **)&c->h_chainFail, irt_context::kSlots * sizeof(uint32_t)));
  memset(c->h_chainFail, 0, irt_context::kSlots * sizeof(uint32_t));
  IRT_HIP(hipHostGetDevicePointer((void **)&c->dh_chainFail, c->h_chainFail, 0));
  if ((rc = dalloc(c, &c->d_queue, (size_t)kQueueWords * irt_context::kSlots))) return rc;
  IRT_HIP(hipMemsetAsync(c->d_queue, 0, (size_t)kQueueWords * irt_context::kSlots * sizeof(uint32_t), c->stream));
  IRT_HIP(hipDeviceGetAttribute(&c->numCU, hipDeviceAttributeMultiprocessorCount, c->device));
  IRT_HIP(hipHostGetDevicePointer((void **)&c->dh_counters, c->h_counters, 0));
  IRT_HIP(hipMemsetAsync(c->d_counters, 0, 16 * irt_context::kSlots * sizeof(unsigned long long), c->stream));

  // ShellAccel{vec3i(1,1024,1024), sphericalBounds} + initGrid + buildShell_ICON
  // (hostCode.cu:652-666), majorants zero until a transfer function arrives
  if ((rc = dalloc(c, &c->d_valueRanges, 2 * c->numMCs))) return rc;
  launch_shell_init(c->d_valueRanges, c->numMCs, c->stream);
  if (numCells) {
    const irt_box3f &sb = c->info.sphericalBounds;
    launch_shell_build(c->d_cells, numCells, make_int3(dims[0], dims[1], dims[2]),
                       make_float3(sb.lower.x, sb.lower.y, sb.lower.z),
                       make_float3(sb.upper.x, sb.upper.y, sb.upper.z), c->d_valueRanges, c->stream);
  }
  prewarm_render(c->variant, c->stream);
  IRT_HIP(hipGetLastError());
  IRT_HIP(hipStreamSynchronize(c->stream));
  mark("shell build");
  // the records themselves are not needed again: the GRID_ACCEL_MODE grid, if ever asked
  // for, is built from the blocks, meta words and corner trig (ensure_grid)
  IRT_HIP(hipFree(c->d_cells));
  c->d_cells = nullptr;
  c->bytes += std::max<size_t>(numCells, 1) * 3 * sizeof(float4);  // d_trig, kept
  c->building = false;
  c->info.deviceBytes = c->bytes;
  // Every scene runs the default 5 waves/SIMD.  (Until the 5-wave kernel lost its scratch
  // spills, scenes past 16 GiB ran the 4-wave build: C5 was 1.9 % faster at 4 waves then,
  // and is 2.8 % slower at 4 waves now -- profiles/r03u_waves/, profiles/r03zg_waves/.)
  return IRT_OK;
}

int irt_create(const irt_icon_cell *cells, size_t numCells, int device, irt_context **out) {
  if (!out || (numCells && !cells)) {
    set_error("irt_create: null argument");
    return IRT_E_INVALID;
  }
  irt_context *c = nullptr;
  int rc = irt_create_begin(numCells, device, &c);
  if (rc) return rc;
  if ((rc = irt_create_append(c, cells, numCells)) || (rc = irt_create_end(c))) {
    irt_destroy(c);
    *out = nullptr;
    return rc;
  }
  *out = c;
  return IRT_OK;
}

// streamed creation helpers: records arrive in chunks of kChunk
static constexpr size_t kChunk = size_t(1) << 20;

int irt_create_from_file(const char *path, long maxNumCells, int device, irt_context **out) {
  if (!path || !out) {
    set_error("irt_create_from_file: null argument");
    return IRT_E_INVALID;
  }
  *out = nullptr;
  FILE *f = fopen(path, "rb");
  if (!f) {
    set_error("irt_create_from_file: cannot open %s", path);
    return IRT_E_IO;
  }
  fseek(f, 0, SEEK_END);
  const long size = ftell(f);
  fseek(f, 0, SEEK_SET);
  size_t n = (size_t)size / sizeof(irt_icon_cell);  // hostCode.cu:725
  if (maxNumCells >= 0) n = std::min(n, (size_t)maxNumCells);  // hostCode.cu:728-730
  irt_context *c = nullptr;
  int rc = irt_create_begin(n, device, &c);
  if (rc) {
    fclose(f);
    return rc;
  }
  std::vector<irt_icon_cell> buf(std::min(n, kChunk));
  for (size_t at = 0; at < n && !rc; at += buf.size()) {
    const size_t m = std::min(buf.size(), n - at);
    if (fread(buf.data(), sizeof(irt_icon_cell), m, f) != m) {
      set_error("irt_create_from_file: short read at record %zu", at);
      rc = IRT_E_IO;
      break;
    }
    rc = irt_create_append(c, buf.data(), m);
  }
  fclose(f);
  if (!rc) rc = irt_create_end(c);
  if (rc) {
    irt_destroy(c);
    return rc;
  }
  *out = c;
  return IRT_OK;
}

int irt_create_synth(int rootN, int bisections, int levels, float topHeight, float noise,
                     uint32_t seed, int device, irt_context **out) {
  return irt_create_synth_terrain(rootN, bisections, levels, topHeight, noise, seed, 0.f, device, out);
}

int irt_create_synth_terrain(int rootN, int bisections, int levels, float topHeight, float noise,
                             uint32_t seed, float terrainHeight, int device, irt_context **out) {
  if (!out) {
    set_error("irt_create_synth: null argument");
    return IRT_E_INVALID;
  }
  *out = nullptr;
  void *gen = nullptr;
  size_t n = 0;
  int rc = synth_open(rootN, bisections, levels, topHeight, noise, seed, terrainHeight, &gen, &n);
  if (rc) return rc;
  irt_context *c = nullptr;
  if ((rc = irt_create_begin(n, device, &c))) {
    synth_close(gen);
    return rc;
  }
  // two pinned chunk buffers: chunk k+1 is synthesised and prepared while chunk k's
  // asynchronous upload runs
  const size_t cap = std::max<size_t>(1, std::min(n, kChunk));
  irt_icon_cell *cb[2] = {nullptr, nullptr};
  float *tb[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  for (int k = 0; k < 2 && !rc; ++k) {
    if (hipHostMalloc((void **)&cb[k], cap * sizeof(irt_icon_cell)) != hipSuccess ||
        hipHostMalloc((void **)&tb[k], cap * 12 * sizeof(float)) != hipSuccess ||
        hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) {
      set_error("irt_create_synth: pinned staging buffers");
      rc = IRT_E_HIP;
    }
  }
  size_t k = 0;
  for (size_t at = 0; at < n && !rc; at += cap, ++k) {
    const int b = (int)(k & 1);
    if (k >= 2 && hipEventSynchronize(ev[b]) != hipSuccess) {
      set_error("irt_create_synth: upload failed");
      rc = IRT_E_HIP;
      break;
    }
    const size_t m = std::min(cap, n - at);
    synth_fill(gen, at, m, cb[b]);
    rc = append_chunk(c, cb[b], m, tb[b]);
    if (!rc && hipEventRecord(ev[b], c->stream) != hipSuccess) rc = IRT_E_HIP;
  }
  if (hipStreamSynchronize(c->stream) != hipSuccess && !rc) {
    set_error("irt_create_synth: upload failed");
    rc = IRT_E_HIP;
  }
  for (int q = 0; q < 2; ++q) {
    if (cb[q]) (void)hipHostFree(cb[q]);
    if (tb[q]) (void)hipHostFree(tb[q]);
    if (ev[q]) (void)hipEventDestroy(ev[q]);
  }
  synth_close(gen);
  if (!rc) rc = irt_create_end(c);
  if (rc) {
    irt_destroy(c);
    return rc;
  }
  *out = c;
  return IRT_OK;
}

void irt_destroy(irt_context *c) {
  if (!c) return;
  if (c->d_probeCounts) (void)hipFree(c->d_probeCounts);
  free_all(c);
  delete c;
}

int irt_get_volume_info(const irt_context *c, irt_volume_info *info) {
  if (!c || !info) {
    set_error("irt_get_volume_info: null argument");
    return IRT_E_INVALID;
  }
  *info = c->info;
  return IRT_OK;
}

int irt_set_transfunc(irt_context *c, const irt_vec4f *lut, int size, irt_box1f valueRange,
                      float opacityScale) {
  if (!c || !lut || size <= 0) {
    set_error("irt_set_transfunc: bad argument");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  // frames still in flight on the caller's stream read the LUT and the majorants: the
  // update is serialized after them, as the reference's TF handler is after its launches
  if (c->launches > 0) {
    const int last = (int)((c->launches - 1) % irt_context::kSlots);
    if (c->pending[last]) IRT_HIP(wait_slot(c, last));
  }
  if (size > c->lutCap) {
    if (c->d_lut) {
      IRT_HIP(hipStreamSynchronize(c->stream));
      IRT_HIP(hipFree(c->d_lut));
      c->bytes -= c->lutCap * sizeof(float4);
      c->d_lut = nullptr;
    }
    int rc = dalloc(c, &c->d_lut, (size_t)size);
    if (rc) return rc;
    c->lutCap = size;
  }
  IRT_HIP(hipMemcpyAsync(c->d_lut, lut, size * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  c->lutSize = size;
  c->tfLo = valueRange.lower;
  c->tfHi = valueRange.upper;
  c->opScale = opacityScale;
  // transfuncUpdateHandler -> computeMaxOpacities (hostCode.cu:878-909); the majorants
  // ignore opacityScale exactly like the reference kernel (hostCode.cu:362-397)
  launch_max_opacities(c->d_valueRanges, c->numMCs, c->d_lut, size, valueRange.lower,
                       valueRange.upper, c->d_maxOp, c->stream);
  if (c->gridBuilt) {  // GRID_ACCEL_MODE's majorants, once its grid exists (ensure_grid)
    launch_max_opacities(c->d_gridVR, (size_t)kGridDim * kGridDim * kGridDim, c->d_lut, size,
                         valueRange.lower, valueRange.upper, c->d_gridMaxOp, c->stream);
    launch_grid_bits(c->d_gridMaxOp, c->d_gridBits, c->stream);
  }
  IRT_HIP(hipGetLastError());
  // a sparse transfer function (many samples per acceptance) on a scene whose table is not used
  // by every launch: the slot table, built on the first such TF (irt_context::slotSparse)
  c->slotSparse = false;
  if (!c->slotAlways && (c->slot.slots || (c->slotLazy && !c->slotTried)) && c->numMCs > 0) {
    if (!c->d_tfStat) {  // once per context (a hipFree per TF change would synchronise the device)
      int rc = dalloc(c, &c->d_tfStat, 2);
      if (rc) return rc;
    }
    double h[2] = {0.0, 0.0};
    IRT_HIP(hipMemsetAsync(c->d_tfStat, 0, 2 * sizeof(double), c->stream));
    launch_accept_stat(c->d_valueRanges, c->d_maxOp, c->numMCs, c->d_lut, size, valueRange.lower,
                       valueRange.upper, c->d_tfStat, c->stream);
    IRT_HIP(hipGetLastError());
    IRT_HIP(hipMemcpyAsync(h, c->d_tfStat, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    IRT_HIP(hipStreamSynchronize(c->stream));
    c->tfSamples = h[1] > 0.0 ? h[0] / h[1] : 0.0;
    if (c->tfSamples >= kSparseTfSamples) {
      if (!c->slot.slots && !c->slotTried) {
        int rc = build_slot_table(c, false);
        if (rc) return rc;
      }
      c->slotSparse = c->slot.slots != nullptr;
    }
  }
  IRT_HIP(hipStreamSynchronize(c->stream));
  c->tfSet = true;
  c->info.deviceBytes = c->bytes;
  return IRT_OK;
}

int irt_clear_frame(irt_context *c, uint32_t *fb, irt_vec4f *accum, size_t n, void *stream) {
  if (!c) {
    set_error("irt_clear_frame: null context");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  launch_clear(fb, (float4 *)accum, n, (hipStream_t)stream);
  IRT_HIP(hipGetLastError());
  return IRT_OK;
}

int irt_render(irt_context *c, const irt_launch_params *lp, int W, int H, uint32_t *fb,
               irt_vec4f *accum, void *stream) {
  return render_impl(c, lp, W, H, 0, 0, 1, fb, accum, nullptr, stream);
}

int irt_render_tiles(irt_context *c, const irt_launch_params *lp, int W, int H, int tileBegin,
                     int tileStride, uint32_t *fb, irt_vec4f *accum, int *numTiles,
                     void *stream) {
  return render_impl(c, lp, W, H, 1, tileBegin, tileStride, fb, accum, numTiles, stream);
}

int irt_render_accumulate(irt_context *c, const irt_launch_params *lp, int W, int H,
                          int numFrames, uint32_t *fb, irt_vec4f *accum, void *stream) {
  return render_impl(c, lp, W, H, 0, 0, 1, fb, accum, nullptr, stream, numFrames);
}

namespace {
// irt_render_sequence and its tile-list form: one chained launch, or one launch per view
int render_sequence(irt_context *c, const irt_launch_params *lps, int numFrames, int W, int H,
                    const int32_t *tiles, int numTiles, uint32_t *fb, irt_vec4f *accum, void *stream) {
  if (!c || !lps || numFrames < 1 || numTiles < 0 || (numTiles > 0 && !tiles)) {
    set_error("irt_render_sequence: bad argument");
    return IRT_E_INVALID;
  }
  // only the camera and accumID may change from frame to frame
  const size_t fixed = offsetof(irt_launch_params, ambientColor);
  for (int k = 1; k < numFrames; ++k)
    if (memcmp((const char *)&lps[k] + fixed, (const char *)&lps[0] + fixed, sizeof(irt_launch_params) - fixed)) {
      set_error("irt_render_sequence: frame %d differs from frame 0 in more than the camera and accumID", k);
      return IRT_E_INVALID;
    }
  const bool chainable = c->chainOn && (c->variant & 65536) == 0 && !c->queueOn && (c->probeExit == 0 || c->probeExit >= 16);
  static const int32_t none = 0;
  const int32_t *list = tiles ? (numTiles > 0 ? tiles : &none) : nullptr;  // null: the whole frame
  const int packed = tiles ? 1 : 0;
  if (numFrames == 1 || !chainable) {  // one launch per frame
    for (int k = 0; k < numFrames; ++k) {
      int rc = render_impl(c, &lps[k], W, H, packed, 0, 1, fb, accum, nullptr, stream, 1, list, numTiles);
      if (rc) return rc;
    }
    return IRT_OK;
  }
  return render_impl(c, &lps[0], W, H, packed, 0, 1, fb, accum, nullptr, stream, numFrames, list, numTiles, lps);
}
}  // namespace

int irt_render_sequence(irt_context *c, const irt_launch_params *lps, int numFrames, int W, int H,
                        uint32_t *fb, irt_vec4f *accum, void *stream) {
  return render_sequence(c, lps, numFrames, W, H, nullptr, 0, fb, accum, stream);
}

int irt_render_tile_list_sequence(irt_context *c, const irt_launch_params *lps, int numFrames, int W, int H,
                                  const int32_t *tiles, int numTiles, uint32_t *fb, irt_vec4f *accum,
                                  void *stream) {
  if (numTiles < 0 || (numTiles > 0 && !tiles)) {
    set_error("irt_render_tile_list_sequence: bad tile list");
    return IRT_E_INVALID;
  }
  static const int32_t none = 0;
  return render_sequence(c, lps, numFrames, W, H, numTiles > 0 ? tiles : &none, numTiles, fb, accum, stream);
}

int irt_render_tiles_accumulate(irt_context *c, const irt_launch_params *lp, int W, int H,
                                int tileBegin, int tileStride, int numFrames, uint32_t *fb,
                                irt_vec4f *accum, int *numTiles, void *stream) {
  return render_impl(c, lp, W, H, 1, tileBegin, tileStride, fb, accum, numTiles, stream, numFrames);
}

int irt_unpack_tiles(irt_context *c, const uint32_t *g, int numRanks, int maxTiles, int W, int H,
                     uint32_t *fb, void *stream) {
  if (!c || !g || !fb || numRanks <= 0 || maxTiles < 0 || W <= 0 || H <= 0) {
    set_error("irt_unpack_tiles: bad argument");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  if (maxTiles > 0) launch_unpack(g, numRanks, maxTiles, W, H, fb, (hipStream_t)stream);
  IRT_HIP(hipGetLastError());
  return IRT_OK;
}

int irt_render_tile_list(irt_context *c, const irt_launch_params *lp, int W, int H,
                         const int32_t *tiles, int numTiles, int numFrames, uint32_t *fb,
                         irt_vec4f *accum, void *stream) {
  if (numTiles < 0 || (numTiles > 0 && !tiles)) {
    set_error("irt_render_tile_list: bad tile list");
    return IRT_E_INVALID;
  }
  static const int32_t none = 0;
  return render_impl(c, lp, W, H, 1, 0, 1, fb, accum, nullptr, stream, numFrames,
                     numTiles > 0 ? tiles : &none, numTiles);
}

int irt_unpack_tile_table(irt_context *c, const uint32_t *g, int numRanks, int maxTiles,
                          const int32_t *table, int W, int H, uint32_t *fb, void *stream) {
  if (!c || !g || !fb || !table || numRanks <= 0 || maxTiles < 0 || W <= 0 || H <= 0) {
    set_error("irt_unpack_tile_table: bad argument");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  if (maxTiles == 0) return IRT_OK;
  const int total = irt_num_tiles(W, H);
  const int32_t *d = nullptr;
  int rc = tile_table(c, table, (size_t)numRanks * (size_t)maxTiles, -1, total, &d);
  if (rc) return rc;
  launch_unpack(g, numRanks, maxTiles, W, H, fb, (hipStream_t)stream, d);
  IRT_HIP(hipGetLastError());
  return IRT_OK;
}

int irt_get_render_stats(const irt_context *cc, irt_render_stats *st) {
  irt_context *c = const_cast<irt_context *>(cc);
  if (!c || !st) {
    set_error("irt_get_render_stats: null argument");
    return IRT_E_INVALID;
  }
  int rc = finish_stats(c);
  if (rc) return rc;
  *st = c->stats;
  return IRT_OK;
}

int irt_get_render_stats_total(const irt_context *cc, irt_render_stats *total, long long *launches) {
  irt_context *c = const_cast<irt_context *>(cc);
  if (!c || !total) {
    set_error("irt_get_render_stats_total: null argument");
    return IRT_E_INVALID;
  }
  int rc = finish_stats(c);
  if (rc) return rc;
  *total = c->total;
  total->kernelMs = c->timedLaunches
                        ? (float)(c->timedMs / (double)c->timedLaunches * (double)c->totalLaunches)
                        : 0.f;
  if (launches) *launches = c->totalLaunches;
  return IRT_OK;
}

int irt_set_timing_interval(irt_context *c, int every) {
  if (!c || every < 1) {
    set_error("irt_set_timing_interval: null context or interval < 1");
    return IRT_E_INVALID;
  }
  c->timingEvery = every;
  return IRT_OK;
}

int irt_reset_render_stats_total(irt_context *c) {
  if (!c) {
    set_error("irt_reset_render_stats_total: null context");
    return IRT_E_INVALID;
  }
  int rc = finish_stats(c);
  if (rc) return rc;
  c->total = irt_render_stats{};
  c->totalLaunches = 0;
  c->timedMs = 0.0;
  c->timedLaunches = 0;
  return IRT_OK;
}

int irt_build_wedge_accel(irt_context *c, const irt_icon_cell *cells, size_t n) {
  if (!c || (n && !cells)) {
    set_error("irt_build_wedge_accel: null argument");
    return IRT_E_INVALID;
  }
  if (n != c->n) {
    set_error("irt_build_wedge_accel: %zu cells, the context has %u", n, c->n);
    return IRT_E_INVALID;
  }
  if (c->wG) return IRT_OK;  // built once per context, like buildCuBQLAccel
  WedgeScene W;
  int rc = build_wedges(cells, n, W);
  if (rc) return rc;
  IRT_HIP(hipSetDevice(c->device));
  if ((rc = upload(c, &c->d_wOff, W.offsets.data(), W.offsets.size())) ||
      (rc = upload(c, &c->d_wRec, W.recs.data(), W.recs.size())) ||
      (rc = upload(c, &c->d_wBox, (const float4 *)W.box.data(), W.box.size() / 4)) ||
      (rc = upload(c, &c->d_wTrig, (const float4 *)W.trig.data(), W.trig.size() / 4)))
    return rc;
  IRT_HIP(hipStreamSynchronize(c->stream));
  c->wG = W.G;
  return IRT_OK;
}

int irt_get_grid(const irt_context *c, float *valueRanges, float *maxOpacities) {
  if (!c) {
    set_error("irt_get_grid: null context");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  // the grid is a cache built on first use: building it changes no observable state
  int rc = ensure_grid(const_cast<irt_context *>(c));
  if (rc) return rc;
  IRT_HIP(hipStreamSynchronize(c->stream));
  const size_t n = (size_t)kGridDim * kGridDim * kGridDim;
  if (valueRanges)
    IRT_HIP(hipMemcpy(valueRanges, c->d_gridVR, 2 * n * sizeof(float), hipMemcpyDeviceToHost));
  if (maxOpacities)
    IRT_HIP(hipMemcpy(maxOpacities, c->d_gridMaxOp, n * sizeof(float), hipMemcpyDeviceToHost));
  return IRT_OK;
}

int irt_get_shell(const irt_context *c, float *valueRanges, float *maxOpacities) {
  if (!c) {
    set_error("irt_get_shell: null context");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  IRT_HIP(hipStreamSynchronize(c->stream));
  if (valueRanges)
    IRT_HIP(hipMemcpy(valueRanges, c->d_valueRanges, 2 * c->numMCs * sizeof(float), hipMemcpyDeviceToHost));
  if (maxOpacities)
    IRT_HIP(hipMemcpy(maxOpacities, c->d_maxOp, c->numMCs * sizeof(float), hipMemcpyDeviceToHost));
  return IRT_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- debug (device math)
namespace {
__global__ void k_debug_math(const float *a, const float *y, const float *x, int n, float *oa,
                             float *ot) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  oa[i] = glibc_asinf(a[i]);
  ot[i] = glibc_atan2f(y[i], x[i]);
}
}  // namespace

extern "C" int irt_debug_device_math(int device, const float *a, const float *y, const float *x,
                                     int n, float *oa, float *ot) {
  if (n <= 0 || !a || !y || !x || !oa || !ot) {
    set_error("irt_debug_device_math: bad argument");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(device));
  float *d = nullptr;
  IRT_HIP(hipMalloc((void **)&d, 5 * (size_t)n * sizeof(float)));
  hipError_t e = hipSuccess;
  e = e == hipSuccess ? hipMemcpy(d, a, n * sizeof(float), hipMemcpyHostToDevice) : e;
  e = e == hipSuccess ? hipMemcpy(d + n, y, n * sizeof(float), hipMemcpyHostToDevice) : e;
  e = e == hipSuccess ? hipMemcpy(d + 2 * (size_t)n, x, n * sizeof(float), hipMemcpyHostToDevice) : e;
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_debug_math, dim3((n + 255) / 256), dim3(256), 0, 0, d, d + n,
                       d + 2 * (size_t)n, n, d + 3 * (size_t)n, d + 4 * (size_t)n);
    e = hipGetLastError();
  }
  e = e == hipSuccess ? hipMemcpy(oa, d + 3 * (size_t)n, n * sizeof(float), hipMemcpyDeviceToHost) : e;
  e = e == hipSuccess ? hipMemcpy(ot, d + 4 * (size_t)n, n * sizeof(float), hipMemcpyDeviceToHost) : e;
  (void)hipFree(d);
  if (e != hipSuccess) {
    set_error("irt_debug_device_math: %s", hipGetErrorString(e));
    return IRT_E_HIP;
  }
  return IRT_OK;
}

namespace {
// Exhaustive error bounds of the certified fast lat/lon (irt_device.h kLatErr / kLonErr),
// as the bit patterns of non-negative doubles (ordered like their values) in out[0..3]:
//   [0] max |fast_asin(x) - glibc_asinf(x)| over every float x in [-1, 1]
//   [1] max |fast_atan(q) - atan(q)|, [2] max |glibc_atanf(q) - atan(q)| over every float q in
//       [0, 2^59] (atan in double)
//   [3] max |rcp(b) b - 1| of the hardware reciprocal over every float b in [2^-100, 2^100]
__device__ __forceinline__ void wave_max_out(unsigned long long *out, double v) {
  unsigned long long b = __double_as_longlong(v);
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(b, off, 64);
    b = o > b ? o : b;
  }
  if (__lane_id() == 0) atomicMax(out, b);
}
__global__ void __launch_bounds__(256) k_fast_math_bounds(unsigned long long *out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
  double m0 = 0.0, m1 = 0.0, m2 = 0.0, m3 = 0.0;
  for (uint32_t u = t; u <= 0x3f800000u; u += stride) {
    const float x = __uint_as_float(u);
    const double a = fabs((double)fast_asin(x) - (double)glibc_asinf(x));
    const double b = fabs((double)fast_asin(-x) - (double)glibc_asinf(-x));
    m0 = fmax(m0, fmax(a, b));
    if (!(a == a) || !(b == b)) m0 = __longlong_as_double(0x7ff8000000000000ll);
  }
  for (uint32_t u = t; u <= 0x5d000000u; u += stride) {
    const float q = __uint_as_float(u);
    const double ref = atan((double)q);
    const double a = fabs((double)fast_atan(q) - ref), b = fabs((double)glibc_atanf(q) - ref);
    m1 = (a == a) ? fmax(m1, a) : __longlong_as_double(0x7ff8000000000000ll);
    m2 = (b == b) ? fmax(m2, b) : __longlong_as_double(0x7ff8000000000000ll);
  }
  for (uint32_t u = 0x0d800000u + t; u <= 0x71800000u; u += stride) {
    const float b = __uint_as_float(u);
    m3 = fmax(m3, fabs((double)__builtin_amdgcn_rcpf(b) * (double)b - 1.0));
  }
  wave_max_out(out + 0, m0);
  wave_max_out(out + 1, m1);
  wave_max_out(out + 2, m2);
  wave_max_out(out + 3, m3);
}
}  // namespace

extern "C" int irt_debug_fast_math_bounds(int device, double *out4) {
  if (!out4) {
    set_error("irt_debug_fast_math_bounds: null argument");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(device));
  unsigned long long *d = nullptr;
  IRT_HIP(hipMalloc((void **)&d, 4 * sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, 4 * sizeof(unsigned long long));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_fast_math_bounds, dim3(8192), dim3(256), 0, 0, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out4, d, 4 * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) {
    set_error("irt_debug_fast_math_bounds: %s", hipGetErrorString(e));
    return IRT_E_HIP;
  }
  return IRT_OK;
}

extern "C" void irt_debug_fast_spherical_consts(float *out2) {
  out2[0] = kLatErr;
  out2[1] = kLonErr;
}

namespace {
__global__ void k_debug_wlog(float *out) {
  __shared__ LogfTab t[16];
  if (threadIdx.x < 16) t[threadIdx.x] = kLogfTab[threadIdx.x];
  __syncthreads();
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  out[j] = woodcock_log(j, t);  // lcg_float uses the low 24 bits only
}
}  // namespace

extern "C" int irt_debug_device_woodcock_log(int device, float *out) {
  if (!out) {
    set_error("irt_debug_device_woodcock_log: null argument");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(device));
  float *d = nullptr;
  const size_t n = (size_t)1 << 24;
  IRT_HIP(hipMalloc((void **)&d, n * sizeof(float)));
  hipLaunchKernelGGL(k_debug_wlog, dim3((unsigned)(n / 256)), dim3(256), 0, 0, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(out, d, n * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) {
    set_error("irt_debug_device_woodcock_log: %s", hipGetErrorString(e));
    return IRT_E_HIP;
  }
  return IRT_OK;
}

namespace {
__global__ void k_debug_srgb(const float *th, const float *x, uint32_t *out, int n) {
  __shared__ float s_th[256];
  s_th[threadIdx.x] = th[threadIdx.x];
  __syncthreads();
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < n) out[j] = srgb_byte(s_th, x[j]);
}
}  // namespace

extern "C" int irt_debug_device_srgb(int device, const float *x, uint32_t *out, int n) {
  if (!x || !out || n < 0) {
    set_error("irt_debug_device_srgb: bad argument");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(device));
  float th[256];
  srgb_thresholds(th);
  float *d = nullptr;
  const size_t m = 256 + 2 * (size_t)n;  // thresholds, x, out
  IRT_HIP(hipMalloc((void **)&d, m * sizeof(float)));
  hipError_t e = hipMemcpy(d, th, sizeof(th), hipMemcpyHostToDevice);
  e = e == hipSuccess ? hipMemcpy(d + 256, x, n * sizeof(float), hipMemcpyHostToDevice) : e;
  if (e == hipSuccess && n > 0) {
    hipLaunchKernelGGL(k_debug_srgb, dim3((n + 255) / 256), dim3(256), 0, 0, d, d + 256,
                       reinterpret_cast<uint32_t *>(d + 256 + n), n);
    e = hipGetLastError();
  }
  e = e == hipSuccess ? hipMemcpy(out, d + 256 + n, n * sizeof(uint32_t), hipMemcpyDeviceToHost) : e;
  (void)hipFree(d);
  if (e != hipSuccess) {
    set_error("irt_debug_device_srgb: %s", hipGetErrorString(e));
    return IRT_E_HIP;
  }
  return IRT_OK;
}

static int debug_locate(irt_context *c, const float *xyz, int n, int *found, float *value, bool wave) {
  if (!c || !xyz || !found || !value || n < 0) {
    set_error("irt_debug_locate: bad argument");
    return IRT_E_INVALID;
  }
  IRT_HIP(hipSetDevice(c->device));
  RenderArgs A;
  memset(&A, 0, sizeof(A));
  A.numCells = c->n;
  A.G = c->G;
  A.binHdr = c->d_binHdr;
  A.fat = c->d_fat;
  A.blocks = c->d_blocks;
  A.slots = c->slot.slots;
  A.slotBins = c->slot.bins;
  A.slotSubs = c->slot.subs;
  for (int k = 0; k < 3; ++k) A.slotEdge[k] = c->slot.edges[k];
  A.numSph = c->numSph;
  A.sphR = c->d_sphR;
  A.sphOff = c->d_sphOff;
  A.sphRec = c->d_sphRec;
  A.sphBits = c->d_sphBits;
  float *d = nullptr;
  IRT_HIP(hipMalloc((void **)&d, (size_t)std::max(n, 1) * 5 * sizeof(float)));
  hipError_t e = hipMemcpy(d, xyz, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice);
  int *dFound = reinterpret_cast<int *>(d + 3 * (size_t)n);
  float *dValue = d + 4 * (size_t)n;
  if (e == hipSuccess) {
    launch_debug_locate(A, d, n, dFound, dValue, 0, wave);
    e = hipGetLastError();
  }
  e = e == hipSuccess ? hipMemcpy(found, dFound, (size_t)n * sizeof(int), hipMemcpyDeviceToHost) : e;
  e = e == hipSuccess ? hipMemcpy(value, dValue, (size_t)n * sizeof(float), hipMemcpyDeviceToHost) : e;
  (void)hipFree(d);
  if (e != hipSuccess) {
    set_error("irt_debug_locate: %s", hipGetErrorString(e));
    return IRT_E_HIP;
  }
  return IRT_OK;
}

extern "C" int irt_debug_locate(irt_context *c, const float *xyz, int n, int *found, float *value) {
  return debug_locate(c, xyz, n, found, value, false);
}

extern "C" int irt_debug_locate_wave(irt_context *c, const float *xyz, int n, int *found, float *value) {
  return debug_locate(c, xyz, n, found, value, true);
}

extern "C" int irt_debug_sched(irt_context *c, int *policy, int *lastApplied, long long *applied) {
  if (!c || !policy || !lastApplied || !applied) {
    set_error("irt_debug_sched: null argument");
    return IRT_E_INVALID;
  }
  *policy = c->schedOn ? c->schedPolicy : 0;
  *lastApplied = c->schedLastApplied ? 1 : 0;
  *applied = c->schedApplied;
  return IRT_OK;
}

extern "C" int irt_debug_counters(irt_context *c, unsigned long long *out16) {
  if (!c || !out16) {
    set_error("irt_debug_counters: null argument");
    return IRT_E_INVALID;
  }
  int rc = finish_stats(c);
  if (rc) return rc;
  memcpy(out16, c->h_last, 16 * sizeof(unsigned long long));
  return IRT_OK;
}

extern "C" int irt_debug_default_variant(void) { return kDefaultVariant; }
// 1 when the context's launches start their candidate scan from the slot table (the OPT_SLOT
// kernels), 0 otherwise; -1 without a context.  *tfSamples (if given): the current transfer
// function's mean Woodcock samples per acceptance (k_accept_stat; 0 when not computed).
extern "C" int irt_debug_slot_use(const irt_context *c, double *tfSamples) {
  if (!c) return -1;
  if (tfSamples) *tfSamples = c->tfSamples;
  return c->slot.slots && (c->slotAlways || c->slotSparse) ? 1 : 0;
}

extern "C" int irt_debug_context_array(const irt_context *c, int which, void *dst, size_t capacity,
                                       size_t *bytes) {
  if (!c || !bytes || c->building) {
    set_error("irt_debug_context_array: null argument or context not built");
    return IRT_E_INVALID;
  }
  const void *src = nullptr;
  size_t n = 0;
  switch (which) {
    case IRT_DEBUG_ARRAY_BIN_HDR: src = c->d_binHdr; n = (size_t)6 * c->G * c->G * kBinHdrWords * 4; break;
    case IRT_DEBUG_ARRAY_FAT: src = c->d_fat; n = c->binEntries * kFatStride4 * 16; break;
    case IRT_DEBUG_ARRAY_BLOCKS: src = c->d_blocks; n = (size_t)c->n * kBlk4 * 16; break;
    case IRT_DEBUG_ARRAY_SPH_R: src = c->d_sphR; n = (size_t)c->numSph * 4; break;
    case IRT_DEBUG_ARRAY_SPH_OFF: src = c->d_sphOff; n = c->numSph ? ((size_t)c->numSph + 1) * 4 : 4; break;
    case IRT_DEBUG_ARRAY_SPH_REC: src = c->d_sphRec; n = (size_t)c->numSphRec * 8; break;
    case IRT_DEBUG_ARRAY_SPH_BITS: src = c->d_sphBits; n = (size_t)kSphBitWords * 4; break;
    case IRT_DEBUG_ARRAY_SLOTS: src = c->slot.slots; n = c->slot.bytes; break;
    default:
      set_error("irt_debug_context_array: unknown array %d", which);
      return IRT_E_INVALID;
  }
  *bytes = n;
  if (dst && capacity >= n && n) {
    IRT_HIP(hipSetDevice(c->device));
    IRT_HIP(hipStreamSynchronize(c->stream));
    IRT_HIP(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
  }
  return IRT_OK;
}

extern "C" int irt_debug_get_variant(const irt_context *c) { return c ? c->variant : -1; }

extern "C" int irt_debug_variants(int *out, int capacity) { return render_variants(out, capacity); }

extern "C" int irt_set_statistics(irt_context *c, int on) {
  if (!c) {
    set_error("irt_set_statistics: null context");
    return IRT_E_INVALID;
  }
  c->statsOff = on == 0;
  return IRT_OK;
}

extern "C" int irt_debug_set_queue(irt_context *c, int on) {
  if (!c) {
    set_error("irt_debug_set_queue: null context");
    return IRT_E_INVALID;
  }
  if (on && !render_queue_compiled()) {
    set_error("irt_debug_set_queue: persistent launches are compiled into the A/B library only "
              "(make VARIANTS=all, libicon_rt_hip_all.so)");
    return IRT_E_INVALID;
  }
  c->queueOn = on != 0;
  return IRT_OK;
}

extern "C" int irt_debug_set_wg_trace(irt_context *c, uint32_t *trace) {
  if (!c) {
    set_error("irt_debug_set_wg_trace: null context");
    return IRT_E_INVALID;
  }
  c->wgTrace = trace;
  return IRT_OK;
}

extern "C" long long irt_debug_launch_workgroups(const irt_context *c, int numTiles, int numFrames) {
  if (!c || numTiles < 0 || numFrames < 1) {
    set_error("irt_debug_launch_workgroups: bad argument");
    return -1;
  }
  RenderArgs A;
  memset(&A, 0, sizeof(A));  // the user-geometry sphere path (sampler 0, accelMode 0)
  const int per = render_wg_per_block(A, c->variant);
  // a single frame in measured-cost order may add its work items (at most kMaxSplit workgroups)
  const size_t extra = c->schedOn && numFrames == 1 && per == 4 ? (size_t)kMaxSplit : 0;
  return (long long)((size_t)numTiles * 16 * per * numFrames + extra);
}

extern "C" int irt_debug_sched_split(const irt_context *c, int *numSplit, int *splitLg) {
  if (!c || !numSplit || !splitLg) {
    set_error("irt_debug_sched_split: null argument");
    return IRT_E_INVALID;
  }
  *numSplit = (int)c->lastNumSplit;
  *splitLg = c->splitLg;
  return IRT_OK;
}

extern "C" int irt_debug_set_chain(irt_context *c, int on) {
  if (!c) {
    set_error("irt_debug_set_chain: null context");
    return IRT_E_INVALID;
  }
  c->chainOn = on != 0;
  return IRT_OK;
}

extern "C" int irt_debug_chain_errors(irt_context *c) {
  if (!c) {
    set_error("irt_debug_chain_errors: null context");
    return -1;
  }
  // retire every launch in flight (each reported hand-off failure is counted, not returned)
  for (long long j = c->launches - irt_context::kSlots; j < c->launches; ++j) {
    if (j < 0) continue;
    const int rc = finish_slot(c, (int)(j % irt_context::kSlots));
    if (rc && rc != IRT_E_CHAIN) return -1;
  }
  return (int)c->chainFailLaunches;
}

extern "C" int irt_debug_set_chain_fault(irt_context *c, uint32_t spins, int withholdFrame) {
  if (!c) {
    set_error("irt_debug_set_chain_fault: null context");
    return IRT_E_INVALID;
  }
  c->chainSpins = spins;
  c->chainWithhold = withholdFrame;
  return IRT_OK;
}

extern "C" int irt_debug_get_queue(const irt_context *c) { return c ? (c->queueOn ? 1 : 0) : -1; }

extern "C" int irt_debug_queue_wgs(const irt_context *c) { return c ? c->lastQueueWG : -1; }

extern "C" int irt_debug_set_variant(irt_context *c, int variant) {
  if (!c || !render_variant_available(variant)) {
    set_error("irt_debug_set_variant: variant %d not compiled", variant);
    return IRT_E_INVALID;
  }
  c->variant = variant;
  return IRT_OK;
}
