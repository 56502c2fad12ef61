// irt_multi.cpp -- include/icon_rt_hip_multi.h: one process driving N GPUs, the frame's 64x64
// tiles dealt by cost over the devices and gathered to the first one over RCCL.
//
// The reference has no multi-GPU path; its CPU launch hands 64x64 tiles
// to a thread pool (common/pipeline.cu:1066-1071, common/thread_pool.h:146-161) and its render
// loop is hostCode.cu:931-965.  Per call, on every device i (its own stream):
//   irt_render_tile_list(ctx_i, rank i's row of the deal) -> packed RGBA8 tiles
// then one RCCL group: every device sends its packed tiles to device 0, device 0 receives
// rank-major into one buffer (ncclSend/ncclRecv, rccl.h:700-720, over the single-process
// communicator of ncclCommInitAll, rccl.h:236), and device 0 scatters them into the caller's
// framebuffer (irt_unpack_tile_table) on the caller's stream.  One host thread drives every
// device, so the sends and receives of all communicators are issued inside one
// ncclGroupStart/ncclGroupEnd (RCCL's rule for a thread that owns several ranks).

#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "icon_rt_hip_multi.h"

namespace {

constexpr int kTilePix = 64 * 64;
// rank 0's extra work per frame (the unpack of the whole frame), as a fraction of a frame's
// render cost: the value the Python pipeline uses (icon-ray-tracing_amd/python/irt_dist.py)
constexpr float kUnpackCost = 0.04f;

thread_local std::string g_err;

int fail(int code, const char *what, const char *detail) {
  g_err = std::string(what) + ": " + (detail ? detail : "");
  return code;
}

#define MHIP(x)                                                        \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) return fail(IRT_E_HIP, #x, hipGetErrorString(e_)); \
  } while (0)
#define MNCCL(x)                                                        \
  do {                                                                  \
    ncclResult_t r_ = (x);                                              \
    if (r_ != ncclSuccess) return fail(IRT_E_HIP, #x, ncclGetErrorString(r_)); \
  } while (0)
#define MIRT(x)                                             \
  do {                                                      \
    int rc_ = (x);                                          \
    if (rc_ != IRT_OK) return fail(rc_, #x, irt_last_error()); \
  } while (0)

}  // namespace

struct irt_multi {
  int n = 0;
  std::vector<int> devices;
  std::vector<irt_context *> ctx;
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> stream;
  irt_volume_info info{};
  // the deal of the current accumulation
  int W = 0, H = 0, maxT = 0;
  float camera[12] = {};                // org, dir_00, dir_du, dir_dv the deal was made for
  std::vector<int32_t> table;           // n x maxT, rank-major, -1 padding
  std::vector<std::vector<int32_t>> tiles;  // row i without padding
  size_t cap = 0;                       // tiles the per-device buffers hold
  std::vector<uint32_t *> d_tiles;      // per device: cap x 4096 packed RGBA8
  std::vector<irt_vec4f *> d_acc;       // per device: cap x 4096 accum
  uint32_t *d_gathered = nullptr;       // device 0: n x cap x 4096
  hipEvent_t gathered = nullptr;        // device 0: the group's receives are done
  hipEvent_t unpacked = nullptr;        // device 0: the last unpack has read d_gathered
  bool haveUnpack = false;
};

extern "C" const char *irt_multi_last_error(void) { return g_err.c_str(); }

static void release(irt_multi *m, bool contexts) {
  for (int i = 0; i < m->n; ++i) {
    if (i < (int)m->devices.size()) (void)hipSetDevice(m->devices[i]);
    if (i < (int)m->stream.size() && m->stream[i]) (void)hipStreamSynchronize(m->stream[i]);
    if (i < (int)m->comm.size() && m->comm[i]) (void)ncclCommDestroy(m->comm[i]);
    if (i < (int)m->d_tiles.size() && m->d_tiles[i]) (void)hipFree(m->d_tiles[i]);
    if (i < (int)m->d_acc.size() && m->d_acc[i]) (void)hipFree(m->d_acc[i]);
    if (i == 0) {
      if (m->d_gathered) (void)hipFree(m->d_gathered);
      if (m->gathered) (void)hipEventDestroy(m->gathered);
      if (m->unpacked) (void)hipEventDestroy(m->unpacked);
    }
    if (i < (int)m->stream.size() && m->stream[i]) (void)hipStreamDestroy(m->stream[i]);
    if (contexts && m->ctx[i]) irt_destroy(m->ctx[i]);
  }
  delete m;
}

extern "C" int irt_multi_create(irt_context *const *contexts, const int *devices, int numDevices, irt_multi **out) {
  if (!contexts || !devices || !out || numDevices < 1) return fail(IRT_E_INVALID, "irt_multi_create", "bad argument");
  *out = nullptr;
  for (int i = 0; i < numDevices; ++i)
    if (!contexts[i]) return fail(IRT_E_INVALID, "irt_multi_create", "null context");
  irt_multi *m = new irt_multi;
  m->n = numDevices;
  m->devices.assign(devices, devices + numDevices);
  m->ctx.assign(contexts, contexts + numDevices);
  m->comm.assign(numDevices, nullptr);
  m->stream.assign(numDevices, nullptr);
  m->d_tiles.assign(numDevices, nullptr);
  m->d_acc.assign(numDevices, nullptr);
  int rc = IRT_OK;
  if ((rc = irt_get_volume_info(m->ctx[0], &m->info)) != IRT_OK) {
    fail(rc, "irt_get_volume_info", irt_last_error());
  } else {
    for (int i = 0; i < numDevices && rc == IRT_OK; ++i) {
      hipError_t e = hipSetDevice(devices[i]);
      if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->stream[i], hipStreamNonBlocking);
      if (e == hipSuccess && i == 0) e = hipEventCreateWithFlags(&m->gathered, hipEventDisableTiming);
      if (e == hipSuccess && i == 0) e = hipEventCreateWithFlags(&m->unpacked, hipEventDisableTiming);
      if (e != hipSuccess) rc = fail(IRT_E_HIP, "irt_multi_create: stream", hipGetErrorString(e));
    }
    if (rc == IRT_OK) {
      ncclResult_t r = ncclCommInitAll(m->comm.data(), numDevices, devices);
      if (r != ncclSuccess) {
        m->comm.assign(numDevices, nullptr);
        rc = fail(IRT_E_HIP, "ncclCommInitAll", ncclGetErrorString(r));
      }
    }
  }
  if (rc != IRT_OK) {
    release(m, false);  // the contexts stay the caller's
    return rc;
  }
  *out = m;
  return IRT_OK;
}

extern "C" int irt_multi_create_cells(const irt_icon_cell *cells, size_t numCells, const int *devices,
                                      int numDevices, irt_multi **out) {
  if (!devices || !out || numDevices < 1) return fail(IRT_E_INVALID, "irt_multi_create_cells", "bad argument");
  std::vector<irt_context *> ctx(numDevices, nullptr);
  int rc = IRT_OK;
  for (int i = 0; i < numDevices && rc == IRT_OK; ++i)
    if ((rc = irt_create(cells, numCells, devices[i], &ctx[i])) != IRT_OK) fail(rc, "irt_create", irt_last_error());
  if (rc == IRT_OK) rc = irt_multi_create(ctx.data(), devices, numDevices, out);
  if (rc != IRT_OK)
    for (irt_context *c : ctx)
      if (c) irt_destroy(c);
  return rc;
}

extern "C" void irt_multi_destroy(irt_multi *m) {
  if (m) release(m, true);
}

extern "C" int irt_multi_num_devices(const irt_multi *m) { return m ? m->n : 0; }

extern "C" irt_context *irt_multi_context(const irt_multi *m, int i) {
  return m && i >= 0 && i < m->n ? m->ctx[i] : nullptr;
}

extern "C" int irt_multi_set_transfunc(irt_multi *m, const irt_vec4f *rgbaLUT, int size, irt_box1f valueRange,
                                       float opacityScale) {
  if (!m) return fail(IRT_E_INVALID, "irt_multi_set_transfunc", "null handle");
  for (int i = 0; i < m->n; ++i) MIRT(irt_set_transfunc(m->ctx[i], rgbaLUT, size, valueRange, opacityScale));
  return IRT_OK;
}

// The deal of a new accumulation (irt_deal_tiles: every tile's estimated cost, heaviest first
// to the least-loaded device, device 0 preloaded with its unpack share), the per-device packed
// and accum buffers sized to the longest row, the accum tiles zeroed.
static int deal(irt_multi *m, const irt_launch_params *lp, int W, int H, int numFrames) {
  const float extra = m->n > 1 ? kUnpackCost / (float)numFrames : 0.f;
  int maxT = 0;
  MIRT(irt_deal_tiles(lp, &m->info, W, H, m->n, extra, nullptr, 0, &maxT));
  std::vector<int32_t> table((size_t)m->n * maxT);
  MIRT(irt_deal_tiles(lp, &m->info, W, H, m->n, extra, table.data(), table.size(), &maxT));
  if ((size_t)maxT > m->cap) {
    for (int i = 0; i < m->n; ++i) {
      MHIP(hipSetDevice(m->devices[i]));
      MHIP(hipStreamSynchronize(m->stream[i]));
      if (m->d_tiles[i]) MHIP(hipFree(m->d_tiles[i]));
      if (m->d_acc[i]) MHIP(hipFree(m->d_acc[i]));
      m->d_tiles[i] = nullptr;
      m->d_acc[i] = nullptr;
      MHIP(hipMalloc((void **)&m->d_tiles[i], (size_t)maxT * kTilePix * sizeof(uint32_t)));
      MHIP(hipMalloc((void **)&m->d_acc[i], (size_t)maxT * kTilePix * sizeof(irt_vec4f)));
      if (i == 0) {
        if (m->d_gathered) MHIP(hipFree(m->d_gathered));
        m->d_gathered = nullptr;
        MHIP(hipMalloc((void **)&m->d_gathered, (size_t)m->n * maxT * kTilePix * sizeof(uint32_t)));
      }
    }
    m->cap = (size_t)maxT;
  }
  for (int i = 0; i < m->n; ++i) {
    MHIP(hipSetDevice(m->devices[i]));
    MHIP(hipMemsetAsync(m->d_acc[i], 0, m->cap * kTilePix * sizeof(irt_vec4f), m->stream[i]));
    MHIP(hipMemsetAsync(m->d_tiles[i], 0, m->cap * kTilePix * sizeof(uint32_t), m->stream[i]));
  }
  m->W = W;
  m->H = H;
  m->maxT = maxT;
  memcpy(m->camera, &lp->org, sizeof(m->camera));
  m->table.swap(table);
  m->tiles.assign(m->n, {});
  for (int i = 0; i < m->n; ++i)
    for (int k = 0; k < maxT; ++k)
      if (m->table[(size_t)i * maxT + k] >= 0) m->tiles[i].push_back(m->table[(size_t)i * maxT + k]);
  return IRT_OK;
}

extern "C" int irt_multi_render(irt_multi *m, const irt_launch_params *lp, int width, int height, int numFrames,
                                uint32_t *d_fb, void *stream) {
  if (!m || !lp || !d_fb || width <= 0 || height <= 0 || numFrames < 1)
    return fail(IRT_E_INVALID, "irt_multi_render", "bad argument");
  static_assert(sizeof(irt_vec3f) * 4 == sizeof(float) * 12, "camera layout");
  if (width != m->W || height != m->H || m->table.empty() || memcmp(m->camera, &lp->org, sizeof(m->camera)) != 0) {
    int rc = deal(m, lp, width, height, numFrames);  // a new view: a new deal, accum tiles zeroed
    if (rc) return rc;
  } else if (lp->accumID == 0) {  // a new accumulation of the same view: clearFramebuffer
    for (int i = 0; i < m->n; ++i) {
      MHIP(hipSetDevice(m->devices[i]));
      MHIP(hipMemsetAsync(m->d_acc[i], 0, m->cap * kTilePix * sizeof(irt_vec4f), m->stream[i]));
    }
  }
  const size_t count = (size_t)m->maxT * kTilePix;
  // device 0's receive buffer is read by the previous call's unpack on the caller's stream
  if (m->haveUnpack) {
    MHIP(hipSetDevice(m->devices[0]));
    MHIP(hipStreamWaitEvent(m->stream[0], m->unpacked, 0));
  }
  for (int i = 0; i < m->n; ++i) {
    if (m->tiles[i].empty()) continue;
    MIRT(irt_render_tile_list(m->ctx[i], lp, width, height, m->tiles[i].data(), (int)m->tiles[i].size(), numFrames,
                              m->d_tiles[i], m->d_acc[i], m->stream[i]));
  }
  MNCCL(ncclGroupStart());
  for (int i = 0; i < m->n; ++i) {
    ncclResult_t r = ncclSend(m->d_tiles[i], count, ncclUint32, 0, m->comm[i], m->stream[i]);
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
      return fail(IRT_E_HIP, "ncclSend", ncclGetErrorString(r));
    }
  }
  for (int r = 0; r < m->n; ++r) {
    ncclResult_t e = ncclRecv(m->d_gathered + (size_t)r * count, count, ncclUint32, r, m->comm[0], m->stream[0]);
    if (e != ncclSuccess) {
      (void)ncclGroupEnd();
      return fail(IRT_E_HIP, "ncclRecv", ncclGetErrorString(e));
    }
  }
  MNCCL(ncclGroupEnd());
  hipStream_t s = (hipStream_t)stream;
  MHIP(hipSetDevice(m->devices[0]));
  MHIP(hipEventRecord(m->gathered, m->stream[0]));
  MHIP(hipStreamWaitEvent(s, m->gathered, 0));
  MIRT(irt_unpack_tile_table(m->ctx[0], m->d_gathered, m->n, m->maxT, m->table.data(), width, height, d_fb, stream));
  MHIP(hipEventRecord(m->unpacked, s));
  m->haveUnpack = true;
  return IRT_OK;
}

extern "C" int irt_multi_synchronize(irt_multi *m) {
  if (!m) return fail(IRT_E_INVALID, "irt_multi_synchronize", "null handle");
  for (int i = 0; i < m->n; ++i) {
    MHIP(hipSetDevice(m->devices[i]));
    MHIP(hipStreamSynchronize(m->stream[i]));
  }
  MHIP(hipSetDevice(m->devices[0]));
  if (m->haveUnpack) MHIP(hipEventSynchronize(m->unpacked));
  return IRT_OK;
}
