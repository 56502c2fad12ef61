// profiles/calib/gather_rate.hip -- what dependent random line reads cost on one MI355X.
//
// k_render's samples are chains of dependent 128-B gathers (cell header -> candidate entry ->
// value block).  This microbenchmark prices that pattern alone: `lanes` lanes (k_render's
// frame: 1024^2 lanes in 256-thread workgroups), each starting at a hashed line of a buffer
// and reading D lines, each line's address taken from the 16 bytes the previous read returned
// ("chain"), or D lines at hashed addresses issued together ("indep", the same line count with
// full memory-level parallelism).  Dynamic LDS pins the occupancy (4 or 8 waves per SIMD;
// k_render runs at 4).  Working sets: 4 GiB (HBM), 192 MiB (fits the 256 MB MALL), 24 MiB.
//
// Output: one JSON line per case: microseconds per launch (HIP events, average of 20 launches
// after 3 warmups), lines per second and the equivalent 128-B bandwidth.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// every line's first 16 bytes: the next line index (hashed), so a chain is a random walk
__global__ void k_init(uint4 *buf, uint32_t lines, uint32_t salt) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += gridDim.x * blockDim.x)
    buf[(size_t)i * 8] = make_uint4(mix(i ^ salt) % lines, i, 0u, 0u);
}

template <int D>
__global__ __launch_bounds__(256) void k_chain(const uint4 *__restrict__ buf, uint32_t lines,
                                               uint32_t *out, uint32_t salt) {
  extern __shared__ uint32_t pad[];
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  uint32_t idx = mix(gid * 2654435761u ^ salt) % lines, acc = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const uint4 v = buf[(size_t)idx * 8];
    acc += v.y;
    idx = v.x;
  }
  if (acc == 0xFFFFFFFFu) pad[threadIdx.x] = acc, out[gid] = pad[threadIdx.x ^ 1];
}

template <int D>
__global__ __launch_bounds__(256) void k_indep(const uint4 *__restrict__ buf, uint32_t lines,
                                               uint32_t *out, uint32_t salt) {
  extern __shared__ uint32_t pad[];
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  uint4 v[D];
#pragma unroll
  for (int d = 0; d < D; ++d)
    v[d] = buf[(size_t)(mix((gid * D + d) ^ salt) % lines) * 8];
  uint32_t acc = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) acc += v[d].y;
  if (acc == 0xFFFFFFFFu) pad[threadIdx.x] = acc, out[gid] = pad[threadIdx.x ^ 1];
}

typedef void (*Kern)(const uint4 *, uint32_t, uint32_t *, uint32_t);

int main() {
  const size_t bytes = 4ull << 30;
  const uint32_t maxLines = (uint32_t)(bytes / 128);
  uint4 *buf;
  uint32_t *out;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, 64u << 20));
  hipLaunchKernelGGL(k_init, dim3(8192), dim3(256), 0, 0, buf, maxLines, 12345u);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  struct Case { const char *name; Kern k; int D; };
  const Case cases[] = {{"chain", k_chain<1>, 1}, {"chain", k_chain<3>, 3}, {"chain", k_chain<6>, 6},
                        {"indep", k_indep<3>, 3}, {"indep", k_indep<6>, 6}};
  const uint32_t workingSets[] = {maxLines, (192u << 20) / 128, (24u << 20) / 128};
  const int wavesPerSimd[] = {4, 8};
  const uint32_t lanesList[] = {1u << 20, 4u << 20};
  for (uint32_t lines : workingSets) {
    // the k_init walk stays inside the first `lines` lines only for the full buffer; re-seed
    hipLaunchKernelGGL(k_init, dim3(8192), dim3(256), 0, 0, buf, lines, 777u);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    for (const Case &c : cases)
      for (int w : wavesPerSimd)
        for (uint32_t lanes : lanesList) {
          // 160 KB of LDS per CU: w waves per SIMD = w workgroups of 4 waves per CU
          const size_t lds = (160u * 1024u) / w - 1024;
          CHECK(hipFuncSetAttribute((const void *)c.k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
          const dim3 grid(lanes / 256);
          for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(c.k, grid, dim3(256), lds, 0, buf, lines, out, (uint32_t)i);
          CHECK(hipGetLastError());
          CHECK(hipEventRecord(e0, 0));
          const int reps = 20;
          for (int i = 0; i < reps; ++i)
            hipLaunchKernelGGL(c.k, grid, dim3(256), lds, 0, buf, lines, out, (uint32_t)(100 + i));
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          float ms = 0.f;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          const double us = ms * 1e3 / reps;
          const double linesPerS = (double)lanes * c.D / (us * 1e-6);
          printf("{\"kind\": \"%s\", \"D\": %d, \"working_set_MiB\": %.0f, \"waves_per_simd\": %d, "
                 "\"lanes\": %u, \"us\": %.2f, \"Glines_per_s\": %.2f, \"GBps_128B\": %.0f}\n",
                 c.name, c.D, lines * 128.0 / (1 << 20), w, lanes, us, linesPerS / 1e9,
                 linesPerS * 128 / 1e9);
          fflush(stdout);
        }
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
