// FETCH_SIZE calibration for the render kernel's access shapes (MI355X_MICROARCH.md: "other
// access widths are uncalibrated: calibrate on a known byte count in your own access
// pattern"). Each kernel reads kPieces pieces at pseudo-random, distinct, aligned positions
// of an 8 GiB buffer (far beyond the 256 MiB Infinity Cache, so no piece is re-read from
// a cache): 16 B per lane (one float4), 64 B per lane (4 float4 of one half line) and
// 128 B per lane (8 float4 of one line). Known bytes = pieces x piece size; rocprofv3
// --pmc FETCH_SIZE gives the tally to compare.
//   hipcc --offload-arch=gfx950 -O3 fetch_calibration.hip -o fetch_calibration
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr size_t kBytes = size_t(8) << 30;
constexpr size_t kLines = kBytes / 128;
constexpr int kPieces = 1 << 22;  // 4 M pieces per kernel

__device__ __forceinline__ size_t line_of(uint32_t i, uint32_t salt) {
  // odd multiplier modulo 2^26 lines: a permutation, so pieces never share a line
  return (size_t)(((uint64_t)(i * 2654435761u + salt * 40503u)) & (kLines - 1));
}

template <int kF4>  // float4 loads per lane (1: 16 B, 4: 64 B, 8: 128 B)
__global__ void k_gather(const float4 *buf, float *out, uint32_t salt) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const float4 *p = buf + line_of(i, salt) * 8;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < kF4; ++k) {
    const float4 v = p[k];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[i] = acc;  // keep the loads
}

int main() {
  float4 *buf = nullptr;
  float *out = nullptr;
  if (hipMalloc((void **)&buf, kBytes) != hipSuccess || hipMalloc((void **)&out, kPieces * 4) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  hipMemset(buf, 0, kBytes);
  hipDeviceSynchronize();
  const dim3 g(kPieces / 256), b(256);
  hipLaunchKernelGGL(k_gather<1>, g, b, 0, 0, buf, out, 1u);
  hipLaunchKernelGGL(k_gather<4>, g, b, 0, 0, buf, out, 2u);
  hipLaunchKernelGGL(k_gather<8>, g, b, 0, 0, buf, out, 3u);
  hipDeviceSynchronize();
  printf("{\"pieces\": %d, \"bytes_16\": %llu, \"bytes_64\": %llu, \"bytes_128\": %llu}\n", kPieces,
         (unsigned long long)kPieces * 16, (unsigned long long)kPieces * 64, (unsigned long long)kPieces * 128);
  hipFree(buf);
  hipFree(out);
  return 0;
}
