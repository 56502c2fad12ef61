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
  float3 amb;
  float ambRad;
  float unitDistance;
  int raygen;
  // volume (Params.h:62-74)
  float3 bmin, bmax;     // Volume::bounds
  int3 dims;             // ShellAccel::dims
  float3 sbLo, sbHi;     // ShellAccel::sphericalBounds
  const float *maxOp;    // ShellAccel::maxOpacities
  // transfer function (Params.h:77-82)
  float tfLo, tfHi, opacityScale;
  const float4 *lut;
  int lutSize;
  // locator + records
  uint32_t numCells;
  int G;
  const uint32_t *offsets;
  const uint4 *entries;
  const float4 *planes;
  const float *hv;
  // libm tables
  const float *logtab;   // 2^24 entries
  const float *srgbTh;   // 256 entries
  // output
  int W, H;
  uint32_t *fb;
  float4 *accum;
  int packed;            // 0: linear x + W*y; 1: packed 64x64 tiles
  int tileBegin, tileStride, numTiles, tilesX;
  unsigned long long *counters;  // [0] launched [1] inBox [2] locate [3] found [4] candidates
  // The render arena (irt_trace.hip): one allocation holding every table the raygen
  // gathers from, addressed by 32-bit float4 indices so a gather step is 4 loads off one
  // base.  Offsets (in float4) of the sub-tables:
  const float4 *arena;
  uint32_t aMaxOp;       // ShellAccel::maxOpacities, numMCs floats
  uint32_t aLog;         // logf table, 2^24 floats
  uint32_t aOffs;        // cube-map CSR offsets, 6G^2+1 uint32
  uint32_t aEnt;         // LocEntry, one float4 each
  uint32_t aRec;         // render records, kRec4 float4 each (irt_common.h)
};

// Render-kernel variants.  Bit 12 selects the state-machine raygen (irt_trace.hip,
// bits 8-11 = minimum waves per SIMD); otherwise the bit set of irt_render.hip's OPT_*
// flags.  All give identical results.
constexpr int kTraceBit = 4096;
constexpr int kDefaultVariant = 9728;  // k_render<OPT_REC, 6 waves/SIMD>: fastest measured (profiles/)
bool trace_variant_available(int variant);
void launch_trace(const RenderArgs &A, int numBlocks, hipStream_t s, int variant);
bool render_variant_available(int variant);
void launch_render(const RenderArgs &A, int numBlocks, hipStream_t s, int variant);
void launch_shell_init(float *valueRanges, size_t numMCs, hipStream_t s);
void launch_shell_build(const irt_icon_cell *cells, size_t n, int3 dims, float3 lo, float3 hi,
                        float *valueRanges, hipStream_t s);
void launch_max_opacities(const float *valueRanges, size_t numMCs, const float4 *lut, int size,
                          float lo, float hi, float *maxOp, hipStream_t s);
void launch_clear(uint32_t *fb, float4 *accum, size_t n, hipStream_t s);
void launch_unpack(const uint32_t *gathered, int numRanks, int maxTiles, int W, int H,
                   uint32_t *fb, hipStream_t s);

}  // namespace irt
