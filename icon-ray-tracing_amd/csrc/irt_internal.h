// irt_internal.h -- C++ internals shared by the host build (host/*.cpp, g++) and the HIP
// runtime layer (csrc/*.hip, hipcc).  No HIP types here.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "icon_rt_hip.h"
#include "irt_common.h"

namespace irt {

void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();


// The scene build's arrays (irt_build.h), restated on the host: the device build
// (irt_build.hip) produces the same bytes.
struct HostScene {
  size_t n = 0;
  irt_volume_info info{};
  std::vector<float> hv;          // n * kHV floats (see irt_common.h), for host checks
  std::vector<float> trig;        // n * 12: per corner {cosf lat, sinf lat, cosf lon, sinf lon}
  std::vector<float> planes;      // n * 12: the side planes of sample() (ICONGrid.h:197-199)
  std::vector<float> rng;         // n * 2: {height[0], height[numLayers]}
  std::vector<uint32_t> meta;     // n: record_meta (numLayers, coarse flag, quantised keys)
  std::vector<float> blocks;      // n * kBlk4 * 4: height/value blocks
  int G = 0;                      // cube-map cells per face edge
  std::vector<uint32_t> offsets;  // 6*G*G + 1 CSR offsets
  std::vector<uint32_t> entryRec; // candidate lists (each sorted by record index) ...
  std::vector<uint32_t> entrySub; // ... and each entry's sub-cell mask
  // the product locator (irt_build.h)
  std::vector<uint32_t> binHdr;   // 6*G*G * kBinHdrWords
  std::vector<float> fat;         // binEntries * kFatStride4 * 4
  size_t binEntries = 0;
  // zero-thickness records (spheres): distinct radii, CSR into record indices (ascending),
  // and a hash bitmap of the radii (irt_common.h sph_hash) the kernel keeps in LDS
  std::vector<float> sphR;
  std::vector<uint32_t> sphOff, sphRec, sphBits;
};

// Build the binned locator (binHdr, fat) from the CSR lists; build_scene calls it.
int build_bins(HostScene &S, int threads);
// Cube-map resolution for a scene with numRuns columns (IRT_LOCATOR_SCALE / _G override).
int locator_resolution(size_t numRuns);
// Point location over the binned locator, as the kernel does it (host restatement).
// getValue of record rec at radius r along its record_path (the kernel's record_value)
float record_value_host(const HostScene &s, uint32_t rec, uint32_t path, float r);
int locate_bins_host(const HostScene &s, float px, float py, float pz, float &value,
                     uint32_t *record, uint32_t *tested);

// Validate, compute volume facts, per-record planes/heights, and the locator.
int build_scene(const irt_icon_cell *cells, size_t n, HostScene &out, int threads = 0);


// Volume facts only (hostCode.cu:792-808, 838-840).
void compute_volume_info(const irt_icon_cell *cells, size_t n, irt_volume_info &info);
// ... as a fold over records in order, for chunked input: per record the corner trig
// (glibc cosf/sinf) and getBounds (ICONGrid.h:78-115), then volume_acc_add in record order.
struct VolumeAcc {
  float vlo[3], vhi[3], slo[3], shi[3], dlo, dhi;
  size_t n;
};
void corner_trig(const irt_icon_cell &c, float *t12);
void cell_bounds(const irt_icon_cell &c, const float *t12, float lo[3], float hi[3]);
void volume_acc_init(VolumeAcc &a);
void volume_acc_add(VolumeAcc &a, const irt_icon_cell &c, const float blo[3], const float bhi[3]);
void volume_acc_merge(VolumeAcc &a, const VolumeAcc &b);  // a's records, then b's
void volume_acc_finish(const VolumeAcc &a, irt_volume_info &info);

// glibc logf(1 - k/2^24) for k in [0, 2^24): the only arguments woodcockTracking's
// `logf(1.f - rnd())` (deviceCode.cu:165) can ever see.
const std::vector<float> &logf_table();

// th[b] (b = 1..255) = smallest float x with make_8bit(linear_to_srgb(x)) >= b, under the
// host glibc powf (dvr_course-common-both.h:30-35, 89-92); th[0] = -inf.
void srgb_thresholds(float th[256]);

// Host restatement of the scalar reference functions the kernels rely on, for checks.
int sample_host(const HostScene &s, uint32_t rec, float px, float py, float pz, float &value);
// Reference-semantics point location over the locator (host side, for CPU tests).
int locate_host(const HostScene &s, float px, float py, float pz, float &value,
                uint32_t *record);

// The unstructured-element locator of CUBQL_MODE (Params.h:31; deviceCode.cu:90-115) and
// TRIANGLE_MODE (61-76), the replacement of buildCuBQLAccel's cuBQL BVH and
// buildTriangleAccel's OptiX BVH (hostCode.cu:557-649, 440-484): per record the glibc corner
// trig and the union box of its wedges' primBounds and its bottom triangle, and a gnomonic
// cube map listing, per cell, every record whose box can hold a point of that direction
// (sorted by index).
struct WedgeScene {
  int G = 0;
  std::vector<float> trig;       // n * 12: per corner {cosf lat, sinf lat, cosf lon, sinf lon}
  std::vector<float> box;        // n * 8: lo.xyz, numLayers (int bits), hi.xyz, 0
  std::vector<uint32_t> offsets; // 6*G*G + 1
  std::vector<uint32_t> recs;    // record indices
};
int build_wedges(const irt_icon_cell *cells, size_t n, WedgeScene &W, int threads = 0);
// CUBQL_MODE sampleVolume over the wedge locator, as the kernel does it (host check).
bool wedge_locate_host(const WedgeScene &W, const irt_icon_cell *cells, float px, float py,
                       float pz, float &value);
// TRIANGLE_MODE sampleVolume over the same locator, as the kernel does it (host check).
bool triangle_locate_host(const WedgeScene &W, const irt_icon_cell *cells, float px, float py,
                          float pz, float &value, uint32_t *record);

int default_threads();

// Synthetic RnBk grid generator (host/irt_synth.cpp): open once, fill any record range.
int synth_open(int rootN, int bisections, int levels, float topHeight, float noise, uint32_t seed,
               float terrainHeight,
               void **gen, size_t *total);
void synth_fill(const void *gen, size_t first, size_t count, irt_icon_cell *out);
void synth_close(void *gen);

}  // namespace irt
