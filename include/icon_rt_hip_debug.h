/*
 * icon_rt_hip_debug.h -- host-only inspection entry points of libicon_rt_hip.so, used by
 * the CPU test-suite to check the pieces the kernels are built from without a GPU.
 * Not part of the drop-in boundary (include/icon_rt_hip.h is).
 */
#ifndef ICON_RT_HIP_DEBUG_H
#define ICON_RT_HIP_DEBUG_H

#include "icon_rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The glibc-exact single-precision restatements the kernels use (csrc/irt_common.h),
 * compiled for the host. */
float irt_debug_asinf(float x);
float irt_debug_atan2f(float y, float x);
/* x86 cvttss2si float->int semantics used by the kernels. */
int irt_debug_f2i(float x);
/* n LCG steps as one affine map, state_n = mul * state + add (mod 2^32), n < 256: the jump
 * table of the cooperative Woodcock loop (irt_common.h lcg_jump). */
void irt_debug_lcg_jump(uint32_t n, uint32_t *mul, uint32_t *add);

/* Host-built tables uploaded to HBM: logf(1 - k/2^24) and the sRGB byte thresholds. */
float irt_debug_logf_entry(uint32_t k);
void irt_debug_srgb_thresholds(float *out256);

/* Number of j in [0, 2^24) where the restated glibc logf (irt_common.h) differs from the
 * host glibc logf at 1 - j/2^24, the only arguments logf(1.f - rnd()) can take. */
uint32_t irt_debug_logf_mismatches(void);
/* The host glibc logf(1 - j/2^24) for every j (out: 2^24 floats). */
void irt_debug_host_woodcock_log(float *out);

/* The locator built by irt_create, on the host: build, query, free. */
typedef struct irt_debug_scene irt_debug_scene;
int irt_debug_scene_build(const irt_icon_cell *cells, size_t n, irt_debug_scene **out);
int irt_debug_scene_info(const irt_debug_scene *s, irt_volume_info *info);
/* Reference-semantics sampleVolume (deviceCode.cu:58-125): returns 1 and the value and
 * record of the lowest-index cell containing p, 0 if none. */
int irt_debug_scene_locate(const irt_debug_scene *s, irt_vec3f p, float *value,
                           uint32_t *record);
/* The same query through the binned locator the render kernel uses (radial bins of fat
 * entries and sub-cell masks, irt_build.h); *tested = candidate entries examined. */
int irt_debug_scene_locate_binned(const irt_debug_scene *s, irt_vec3f p, float *value,
                                  uint32_t *record, uint32_t *tested);
/* findHeight + value of record `rec` at radius r two ways: out2[0] from the literal
 * binary search (ICONGrid.h:117-164), out2[1] the way the render kernel reads it (coarse
 * keys + one 64-B block of the height/value blocks, irt_common.h).  Bit for bit equal. */
int irt_debug_scene_values(const irt_debug_scene *s, uint32_t rec, float r, float *out2);
/* Candidate list of the cube-map cell containing direction p. */
int irt_debug_scene_candidates(const irt_debug_scene *s, irt_vec3f p, uint32_t *records,
                               int capacity);
/* Per-record side planes (3 x vec4) as uploaded. */
int irt_debug_scene_planes(const irt_debug_scene *s, uint32_t record, float *out12);
void irt_debug_scene_free(irt_debug_scene *s);
/* CUBQL_MODE (deviceCode.cu:90-115): build the wedge locator irt_build_wedge_accel
 * uploads, then sampleVolume through it as the kernel does (first wedge in index order
 * whose primBounds contain p and whose intersectWedgeEXT accepts it). */
int irt_debug_scene_build_wedges(irt_debug_scene *s, const irt_icon_cell *cells, size_t n);
int irt_debug_scene_locate_wedge(irt_debug_scene *s, irt_vec3f p, float *value);
/* TRIANGLE_MODE sampleVolume (deviceCode.cu:61-76) through the same locator, as the kernel
 * does it; *record = the hit cell. */
int irt_debug_scene_locate_triangle(irt_debug_scene *s, irt_vec3f p, float *value,
                                    uint32_t *record);
/* intersectWedgeEXT (UElems.h:214-311) as the kernel evaluates it; v24 = 6 x (xyz, scalar). */
int irt_debug_intersect_wedge(const float *v24, irt_vec3f p, float *value);

/* The scene arrays the render kernel reads, byte for byte: from a context (the device
 * build, csrc/irt_build.hip; waits for it) or from the host restatement of the build
 * (host/irt_scene.cpp).  which: IRT_DEBUG_ARRAY_*.  With dst null (or capacity too small)
 * only *bytes is set. */
enum {
  IRT_DEBUG_ARRAY_BIN_HDR = 0,  /* cube-map cell headers, kBinHdrWords u32 each */
  IRT_DEBUG_ARRAY_FAT = 1,      /* fat candidate entries, 64 B each */
  IRT_DEBUG_ARRAY_BLOCKS = 2,   /* per-record height/value blocks, 256 B each */
  IRT_DEBUG_ARRAY_SPH_R = 3,    /* sphere radii (f32) */
  IRT_DEBUG_ARRAY_SPH_OFF = 4,  /* CSR offsets (u32) */
  IRT_DEBUG_ARRAY_SPH_REC = 5,  /* (record, numLayers) u32 pairs */
  IRT_DEBUG_ARRAY_SPH_BITS = 6, /* radius hash bitmap (u32) */
  IRT_DEBUG_ARRAY_SLOTS = 7     /* the slot table (irt_common.h kSlot4), 128 B per (cell, sub-cell,
                                   bin); 0 bytes when the scene has none (context only) */
};
int irt_debug_context_array(const irt_context *ctx, int which, void *dst, size_t capacity,
                            size_t *bytes);
int irt_debug_scene_array(const irt_debug_scene *s, int which, void *dst, size_t capacity,
                          size_t *bytes);

/* Select the render-kernel variant (bit set of irt_render.hip's OPT_* flags; every
 * variant gives identical results -- used for in-process A/B timing). */
int irt_debug_set_variant(irt_context *ctx, int variant);
/* The variant a new context launches (IRT_RENDER_VARIANT overrides it per context). */
int irt_debug_default_variant(void);
/* 1 when the context's launches start their candidate scan from the slot table (the OPT_SLOT
 * kernels: every launch on scenes whose headers outgrow the last-level cache or with IRT_SLOTS=1;
 * otherwise while a sparse transfer function is set), 0 otherwise, -1 without a context.
 * *tfSamples (if not null): the transfer function's mean Woodcock samples per acceptance over the
 * shell's macrocells, the measure of "sparse" (>= 8; 0 when it was not computed). */
int irt_debug_slot_use(const irt_context *ctx, double *tfSamples);
/* The variant this context launches: the default on scenes with holes (columns starting at
 * different radii, as convert_icon's terrain does, or gaps inside columns: the raygen's miss
 * mode), the default | 262144 (no miss mode) on scenes without, unless IRT_RENDER_VARIANT or
 * irt_debug_set_variant chose another; -1 for NULL. */
int irt_debug_get_variant(const irt_context *ctx);
/* The variants this build compiled: returns their count and writes the first `capacity` of
 * them to `out` (may be NULL).  The product build has the default and the statistics
 * variant; `make VARIANTS=all` (libicon_rt_hip_all.so) adds the A/B variants. */
int irt_debug_variants(int *out, int capacity);
/* Persistent launches on or off for this context (IRT_QUEUE sets the default): every
 * resident wave pulls 8x8-pixel packets from a per-launch counter (RenderArgs::queue) instead
 * of one workgroup per 16x16 block.  Frames are identical either way.  Only the A/B library
 * (make VARIANTS=all) compiles the persistent kernels: the product library refuses on = 1
 * (IRT_E_INVALID).  get: 1/0, -1 for NULL. */
int irt_debug_set_queue(irt_context *ctx, int on);
int irt_debug_get_queue(const irt_context *ctx);
/* Workgroups of this context's last persistent launch (0 if none yet; -1 for NULL):
 * every CU's resident share by the kernel's occupancy, or IRT_QUEUE_WGS per CU. */
int irt_debug_queue_wgs(const irt_context *ctx);
/* The raw per-frame counters of the last render (waits for it): [0] launched [1] in box
 * [2] sampleVolume calls [3] found [4] candidates; with the statistics variant bit also
 * [5] Woodcock draws [6] sum over waves of the per-wave max draws [7] zero-length leaves
 * [8] sum over waves of the per-wave max zero-length leaves [9] rays reaching range 1. */
int irt_debug_counters(irt_context *ctx, unsigned long long *out16);

/* Evaluate the kernels' device versions of asinf(a[i]) and atan2f(y[i], x[i]) on GPU
 * `device` (host arrays in/out; n elements each).  Used to prove the device restatements
 * round exactly like the host glibc. */
int irt_debug_device_math(int device, const float *a, const float *y, const float *x, int n,
                          float *out_asinf, float *out_atan2f);
/* Exhaustive device error bounds of the certified fast lat/lon (irt_device.h), into out4:
 * [0] max |fast_asin(x) - glibc asinf(x)| over every float in [-1, 1]; [1] / [2] max
 * |fast_atan(q) - atan(q)| / |glibc atanf(q) - atan(q)| over every float q in [0, 2^59];
 * [3] max relative error of the hardware reciprocal over every float in [2^-100, 2^100]. */
int irt_debug_fast_math_bounds(int device, double *out4);
/* The bounds the kernel assumes: out2 = {kLatErr, kLonErr}. */
void irt_debug_fast_spherical_consts(float *out2);
/* The device logf(1.f - rnd()) for every LCG low-24-bit value j (out: 2^24 floats, index j). */
int irt_debug_device_woodcock_log(int device, float *out);
/* The kernels' make_8bit(linear_to_srgb(x[i])) (csrc/irt_device.h srgb_byte) for n host
 * values on GPU `device`; out: n bytes widened to uint32. */
int irt_debug_device_srgb(int device, const float *x, uint32_t *out, int n);
/* The render kernel's point location (sampleVolume over the context's binned lists,
 * csrc/irt_render.hip Tracer::locate) for n points xyz[3i..3i+2]: found[i] 0/1, value[i]. */
int irt_debug_locate(irt_context *ctx, const float *xyz, int n, int *found, float *value);
/* The same through the cooperative kernel's wave-wide candidate scan (Tracer::locate_wave):
 * the first candidates tested per lane, the rest dealt out over the wave, the second pass
 * for points exactly on a radial bin edge.  Must equal irt_debug_locate point for point. */
int irt_debug_locate_wave(irt_context *ctx, const float *xyz, int n, int *found, float *value);
/* Measured-cost scheduling state: the policy (IRT_SCHED; 0 = off), whether the last launch
 * ran its workgroups in a measured-cost order, and how many launches have. */
int irt_debug_sched(irt_context *ctx, int *policy, int *lastApplied, long long *applied);
/* Measurement only: the next renders' workgroups each write 4 words to the device buffer
 * `trace` (NULL: off): {start, end} of the workgroup (s_memrealtime, 100 MHz, low 32 bits),
 * the wave's HW_ID and XCC_ID registers; workgroup b of a launch at trace[4b].  The buffer
 * must hold 4 words per workgroup of the launch: irt_debug_launch_workgroups gives the count
 * (the default variant's one-wave workgroups: 64 per 64x64 tile and frame); frames are
 * unchanged. */
int irt_debug_set_wg_trace(irt_context *ctx, uint32_t *trace);
/* Workgroups one launch of numTiles 64x64 tiles x numFrames frames runs with this context's
 * variant and settings, at most (the size irt_debug_set_wg_trace's buffer needs, in units of 4
 * words; with measured-cost scheduling a single frame adds up to 4096 workgroups for its work
 * items, which come first; rows a launch does not use stay as they were). */
long long irt_debug_launch_workgroups(const irt_context *ctx, int numTiles, int numFrames);
/* Measured-cost scheduling (IRT_SCHED; on by default for scenes with holes): the last launch's
 * split WORK ITEMS in *numSplit -- every split packet (one longer than IRT_SPLIT_FACTOR (0.35 with holes, else 1) x
 * the frame's ideal span, the packets' durations over the resident slots) is rendered first in
 * 2^splitLg parts of 64 >> splitLg rays (IRT_SPLIT_LG, default 2; 0: no splits), one work item
 * per part, and the items are padded with empty ones to a multiple of 8 (so *numSplit is parts x
 * packets rounded up, not the packet count) -- and splitLg.  Frames are unchanged. */
int irt_debug_sched_split(const irt_context *ctx, int *numSplit, int *splitLg);
/* Chained progressive frames on (default; IRT_CHAIN=0 turns it off per context) or off: a
 * launch of several frames (irt_render_accumulate, irt_render_tiles_accumulate,
 * irt_render_tile_list) lerps each frame straight into accum/fb, frame f's workgroup waiting for
 * frame f - 1's to publish the same pixels; off: every frame's colour goes to a sample buffer
 * and a second kernel runs the lerp chain.  Frames are identical either way. */
int irt_debug_set_chain(irt_context *ctx, int on);
/* Launches whose chained-frame waits timed out since the context was created (a wait gives up
 * after 2^20 polls, about a second); retires every launch in flight first (waits for them),
 * counting -- not returning -- their IRT_E_CHAIN.  0 in every correct run; -1 on error. */
int irt_debug_chain_errors(irt_context *ctx);
/* Test hook for the failure path: chained waits give up after `spins` polls (0: the default),
 * and the waves of frame `withholdFrame` of every chained launch (-1: none) never publish, so
 * frame withholdFrame + 1's waves time out. */
int irt_debug_set_chain_fault(irt_context *ctx, uint32_t spins, int withholdFrame);

#ifdef __cplusplus
}
#endif
#endif
