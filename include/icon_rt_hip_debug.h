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

/* Host-built tables uploaded to HBM: logf(1 - k/2^24) and the sRGB byte thresholds. */
float irt_debug_logf_entry(uint32_t k);
void irt_debug_srgb_thresholds(float *out256);

/* The locator built by irt_create, on the host: build, query, free. */
typedef struct irt_debug_scene irt_debug_scene;
int irt_debug_scene_build(const irt_icon_cell *cells, size_t n, irt_debug_scene **out);
int irt_debug_scene_info(const irt_debug_scene *s, irt_volume_info *info);
/* Reference-semantics sampleVolume (deviceCode.cu:58-125): returns 1 and the value and
 * record of the lowest-index cell containing p, 0 if none. */
int irt_debug_scene_locate(const irt_debug_scene *s, irt_vec3f p, float *value,
                           uint32_t *record);
/* Candidate list of the cube-map cell containing direction p. */
int irt_debug_scene_candidates(const irt_debug_scene *s, irt_vec3f p, uint32_t *records,
                               int capacity);
/* Per-record side planes (3 x vec4) as uploaded. */
int irt_debug_scene_planes(const irt_debug_scene *s, uint32_t record, float *out12);
void irt_debug_scene_free(irt_debug_scene *s);

/* Evaluate the kernels' device versions of asinf(a[i]), atan2f(y[i], x[i]) and the
 * LCG draw sequence on GPU `device` (host arrays in/out; n elements each).  Used to prove
 * the device restatements round exactly like the host glibc. */
int irt_debug_device_math(int device, const float *a, const float *y, const float *x, int n,
                          float *out_asinf, float *out_atan2f);

#ifdef __cplusplus
}
#endif
#endif
