/*
 * icon_oracle.h -- C API of the CPU ORACLE (test infrastructure only).
 *
 * The oracle is a plain C++ restatement of the reference's CPU render path
 * (szellmann/icon-ray-tracing, `icon_rt` non-RTCORE build).  It exists so that
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg can CHECK the
 * MI355X product; nothing in icon-ray-tracing_amd/ links, loads or calls it.
 *
 * Every function cites the reference file:line it restates.  The oracle uses the
 * host glibc libm exactly where the reference does (asinf, atan2f, sinf, cosf,
 * logf, powf, tanf, atanf, log10f), compiled by g++ with -ffp-contract=off,
 * which is how the reference's CPU build evaluates them.
 */
#ifndef ICON_ORACLE_H
#define ICON_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* icon_rt::ICONCell (icon_rt/ICONGrid.h:59-76): 284 bytes, no padding. */
typedef struct oc_cell {
  float lat[3];
  float lon[3];
  int32_t numLayers;
  float height[32];
  float value[32];
} oc_cell;

typedef struct oc_vec3 { float x, y, z; } oc_vec3;
typedef struct oc_box3 { oc_vec3 lower, upper; } oc_box3;

/* Everything the raygen reads from icon_rt::LaunchParams (icon_rt/Params.h:92-119). */
typedef struct oc_params {
  /* camera (Params.h:100-105) */
  oc_vec3 org, dir_00, dir_du, dir_dv;
  int32_t accumID;                /* Params.h:111 */
  oc_vec3 ambientColor;           /* Params.h:114 */
  float ambientRadiance;          /* Params.h:115 */
  float unitDistance;             /* Params.h:118 */
  int32_t raygen;                 /* 0: woodcockTrackingWithAccel (deviceCode.cu:281), 1: woodcockTrackingAE (deviceCode.cu:239) */
  /* volume (Params.h:51-75) */
  oc_box3 bounds;
  int32_t dims[3];                /* ShellAccel::dims (ShellAccel.h:23) */
  oc_box3 sphericalBounds;        /* ShellAccel::sphericalBounds (ShellAccel.h:24) */
  const float *maxOpacities;      /* ShellAccel::maxOpacities (ShellAccel.h:26) */
  /* transfunc (Params.h:77-82) */
  float tf_lower, tf_upper, opacityScale;
  const float *lut;               /* vec4f[lut_size] as 4*lut_size floats */
  int32_t lut_size;
  /* GRID_ACCEL_MODE (Params.h:34, 44-49): accelMode 1 traverses gridMaxOpacities with
     dda3 (DDA.h:35-136) instead of the shell accelerator with sdda */
  int32_t accelMode;
  int32_t gridDims[3];
  oc_box3 gridBounds;
  const float *gridMaxOpacities;
  /* Volume::mode (Params.h:60): 0 the cell sample() scan (the CPU build, deviceCode.cu:
     116-123), 1 TRIANGLE_MODE (61-76), 2 CUBQL_MODE wedges (90-115) */
  int32_t mode;
} oc_params;

typedef struct oc_stats {
  uint64_t rays_launched;     /* pixels the raygen ran for */
  uint64_t rays_in_box;       /* rays that passed boxTest (deviceCode.cu:294) */
  uint64_t locate_calls;      /* sampleVolume calls (deviceCode.cu:173) outside zero-length sdda leaves */
  uint64_t samples_found;     /* sampleVolume calls that found a cell */
  uint64_t rng_draws;         /* total LCG draws */
  uint64_t leaves;            /* sdda func() invocations (ShellAccel.h:389) */
} oc_stats;

/* ---- host-side setup restated from hostCode.cu main() ---- */

/* lat/lon filter (hostCode.cu:736-758); ranges in degrees, returns kept count,
   compacting cells in place (stable). */
size_t oracle_filter_cells(oc_cell *cells, size_t n, float latLo, float latHi,
                           float lonLo, float lonHi);

/* sphericalBounds, volbounds, dataRange (hostCode.cu:792-808). */
void oracle_compute_bounds(const oc_cell *cells, size_t n, oc_box3 *sphericalBounds,
                           oc_box3 *volbounds, float *dataRange /*[2]*/);

/* unitDistance (hostCode.cu:838-840). */
float oracle_unit_distance(float innerRadius);

/* Default 5-entry LUT (hostCode.cu:828-834); writes 20 floats. */
void oracle_default_lut5(float *out);

/* resampleLUT (common/dvr_course-common.h:44-70); src/dst are vec4f arrays. */
void oracle_resample_lut(const float *src, int nsrc, float *dst, int ndst);

/* Camera (common/camera.h): viewAll (98-104) / setOrientation (34-54) then getScreen (86-96).
   fovy_rad is the camera's stored fovy (radians).  out: org, lower_left, horizontal, vertical. */
void oracle_camera_view_all(oc_box3 box, float fovy_rad, float aspect, oc_vec3 *out4);
void oracle_camera_orient(oc_vec3 vp, oc_vec3 vi, oc_vec3 vu, float fovy_rad, float aspect,
                          oc_vec3 *out4);

/* Shell accelerator build: initGrid + buildShell_ICON (hostCode.cu:216-225, 299-336).
   valueRanges: 2*dims.x*dims.y*dims.z floats (box1f). */
void oracle_build_shell(const oc_cell *cells, size_t n, const int32_t dims[3],
                        oc_box3 sphericalBounds, float *valueRanges);

/* computeMaxOpacities(ShellAccel) (hostCode.cu:362-397). */
/* initGrid(Grid) + buildGrid_ICON + rasterizeBox (hostCode.cu:205-214, 227-297):
   valueRanges = 2*dims^3 floats over worldBounds (the volume bounds). */
void oracle_build_grid(const oc_cell *cells, size_t n, const int32_t dims[3], oc_box3 worldBounds,
                       float *valueRanges);
void oracle_max_opacities(const float *valueRanges, size_t numMCs, const float *lut,
                          int size, float tfLo, float tfHi, float *maxOpacities);

/* clearFramebuffer (common/pipeline.cu:171-199): fb=make_rgba(0)=0, accum=0. */
void oracle_clear(uint32_t *fb, float *accum, size_t numPixels);

/* One frame of the raygen over pixel rectangle [x0,x1)x[y0,y1) of a W x H launch,
   on `nthreads` threads pulling 64x64 tiles from an atomic counter (mirrors
   common/thread_pool.h:129-163 + common/parallel_for.h:62-82).  accum (4*W*H floats)
   and fb (W*H) are read/modified in place.  fast!=0 skips the dead asinf/atan2f of
   toSpherical inside sample() and tests the radius first (identical results); fast==2
   locates samples through the direction-voxel locator (identical results).
   Returns 0 on success. */
int oracle_render(const oc_cell *cells, size_t n, const oc_params *p, int W, int H,
                  int x0, int y0, int x1, int y1, float *accum, uint32_t *fb,
                  int nthreads, int fast, oc_stats *stats);

/* A scene whose locator tables are built once (fast as above; 2 = the direction-voxel
   locator), then frames rendered on it as oracle_render does: the CPU baseline times the
   render only, as the reference's own timer does (pipeline.cu:1062-1073). */
typedef struct oc_scene oc_scene;
oc_scene *oracle_scene_new(const oc_cell *cells, size_t n, int fast, int nthreads);
int oracle_scene_render(oc_scene *s, const oc_params *p, int W, int H, int x0, int y0, int x1,
                        int y1, float *accum, uint32_t *fb, int nthreads, oc_stats *stats);
void oracle_scene_free(oc_scene *s);

/* The same raygen for an explicit list of pixels (xy pairs), scheduled one pixel at a
   time over `nthreads` threads -- used to time a bounded, unbiased sample of a frame
   (bench.py's cpu_baseline).  Writes accum/fb at the pixels' frame positions. */
int oracle_render_pixels(const oc_cell *cells, size_t n, const oc_params *p, int W, int H,
                         const int32_t *xy, int numPixels, float *accum, uint32_t *fb,
                         int nthreads, int fast, oc_stats *stats);
/* Analysis only: each pixel's sample outcomes as letters ('|' a woodcockFunc call, 'm' outside
 * every cell, 'l' located and rejected, 'A' accepted, 'E' past tmax), NUL-terminated at
 * out + i * stride (profiles/sample_pattern.py). */
int oracle_trace_pixels(const oc_cell *cells, size_t n, const oc_params *p, int W, int H,
                        const int32_t *xy, int numPixels, char *out, int stride, int nthreads);
/* Analysis only: the points (xyz) of the traced rays' samples outside every cell. */
long oracle_trace_misses(const oc_cell *cells, size_t n, const oc_params *p, int W, int H,
                         const int32_t *xy, int numPixels, float *out, long cap, int nthreads);

/* ---- known-answer helpers (single functions) ---- */
void oracle_lcg(uint32_t seed0, uint32_t seed1, int n, float *out);            /* dvr_course-common-both.h:41-86 */
int oracle_sample(const oc_cell *cell, oc_vec3 pos, float *value);              /* ICONGrid.h:181-208 */
int oracle_find_height(const oc_cell *cell, float h);                           /* ICONGrid.h:117-145 */
int oracle_intersect_sphere(oc_vec3 org, oc_vec3 dir, float radius, float *tn, float *tf); /* ShellAccel.h:34-53 */
int oracle_box_test(oc_vec3 org, oc_vec3 dir, float tmin, float tmax, oc_box3 box,
                    float *t0, float *t1);                                      /* vecmath.h:1926-1937 */
/* sdda leaf sequence (ShellAccel.h:82-229) with a callback that always continues;
   writes up to maxOut (leaf, t0, t1) triples, returns the number of leaves visited. */
int oracle_sdda_trace(oc_vec3 org, oc_vec3 dir, float tmin, float tmax, const int32_t dims[3],
                      oc_box3 sphericalBounds, int maxOut, int32_t *leaf, float *t0, float *t1);
/* dda3 (DDA.h:35-136) leaf sequence over a dims grid of worldBounds. */
int oracle_dda3_trace(oc_vec3 org, oc_vec3 dir, float tmin, float tmax, const int32_t dims[3],
                      oc_box3 worldBounds, int maxOut, int32_t *leaf, float *t0, float *t1);
/* intersectWedgeEXT (UElems.h:214-311): v24 = 6 vertices as (x,y,z,scalar). */
int oracle_intersect_wedge(const float *v24, oc_vec3 p, float *value);
/* CUBQL_MODE sampleVolume over the wedges of `cells` (hostCode.cu:557-600). */
int oracle_wedge_sample(const oc_cell *cells, size_t n, oc_vec3 p, float *value);
/* TRIANGLE_MODE sampleVolume over the cells' bottom triangles (deviceCode.cu:61-76). */
int oracle_triangle_sample(const oc_cell *cells, size_t n, oc_vec3 p, float *value);
float oracle_linear_to_srgb(float x);                                          /* dvr_course-common-both.h:30-35 */
uint32_t oracle_make_rgba(const float *rgba4);                                 /* dvr_course-common-both.h:103-110 */
void oracle_to_spherical(oc_vec3 c, oc_vec3 *out);                             /* ICONGrid.h:36-42 */
void oracle_to_cartesian(oc_vec3 s, oc_vec3 *out);                             /* ICONGrid.h:44-54 */
void oracle_get_bounds(const oc_cell *cell, oc_box3 *out);                     /* ICONGrid.h:78-115 */
/* postClassify (deviceCode.cu:127-135) */
void oracle_post_classify(const float *lut, int size, float lo, float hi, float opacityScale,
                          float v, float *out4);

#ifdef __cplusplus
}
#endif
#endif
