/*
 * icon_rt_hip.h -- C ABI of the MI355X-native ICON volume renderer.
 *
 * Drop-in boundary for the hot path of szellmann/icon-ray-tracing `icon_rt`:
 * the reference renders one frame with
 *     SET_LAUNCH_PARAMS(parms); pl.launch();            (icon_rt/hostCode.cu:961-963)
 * which runs the raygen `woodcockTrackingWithAccel` (icon_rt/deviceCode.cu:281-341)
 * once per pixel -- on the CPU through parallel::for_each (common/pipeline.cu:1066-1071),
 * on NVIDIA through owlLaunch2D (common/pipeline.cu:1064).  This library replaces that
 * launch (and the accelerator builds that feed it) with hand-written HIP kernels for
 * gfx950.  Plain C types, plain pointers and sizes; no C++ or torch types.
 *
 * Conventions
 *  - Every function returns IRT_OK (0) or a negative IRT_E_* code; irt_last_error()
 *    returns a thread-local message for the last failure.  (The reference prints and
 *    continues or abort()s; pipeline.cu:992-995, hostCode.cu:19-34.)
 *  - Input arrays are copied; the context never retains caller pointers beyond a call
 *    (the reference's LaunchParams borrow pointers owned by Buffer/Frame/Transfunc).
 *  - Framebuffer pointers passed to irt_render* are DEVICE pointers on the context's
 *    device (HBM-resident, as the reference's fbPointer/accumBuffer in RTCORE builds).
 *  - `stream` is a hipStream_t passed as void*; NULL is HIP's null (legacy default) stream,
 *    so work launched there is ordered with every blocking stream of the process (torch's
 *    default stream included).
 *  - A context is single-caller.  Multi-GPU = one process (one context) per GPU.
 *  - Launches of one context execute in call order, whatever streams they are given: a call
 *    on another stream than the previous call's makes its stream wait for the previous launch
 *    first (the reference has one launch stream per pipeline, pipeline.cu:1064).
 */
#ifndef ICON_RT_HIP_H
#define ICON_RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IRT_OK 0
#define IRT_E_INVALID (-1)   /* bad argument */
#define IRT_E_HIP (-2)       /* HIP runtime error (no device, OOM, launch failure) */
#define IRT_E_DATA (-3)      /* unusable cell data (numLayers out of [0,31], non-finite) */
#define IRT_E_IO (-4)        /* file I/O */
#define IRT_E_CHAIN (-5)     /* a chained multi-frame launch's per-pixel hand-off timed out: that
                                launch's frames were lerped out of order (see
                                irt_render_accumulate) */

/* == icon_rt::ICONCell (icon_rt/ICONGrid.h:59-76); 284 bytes; the `.ic` record. */
typedef struct irt_icon_cell {
  float lat[3];        /* radians, per triangle corner, ccw */
  float lon[3];        /* radians */
  int32_t numLayers;   /* <= 31 (MAX_LAYERS 32, ICONGrid.h:57) */
  float height[32];    /* metres from the Earth centre, [0:numLayers] used */
  float value[32];     /* per layer, [0:numLayers) used */
} irt_icon_cell;

typedef struct irt_vec3f { float x, y, z; } irt_vec3f;
typedef struct irt_vec4f { float x, y, z, w; } irt_vec4f;
typedef struct irt_box1f { float lower, upper; } irt_box1f;
typedef struct irt_box3f { irt_vec3f lower, upper; } irt_box3f;

/* Raygen selector == Pipeline::setRayGen(...) choice (hostCode.cu:138-149, 863). */
#define IRT_RAYGEN_WITH_ACCEL 0 /* woodcockTrackingWithAccel, deviceCode.cu:281-341 */
#define IRT_RAYGEN_AE 1         /* woodcockTrackingAE, deviceCode.cu:239-275 */
#define IRT_ACCEL_SPHERE 0      /* SPHERE_ACCEL_MODE (Params.h:33): sdda, ShellAccel.h:82-229 */
#define IRT_ACCEL_GRID 1        /* GRID_ACCEL_MODE (Params.h:34): dda3, DDA.h:35-136 */
/* Sampler == Volume::mode (Params.h:29-31, 60; the -mode flag, hostCode.cu:125-127). */
#define IRT_MODE_USER_GEOM 0    /* sample() on the cells (ICONGrid.h:181-208): the CPU build's
                                   scan (deviceCode.cu:116-123), lowest index wins */
#define IRT_MODE_TRIANGLES 1    /* the OptiX triangle trace (deviceCode.cu:61-76): closest
                                   bottom triangle toward the Earth's centre (needs
                                   irt_build_wedge_accel); OptiX's own intersection test is
                                   not reproducible, see ray_triangle in csrc/irt_common.h */
#define IRT_MODE_CUBQL 2        /* wedges + intersectWedgeEXT (deviceCode.cu:90-115) */

/* Per-frame part of icon_rt::LaunchParams (icon_rt/Params.h:92-119).  The volume,
 * accelerator and transfer-function members live in the context (set by irt_create /
 * irt_set_transfunc); the framebuffer pointers are arguments of irt_render. */
typedef struct irt_launch_params {
  irt_vec3f org;            /* camera.org    (Params.h:101; hostCode.cu:942) */
  irt_vec3f dir_00;         /* camera.dir_00 (Params.h:102; hostCode.cu:943) */
  irt_vec3f dir_du;         /* camera.dir_du (Params.h:103; hostCode.cu:944) */
  irt_vec3f dir_dv;         /* camera.dir_dv (Params.h:104; hostCode.cu:945) */
  int32_t accumID;          /* Params.h:111; hostCode.cu:958 */
  irt_vec3f ambientColor;   /* Params.h:114; hostCode.cu:925 */
  float ambientRadiance;    /* Params.h:115; hostCode.cu:926 */
  float unitDistance;       /* Params.h:118; hostCode.cu:956 */
  int32_t raygen;           /* IRT_RAYGEN_* */
  int32_t accelMode;        /* volume.accelMode (Params.h:33-34; hostCode.cu:170-200, the
                               "Accel mode" UI option 853-857): IRT_ACCEL_SPHERE (sdda over
                               the shell grid, the default) or IRT_ACCEL_GRID (dda3 over the
                               256^3 Cartesian grid) */
  int32_t mode;             /* volume.mode: IRT_MODE_USER_GEOM (default), IRT_MODE_TRIANGLES
                               or IRT_MODE_CUBQL (both need irt_build_wedge_accel) */
} irt_launch_params;

/* Scene facts computed at irt_create exactly as hostCode.cu:792-808, 838-840. */
typedef struct irt_volume_info {
  uint64_t numCells;            /* Volume::numCells (Params.h:63) */
  irt_box3f bounds;             /* Volume::bounds = union of ICONCell::getBounds() */
  irt_box3f sphericalBounds;    /* ShellAccel::sphericalBounds (r, lat, lon) */
  irt_box1f dataRange;          /* min/max of value[0:numLayers) */
  float unitDistance;           /* 10^(floor(log10(sphericalBounds.lower.x))-3) */
  int32_t shellDims[3];         /* ShellAccel::dims = (1,1024,1024) (hostCode.cu:654) */
  /* locator facts (MI355X point-location structure replacing OptiX/cuBQL) */
  int32_t locatorFaceRes;       /* cube-map cells per face edge */
  uint64_t locatorEntries;      /* candidate-list entries */
  uint64_t deviceBytes;         /* HBM held by the context */
} irt_volume_info;

/* Statistics of the most recent irt_render* call on a context. */
typedef struct irt_render_stats {
  uint64_t raysLaunched;        /* pixels the raygen ran for */
  uint64_t raysInBox;           /* rays that passed boxTest (deviceCode.cu:294) */
  uint64_t locateCalls;         /* sampleVolume calls (deviceCode.cu:173) */
  uint64_t samplesFound;        /* sampleVolume calls that found a cell */
  uint64_t candidatesTested;    /* locator candidate-list entries examined */
  float kernelMs;               /* render kernel time, HIP events on the launch stream
                                   (most recent timed launch, irt_set_timing_interval) */
} irt_render_stats;

typedef struct irt_context irt_context;

/* ---------------------------------------------------------------- errors */
const char *irt_last_error(void);

/* ---------------------------------------------------------------- context
 * irt_create: validate and copy `cells` (already lat/lon-filtered, see irt_filter_cells),
 * compute the volume facts (hostCode.cu:792-808), build the cell locator that replaces the
 * OptiX/cuBQL accelerators (hostCode.cu:440-650), upload to HBM on `device`, and build the
 * spherical-shell accelerator on the GPU: initGrid + buildShell_ICON
 * (hostCode.cu:216-225, 299-336, 652-666).  Majorants stay zero until irt_set_transfunc.
 * Everything but the per-record glibc corner trig (toCartesian's cosf/sinf) is built on
 * the device.  irt_create = irt_create_begin + irt_create_append(all) + irt_create_end. */
int irt_create(const irt_icon_cell *cells, size_t numCells, int device, irt_context **out);

/* Streaming creation, for scenes larger than host memory should hold at once (the cells
 * go to HBM chunk by chunk, host memory stays at one chunk): `numCells` records arrive
 * through any number of irt_create_append calls, in record order; irt_create_end builds
 * the scene on the device.  The context is unusable (and irt_create_end fails) unless
 * exactly numCells records were appended. */
int irt_create_begin(size_t numCells, int device, irt_context **out);
int irt_create_append(irt_context *ctx, const irt_icon_cell *cells, size_t n);
int irt_create_end(irt_context *ctx);

/* The load of hostCode.cu:717-734 streamed straight into a context: records of the `.ic`
 * file (N = filesize / 284, truncated to maxNumCells when >= 0, `--num-cells`). */
int irt_create_from_file(const char *path, long maxNumCells, int device, irt_context **out);

/* A synthetic RnBk grid (irt_synth_grid) generated chunk by chunk straight into a context. */
int irt_create_synth(int rootN, int bisections, int levels, float topHeight, float noise,
                     uint32_t seed, int device, irt_context **out);
/* ... with terrain (irt_synth_grid_terrain). */
int irt_create_synth_terrain(int rootN, int bisections, int levels, float topHeight, float noise,
                             uint32_t seed, float terrainHeight, int device, irt_context **out);
void irt_destroy(irt_context *ctx);
int irt_get_volume_info(const irt_context *ctx, irt_volume_info *info);

/* == Pipeline::setTransfunc -> transfuncUpdateHandler -> computeMaxOpacities
 * (pipeline.cu:456-478; hostCode.cu:878-909, 362-397).  `rgbaLUT` is the final LUT
 * (the reference resamples to 300 entries first when size < 300; irt_resample_lut). */
int irt_set_transfunc(irt_context *ctx, const irt_vec4f *rgbaLUT, int size,
                      irt_box1f valueRange, float opacityScale);

/* == clearFramebuffer (common/pipeline.cu:171-199): fb = make_rgba(0), accum = 0. */
int irt_clear_frame(irt_context *ctx, uint32_t *d_fb, irt_vec4f *d_accum, size_t numPixels,
                    void *stream);

/* == one Pipeline::launch() of the raygen over the full width x height launch
 * (pipeline.cu:1061-1074 / owlLaunch2D 1064).  d_fb / d_accum are device arrays of
 * width*height, pixel (x,y) at x + width*y (deviceCode.cu:286). */
int irt_render(irt_context *ctx, const irt_launch_params *lp, int width, int height,
               uint32_t *d_fb, irt_vec4f *d_accum, void *stream);

/* Frame-tile subset of the same launch, for multi-GPU frame splitting: renders the
 * 64x64 tiles t = tileBegin, tileBegin+tileStride, ... (row-major tile ids over
 * ceil(width/64) x ceil(height/64)) into PACKED buffers: tile k of this subset at
 * d_fb_tiles[k*4096 + ly*64 + lx].  Pixel seeds/cameras use the full-launch (x,y,width,
 * height), so every pixel is bit-identical to irt_render's.  Returns the tile count in
 * *numTiles when non-NULL. */
int irt_render_tiles(irt_context *ctx, const irt_launch_params *lp, int width, int height,
                     int tileBegin, int tileStride, uint32_t *d_fb_tiles,
                     irt_vec4f *d_accum_tiles, int *numTiles, void *stream);

/* The reference's progressive accumulation (`--sample-limit N`: Pipeline::isRunning /
 * launch, pipeline.cu:991-1075, with accumID = frameID, hostCode.cu:947-958) batched:
 * numFrames consecutive frames accumID = lp->accumID .. lp->accumID+numFrames-1 in one
 * launch, bit-identical to numFrames irt_render calls with accumID incremented (each
 * frame's lerp(new, old, 1/(accumID+1)), deviceCode.cu:333-334, applied in order; fb holds
 * the last frame's make_rgba(linear_to_srgb(accum))).  The _tiles form packs like
 * irt_render_tiles and is what each rank runs in the multi-GPU weak-scaling split.
 * The frames are chained per pixel inside the one launch (frame f's workgroup of a block
 * lerps once frame f - 1's has published the same pixels), so the next frame's workgroups
 * fill the chip while the previous frame's last ones finish; every frame's accum and fb
 * are written, as numFrames separate launches would.
 * A hand-off wait is bounded (~1 s).  If one ever gives up, the launch's frames were lerped
 * out of order, and the launch fails loudly instead of returning wrong pixels silently: the
 * next call on the context that sees it -- any irt_render* call, irt_get_render_stats*,
 * irt_reset_render_stats_total -- returns IRT_E_CHAIN, irt_last_error() names the launch, and
 * the context renders later multi-frame launches without chaining (per-frame sample buffer +
 * a lerp pass).  The call that returns IRT_E_CHAIN has NOT enqueued its own work: its frame(s)
 * were not rendered, and the caller re-issues the call (or restarts the accumulation from
 * accumID 0).  (The reference's launch either renders the frame or aborts,
 * pipeline.cu:1038-1075.)  Frames of 2^27 pixels or more are never chained. */
int irt_render_accumulate(irt_context *ctx, const irt_launch_params *lp, int width, int height,
                          int numFrames, uint32_t *d_fb, irt_vec4f *d_accum, void *stream);
/* A sequence of views in one launch: frame k renders lps[k] -- its own camera (org, dir_00,
 * dir_du, dir_dv) and accumID; every other member must equal lps[0]'s -- into the same fb and
 * accum, bit-identical to numFrames irt_render calls in order (the reference's render loop,
 * pipeline.cu:991-1075, with the camera moved between frames: an orbit or a camera path).  The
 * frames are chained per pixel in the launch, as in irt_render_accumulate; with a variant or
 * setting that cannot chain, one launch per frame. */
int irt_render_sequence(irt_context *ctx, const irt_launch_params *lps, int numFrames, int width,
                        int height, uint32_t *d_fb, irt_vec4f *d_accum, void *stream);
/* The same over one rank's tile list, packed as irt_render_tile_list packs it (the multi-GPU
 * split of a camera path: every rank renders its tiles of the same views). */
int irt_render_tile_list_sequence(irt_context *ctx, const irt_launch_params *lps, int numFrames,
                                  int width, int height, const int32_t *tiles, int numTiles,
                                  uint32_t *d_fb_tiles, irt_vec4f *d_accum_tiles, void *stream);
int irt_render_tiles_accumulate(irt_context *ctx, const irt_launch_params *lp, int width,
                                int height, int tileBegin, int tileStride, int numFrames,
                                uint32_t *d_fb_tiles, irt_vec4f *d_accum_tiles, int *numTiles,
                                void *stream);

/* Scatter packed tiles (as produced by irt_render_tiles on `numRanks` ranks and gathered
 * rank-major into d_gathered[rank][maxTilesPerRank][4096]) into a linear framebuffer. */
int irt_unpack_tiles(irt_context *ctx, const uint32_t *d_gathered, int numRanks,
                     int maxTilesPerRank, int width, int height, uint32_t *d_fb, void *stream);

/* Cost-balanced multi-GPU deal of a width x height launch's 64x64 tiles (no GPU needed;
 * the reference's CPU path hands the same tiles to a thread pool dynamically,
 * common/thread_pool.h:146-161, for_each.h:70-85).  Each tile's cost is estimated from the
 * camera (lp) and the shell radii (info->sphericalBounds): rays through an 8x8 subset of
 * its pixels, weighted by whether they reach the box and the shell and by their chord
 * through the shell.  Tiles go, heaviest first (ties by id), to the least-loaded rank
 * (longest-processing-time first; ties to the lowest rank); rank 0 starts loaded with
 * rank0Extra x the frame's total estimated cost (in [0, 1): the work rank 0 does beyond its
 * tiles, e.g. the framebuffer unpack per rendered frame).  Deterministic: every rank
 * computes the same table.  table: numRanks x maxTilesPerRank, rank-major, row r = rank r's
 * tiles in render order (heaviest first), -1 padding; table == NULL returns only
 * *maxTilesPerRank (the longest row). */
int irt_deal_tiles(const irt_launch_params *lp, const irt_volume_info *info, int width,
                   int height, int numRanks, float rank0Extra, int32_t *table, size_t capacity,
                   int *maxTilesPerRank);

/* irt_render_tiles / irt_render_tiles_accumulate over an explicit tile list (host array of
 * row-major tile ids, e.g. one row of irt_deal_tiles' table without its -1 padding):
 * list entry k is packed at d_fb_tiles[k*4096 ...].  numFrames >= 1 consecutive progressive
 * frames as irt_render_tiles_accumulate.  Every pixel is bit-identical to irt_render's. */
int irt_render_tile_list(irt_context *ctx, const irt_launch_params *lp, int width, int height,
                         const int32_t *tiles, int numTiles, int numFrames,
                         uint32_t *d_fb_tiles, irt_vec4f *d_accum_tiles, void *stream);

/* Scatter packed tiles gathered rank-major (d_gathered[rank][maxTilesPerRank][4096]) whose
 * tile ids are the host table[rank * maxTilesPerRank + k] (irt_deal_tiles; -1: empty). */
int irt_unpack_tile_table(irt_context *ctx, const uint32_t *d_gathered, int numRanks,
                          int maxTilesPerRank, const int32_t *table, int width, int height,
                          uint32_t *d_fb, void *stream);

/* Statistics of the most recent launch (waits for it).  Launches never wait for earlier
 * ones' statistics: counters are read back through a ring, so frames queue back to back
 * like the reference's GPU path (owlLaunch2D is asynchronous, pipeline.cu:1064).
 * Returns IRT_E_CHAIN once for a chained launch whose hand-off timed out (see
 * irt_render_accumulate). */
int irt_get_render_stats(const irt_context *ctx, irt_render_stats *stats);
/* Sums over every launch since the last reset; *launches = count.  kernelMs is the mean
 * of the timed launches times the launch count (see irt_set_timing_interval). */
int irt_get_render_stats_total(const irt_context *ctx, irt_render_stats *total,
                               long long *launches);
int irt_reset_render_stats_total(irt_context *ctx);
/* Kernel timing (HIP events on the launch stream) on every `every`-th launch only (default
 * 8; 1 = every launch): an event pair per frame adds ~10 us of stream gaps to a 0.17 ms
 * frame.  irt_render_stats.kernelMs of a launch is that of the most recent timed launch.
 * No counterpart in the reference, which times on the host (pipeline.cu:1062-1073). */
int irt_set_timing_interval(irt_context *ctx, int every);
/* The per-launch event counts of irt_render_stats (rays, sampleVolume calls, samples found,
 * candidates) on (1, the default) or off (0).  Counting costs each launch a store of every
 * workgroup's counts into pinned host memory -- ~1.5 % of a C3 frame, more of a small
 * multi-GPU share -- and the reference renders without it; with counting off the counts
 * read 0 (kernelMs stays).  Frames are identical either way.  No reference counterpart. */
int irt_set_statistics(irt_context *ctx, int on);

/* buildCuBQLAccel (hostCode.cu:557-649) for IRT_MODE_CUBQL: the wedges of every (cell,
 * layer) -- corners toCartesian(height[h|h+1], lat, lon), scalar
 * h == 0 ? getValue(height[0]) : (getValue(height[h-1]) + getValue(height[h])) * 0.5 on
 * all six vertices -- behind a cube-map locator of their primBounds (replacing the cuBQL
 * BVH).  `cells` must be the array given to irt_create.  A sample takes the first wedge,
 * in (cell, layer) order, whose bounds contain it and whose intersectWedgeEXT
 * (UElems.h:214-311) accepts it; cuBQL's own traversal order is not reproducible here
 * (the submodule is not vendored), so that order is the documented choice. */
int irt_build_wedge_accel(irt_context *ctx, const irt_icon_cell *cells, size_t n);
/* The same locator also serves IRT_MODE_TRIANGLES (buildTriangleAccel, hostCode.cu:440-484):
 * every cell's bottom triangle toCartesian(height[0], lat, lon) is listed too. */

/* Download the GRID_ACCEL_MODE grid (256^3 macrocells over the volume bounds,
 * hostCode.cu:668-682; index x + 256*(y + 256*z)), same conventions as irt_get_shell.
 * The grid (201 MB) is built on first use -- this call or the first IRT_ACCEL_GRID render --
 * not at irt_create as the reference's main() does (hostCode.cu:875): same grid, no cost to
 * sphere-mode runs. */
int irt_get_grid(const irt_context *ctx, float *valueRanges, float *maxOpacities);

/* Download the shell accelerator (for checking): valueRanges as 2 floats per
 * macrocell, maxOpacities as 1 float per macrocell; either may be NULL. */
int irt_get_shell(const irt_context *ctx, float *valueRanges, float *maxOpacities);

/* Number of tiles of a width x height launch. */
int irt_num_tiles(int width, int height);

/* ---------------------------------------------------------------- host helpers
 * (no GPU needed) -- the host-side setup of icon_rt's main() and common/, so a host
 * program (the C++ Pipeline mirror under icon-ray-tracing_amd/host, or Python) can
 * reproduce the reference's frame setup bit for bit. */

/* Load a raw `.ic` file (hostCode.cu:717-734): N = filesize/284; the first
 * min(N, maxNumCells) records if maxNumCells >= 0.  Call with out == NULL to get the
 * count in *count; then with capacity >= count. */
int irt_load_ic(const char *path, long maxNumCells, irt_icon_cell *out, size_t capacity,
                size_t *count);
int irt_save_ic(const char *path, const irt_icon_cell *cells, size_t count);

/* convert_icon (tools/convert_icon/convert_icon.cpp:168-391): DWD ICON netCDF inputs ->
 * `.ic` records, the convertToIC branch (353-391) evaluated exactly, including its
 * quirks: at most maxLayers data levels (24, 345-349), the last record of a column gets
 * `numLayers % 32 - 1` layers (365), heights R + HHL - HSURF with float/double mixing as
 * written (361, 371), values min/max-normalised in double (317-328), HHL and data files
 * sorted by their `height` level index, descending (274, 337).  Inputs are netCDF
 * classic files (CDF-1/2/5; the netCDF library is replaced by host/irt_netcdf.cpp);
 * netCDF-4/HDF5 inputs fail with IRT_E_IO.  Where the reference reads out of bounds
 * (too few HHL/data files for the layers, a data file with fewer than `cell` values)
 * this returns IRT_E_DATA.  Slots the reference leaves uninitialised are zero.
 * Two-call pattern: out == NULL returns the record count in *count. */
typedef struct irt_convert_opts {
  const char *hgridFile;          /* -hgrid: clon_vertices/clat_vertices (200-203) */
  const char *hsurfFile;          /* -hsurf: HSURF (225) */
  const char *const *hhlFiles;    /* -hhl: height + HHL per file (239-272) */
  int numHhlFiles;
  const char *const *dataFiles;   /* -data: ncells, height + the variable (282-335) */
  int numDataFiles;
  const char *varName;            /* NULL = "pres" (308) */
  int maxLayers;                  /* <= 0: 5 (24) */
} irt_convert_opts;
int irt_convert_icon(const irt_convert_opts *opts, irt_icon_cell *out, size_t capacity,
                     size_t *count);

/* convert_icon's UMesh output (tools/convert_icon/convert_icon.cpp:393-452, the tool's
 * default convertToUMesh branch): one wedge per (cell, layer) with six vertices of its own
 * at R + HSURF*50 / R + (HHL - HSURF)*50, each carrying the layer's value, written to
 * `path` in umesh's binary layout (u64 magic 0x234235567, then u64-counted arrays:
 * vertices vec3f, per-vertex f32 scalars, triangles, quads, tets, pyramids, wedges
 * (6 x i32), hexes).  Needs numLayers+1 HHL files (the reference reads hhl[j+1]).
 * The counts written go to *numVertices / *numWedges (either may be NULL). */
int irt_convert_icon_umesh(const irt_convert_opts *opts, const char *path, size_t *numVertices,
                           size_t *numWedges);

/* Lat/lon filter in degrees (hostCode.cu:736-758); stable, in place; returns the kept
 * count in *count. */
int irt_filter_cells(irt_icon_cell *cells, size_t n, irt_box1f latRangeDeg,
                     irt_box1f lonRangeDeg, size_t *count);

/* Volume facts without a GPU (same values irt_get_volume_info reports). */
int irt_compute_volume_info(const irt_icon_cell *cells, size_t n, irt_volume_info *info);

/* Default transfer function of hostCode.cu:823-836 after Pipeline::setTransfunc's
 * resampling to 300 entries (pipeline.cu:469-473): writes 300 entries to out300 and the
 * value range (dataRange, or [0,1] if empty) to *valueRange. */
int irt_default_transfunc(irt_box1f dataRange, irt_vec4f *out300, irt_box1f *valueRange);

/* resampleLUT (common/dvr_course-common.h:44-70). */
int irt_resample_lut(const irt_vec4f *src, int nsrc, irt_vec4f *dst, int ndst);

/* Camera (common/camera.h) -> LaunchParams.camera as hostCode.cu:939-945 computes it:
 * org = getPosition(), dir_00 = lower_left, dir_du = horizontal/imgW, dir_dv =
 * vertical/imgH.  irt_camera_view_all: Camera::viewAll (camera.h:98-104) with the
 * default fovy of 90 degrees; irt_camera_look_at: Pipeline's --camera vp vi vu / -fovy
 * path (pipeline.cu:444-454; fovy in degrees, <1e-3 -> 90). */
int irt_camera_view_all(irt_box3f bounds, float fovyDeg, int imgW, int imgH,
                        irt_launch_params *lp);
int irt_camera_look_at(irt_vec3f vp, irt_vec3f vi, irt_vec3f vu, float fovyDeg, int imgW,
                       int imgH, irt_launch_params *lp);

/* Synthetic RnBk icosahedral ICON grid (no netCDF offline): 20*rootN^2*4^bisections
 * triangles, `levels` layers with heights R + topHeight*(l/levels)^2, a smooth value
 * field normalised to [0,1] (plus `noise` * hash noise, seeded), stored as `.ic` records
 * of <= 31 layers, bottom to top, consecutive per column.  out == NULL -> count only. */
int irt_synth_grid(int rootN, int bisections, int levels, float topHeight, float noise,
                   uint32_t seed, irt_icon_cell *out, size_t capacity, size_t *count);
/* The same grid over terrain, as tools/convert_icon's `.ic` branch (convert_icon.cpp:353-391)
 * would write it from DWD-like fields: HSURF per column up to terrainHeight metres (~60 % of the
 * columns land), HHL terrain-following near the ground and flat above (the per-column offset
 * HSURF (1 - z/Zd)^2 shrinking with height z, Zd = min(topHeight, 20 km)), records with
 * H[0] = R + HSURF and H[j] = R + HHL - HSURF (so every land column's first layer is inverted)
 * and the last record of a column holding levels % 32 - 1 layers.  terrainHeight 0 ==
 * irt_synth_grid; needs levels % 32 != 0 and 2 terrainHeight < Zd. */
int irt_synth_grid_terrain(int rootN, int bisections, int levels, float topHeight, float noise,
                           uint32_t seed, float terrainHeight, irt_icon_cell *out,
                           size_t capacity, size_t *count);

#ifdef __cplusplus
}
#endif
#endif /* ICON_RT_HIP_H */
