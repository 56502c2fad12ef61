/*
 * icon_rt_hip_multi.h -- one process, N GPUs: the frame-tile split of the ICON renderer with
 * an RCCL gather of the framebuffer, for C/C++ integrators (no torch, no MPI).
 * Library: icon-ray-tracing_amd/libicon_rt_multi.so (links libicon_rt_hip.so and RCCL).
 *
 * The reference is single-device: its main loop renders a frame with
 *     SET_LAUNCH_PARAMS(parms); pl.launch(); pl.present();   (icon_rt/hostCode.cu:931-965)
 * and its CPU path already cuts the frame into 64x64 tiles pulled by a thread pool
 * (common/pipeline.cu:1066-1071, thread_pool.h:146-161).  Here the same tiles are dealt to
 * the N devices by estimated cost (irt_deal_tiles), every device renders its tiles into a
 * packed buffer (irt_render_tile_list, one context per device, one stream per device), the
 * packed tiles go to the first device over RCCL (single-process communicator,
 * ncclCommInitAll, rccl.h:236; grouped ncclSend/ncclRecv, rccl.h:700-720) and are scattered
 * into the caller's framebuffer there (irt_unpack_tile_table).  Pixel seeds depend only on
 * (accumID, W, H, x, y) (deviceCode.cu:288-289), so the frame is bit-identical to irt_render's
 * on one device.  The accumulation buffer stays sharded: each device keeps the accum of its
 * own tiles across the frames of a progressive accumulation (no exchange needed).
 *
 * Conventions as in icon_rt_hip.h: IRT_OK / IRT_E_* codes, single caller per handle.
 */
#ifndef ICON_RT_HIP_MULTI_H
#define ICON_RT_HIP_MULTI_H

#include "icon_rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct irt_multi irt_multi;

/* Message of the last failed irt_multi_* call on this thread (an RCCL/HIP failure of the
 * multi layer, or the irt_last_error() text of the irt_* call that failed under it). */
const char *irt_multi_last_error(void);

/* Take ownership of numDevices contexts of the SAME scene, contexts[i] created on devices[i]
 * (any irt_create* call; the C++ app streams the `.ic` file into each).  Creates one stream per
 * device and the RCCL communicator over the devices (ncclCommInitAll).  The first device
 * holds the assembled framebuffer.  On failure the contexts stay the caller's. */
int irt_multi_create(irt_context *const *contexts, const int *devices, int numDevices, irt_multi **out);
/* irt_create(cells) on every device, then irt_multi_create. */
int irt_multi_create_cells(const irt_icon_cell *cells, size_t numCells, const int *devices, int numDevices,
                           irt_multi **out);
/* Destroys the communicator, the buffers and the contexts. */
void irt_multi_destroy(irt_multi *m);
int irt_multi_num_devices(const irt_multi *m);
/* The context of device i (statistics, debug calls); owned by m. */
irt_context *irt_multi_context(const irt_multi *m, int i);

/* irt_set_transfunc on every device (Pipeline::setTransfunc -> computeMaxOpacities,
 * pipeline.cu:456-478, hostCode.cu:878-909). */
int irt_multi_set_transfunc(irt_multi *m, const irt_vec4f *rgbaLUT, int size, irt_box1f valueRange,
                            float opacityScale);

/* numFrames >= 1 consecutive progressive frames accumID = lp->accumID ... of a width x height
 * launch (the reference's render loop, hostCode.cu:931-965; numFrames > 1 as
 * irt_render_accumulate), split over the devices, the last frame's RGBA8 assembled in d_fb
 * (a device array of width*height on the FIRST device, pixel (x,y) at x + width*y) on
 * `stream` (a hipStream_t of the first device, NULL: the null stream).  The tiles are dealt
 * (irt_deal_tiles) for the first call and again whenever the camera (org, dir_00, dir_du,
 * dir_dv) or the frame size changes; the devices' accum tiles are zeroed then and whenever
 * accumID is 0 (clearFramebuffer, pipeline.cu:171-199).  Work on `stream` after this
 * call sees the whole frame; the call itself does not wait for the GPUs. */
int irt_multi_render(irt_multi *m, const irt_launch_params *lp, int width, int height, int numFrames,
                     uint32_t *d_fb, void *stream);

/* Wait for every device's work of this handle. */
int irt_multi_synchronize(irt_multi *m);

#ifdef __cplusplus
}
#endif
#endif /* ICON_RT_HIP_MULTI_H */
