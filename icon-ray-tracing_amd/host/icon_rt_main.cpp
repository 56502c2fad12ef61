// icon_rt_main.cpp -- the icon_rt application on the MI355X backend: mirrors
// icon_rt/hostCode.cu main() (703-968) step by step, with the launch going through the C
// ABI of include/icon_rt_hip.h.
//
//   icon_rt <file.ic> [--num-cells N] [--lat-range a:b] [--lon-range a:b]
//           [-mode 0|1|2]                       (0 cell sample(), 1 triangles, 2 wedges)
//           [Pipeline flags: --size W H, --camera ..., -fovy f, --xf f, --sample-limit N]
//           [--synth rootN bisections levels]   (no .ic file: synthetic ICON grid)
//           [--bench K]                         (render K extra frames, print timing)
//           [--frames-per-launch B]             (--bench: B consecutive progressive frames
//                                                per launch, irt_render_accumulate)
//           [--true-size]                       (dir_du/dir_dv over the real W/H instead
//                                                of the reference's hard-coded 512)
//           [--accel sphere|grid]               (the "Accel mode" UI option,
//                                                hostCode.cu:853-857, 170-199)
//           [--gpus N]                          (N devices in this process: the frame's
//                                                64x64 tiles dealt over them, RCCL gather
//                                                to device 0; include/icon_rt_hip_multi.h)
//           [--dump-fb file]                    (the final RGBA8 framebuffer, raw W*H u32)

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "icon_rt_hip.h"
#include "icon_rt_hip_multi.h"
#include "pipeline.h"

using namespace irt_host;

namespace {

struct AppState {  // hostCode.cu:65-92 (the parts this backend uses)
  std::string filepath;
  long maxNumCells = -1;
  irt_box1f latRange{-INFINITY, INFINITY};
  irt_box1f lonRange{-INFINITY, INFINITY};
  int synth[3] = {0, 0, 0};
  int benchFrames = 0;
  int framesPerLaunch = 1;
  bool trueSize = false;
  int accelMode = IRT_ACCEL_SPHERE;  // g_appState.accelMode (hostCode.cu:75)
  int mode = IRT_MODE_USER_GEOM;     // g_appState.mode: the sampler (Params.h:29-31)
  int gpus = 0;                      // > 0: the multi-GPU split over devices 0..gpus-1
  std::string dumpFb;
} g;

bool endsWith(const std::string &s, const std::string &suffix) {
  return s.size() >= suffix.size() && s.compare(s.size() - suffix.size(), suffix.size(), suffix) == 0;
}

void parseRange(const std::string &s, irt_box1f &r) {  // hostCode.cu:115-124
  r.lower = std::stof(s.substr(0, s.find(':')));
  r.upper = std::stof(s.substr(s.find(':') + 1));
}

void parseCommandLine(int argc, char *argv[]) {  // hostCode.cu:106-129
  for (int i = 1; i < argc; ++i) {
    std::string arg = argv[i];
    if (arg[0] != '-' && endsWith(arg, ".ic"))
      g.filepath = arg;
    else if (arg == "--num-cells" && i + 1 < argc)
      g.maxNumCells = atol(argv[++i]);
    else if (arg == "--lat-range" && i + 1 < argc)
      parseRange(argv[++i], g.latRange);
    else if (arg == "--lon-range" && i + 1 < argc)
      parseRange(argv[++i], g.lonRange);
    else if (arg == "-mode" && i + 1 < argc)
      g.mode = atoi(argv[++i]);  // hostCode.cu:125-127
    else if (arg == "--synth" && i + 3 < argc) {
      for (int k = 0; k < 3; ++k) g.synth[k] = atoi(argv[++i]);
    } else if (arg == "--bench" && i + 1 < argc)
      g.benchFrames = atoi(argv[++i]);
    else if (arg == "--frames-per-launch" && i + 1 < argc)
      g.framesPerLaunch = atoi(argv[++i]) < 1 ? 1 : atoi(argv[i]);
    else if (arg == "--true-size")
      g.trueSize = true;
    else if (arg == "--accel" && i + 1 < argc)
      g.accelMode = std::string(argv[++i]) == "grid" ? IRT_ACCEL_GRID : IRT_ACCEL_SPHERE;
    else if (arg == "--gpus" && i + 1 < argc)
      g.gpus = atoi(argv[++i]);
    else if (arg == "--dump-fb" && i + 1 < argc)
      g.dumpFb = argv[++i];
  }
}

void die(const char *what) {
  fprintf(stderr, "%s: %s\n", what, irt_last_error());
  exit(1);
}

void dieMulti(const char *what) {
  fprintf(stderr, "%s: %s\n", what, irt_multi_last_error());
  exit(1);
}

}  // namespace

int main(int argc, char *argv[]) {
  if (argc < 2) {
    fprintf(stderr, "Usage: icon_rt <file.ic> [options]\n");
    return -1;
  }
  parseCommandLine(argc, argv);

  // load (hostCode.cu:717-734) or synthesise
  std::vector<irt_icon_cell> cells;
  size_t n = 0;
  if (!g.filepath.empty()) {
    if (irt_load_ic(g.filepath.c_str(), g.maxNumCells, nullptr, 0, &n)) die("load");
    cells.resize(n);
    if (irt_load_ic(g.filepath.c_str(), g.maxNumCells, cells.data(), n, &n)) die("load");
  } else if (g.synth[0] > 0) {
    if (irt_synth_grid(g.synth[0], g.synth[1], g.synth[2], 75e3f, 0.f, 1234, nullptr, 0, &n)) die("synth");
    cells.resize(n);
    if (irt_synth_grid(g.synth[0], g.synth[1], g.synth[2], 75e3f, 0.f, 1234, cells.data(), n, &n))
      die("synth");
    if (g.maxNumCells >= 0 && (size_t)g.maxNumCells < n) cells.resize(g.maxNumCells);
  } else {
    fprintf(stderr, "Usage: icon_rt <file.ic> [options]\n");
    return -1;
  }
  // lat/lon filter (hostCode.cu:736-758)
  if (irt_filter_cells(cells.data(), cells.size(), g.latRange, g.lonRange, &n)) die("filter");
  cells.resize(n);

  // bounds, dataRange, unitDistance (hostCode.cu:792-808, 838-840)
  irt_volume_info info;
  if (irt_compute_volume_info(cells.data(), cells.size(), &info)) die("volume info");

  Pipeline pl(argc, argv, "icon_rt");  // hostCode.cu:813
  const int imgWidth = 512, imgHeight = 512;  // hostCode.cu:815
  Frame fb(imgWidth, imgHeight);
  pl.setFrame(&fb);

  // default transfer function (hostCode.cu:823-836)
  Transfunc defaultTF;
  if (!pl.transfuncValid()) {
    irt_vec4f lut300[300];
    irt_box1f vr;
    irt_default_transfunc(info.dataRange, lut300, &vr);
    defaultTF.valueRange = vr;
    defaultTF.lut.assign(lut300, lut300 + 300);
    pl.setTransfunc(&defaultTF);
  }

  // the accelerators (hostCode.cu:868-910): one HIP context replaces OptiX/cuBQL/shell
  irt_context *ctx = nullptr;
  irt_multi *multi = nullptr;
  auto t0 = std::chrono::steady_clock::now();
  if (g.gpus > 0) {  // one context per device, an RCCL communicator over them
    std::vector<int> devs(g.gpus);
    for (int d = 0; d < g.gpus; ++d) devs[d] = d;
    if (irt_multi_create_cells(cells.data(), cells.size(), devs.data(), g.gpus, &multi))
      dieMulti("irt_multi_create_cells");
    ctx = irt_multi_context(multi, 0);
    fprintf(stderr, "icon_rt: %d devices, frame tiles dealt by cost, RCCL gather to device 0\n", g.gpus);
  } else if (irt_create(cells.data(), cells.size(), 0, &ctx)) {
    die("irt_create");
  }
  auto t1 = std::chrono::steady_clock::now();
  irt_get_volume_info(ctx, &info);
  fprintf(stderr, "icon_rt: %zu cells, %.2f GiB HBM, locator %d^2 x 6, build %.2f s\n",
          cells.size(), info.deviceBytes / 1073741824.0, info.locatorFaceRes,
          std::chrono::duration<double>(t1 - t0).count());
  pl.setTransfuncUpdateHandler([&](const Transfunc *tf, int) {
    if (multi) {
      if (irt_multi_set_transfunc(multi, tf->lut.data(), tf->size(), tf->valueRange, tf->opacity))
        dieMulti("irt_multi_set_transfunc");
    } else if (irt_set_transfunc(ctx, tf->lut.data(), tf->size(), tf->valueRange, tf->opacity)) {
      die("irt_set_transfunc");
    }
  });

  // camera (hostCode.cu:819-821 viewAll, pipeline.cu:444-454 cmdline override, 939-945)
  const int divW = g.trueSize ? fb.width : imgWidth, divH = g.trueSize ? fb.height : imgHeight;
  irt_launch_params lp;
  memset(&lp, 0, sizeof(lp));
  if (pl.camera.fromCmdline) {
    irt_camera_look_at(pl.camera.vp, pl.camera.vi, pl.camera.vu, pl.camera.fovyDeg, divW, divH, &lp);
  } else {
    irt_camera_view_all(info.bounds, 90.f, divW, divH, &lp);
  }
  lp.ambientColor = {1.f, 1.f, 1.f};  // hostCode.cu:925-926
  lp.ambientRadiance = 1.f;
  lp.unitDistance = info.unitDistance;
  lp.raygen = IRT_RAYGEN_WITH_ACCEL;  // setRayGen(woodcockTrackingWithAccel) (863)
  lp.accelMode = g.accelMode;         // toggleAccelMode (hostCode.cu:170-199)
  if (g.mode == IRT_MODE_CUBQL || g.mode == IRT_MODE_TRIANGLES) {
    // toggleMode (hostCode.cu:152-168): buildCuBQLAccel / buildTriangleAccel's geometry
    for (int d = 0; d < (multi ? g.gpus : 1); ++d)
      if (irt_build_wedge_accel(multi ? irt_multi_context(multi, d) : ctx, cells.data(), cells.size()))
        die("irt_build_wedge_accel");
    lp.mode = g.mode;
  } else if (g.mode != IRT_MODE_USER_GEOM) {
    fprintf(stderr, "icon_rt: unknown -mode %d; using the cell sampler (-mode 0)\n", g.mode);
  }

  pl.clearFramebuffer = [&] {
    if (irt_clear_frame(ctx, fb.fbPointer, fb.accumBuffer, (size_t)fb.width * fb.height, nullptr))
      die("clear");
  };
  pl.setRayGen([&] {
    if (multi) {
      if (irt_multi_render(multi, &lp, fb.width, fb.height, 1, fb.fbPointer, nullptr)) dieMulti("irt_multi_render");
      return;
    }
    if (irt_render(ctx, &lp, fb.width, fb.height, fb.fbPointer, fb.accumBuffer, nullptr))
      die("irt_render");
    irt_render_stats st;
    irt_get_render_stats(ctx, &st);
  });

  do {  // hostCode.cu:931-965
    lp.accumID = pl.frameID;
    pl.launch();
    pl.present();
  } while (pl.isRunning());

  if (g.benchFrames > 0) {
    // as bench.py: per-launch counting off, the launches back to back, one wait at the end
    for (int d = 0; d < (multi ? g.gpus : 1); ++d)
      if (irt_set_statistics(multi ? irt_multi_context(multi, d) : ctx, 0)) die("irt_set_statistics");
    const int B = g.framesPerLaunch;
    auto render = [&](int k, int n) {  // B > 1: frames k .. k+n-1 of the accumulation in one launch
      lp.accumID = B > 1 ? k : 0;
      if (multi) {
        if (irt_multi_render(multi, &lp, fb.width, fb.height, n, fb.fbPointer, nullptr)) dieMulti("irt_multi_render");
        return;
      }
      const int rc = n > 1 ? irt_render_accumulate(ctx, &lp, fb.width, fb.height, n, fb.fbPointer,
                                                   fb.accumBuffer, nullptr)
                           : irt_render(ctx, &lp, fb.width, fb.height, fb.fbPointer, fb.accumBuffer, nullptr);
      if (rc) die("irt_render");
    };
    auto sync = [&] {
      if (multi && irt_multi_synchronize(multi)) dieMulti("irt_multi_synchronize");
      if (hipDeviceSynchronize() != hipSuccess) die("hipDeviceSynchronize");
    };
    render(0, B);  // warm-up
    sync();
    const auto a = std::chrono::steady_clock::now();
    for (int k = 0; k < g.benchFrames; k += B) render(B + k, std::min(B, g.benchFrames - k));
    sync();
    const double total = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    const double px = (double)fb.width * fb.height * g.benchFrames;
    printf("bench: %d frames %dx%d, %d per launch, %d device(s): %.4f ms/frame, %.1f Mray/s\n", g.benchFrames,
           fb.width, fb.height, B, multi ? g.gpus : 1, 1e3 * total / g.benchFrames, px / total / 1e6);
  }
  if (!g.dumpFb.empty()) {  // the final framebuffer (after --bench's frames), raw (x + W*y, RGBA8 with r in the low byte)
    if (multi && irt_multi_synchronize(multi)) dieMulti("irt_multi_synchronize");
    std::vector<uint32_t> h((size_t)fb.width * fb.height);
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h.data(), fb.fbPointer, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
      die("dump-fb copy");
    FILE *f = fopen(g.dumpFb.c_str(), "wb");
    if (!f || fwrite(h.data(), 4, h.size(), f) != h.size()) die("dump-fb write");
    fclose(f);
  }
  if (multi)
    irt_multi_destroy(multi);
  else
    irt_destroy(ctx);
  return 0;
}
