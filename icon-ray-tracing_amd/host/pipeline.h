// pipeline.h -- C++ mirror of dvr_course::Pipeline (common/pipeline.h:53-147) for the
// MI355X backend: same command-line flags, same frame-ID sequencing and clear-on-frame-0
// (common/pipeline.cu:991-1075), PNG presentation (733-739); the launch itself goes
// through the C ABI (irt_render) instead of parallel::for_each / owlLaunch2D.
#pragma once

#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

#include "icon_rt_hip.h"

namespace irt_host {

// dvr_course::Frame (common/fb.h:27-48) with device (HBM) buffers.
struct Frame {
  Frame(int w, int h) { resize(w, h); }
  ~Frame();
  Frame(const Frame &) = delete;
  Frame &operator=(const Frame &) = delete;
  void resize(int w, int h);
  uint32_t *fbPointer = nullptr;
  float *fbDepth = nullptr;
  irt_vec4f *accumBuffer = nullptr;
  int width = 0, height = 0;
};

// dvr_course::Transfunc (common/transfunc.h:29-49), host-side LUT.
struct Transfunc {
  float opacity = 1.f;
  irt_box1f valueRange{0.f, 1.f};
  irt_box1f relRange{0.f, 1.f};
  std::vector<irt_vec4f> lut;
  int size() const { return (int)lut.size(); }
};

// Camera state the Pipeline can override from --camera/-fovy (pipeline.cu:444-454).
struct CameraSpec {
  bool fromCmdline = false;
  irt_vec3f vp{0, 0, 0}, vi{0, 0, 0}, vu{0, 0, 0};
  float fovyDeg = 70.f;  // pipeline.cu:782
};

struct Pipeline {
  Pipeline(int argc, char *argv[], std::string name = "dvr-course-cpp");
  ~Pipeline();

  // ray generation: the app installs the frame launch (irt_render) here
  void setRayGen(const std::function<void()> &f) { func = f; }
  std::function<void()> func;
  // clearFramebuffer (pipeline.cu:171-199): the app installs irt_clear_frame here
  std::function<void()> clearFramebuffer;

  void setFrame(Frame *f);
  Frame *fb = nullptr;
  int frameID = 0;

  CameraSpec camera;  // setCamera(): cmdline override if --camera was given

  void setTransfunc(Transfunc *tf, int index = 0);
  Transfunc *getTransfunc(int index = 0) const;
  bool transfuncValid(int index = 0) const;
  typedef std::function<void(const Transfunc *, int)> TransfuncUpdateHandler;
  void setTransfuncUpdateHandler(TransfuncUpdateHandler h) { updateHandler = h; }

  bool isRunning();
  void launch();
  void present() const;
  void resetAccumulation() { frameID = 0; }

  double avgSeconds() const { return avg_t; }
  int sampleLimit = 1;  // non-interactive default (pipeline.cu:764)
  std::string name;

 private:
  void init();
  bool running = false;
  bool inited = false;
  TransfuncUpdateHandler updateHandler;
  std::vector<Transfunc *> transfuncs;
  Transfunc ourTransfunc;
  std::string xfFile;
  int cmdWidth = -1, cmdHeight = -1;
  double avg_t = 0.0;
  void *ev0 = nullptr, *ev1 = nullptr;
};

// .xf transfer-function files (pipeline.cu:127-169)
bool loadXF(const std::string &file, Transfunc &tf);
bool saveXF(const std::string &file, const Transfunc &tf);

// Minimal PNG writer (stored deflate blocks), RGBA8, optionally flipped vertically.
bool writePNG(const std::string &file, const uint32_t *rgba, int w, int h, bool flip);

}  // namespace irt_host
