// pipeline.cpp -- see pipeline.h.

#include "pipeline.h"

#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>

namespace irt_host {

static void hipCheck(hipError_t e, const char *what) {
  if (e != hipSuccess) {
    fprintf(stderr, "HIP error in %s: %s\n", what, hipGetErrorString(e));
    exit(1);
  }
}

Frame::~Frame() {
  if (fbPointer) (void)hipFree(fbPointer);
  if (fbDepth) (void)hipFree(fbDepth);
  if (accumBuffer) (void)hipFree(accumBuffer);
}

void Frame::resize(int w, int h) {  // fb.cu:49-67 (device buffers)
  if (fbPointer) (void)hipFree(fbPointer);
  if (fbDepth) (void)hipFree(fbDepth);
  if (accumBuffer) (void)hipFree(accumBuffer);
  width = w;
  height = h;
  hipCheck(hipMalloc((void **)&fbPointer, (size_t)w * h * sizeof(uint32_t)), "Frame");
  hipCheck(hipMalloc((void **)&fbDepth, (size_t)w * h * sizeof(float)), "Frame");
  hipCheck(hipMalloc((void **)&accumBuffer, (size_t)w * h * sizeof(irt_vec4f)), "Frame");
}

bool loadXF(const std::string &file, Transfunc &tf) {  // pipeline.cu:127-150
  std::ifstream in(file, std::ios::binary);
  if (!in.good()) return false;
  in.read((char *)&tf.opacity, sizeof(tf.opacity));
  in.read((char *)&tf.valueRange, sizeof(tf.valueRange));
  in.read((char *)&tf.relRange, sizeof(tf.relRange));
  int n = 0;
  in.read((char *)&n, sizeof(n));
  if (n <= 0) return false;
  tf.lut.resize(n);
  in.read((char *)tf.lut.data(), sizeof(irt_vec4f) * n);
  return (bool)in;
}

bool saveXF(const std::string &file, const Transfunc &tf) {  // pipeline.cu:152-169
  std::ofstream out(file, std::ios::binary);
  if (!out.good()) return false;
  out.write((const char *)&tf.opacity, sizeof(tf.opacity));
  out.write((const char *)&tf.valueRange, sizeof(tf.valueRange));
  out.write((const char *)&tf.relRange, sizeof(tf.relRange));
  int n = tf.size();
  out.write((const char *)&n, sizeof(n));
  out.write((const char *)tf.lut.data(), sizeof(irt_vec4f) * n);
  return true;
}

Pipeline::Pipeline(int argc, char *argv[], std::string nm) : name(nm) {
  // Pipeline::Impl::parseCommandLine (pipeline.cu:224-253)
  for (int i = 1; i < argc; ++i) {
    std::string arg = argv[i];
    auto need = [&](int k) {
      if (i + k >= argc) {
        fprintf(stderr, "missing value for %s\n", arg.c_str());
        exit(1);
      }
    };
    if (arg == "--bgcolor") {
      need(3);
      i += 3;  // only used by the interactive viewer
    } else if (arg == "--sample-limit") {
      need(1);
      sampleLimit = atoi(argv[++i]);
    } else if (arg == "--xf") {
      need(1);
      xfFile = argv[++i];
    } else if (arg == "-win" || arg == "--win" || arg == "--size") {
      need(2);
      cmdWidth = atoi(argv[++i]);
      cmdHeight = atoi(argv[++i]);
    } else if (arg == "-fovy") {
      need(1);
      camera.fovyDeg = (float)atof(argv[++i]);
    } else if (arg == "--camera") {
      need(9);
      float v[9];
      for (int k = 0; k < 9; ++k) v[k] = (float)atof(argv[++i]);
      camera.vp = {v[0], v[1], v[2]};
      camera.vi = {v[3], v[4], v[5]};
      camera.vu = {v[6], v[7], v[8]};
    }
  }
  // setCamera applies the override iff vu != 0 (pipeline.cu:446)
  camera.fromCmdline = camera.vu.x != 0.f || camera.vu.y != 0.f || camera.vu.z != 0.f;
  if (!xfFile.empty() && loadXF(xfFile, ourTransfunc)) transfuncs = {&ourTransfunc};
}

Pipeline::~Pipeline() {
  if (ev0) (void)hipEventDestroy((hipEvent_t)ev0);
  if (ev1) (void)hipEventDestroy((hipEvent_t)ev1);
}

void Pipeline::setFrame(Frame *f) {  // pipeline.cu:430-442
  fb = f;
  if (cmdWidth > 0 && cmdHeight > 0) f->resize(cmdWidth, cmdHeight);
}

void Pipeline::setTransfunc(Transfunc *tf, int index) {  // pipeline.cu:456-478
  if (index >= (int)transfuncs.size()) transfuncs.resize(index + 1);
  transfuncs[index] = tf;
  if (tf->size() < 300) {
    std::vector<irt_vec4f> newLUT(300);
    irt_resample_lut(tf->lut.data(), tf->size(), newLUT.data(), 300);
    tf->lut = newLUT;
  }
  if (updateHandler) updateHandler(tf, index);
}

Transfunc *Pipeline::getTransfunc(int index) const { return transfuncs[index]; }
bool Pipeline::transfuncValid(int index) const {
  return (int)transfuncs.size() > index && transfuncs[index] != nullptr;
}

void Pipeline::init() {  // pipeline.cu:255-308
  if (!fb) {
    fprintf(stderr, "Pipeline invalid on init, aborting...\n");
    abort();
  }
  if (updateHandler)
    for (int i = 0; i < (int)transfuncs.size(); ++i) updateHandler(transfuncs[i], i);
  if (!ev0) {
    hipCheck(hipEventCreate((hipEvent_t *)&ev0), "event");
    hipCheck(hipEventCreate((hipEvent_t *)&ev1), "event");
  }
  inited = true;
}

bool Pipeline::isRunning() {  // pipeline.cu:991-1036 (non-interactive)
  if (!fb) {
    fprintf(stderr, "Pipeline invalid, aborting...\n");
    abort();
  }
  running = (frameID < sampleLimit - 1);
  if (!running) return false;
  frameID++;
  return running;
}

void Pipeline::launch() {  // pipeline.cu:1038-1075
  if (!fb) {
    fprintf(stderr, "Pipeline invalid, aborting...\n");
    abort();
  }
  if (!running) {
    init();
    isRunning();  // first time is always running (frameID may become 1 here)
  }
  if (!func) return;
  if (frameID == 0 && clearFramebuffer) clearFramebuffer();  // pipeline.cu:1058-1059
  if (frameID < sampleLimit) {
    hipCheck(hipEventRecord((hipEvent_t)ev0, 0), "event");
    func();
    hipCheck(hipEventRecord((hipEvent_t)ev1, 0), "event");
    hipCheck(hipEventSynchronize((hipEvent_t)ev1), "event");
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, (hipEvent_t)ev0, (hipEvent_t)ev1), "event");
    double elapsed = ms / 1000.0;
    if (avg_t <= 0) avg_t = elapsed;
    avg_t = 0.8 * avg_t + 0.2 * elapsed;
  }
}

void Pipeline::present() const {  // pipeline.cu:608-741 (non-interactive PNG)
  std::vector<uint32_t> pixels((size_t)fb->width * fb->height);
  hipCheck(hipMemcpy(pixels.data(), fb->fbPointer, pixels.size() * 4, hipMemcpyDeviceToHost),
           "present");
  std::string fileName = name + ".png";
  writePNG(fileName, pixels.data(), fb->width, fb->height, /*flip*/ true);
  printf("Output: %s\n", fileName.c_str());
  printf("FPS: %.2f\n", 1.f / (avg_t > 1e-8 ? avg_t : 1e-8));
}

// ----------------------------------------------------------------- PNG (stored deflate)
static uint32_t crc32(const uint8_t *p, size_t n, uint32_t c = 0xffffffffu) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t v = i;
      for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xedb88320u ^ (v >> 1) : v >> 1;
      table[i] = v;
    }
    init = true;
  }
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c;
}

bool writePNG(const std::string &file, const uint32_t *rgba, int w, int h, bool flip) {
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (w * 4 + 1));
  for (int y = 0; y < h; ++y) {
    const int sy = flip ? h - 1 - y : y;
    raw.push_back(0);
    const uint8_t *row = (const uint8_t *)(rgba + (size_t)sy * w);
    raw.insert(raw.end(), row, row + 4 * w);
  }
  std::vector<uint8_t> z = {0x78, 0x01};
  uint32_t a = 1, b = 0;
  for (uint8_t v : raw) {
    a = (a + v) % 65521;
    b = (b + a) % 65521;
  }
  for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
    size_t len = std::min<size_t>(65535, raw.size() - off);
    bool last = off + len >= raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back(len & 0xff);
    z.push_back(len >> 8);
    z.push_back(~len & 0xff);
    z.push_back((~len >> 8) & 0xff);
    z.insert(z.end(), raw.begin() + off, raw.begin() + off + len);
    if (last) break;
  }
  uint32_t adler = (b << 16) | a;
  for (int s = 24; s >= 0; s -= 8) z.push_back((adler >> s) & 0xff);
  FILE *f = fopen(file.c_str(), "wb");
  if (!f) return false;
  auto be32 = [&](uint32_t v) {
    uint8_t q[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    fwrite(q, 1, 4, f);
  };
  auto chunk = [&](const char *type, const std::vector<uint8_t> &data) {
    be32((uint32_t)data.size());
    std::vector<uint8_t> td(type, type + 4);
    td.insert(td.end(), data.begin(), data.end());
    fwrite(td.data(), 1, td.size(), f);
    be32(crc32(td.data(), td.size()) ^ 0xffffffffu);
  };
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  fwrite(sig, 1, 8, f);
  std::vector<uint8_t> ihdr = {(uint8_t)(w >> 24), (uint8_t)(w >> 16), (uint8_t)(w >> 8), (uint8_t)w,
                               (uint8_t)(h >> 24), (uint8_t)(h >> 16), (uint8_t)(h >> 8), (uint8_t)h,
                               8, 6, 0, 0, 0};
  chunk("IHDR", ihdr);
  chunk("IDAT", z);
  chunk("IEND", {});
  fclose(f);
  return true;
}

}  // namespace irt_host
