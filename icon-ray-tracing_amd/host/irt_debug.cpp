// irt_debug.cpp -- host-only inspection entry points (include/icon_rt_hip_debug.h).

#include <string.h>

#include "icon_rt_hip_debug.h"
#include "irt_internal.h"

using namespace irt;

struct irt_debug_scene {
  HostScene s;
};

extern "C" {

float irt_debug_asinf(float x) { return glibc_asinf(x); }
float irt_debug_atan2f(float y, float x) { return glibc_atan2f(y, x); }
int irt_debug_f2i(float x) { return f2i_x86(x); }

float irt_debug_logf_entry(uint32_t k) { return logf_table()[k & 0x00FFFFFFu]; }

void irt_debug_srgb_thresholds(float *out256) { srgb_thresholds(out256); }

int irt_debug_scene_build(const irt_icon_cell *cells, size_t n, irt_debug_scene **out) {
  if (!out || (n && !cells)) {
    set_error("irt_debug_scene_build: null argument");
    return IRT_E_INVALID;
  }
  irt_debug_scene *d = new irt_debug_scene();
  int rc = build_scene(cells, n, d->s);
  if (rc) {
    delete d;
    return rc;
  }
  *out = d;
  return IRT_OK;
}

int irt_debug_scene_info(const irt_debug_scene *s, irt_volume_info *info) {
  if (!s || !info) return IRT_E_INVALID;
  *info = s->s.info;
  return IRT_OK;
}

int irt_debug_scene_locate(const irt_debug_scene *s, irt_vec3f p, float *value,
                           uint32_t *record) {
  if (!s || !value) return IRT_E_INVALID;
  float v = 0.f;
  uint32_t r = 0;
  int hit = locate_host(s->s, p.x, p.y, p.z, v, &r);
  if (hit) {
    *value = v;
    if (record) *record = r;
  }
  return hit;
}

int irt_debug_scene_candidates(const irt_debug_scene *s, irt_vec3f p, uint32_t *records,
                               int capacity) {
  if (!s || s->s.G == 0) return 0;
  const uint32_t cell = cubemap_cell(p.x, p.y, p.z, s->s.G);
  const uint32_t b = s->s.offsets[cell], e = s->s.offsets[cell + 1];
  int k = 0;
  for (uint32_t i = b; i < e; ++i, ++k)
    if (records && k < capacity) records[k] = s->s.entries[i].idx;
  return k;
}

int irt_debug_scene_planes(const irt_debug_scene *s, uint32_t record, float *out12) {
  if (!s || !out12 || record >= s->s.n) return IRT_E_INVALID;
  memcpy(out12, &s->s.planes[3 * (size_t)record], 12 * sizeof(float));
  return IRT_OK;
}

void irt_debug_scene_free(irt_debug_scene *s) { delete s; }

}  // extern "C"
