// irt_debug.cpp -- host-only inspection entry points (include/icon_rt_hip_debug.h).

#include <math.h>
#include <vector>
#include <string.h>

#include "icon_rt_hip_debug.h"
#include "irt_internal.h"

using namespace irt;

struct irt_debug_scene {
  HostScene s;
  std::vector<irt_icon_cell> cells;  // kept for the CUBQL_MODE wedge queries
  WedgeScene w;
};

extern "C" {

float irt_debug_asinf(float x) { return glibc_asinf(x); }
float irt_debug_atan2f(float y, float x) { return glibc_atan2f(y, x); }
int irt_debug_f2i(float x) { return f2i_x86(x); }
void irt_debug_lcg_jump(uint32_t n, uint32_t *mul, uint32_t *add) { lcg_jump(n, *mul, *add); }

float irt_debug_logf_entry(uint32_t k) { return logf_table()[k & 0x00FFFFFFu]; }

void irt_debug_srgb_thresholds(float *out256) { srgb_thresholds(out256); }

void irt_debug_host_woodcock_log(float *out) {
  for (uint32_t k = 0; k < (1u << 24); ++k) out[k] = logf(1.f - (float)k / (float)0x01000000);
}

uint32_t irt_debug_logf_mismatches(void) {
  // glibc_logf_unit (irt_common.h) vs the host glibc logf over the Woodcock domain
  uint32_t bad = 0;
  for (uint32_t k = 0; k < (1u << 24); ++k) {
    const float x = 1.f - (float)k / (float)0x01000000;
    if (f2u(glibc_logf_unit(x, kLogfTab)) != f2u(logf(x))) ++bad;
  }
  return bad;
}

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

int irt_debug_scene_locate_binned(const irt_debug_scene *s, irt_vec3f p, float *value,
                                  uint32_t *record, uint32_t *tested) {
  if (!s || !value) return IRT_E_INVALID;
  float v = 0.f;
  uint32_t r = 0;
  int hit = locate_bins_host(s->s, p.x, p.y, p.z, v, &r, tested);
  if (hit) {
    *value = v;
    if (record) *record = r;
  }
  return hit;
}

int irt_debug_scene_values(const irt_debug_scene *s, uint32_t rec, float r, float *out2) {
  if (!s || !out2 || rec >= s->s.n) return IRT_E_INVALID;
  const float *hv = &s->s.hv[(size_t)rec * kHV];
  int32_t nl;
  memcpy(&nl, hv + 63, 4);
  out2[0] = hv[32 + find_height(hv, nl, r)];
  // the kernel's path (irt_render.hip record_value): the quantised coarse keys pick one
  // 64-B block for sorted heights (exact keys near a key), else the literal binary search
  out2[1] = record_value_host(s->s, rec,
                              record_path(s->s.meta[rec], s->s.rng[2 * (size_t)rec],
                                          s->s.rng[2 * (size_t)rec + 1], r), r);
  return IRT_OK;
}

int irt_debug_scene_candidates(const irt_debug_scene *s, irt_vec3f p, uint32_t *records,
                               int capacity) {
  if (!s || s->s.G == 0) return 0;
  const uint32_t cell = cubemap_cell(p.x, p.y, p.z, s->s.G);
  const uint32_t b = s->s.offsets[cell], e = s->s.offsets[cell + 1];
  int k = 0;
  for (uint32_t i = b; i < e; ++i, ++k)
    if (records && k < capacity) records[k] = s->s.entryRec[i];
  return k;
}

int irt_debug_scene_planes(const irt_debug_scene *s, uint32_t record, float *out12) {
  if (!s || !out12 || record >= s->s.n) return IRT_E_INVALID;
  memcpy(out12, &s->s.planes[12 * (size_t)record], 12 * sizeof(float));
  return IRT_OK;
}

void irt_debug_scene_free(irt_debug_scene *s) { delete s; }

int irt_debug_scene_array(const irt_debug_scene *s, int which, void *dst, size_t capacity,
                          size_t *bytes) {
  if (!s || !bytes) {
    set_error("irt_debug_scene_array: null argument");
    return IRT_E_INVALID;
  }
  const HostScene &S = s->s;
  std::vector<uint32_t> rec;
  const void *src = nullptr;
  size_t n = 0;
  switch (which) {
    case IRT_DEBUG_ARRAY_BIN_HDR: src = S.binHdr.data(); n = S.binHdr.size() * 4; break;
    case IRT_DEBUG_ARRAY_FAT: src = S.fat.data(); n = S.fat.size() * 4; break;
    case IRT_DEBUG_ARRAY_BLOCKS: src = S.blocks.data(); n = S.blocks.size() * 4; break;
    case IRT_DEBUG_ARRAY_SPH_R: src = S.sphR.data(); n = S.sphR.size() * 4; break;
    case IRT_DEBUG_ARRAY_SPH_OFF: src = S.sphOff.data(); n = S.sphOff.size() * 4; break;
    case IRT_DEBUG_ARRAY_SPH_REC:
      for (uint32_t r : S.sphRec) {
        int32_t nl;
        memcpy(&nl, &S.hv[(size_t)r * kHV + 63], 4);
        rec.push_back(r);
        rec.push_back((uint32_t)nl);
      }
      src = rec.data();
      n = rec.size() * 4;
      break;
    case IRT_DEBUG_ARRAY_SPH_BITS: src = S.sphBits.data(); n = S.sphBits.size() * 4; break;
    default:
      set_error("irt_debug_scene_array: unknown array %d", which);
      return IRT_E_INVALID;
  }
  *bytes = n;
  if (dst && capacity >= n && n) memcpy(dst, src, n);
  return IRT_OK;
}

int irt_debug_scene_locate_wedge(irt_debug_scene *s, irt_vec3f p, float *value) {
  if (!s || !value) return IRT_E_INVALID;
  if (s->w.G == 0) {
    set_error("irt_debug_scene_locate_wedge: call irt_debug_scene_build_wedges first");
    return IRT_E_INVALID;
  }
  return wedge_locate_host(s->w, s->cells.data(), p.x, p.y, p.z, *value) ? 1 : 0;
}

int irt_debug_scene_build_wedges(irt_debug_scene *s, const irt_icon_cell *cells, size_t n) {
  if (!s || (n && !cells) || n != s->s.n) {
    set_error("irt_debug_scene_build_wedges: cells do not match the scene");
    return IRT_E_INVALID;
  }
  s->cells.assign(cells, cells + n);
  return build_wedges(cells, n, s->w);
}

int irt_debug_scene_locate_triangle(irt_debug_scene *s, irt_vec3f p, float *value,
                                    uint32_t *record) {
  if (!s || !value) return IRT_E_INVALID;
  if (s->w.G == 0) {
    set_error("irt_debug_scene_locate_triangle: call irt_debug_scene_build_wedges first");
    return IRT_E_INVALID;
  }
  return triangle_locate_host(s->w, s->cells.data(), p.x, p.y, p.z, *value, record) ? 1 : 0;
}

int irt_debug_intersect_wedge(const float *v24, irt_vec3f p, float *value) {
  WV4 V[6];
  memcpy(V, v24, sizeof(V));
  float v = 0.f;
  const bool hit = intersect_wedge(v, p.x, p.y, p.z, V);
  if (hit) *value = v;
  return hit ? 1 : 0;
}

}  // extern "C"
