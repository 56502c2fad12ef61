// irt_convert.cpp -- convert_icon's DWD ICON netCDF -> `.ic` conversion
// (tools/convert_icon/convert_icon.cpp:168-391) over the netCDF-classic reader in
// irt_netcdf.cpp.  Compiled with g++ -ffp-contract=off like the reference tool, and the
// arithmetic keeps the reference's float/double mixing expression by expression.
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "icon_rt_hip.h"
#include "irt_internal.h"
#include "irt_netcdf.h"

using irt::set_error;

namespace {

struct DataField {  // convert_icon.cpp:213-216
  int height = 0;
  std::vector<float> value;
};

// readDoubleVar (convert_icon.cpp:98-118): the whole variable, which must hold len values
int readDoubleVar(const irt_nc::File &f, const char *file, const char *name, size_t len,
                  std::vector<double> &out) {
  const irt_nc::Var *v = f.findVar(name);
  if (!v) {
    set_error("irt_convert_icon: variable %s not found in %s", name, file);
    return IRT_E_DATA;
  }
  if (f.numValues(*v) != len) {
    set_error("irt_convert_icon: variable %s in %s has %llu values, expected %zu", name, file,
              (unsigned long long)f.numValues(*v), len);
    return IRT_E_DATA;
  }
  std::string err;
  if (!f.readDouble(*v, out, err)) {
    set_error("irt_convert_icon: %s", err.c_str());
    return IRT_E_IO;
  }
  return IRT_OK;
}

int openNc(irt_nc::File &f, const char *path) {
  std::string err;
  if (!path || !f.open(path, err)) {
    set_error("irt_convert_icon: %s", path ? err.c_str() : "missing input file");
    return IRT_E_IO;
  }
  return IRT_OK;
}

int readDim(const irt_nc::File &f, const char *file, const char *name, size_t &len) {
  uint64_t l = 0;
  if (!f.dimLength(name, l)) {
    set_error("irt_convert_icon: dim %s not found in %s", name, file);
    return IRT_E_DATA;
  }
  len = (size_t)l;
  return IRT_OK;
}

// One HHL or data file: `height` (level index) + the cell field (convert_icon.cpp:239-335)
int readField(const char *path, const char *varName, bool isData, size_t cell,
              DataField &field) {
  irt_nc::File f;
  int rc;
  if ((rc = openNc(f, path))) return rc;
  size_t n = cell;
  if (isData && (rc = readDim(f, path, "ncells", n))) return rc;  // 292
  if (isData && n < cell) {  // the reference reads var[0..cell) (330-332)
    set_error("irt_convert_icon: %s has %zu cells, the grid %zu", path, n, cell);
    return IRT_E_DATA;
  }
  std::vector<double> height, var;
  if ((rc = readDoubleVar(f, path, "height", 1, height))) return rc;
  field.height = (int)height[0];
  if ((rc = readDoubleVar(f, path, varName, n, var))) return rc;
  if (isData) {  // normalise to [0,1] in double (317-328)
    double minValue(DBL_MAX);
    double maxValue(-DBL_MAX);
    for (size_t j = 0; j < n; ++j) {
      minValue = fmin(minValue, var[j]);
      maxValue = fmax(maxValue, var[j]);
    }
    for (size_t j = 0; j < n; ++j) {
      var[j] -= minValue;
      var[j] /= maxValue - minValue;
    }
  }
  field.value.resize(cell);
  for (size_t j = 0; j < cell; ++j) field.value[j] = (float)var[j];
  return IRT_OK;
}

constexpr int LMAX = 32;  // convert_icon.cpp:351
constexpr uint64_t kUMeshMagic = 0x234235567ull;  // umesh binary files (UMesh::saveTo)

inline int div_up(int a, int b) { return (a + b - 1) / b; }  // 47-49

// The netCDF inputs of both outputs (convert_icon.cpp:168-349)
struct Inputs {
  size_t cell = 0;
  std::vector<double> clon, clat, hsurf;
  std::vector<DataField> hhl, values;
  int numLayers = 0;  // data files, at most maxLayers (345-349)
};

int load_inputs(const irt_convert_opts *o, Inputs &in) {
  if (!o || !o->hgridFile || !o->hsurfFile || o->numHhlFiles <= 0 ||
      (o->numHhlFiles && !o->hhlFiles) || o->numDataFiles < 0 ||
      (o->numDataFiles && !o->dataFiles)) {
    set_error("irt_convert_icon: need -hgrid, -hsurf and -hhl files (convert_icon.cpp:176-181)");
    return IRT_E_INVALID;
  }
  const char *varName = o->varName ? o->varName : "pres";
  const int maxLayers = o->maxLayers > 0 ? o->maxLayers : 5;
  int rc;
  // horizontal grid (187-211)
  size_t &cell = in.cell;
  {
    irt_nc::File f;
    if ((rc = openNc(f, o->hgridFile)) || (rc = readDim(f, o->hgridFile, "cell", cell)))
      return rc;
    if (cell > (size_t)INT32_MAX) {  // cellID * 3 below, and the record's int fields
      set_error("irt_convert_icon: %s: cell dimension %zu too large", o->hgridFile, cell);
      return IRT_E_INVALID;
    }
    if ((rc = readDoubleVar(f, o->hgridFile, "clon_vertices", cell * 3, in.clon)) ||
        (rc = readDoubleVar(f, o->hgridFile, "clat_vertices", cell * 3, in.clat)))
      return rc;
  }
  // HSURF (220-231)
  {
    irt_nc::File f;
    if ((rc = openNc(f, o->hsurfFile)) || (rc = readDoubleVar(f, o->hsurfFile, "HSURF", cell, in.hsurf)))
      return rc;
  }
  // HHL and data files, sorted by level index, descending (236-337)
  in.hhl.resize(o->numHhlFiles);
  in.values.resize(o->numDataFiles);
  for (int i = 0; i < o->numHhlFiles; ++i)
    if ((rc = readField(o->hhlFiles[i], "HHL", false, cell, in.hhl[i]))) return rc;
  for (int i = 0; i < o->numDataFiles; ++i)
    if ((rc = readField(o->dataFiles[i], varName, true, cell, in.values[i]))) return rc;
  // std::sort in the reference: equal level indices (malformed input) have no defined
  // order there; stable here
  auto desc = [](const DataField &a, const DataField &b) { return a.height > b.height; };
  std::stable_sort(in.hhl.begin(), in.hhl.end(), desc);
  std::stable_sort(in.values.begin(), in.values.end(), desc);
  in.numLayers = o->numDataFiles;  // 345-349
  if (in.numLayers > maxLayers) in.numLayers = maxLayers;
  return IRT_OK;
}

}  // namespace

extern "C" int irt_convert_icon(const irt_convert_opts *o, irt_icon_cell *out, size_t capacity,
                                size_t *count) {
  if (!count) {
    set_error("irt_convert_icon: null count");
    return IRT_E_INVALID;
  }
  Inputs in;
  if (int rc = load_inputs(o, in)) return rc;
  const size_t cell = in.cell;
  const std::vector<double> &clon = in.clon, &clat = in.clat, &hsurf = in.hsurf;
  const std::vector<DataField> &hhl = in.hhl, &values = in.values;
  const int numLayers = in.numLayers;
  // records per column and the layers they consume (362-377)
  const int numRecs = div_up(numLayers, LMAX - 1);
  int used = 0;
  for (int i = 0; i < numRecs; ++i) {
    int numLayersLocal = LMAX - 1;
    if ((i + 1) * numLayersLocal > numLayers) numLayersLocal = numLayers % LMAX - 1;
    used += numLayersLocal > 0 ? numLayersLocal : 0;
  }
  if (used > (int)hhl.size() || used > (int)values.size()) {
    set_error("irt_convert_icon: %d layers need %d HHL and data files (have %zu, %zu)",
              numLayers, used, hhl.size(), values.size());
    return IRT_E_DATA;
  }
  const size_t total = cell * (size_t)numRecs;
  *count = total;
  if (!out) return IRT_OK;
  if (capacity < total) {
    set_error("irt_convert_icon: capacity %zu < %zu", capacity, total);
    return IRT_E_INVALID;
  }
  size_t k = 0;
  for (size_t cellID = 0; cellID < cell; ++cellID) {  // 356-389
    float lat[3]{(float)clat[cellID * 3], (float)clat[cellID * 3 + 1], (float)clat[cellID * 3 + 2]};
    float lon[3]{(float)clon[cellID * 3], (float)clon[cellID * 3 + 1], (float)clon[cellID * 3 + 2]};
    constexpr float R = 6.371229E6f;
    int valueIt = 0, hhlIt = 0;
    float prevH = R + hsurf[cellID];
    for (int i = 0; i < numRecs; ++i) {
      int numLayersLocal = LMAX - 1;
      if ((i + 1) * numLayersLocal > numLayers) numLayersLocal = numLayers % LMAX - 1;
      irt_icon_cell &c = out[k++];
      memset(&c, 0, sizeof(c));
      c.height[0] = prevH;
      for (int j = 1; j <= numLayersLocal; ++j) {
        c.height[j] = R + hhl[hhlIt++].value[cellID] - hsurf[cellID];
        prevH = c.height[j];
      }
      for (int j = 0; j < numLayersLocal; ++j) c.value[j] = values[valueIt++].value[cellID];
      memcpy(c.lat, lat, sizeof(lat));
      memcpy(c.lon, lon, sizeof(lon));
      c.numLayers = numLayersLocal;
    }
  }
  return IRT_OK;
}

// The UMesh branch (convert_icon.cpp:393-452): one wedge per (cell, layer j < numLayers),
// six vertices of its own (toCartesian with glibc cosf/sinf, 48-57), bottom and top at
// h1 = R + HSURF*50 for j == 0, else R + (HHL[j] - HSURF)*50, and h2 = R + (HHL[j+1] -
// HSURF)*50 (double arithmetic, rounded to float); all six vertices carry values[j] (the
// reference's "TODO: interpolate").  Written in umesh's binary layout (UMesh::saveTo; the
// umesh library is not part of the reference snapshot): u64 magic, then u64-counted arrays
// -- vertices (3 f32), per-vertex scalars (f32), triangles, quads, tets, pyramids (empty),
// wedges (6 i32), hexes (empty).
extern "C" int irt_convert_icon_umesh(const irt_convert_opts *o, const char *path, size_t *numVertices,
                                      size_t *numWedges) {
  if (!path) {
    set_error("irt_convert_icon_umesh: null path");
    return IRT_E_INVALID;
  }
  Inputs in;
  if (int rc = load_inputs(o, in)) return rc;
  const int numLayers = in.numLayers;
  if (numLayers + 1 > (int)in.hhl.size() || numLayers > (int)in.values.size()) {
    // the reference reads hhl[j+1] and values[j] unchecked (409-412)
    set_error("irt_convert_icon_umesh: %d layers need %d HHL and %d data files (have %zu, %zu)",
              numLayers, numLayers + 1, numLayers, in.hhl.size(), in.values.size());
    return IRT_E_DATA;
  }
  const size_t nw = in.cell * (size_t)numLayers;
  if (nw * 6 > (size_t)INT32_MAX) {  // UMesh::Wedge holds int indices
    set_error("irt_convert_icon_umesh: %zu wedges exceed int vertex indices", nw);
    return IRT_E_INVALID;
  }
  std::vector<float> verts(nw * 18), scalars(nw * 6);
  std::vector<int32_t> wedges(nw * 6);
  size_t w = 0;
  for (size_t cellID = 0; cellID < in.cell; ++cellID) {
    const float lat[3]{(float)in.clat[cellID * 3], (float)in.clat[cellID * 3 + 1], (float)in.clat[cellID * 3 + 2]};
    const float lon[3]{(float)in.clon[cellID * 3], (float)in.clon[cellID * 3 + 1], (float)in.clon[cellID * 3 + 2]};
    constexpr float R = 6.371229E6f;
    constexpr float scale = 50.f;
    for (int j = 0; j < numLayers; ++j, ++w) {
      const float h1 = j == 0 ? R + in.hsurf[cellID] * scale
                              : R + (in.hhl[j].value[cellID] - in.hsurf[cellID]) * scale;
      const float h2 = R + (in.hhl[j + 1].value[cellID] - in.hsurf[cellID]) * scale;
      const float v = in.values[j].value[cellID];
      for (int k = 0; k < 6; ++k) {  // bv1 bv2 bv3 tv1 tv2 tv3
        const float r = k < 3 ? h1 : h2;
        float *x = &verts[(6 * w + k) * 3];
        x[0] = r * cosf(lat[k % 3]) * cosf(lon[k % 3]);
        x[1] = r * cosf(lat[k % 3]) * sinf(lon[k % 3]);
        x[2] = r * sinf(lat[k % 3]);
        scalars[6 * w + k] = v;
        wedges[6 * w + k] = (int32_t)(6 * w + k);
      }
    }
  }
  FILE *f = fopen(path, "wb");
  if (!f) {
    set_error("irt_convert_icon_umesh: cannot write %s", path);
    return IRT_E_IO;
  }
  const uint64_t magic = kUMeshMagic, zero = 0, nv = nw * 6, nw64 = nw;
  bool ok = fwrite(&magic, 8, 1, f) == 1;
  ok = ok && fwrite(&nv, 8, 1, f) == 1 && fwrite(verts.data(), 4, verts.size(), f) == verts.size();
  ok = ok && fwrite(&nv, 8, 1, f) == 1 && fwrite(scalars.data(), 4, scalars.size(), f) == scalars.size();
  for (int k = 0; k < 4 && ok; ++k) ok = fwrite(&zero, 8, 1, f) == 1;  // triangles quads tets pyrs
  ok = ok && fwrite(&nw64, 8, 1, f) == 1 && fwrite(wedges.data(), 4, wedges.size(), f) == wedges.size();
  ok = ok && fwrite(&zero, 8, 1, f) == 1;  // hexes
  ok = (fclose(f) == 0) && ok;
  if (!ok) {
    set_error("irt_convert_icon_umesh: short write to %s", path);
    return IRT_E_IO;
  }
  if (numVertices) *numVertices = (size_t)nv;
  if (numWedges) *numWedges = nw;
  return IRT_OK;
}
