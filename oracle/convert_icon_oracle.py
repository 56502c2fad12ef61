"""convert_icon_oracle.py -- CPU restatement of the reference's convert_icon `.ic` branch
(TEST INFRASTRUCTURE ONLY; only tests/ may import this).

Follows tools/convert_icon/convert_icon.cpp:168-391 with numpy, reading the netCDF inputs
through scipy.io.netcdf_file -- a reader independent of the product's C++ one
(icon-ray-tracing_amd/host/irt_netcdf.cpp).  Float/double mixing is spelled out per
expression:
  prevH  = (float)(R + hsurf)                       R float, hsurf double      (361)
  H[j]   = (float)((double)(R + hhl_f32) - hsurf)   R + hhl in float first     (371)
  value  = (float)((var - min) / (max - min))       double, fmin/fmax          (317-332)
  numLayersLocal = numLayers % 32 - 1 for the last record of a column          (365)

Parity: the netCDF C library and the reference tool are not buildable here (netcdf.h is
absent), and the reference ships no converted fixtures, so this restatement is *parity
unpinned*: it pins the product converter to the reference's source semantics only.
"""
from __future__ import annotations

import numpy as np
from scipy.io import netcdf_file

CELL_DTYPE = np.dtype(
    [("lat", "<f4", (3,)), ("lon", "<f4", (3,)), ("numLayers", "<i4"),
     ("height", "<f4", (32,)), ("value", "<f4", (32,))], align=False)

LMAX = 32
R = np.float32(6.371229e6)


def _read(path, name):
    with netcdf_file(path, "r", mmap=False) as f:
        return np.array(f.variables[name][:], dtype=np.float64).ravel()


def _dim(path, name):
    with netcdf_file(path, "r", mmap=False) as f:
        n = f.dimensions[name]
        if n is None:  # record dimension: the number of records
            n = f._recs
        return int(n)


def convert(hgrid, hsurf, hhl_files, data_files, var="pres", max_layers=5) -> np.ndarray:
    cell = _dim(hgrid, "cell")
    clon = _read(hgrid, "clon_vertices").reshape(cell, 3)
    clat = _read(hgrid, "clat_vertices").reshape(cell, 3)
    hs = _read(hsurf, "HSURF")
    hhl = []
    for p in hhl_files:  # 239-272
        h = int(np.trunc(_read(p, "height")[0]))
        hhl.append((h, _read(p, "HHL").astype(np.float32)))
    vals = []
    for p in data_files:  # 282-335
        h = int(np.trunc(_read(p, "height")[0]))
        v = _read(p, var)
        mn = np.fmin.reduce(v, initial=np.finfo(np.float64).max)
        mx = np.fmax.reduce(v, initial=-np.finfo(np.float64).max)
        v = (v - mn) / (mx - mn)
        vals.append((h, v[:cell].astype(np.float32)))
    hhl.sort(key=lambda t: -t[0])   # stable, descending (274)
    vals.sort(key=lambda t: -t[0])  # (337)
    num_layers = min(len(data_files), max_layers)
    num_recs = (num_layers + LMAX - 2) // (LMAX - 1)
    out = np.zeros(cell * num_recs, CELL_DTYPE)
    lat32 = clat.astype(np.float32)
    lon32 = clon.astype(np.float32)
    prev = (np.float64(R) + hs).astype(np.float32)
    hit = vit = 0
    for i in range(num_recs):
        nl = LMAX - 1
        if (i + 1) * nl > num_layers:
            nl = num_layers % LMAX - 1
        rec = out[i::num_recs]
        rec["lat"] = lat32
        rec["lon"] = lon32
        rec["numLayers"] = nl
        rec["height"][:, 0] = prev
        for j in range(1, nl + 1):
            hj = ((R + hhl[hit][1]).astype(np.float64) - hs).astype(np.float32)
            hit += 1
            rec["height"][:, j] = hj
            prev = hj
        for j in range(max(nl, 0)):
            rec["value"][:, j] = vals[vit][1]
            vit += 1
        out[i::num_recs] = rec
    return out


def _glibc_trig():
    """cosf/sinf from glibc (the reference tool's toCartesian, convert_icon.cpp:48-57):
    numpy's float32 cos/sin are not glibc's."""
    import ctypes
    m = ctypes.CDLL("libm.so.6")
    for fn in (m.cosf, m.sinf):
        fn.restype = ctypes.c_float
        fn.argtypes = [ctypes.c_float]
    cosf = np.vectorize(lambda x: np.float32(m.cosf(float(x))), otypes=[np.float32])
    sinf = np.vectorize(lambda x: np.float32(m.sinf(float(x))), otypes=[np.float32])
    return cosf, sinf


def convert_umesh(hgrid, hsurf, hhl_files, data_files, var="pres", max_layers=5) -> dict:
    """The UMesh branch (convert_icon.cpp:393-452): per (cell, layer j) six vertices
    bv1..bv3 at h1, tv1..tv3 at h2, every one carrying values[j]; one wedge of their indices.
      h1 = (float)(R + hsurf*50)            j == 0   (double: hsurf is double)  (403-404)
      h1 = (float)(R + (hhl_j - hsurf)*50)  j > 0    (hhl float, promoted)      (404-405)
      h2 = (float)(R + (hhl_{j+1} - hsurf)*50)                                  (406)
      x, y, z = (r*cosf(lat))*cosf(lon), (r*cosf(lat))*sinf(lon), r*sinf(lat)   (48-57)"""
    cell = _dim(hgrid, "cell")
    clat = _read(hgrid, "clat_vertices").reshape(cell, 3).astype(np.float32)
    clon = _read(hgrid, "clon_vertices").reshape(cell, 3).astype(np.float32)
    hs = _read(hsurf, "HSURF")
    hhl = sorted(((int(np.trunc(_read(p, "height")[0])), _read(p, "HHL").astype(np.float32))
                  for p in hhl_files), key=lambda t: -t[0])
    vals = []
    for p in data_files:
        h = int(np.trunc(_read(p, "height")[0]))
        v = _read(p, var)
        mn = np.fmin.reduce(v, initial=np.finfo(np.float64).max)
        mx = np.fmax.reduce(v, initial=-np.finfo(np.float64).max)
        vals.append((h, ((v - mn) / (mx - mn))[:cell].astype(np.float32)))
    vals.sort(key=lambda t: -t[0])
    L = min(len(data_files), max_layers)
    cosf, sinf = _glibc_trig()
    cl, sl, co, so = cosf(clat), sinf(clat), cosf(clon), sinf(clon)
    R64, S64 = float(np.float32(6.371229e6)), 50.0
    verts = np.zeros((cell, L, 6, 3), np.float32)
    scal = np.zeros((cell, L, 6), np.float32)
    for j in range(L):
        h1 = (R64 + hs * S64) if j == 0 else (R64 + (hhl[j][1].astype(np.float64) - hs) * S64)
        h2 = R64 + (hhl[j + 1][1].astype(np.float64) - hs) * S64
        for k in range(6):
            r = (h1 if k < 3 else h2).astype(np.float32)
            c = k % 3
            verts[:, j, k, 0] = (r * cl[:, c]) * co[:, c]
            verts[:, j, k, 1] = (r * cl[:, c]) * so[:, c]
            verts[:, j, k, 2] = r * sl[:, c]
            scal[:, j, k] = vals[j][1]
    n = cell * L
    return {"vertices": verts.reshape(n * 6, 3), "scalars": scal.reshape(n * 6),
            "wedges": np.arange(n * 6, dtype=np.int32).reshape(n, 6)}
