"""Synthetic DWD-ICON-style netCDF inputs for convert_icon tests.

Writes, with scipy.io.netcdf_file (netCDF classic, CDF-1 or CDF-2), the four kinds of
files convert_icon reads (tools/convert_icon/convert_icon.cpp:185-335):
  - the horizontal grid: dims cell, vertex, nv; clon_vertices/clat_vertices (cell, nv), rad;
  - HSURF (cell);
  - one HHL file per half level: height (1) = level index, HHL (time=UNLIMITED?, ncells);
  - one data file per full level: dim ncells, height (1), the variable (default "pres").
Geometry comes from the package's icosahedral generator; heights/values are smooth
synthetic fields (real DWD data is not available offline).
"""
import os

import numpy as np
from scipy.io import netcdf_file

import irt


def write_icon_set(d, bisections=1, levels=6, var="pres", version=2, record_hhl=False,
                   float32_data=False, shuffle=True, seed=3):
    """Returns (hgrid, hsurf, hhl_files, data_files); levels = number of full levels."""
    rng = np.random.default_rng(seed)
    cells = irt.synth_grid(2, bisections, 1)  # one record per column: lat/lon only
    ncell = cells.size
    clat = cells["lat"].astype(np.float64) + rng.normal(0, 1e-9, (ncell, 3))
    clon = cells["lon"].astype(np.float64) + rng.normal(0, 1e-9, (ncell, 3))
    hgrid = os.path.join(d, "grid.nc")
    with netcdf_file(hgrid, "w", version=version) as f:
        f.createDimension("cell", ncell)
        f.createDimension("vertex", ncell // 2 + 2)
        f.createDimension("nv", 3)
        f.title = b"synthetic ICON grid"
        for name, a in (("clon_vertices", clon), ("clat_vertices", clat)):
            v = f.createVariable(name, "d", ("cell", "nv"))
            v[:] = a
            v.units = b"radian"
    cx = np.cos(clat.mean(1)) * np.cos(clon.mean(1))
    cz = np.sin(clat.mean(1))
    hs = np.maximum(0.0, 2500.0 * np.sin(3 * cx) * np.cos(2 * cz)) + rng.uniform(0, 5, ncell)
    hsurf = os.path.join(d, "hsurf.nc")
    with netcdf_file(hsurf, "w", version=version) as f:
        f.createDimension("cell", ncell)
        v = f.createVariable("HSURF", "d", ("cell",))
        v[:] = hs
    # half levels 1..levels+1 (1 = model top); HHL = height above sea level
    hhl_files, data_files = [], []
    top = 75e3
    for lev in range(1, levels + 2):
        eta = 1.0 - (lev - 1) / levels  # 1 at the top, 0 at the surface
        h = hs + (top - hs) * eta ** 2 + rng.uniform(0, 1e-3, ncell)
        p = os.path.join(d, f"hhl_{lev:03d}.nc")
        with netcdf_file(p, "w", version=version) as f:
            if record_hhl:  # the UNLIMITED dimension must come first
                f.createDimension("time", None)
            f.createDimension("ncells", ncell)
            f.createDimension("height", 1)
            hv = f.createVariable("height", "d", ("height",))
            hv[:] = [float(lev)]
            if record_hhl:  # two record variables: padded, interleaved record slabs
                t = f.createVariable("time_flag", "h", ("time",))
                t[0] = 7
                v = f.createVariable("HHL", "d", ("time", "ncells"))
                v[0, :] = h
            else:
                v = f.createVariable("HHL", "d", ("ncells",))
                v[:] = h
        hhl_files.append(p)
    for lev in range(1, levels + 1):
        val = 1e5 * np.exp(-(levels - lev) / 8.0) * (1 + 0.05 * np.sin(5 * cx + lev))
        p = os.path.join(d, f"data_{lev:03d}.nc")
        with netcdf_file(p, "w", version=version) as f:
            f.createDimension("ncells", ncell)
            f.createDimension("height", 1)
            hv = f.createVariable("height", "d", ("height",))
            hv[:] = [float(lev)]
            v = f.createVariable(var, "f" if float32_data else "d", ("ncells",))
            v[:] = val
        data_files.append(p)
    if shuffle:  # the tool sorts by level index itself
        rng.shuffle(hhl_files)
        rng.shuffle(data_files)
    return hgrid, hsurf, hhl_files, data_files
