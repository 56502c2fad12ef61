"""convert_icon (tools/convert_icon/convert_icon.cpp:168-391): the product's C++ converter
and netCDF-classic reader (irt_convert_icon, host/irt_convert.cpp + host/irt_netcdf.cpp)
against the numpy restatement in oracle/convert_icon_oracle.py, which reads the same files
through scipy's independent netCDF reader.  Bit-exact on every record byte.

Parity note: the reference tool needs the netCDF C library (absent here) and ships no
converted fixtures, so this path is "parity unpinned" beyond the reference's source
semantics."""
import os
import subprocess

import numpy as np
import pytest

import convert_icon_oracle as CO
import irt
from icon_nc import write_icon_set

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "icon-ray-tracing_amd", "convert_icon")


def same_records(a, b):
    assert a.shape == b.shape
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))


def got_hsurf(hs):
    from scipy.io import netcdf_file
    with netcdf_file(hs, "r", mmap=False) as f:
        return np.array(f.variables["HSURF"][:], np.float64)


CASES = [
    # (levels, max_layers, expected numLayers per record) -- convert_icon.cpp:345-366
    (6, 5, [4]),        # defaults: maxLayers 5 -> `5 % 32 - 1` = 4 layers written
    (31, 31, [31]),
    (33, 40, [31, 0]),  # numLayers % 32 == 1: a zero-thickness second record
    (40, 40, [31, 7]),  # the last record gets 40 % 32 - 1 = 7, not the remaining 9
    (62, 90, [31, 31]),
]


@pytest.mark.parametrize("levels,max_layers,expect", CASES)
def test_convert_matches_restatement(tmp_path, levels, max_layers, expect):
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=levels)
    got = irt.convert_icon(hg, hs, hhl, data, max_layers=max_layers)
    ref = CO.convert(hg, hs, hhl, data, max_layers=max_layers)
    assert same_records(got, ref)
    ncol = got.size // len(expect)
    assert list(got["numLayers"][:len(expect)]) == expect
    assert got.size == ncol * len(expect)
    # columns are contiguous bottom-to-top stacks
    h = got["height"]
    nl = got["numLayers"]
    if len(expect) > 1 and expect[1] > 0:
        assert np.array_equal(h[1::2, 0], h[0::2, 30 + 1])
    # H[0] = R + HSURF but H[j] = R + HHL - HSURF (361 vs 371): with HHL at the surface
    # equal to HSURF the first layer is inverted by HSURF; above it the stack ascends
    assert np.all(np.diff(h[0, 1:nl[0] + 1]) > 0)
    first = h[::len(expect)]  # each column's first record
    assert np.allclose(first[:, 1], 6.371229e6)
    assert np.allclose(first[:, 0] - first[:, 1], got_hsurf(hs), atol=1.0)


def test_convert_classic_cdf1_record_dims_and_float_data(tmp_path):
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=8, version=1, record_hhl=True,
                                       float32_data=True)
    got = irt.convert_icon(hg, hs, hhl, data, max_layers=8)
    ref = CO.convert(hg, hs, hhl, data, max_layers=8)
    assert same_records(got, ref)
    assert got["numLayers"][0] == 7


def test_convert_other_variable_name(tmp_path):
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=5, var="t")
    got = irt.convert_icon(hg, hs, hhl, data, var="t")
    assert same_records(got, CO.convert(hg, hs, hhl, data, var="t"))
    with pytest.raises(irt.IrtError, match="variable pres not found"):
        irt.convert_icon(hg, hs, hhl, data)


def test_convert_errors(tmp_path):
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=6)
    h5 = tmp_path / "hdf5.nc"
    h5.write_bytes(b"\x89HDF\r\n\x1a\n" + bytes(64))
    with pytest.raises(irt.IrtError, match="netCDF-4/HDF5"):
        irt.convert_icon(str(h5), hs, hhl, data)
    junk = tmp_path / "junk.nc"
    junk.write_bytes(b"CDF\x02" + bytes(3))
    with pytest.raises(irt.IrtError, match="truncated or malformed"):
        irt.convert_icon(str(junk), hs, hhl, data)
    with pytest.raises(irt.IrtError, match="need 4 HHL"):  # reference reads out of bounds
        irt.convert_icon(hg, hs, hhl[:2], data)
    with pytest.raises(irt.IrtError, match="HSURF"):
        irt.convert_icon(hg, hg, hhl, data)
    with pytest.raises(irt.IrtError, match="cannot open"):
        irt.convert_icon(hg, str(tmp_path / "missing.nc"), hhl, data)


def test_convert_tool_writes_loadable_ic(tmp_path):
    """The convert_icon CLI (same flags as the reference) -> .ic -> irt_load_ic -> the
    scene facts icon_rt's main() derives."""
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=12)
    base = str(tmp_path / "out")
    r = subprocess.run([TOOL, "-hgrid", hg, "-hsurf", hs, "-hhl", *hhl, "-data", *data,
                        "-o", base, "--max-layers", "12"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert not os.path.exists(base + ".umesh")  # the UMesh branch only with --umesh
    cells = irt.load_ic(base + ".ic")
    assert same_records(cells, CO.convert(hg, hs, hhl, data, max_layers=12))
    info = irt.volume_info(cells)
    assert info.dataRange.lower == 0.0 and info.dataRange.upper <= 1.0
    assert 6.371e6 < info.sphericalBounds.lower.x < info.sphericalBounds.upper.x < 6.45e6
    r = subprocess.run([TOOL, "-hgrid", hg], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stderr


def _cdf5(path, dims, variables):
    """A minimal CDF-5 header: dims [(name, length)], variables [(name, [dim index])] of
    doubles with no data behind them (the reader must not trust the header's sizes)."""
    import struct

    def name(s):
        b = s.encode()
        return struct.pack(">Q", len(b)) + b + bytes((4 - len(b) % 4) % 4)

    out = b"CDF\x05" + struct.pack(">Q", 1)
    out += struct.pack(">IQ", 0x0A, len(dims))
    for n, length in dims:
        out += name(n) + struct.pack(">Q", length)
    out += struct.pack(">IQ", 0, 0)  # no global attributes
    out += struct.pack(">IQ", 0x0B, len(variables))
    for n, ids in variables:
        out += name(n) + struct.pack(">Q", len(ids)) + b"".join(struct.pack(">Q", i) for i in ids)
        out += struct.pack(">IQ", 0, 0) + struct.pack(">IQQ", 6, 8, 4096)  # NC_DOUBLE, vsize, begin
    path.write_bytes(out + bytes(64))
    return str(path)


def test_convert_rejects_crafted_header_sizes(tmp_path):
    """header dimension products that wrap 64 bits, or claim more bytes than
    the file holds, fail cleanly instead of sizing a buffer from a wrapped product."""
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=6)
    verts = [("clon_vertices", [0, 1]), ("clat_vertices", [0, 1])]
    wrap = _cdf5(tmp_path / "wrap.nc", [("cell", 3), ("nv", (1 << 63) + 1)], verts)
    with pytest.raises(irt.IrtError, match="expected 9"):
        irt.convert_icon(wrap, hs, hhl, data)
    big = _cdf5(tmp_path / "big.nc", [("cell", 1 << 20), ("nv", 3)], verts)
    with pytest.raises(irt.IrtError, match="larger than the file"):
        irt.convert_icon(big, hs, hhl, data)
    huge = _cdf5(tmp_path / "huge.nc", [("cell", 1 << 40), ("nv", 3)], verts)
    with pytest.raises(irt.IrtError, match="too large"):
        irt.convert_icon(huge, hs, hhl, data)


@pytest.mark.parametrize("levels,max_layers", [(6, 5), (8, 3), (31, 31)])
def test_umesh_matches_restatement(tmp_path, levels, max_layers):
    """The UMesh branch (convert_icon.cpp:393-452) vs the numpy restatement: vertex and
    scalar bits, wedge indices, the file layout (parity unpinned: umesh is absent)."""
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=levels)
    out = str(tmp_path / "o.umesh")
    nv, nw = irt.convert_icon_umesh(hg, hs, hhl, data, out, max_layers=max_layers)
    got = irt.read_umesh(out)
    ref = CO.convert_umesh(hg, hs, hhl, data, max_layers=max_layers)
    assert got["magic"] == 0x234235567
    assert nw == ref["wedges"].shape[0] and nv == 6 * nw
    assert np.array_equal(got["vertices"].view(np.uint32), ref["vertices"].view(np.uint32))
    assert np.array_equal(got["scalars"].view(np.uint32), ref["scalars"].view(np.uint32))
    assert np.array_equal(got["wedges"], ref["wedges"])
    for k in ("triangles", "quads", "tets", "pyrs", "hexes"):
        assert got[k].shape[0] == 0
    # bottom below top where HHL ascends past the surface layer
    v = got["vertices"].reshape(nw, 6, 3).astype(np.float64)
    assert np.all(np.linalg.norm(v[:, 3:], axis=2) > 0)


def test_umesh_needs_one_more_hhl_level(tmp_path):
    """hhl[j+1] for every layer j < numLayers (convert_icon.cpp:406): one HHL file short is
    an error here, an out-of-bounds read in the reference."""
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=6)
    with pytest.raises(irt.IrtError):
        irt.convert_icon_umesh(hg, hs, hhl[:5], data, str(tmp_path / "x.umesh"), max_layers=5)


def test_umesh_cli(tmp_path):
    hg, hs, hhl, data = write_icon_set(str(tmp_path), levels=6)
    base = str(tmp_path / "cli")
    r = subprocess.run([TOOL, "-hgrid", hg, "-hsurf", hs, "-hhl", *hhl, "-data", *data, "-o", base,
                        "--umesh", "--no-ic"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = irt.read_umesh(base + ".umesh")
    ref = CO.convert_umesh(hg, hs, hhl, data)
    assert np.array_equal(got["vertices"].view(np.uint32), ref["vertices"].view(np.uint32))
    assert not os.path.exists(base + ".ic")
