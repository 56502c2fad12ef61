"""Host logic of the product (no GPU): the setup of icon_rt's main() as the C ABI exposes
it, the libm restatements and tables the kernels use, and the cell locator that replaces
the reference's cell location -- each checked against the oracle / golden fixtures."""
import ctypes as C
import os
import tempfile

import numpy as np
import pytest

import irt
import oracle as O
from golden_util import FRAME_FIXTURES, load
from helpers import FRAMING, bits, terrain_cells


@pytest.mark.parametrize("name", FRAME_FIXTURES)
def test_volume_info_tf_camera_match_fixture(name):
    d = load(name)
    cells = d["cells"]
    info = irt.volume_info(cells)
    sb = [info.sphericalBounds.lower.x, info.sphericalBounds.lower.y, info.sphericalBounds.lower.z,
          info.sphericalBounds.upper.x, info.sphericalBounds.upper.y, info.sphericalBounds.upper.z]
    vb = [info.bounds.lower.x, info.bounds.lower.y, info.bounds.lower.z, info.bounds.upper.x,
          info.bounds.upper.y, info.bounds.upper.z]
    assert np.array_equal(bits(sb), bits(d["spherical_bounds"]))
    assert np.array_equal(bits(vb), bits(d["volume_bounds"]))
    assert np.array_equal(bits([info.dataRange.lower, info.dataRange.upper]), bits(d["data_range"]))
    assert np.float32(info.unitDistance) == d["unit_distance"]
    if float(d["opacity_scale"]) == 1.0:  # default-TF fixtures
        lut, vr = irt.default_transfunc((info.dataRange.lower, info.dataRange.upper))
        assert np.array_equal(bits(lut), bits(d["lut"]))
        assert np.array_equal(bits(vr), bits(d["value_range"]))


def test_cameras_match_reference_kats():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "kats.npz"))
    b6 = z["camera_box6"]
    box = irt.Box3(irt.vec3(b6[:3]), irt.vec3(b6[3:]))
    lp = irt.camera_view_all(box, 1, 1)
    assert np.array_equal(bits(lp.camera12()), bits(z["cameras"][0]))
    for spec, ref in zip(z["camera_specs"], z["cameras"][1:]):
        lp = irt.camera_look_at(spec[0:3], spec[3:6], spec[6:9], float(spec[9]), 1, 1)
        assert np.array_equal(bits(lp.camera12()), bits(ref))
    src = z["lut_src"]
    assert np.array_equal(bits(irt.resample_lut(src, 300)), bits(z["lut_300"]))


def test_filter_and_ic_io_roundtrip():
    cells = irt.synth_grid(2, 2, 35)
    for lat, lon in [((-30, 60), (-90, 45)), ((0, 90), (-180, 180)), ((-5, 5), (10, 11))]:
        a = irt.filter_cells(cells, lat, lon)
        b = np.array(cells, copy=True)
        n = O.olib().oracle_filter_cells(b.ctypes.data, b.size, lat[0], lat[1], lon[0], lon[1])
        assert a.size == n and a.tobytes() == b[:n].tobytes()
    with tempfile.TemporaryDirectory() as t:
        p = os.path.join(t, "grid.ic")
        irt.save_ic(p, cells)
        assert os.path.getsize(p) == 284 * cells.size
        back = irt.load_ic(p)
        assert back.tobytes() == cells.tobytes()
        assert irt.load_ic(p, 12).tobytes() == cells[:12].tobytes()  # --num-cells 12


def test_synthetic_grid_shape():
    for rn, bis, L in [(1, 0, 4), (2, 0, 90), (2, 3, 31), (2, 2, 32)]:
        cells = irt.synth_grid(rn, bis, L)
        per_col = (L + 30) // 31
        assert cells.size == 20 * rn * rn * 4 ** bis * per_col
        nl = cells["numLayers"].reshape(-1, per_col)
        assert (nl.sum(1) == L).all() and (nl <= 31).all()
        h = cells["height"].reshape(-1, per_col, 32)
        for r in range(per_col - 1):  # consecutive records share the boundary height
            assert (h[:, r, nl[0, r]] == h[:, r + 1, 0]).all()
        assert cells["value"].max() <= 1.0 and cells["value"].min() >= 0.0


@pytest.mark.parametrize("L", [90, 65, 40])
def test_terrain_grid_follows_convert_icon(L):
    """irt_synth_grid_terrain writes the records convert_icon.cpp:353-391 would: per column the
    first record starts at H[0] = R + HSURF (361), every later height is R + HHL - HSURF (371)
    with HHL - HSURF increasing with height (so H[0] > H[1] on land: the inverted first layer),
    records chain (H[0] of record i = the last height of record i - 1), and the last record holds
    L % 32 - 1 layers (365).  Ocean columns (HSURF = 0) have the flat grid's heights."""
    R = np.float32(6.371229e6)
    t = irt.synth_grid(2, 1, L, terrain=4000.0)
    f = irt.synth_grid(2, 1, L)
    per_col = (L + 30) // 31
    assert t.size == f.size == 20 * 4 * 4 * per_col
    nl = t["numLayers"].reshape(-1, per_col)
    want = [31] * (per_col - 1) + [L % 32 - 1]
    assert (nl == np.array(want)).all()
    h = t["height"].reshape(-1, per_col, 32)
    hs = h[:, 0, 0].astype(np.float64) - float(R)
    land = hs > 0
    assert 0.3 < land.mean() < 0.8 and hs.max() <= 4000.0 and hs.min() >= 0.0
    dz1 = float(f["height"][0][1]) - float(R)  # the first half level above the ground
    steep = hs > dz1 + 1.0
    assert steep.mean() > 0.3
    assert (h[steep, 0, 0] > h[steep, 0, 1]).all()  # the inverted first layer
    for r in range(per_col):
        k = nl[0, r]
        if r:
            assert (h[:, r, 0] == h[:, r - 1, nl[0, r - 1]]).all()
        lo = 1 if r == 0 else 0
        if k > lo:
            assert (np.diff(h[:, r, lo:k + 1], axis=1) > 0).all()
    # ocean columns (H[0] = R): the flat grid's heights (R + z in double, rounded), layer for
    # layer, to within one float step at 6.4e6 m (a coast's HSURF can be far below a metre)
    hf = f["height"].reshape(-1, per_col, 32)
    ocean = ~land
    assert ocean.sum() > 10
    assert (np.abs(h[ocean, 0, :32].astype(np.float64) - hf[ocean, 0, :32]) <= 0.5).all()
    assert t["value"].max() <= 1.0 and t["value"].min() >= 0.0
    # deterministic, and the count-only call agrees
    assert t.tobytes() == irt.synth_grid(2, 1, L, terrain=4000.0).tobytes()


def test_libm_restatements_match_glibc():
    libm = C.CDLL("libm.so.6")
    libm.asinf.restype = libm.atan2f.restype = libm.logf.restype = C.c_float
    libm.asinf.argtypes = [C.c_float]
    libm.atan2f.argtypes = [C.c_float, C.c_float]
    libm.logf.argtypes = [C.c_float]
    L = irt.lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(-1, 1, 30000), [0.0, -0.0, 1.0, -1.0, 0.975, 0.5, 1e-30, -1e-9]]).astype(np.float32)
    for x in xs:
        assert np.float32(L.irt_debug_asinf(float(x))).view(np.uint32) == np.float32(libm.asinf(float(x))).view(np.uint32)
    ys = (rng.normal(size=30000) * 7e6).astype(np.float32)
    xs2 = (rng.normal(size=30000) * 7e6).astype(np.float32)
    ys[:50] = 0
    xs2[50:100] = 0
    for y, x in zip(ys, xs2):
        a, b = L.irt_debug_atan2f(float(y), float(x)), libm.atan2f(float(y), float(x))
        assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32)
    for k in list(range(0, 1 << 24, 9973)) + [0, 1, 2, 12, (1 << 24) - 1]:
        x = np.float32(1.0) - np.float32(k) / np.float32(1 << 24)
        assert np.float32(L.irt_debug_logf_entry(k)).view(np.uint32) == np.float32(libm.logf(float(x))).view(np.uint32)
    # the kernels' logf(1.f - rnd()) is glibc's algorithm restated (irt_common.h): exhaustive
    # over the 2^24 arguments it can take
    assert L.irt_debug_logf_mismatches() == 0
    for f in [0.5, -0.5, 1e10, -1e10, 2147483520.0, 2147483648.0, -2147483648.0, float("nan"), float("inf")]:
        v = L.irt_debug_f2i(f)
        ref = int(f) if np.isfinite(f) and -2147483648.0 <= f < 2147483648.0 else -2147483648
        assert v == ref, f


def test_srgb_thresholds_reproduce_make_8bit():
    """The kernels map accum -> RGBA8 by binary search in 255 host-built thresholds; that
    must equal make_8bit(linear_to_srgb(x)) for every x (checked on a dense sweep and
    around every threshold)."""
    th = np.zeros(256, np.float32)
    irt.lib().irt_debug_srgb_thresholds(th.ctypes.data)
    assert np.all(np.diff(th[1:]) >= 0)
    L = O.olib()

    def ref_byte(x):  # deviceCode.cu:336-340: srgb on rgb, then make_rgba
        c = np.array([L.oracle_linear_to_srgb(x), 0, 0, 0], np.float32)
        return L.oracle_make_rgba(c.ctypes.data) & 0xFF

    def byte(x):
        return int(np.searchsorted(th[1:], np.float32(x), side="right"))
    xs = np.concatenate([np.linspace(-0.1, 1.1, 20001, dtype=np.float32),
                         np.float32([0.0, 0.0031308, 1.0, 2.0, -1.0])])
    for x in xs:
        assert byte(x) == ref_byte(float(x)), x
    for b in range(1, 256):
        t = th[b]
        below = np.nextafter(t, np.float32(-1))
        assert byte(t) == ref_byte(float(t)) and byte(below) == ref_byte(float(below))


@pytest.mark.parametrize("rn,bis,L", [(1, 0, 4), (2, 2, 40), (2, 3, 90)])
def test_locator_is_conservative_and_lowest_index(rn, bis, L):
    """sampleVolume over the cube-map lists == the reference's first-hit linear scan, on
    random points, points exactly on layer boundaries and points on shared triangle
    edges (where neighbouring cells tie and the lower index must win)."""
    cells = irt.synth_grid(rn, bis, L)
    D = irt.DebugScene(cells)
    Lb = O.olib()
    rng = np.random.default_rng(rn * 100 + bis)
    pts = []
    sbl = float(cells["height"][:, 0].min())
    sbu = float(np.max(cells["height"][np.arange(cells.size), cells["numLayers"]]))
    d = rng.normal(size=(400, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pts += list((d * rng.uniform(sbl - 50, sbu + 50, (400, 1))).astype(np.float32))
    for i in rng.choice(cells.size, 60):
        c = cells[i]
        lat, lon = c["lat"].astype(np.float64), c["lon"].astype(np.float64)
        cd = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
        for j in (0, c["numLayers"] // 2, c["numLayers"]):
            v = cd.mean(0)
            pts.append((v / np.linalg.norm(v) * np.float64(c["height"][j])).astype(np.float32))
        for a, b in ((0, 1), (1, 2), (2, 0)):  # edge midpoints and a corner
            v = cd[a] + cd[b]
            pts.append((v / np.linalg.norm(v) * np.float64(c["height"][1])).astype(np.float32))
        pts.append((cd[0] * np.float64(c["height"][2])).astype(np.float32))
    n_hit = 0
    for p in pts:
        hit, v, rec = D.locate(p)
        hb, vb, recb, _ = D.locate_binned(p)  # the render kernel's binned lists
        assert (hb, recb, np.float32(vb)) == (hit, rec, np.float32(v)), p
        val = C.c_float()
        found = None
        for i in range(cells.size):
            if Lb.oracle_sample(cells[i:i + 1].ctypes.data, O.v3(p), C.byref(val)):
                found = (i, np.float32(val.value))
                break
        assert (found is not None) == hit, p
        if hit:
            n_hit += 1
            assert found[0] == rec and found[1] == np.float32(v), p
    assert n_hit > len(pts) // 2


def test_render_record_layout_gives_findheight_value():
    """The state-machine kernel reads findHeight's answer from the render-record layout
    (irt_common.h: coarse keys + one height/value block, or the literal search for
    unsorted columns).  Host evaluation of that path == the literal binary search
    (ICONGrid.h:117-164) at every layer boundary, its float neighbours and random radii,
    for sorted and deliberately unsorted columns of every layer count, and for records whose
    height[0] sits above some of their other heights (convert_icon's inverted first layer)."""
    cells = irt.synth_grid(2, 1, 93)  # records of 31, 31, 31 layers (and a short tail)
    rng = np.random.default_rng(7)
    cells = cells[:400].copy()
    nls = set()
    for i in range(cells.size):
        nl = int(rng.integers(0, 32))
        cells["numLayers"][i] = nl
        nls.add(nl)
        if i % 3 == 0 and nl >= 2:  # unsorted column: swap two interior heights
            a, b = rng.choice(np.arange(1, nl + 1), 2, replace=False)
            h = cells["height"][i]
            h[a], h[b] = h[b], h[a]
        elif i % 3 == 1 and nl >= 2:
            # convert_icon's inverted first layer (H[0] = R + HSURF above H[1..j]): height[0]
            # moved up to (or just past) height[j], so coarse keys fall below it
            j = int(rng.integers(1, nl + 1))
            h = cells["height"][i]
            h[0] = h[j] if i % 2 else np.nextafter(h[j], np.float32(np.inf))
    D = irt.DebugScene(cells)
    checked = 0
    for i in range(cells.size):
        nl = int(cells["numLayers"][i])
        hs = cells["height"][i][:nl + 1].astype(np.float32)
        rs = list(hs) + list(np.nextafter(hs, np.float32(np.inf))) + \
            list(np.nextafter(hs, np.float32(-np.inf))) + \
            list(rng.uniform(hs.min() - 10, hs.max() + 10, 8).astype(np.float32))
        for r in rs:
            if r < hs[0] or r > hs[nl]:
                continue  # sample() rejects it before findHeight (ICONGrid.h:184)
            a, b = D.values(i, float(r))
            assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32), (i, nl, r)
            checked += 1
    assert len(nls) > 25 and checked > 5000


def _norm32(p):
    p = p.astype(np.float32)
    return np.sqrt(np.float32(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]))


def _on_radius(v, r):
    """A float32 point in direction v whose float32 |p| (sqrtf(x*x+y*y+z*z), as
    toSpherical computes it) equals r exactly, when one is found nearby."""
    v = np.asarray(v, np.float64)
    v = v / np.linalg.norm(v)
    r = np.float32(r)
    s = np.float64(r)
    p = (v * s).astype(np.float32)
    for _ in range(64):
        q = _norm32(p)
        if q == r:
            break
        s *= 1 + (float(r) - float(q)) / float(r) * 0.999 + (1e-8 if q < r else -1e-8)
        p = (v * s).astype(np.float32)
    return p


@pytest.mark.parametrize("kind", ["perturbed", "convert_icon"])
def test_binned_locator_on_terrain_following_columns(kind):
    """The binned lists (per-cell radial edges, fat entries) against the brute-force first
    hit on columns whose record boundaries differ from column to column (terrain-following
    levels, like ICON's HHL), records with unsorted heights, zero-thickness records and
    inverted records -- at random radii, exactly on every record boundary and its float
    neighbours.  "convert_icon": the terrain grid as convert_icon writes it (inverted first
    layers over land; 65 levels, so the last record of every column is a zero-thickness
    sphere at the top)."""
    cells = terrain_cells(11) if kind == "perturbed" else irt.synth_grid(2, 1, 65, terrain=4000.0)
    rng = np.random.default_rng(12)
    D = irt.DebugScene(cells)
    Lb = O.olib()
    pts = []
    d = rng.normal(size=(300, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    sbl = float(cells["height"][:, 0].min())
    sbu = float(cells["height"].max())
    pts += list((d * rng.uniform(sbl - 50, sbu + 50, (300, 1))).astype(np.float32))
    for i in rng.choice(cells.size, 80):
        c = cells[i]
        lat, lon = c["lat"].astype(np.float64), c["lon"].astype(np.float64)
        cd = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
        v = cd.mean(0)
        v /= np.linalg.norm(v)
        for hh in (c["height"][0], c["height"][c["numLayers"]]):
            for rr in (hh, np.nextafter(hh, np.float32(np.inf)), np.nextafter(hh, np.float32(0))):
                pts.append(_on_radius(v, rr))
    # a direction far from any column of a zero-thickness record, on its radius exactly
    zt = [i for i in range(cells.size) if cells["height"][i][0] == cells["height"][i][cells["numLayers"][i]]]
    assert zt
    for i in zt[:10]:
        pts.append(_on_radius(rng.normal(size=3), cells["height"][i][0]))
    n_hit = n_sph = n_void = 0
    zt = set(zt)
    for p in pts:
        hb, vb, recb, tested = D.locate_binned(p)
        # outside the radial range of every record that can reach its quad (the header's bounds):
        # decided without a candidate test -- and the brute-force scan below must agree
        n_void += (not hb) and tested == 0
        val = C.c_float()
        found = None
        for i in range(cells.size):
            if Lb.oracle_sample(cells[i:i + 1].ctypes.data, O.v3(p), C.byref(val)):
                found = (i, np.float32(val.value))
                break
        assert (found is not None) == hb, p
        if hb:
            n_hit += 1
            assert found[0] == recb and found[1] == np.float32(vb), (p, found, recb)
            n_sph += found[0] in zt
    assert n_hit > len(pts) // 3 and n_sph >= 3
    # the convert_icon layout's voids over land (tops HSURF below the ocean's) and under it
    assert kind != "convert_icon" or n_void > 20, n_void


# ------------------------------------------------------------------ CUBQL_MODE wedges
def _wedge_lib():
    import ctypes as C
    L = irt.lib()
    P = C.c_void_p
    L.irt_debug_scene_build.argtypes = [P, C.c_size_t, C.POINTER(P)]
    L.irt_debug_scene_build_wedges.argtypes = [P, P, C.c_size_t]
    L.irt_debug_scene_locate_wedge.argtypes = [P, irt.Vec3, C.POINTER(C.c_float)]
    L.irt_debug_intersect_wedge.argtypes = [P, irt.Vec3, C.POINTER(C.c_float)]
    L.irt_debug_scene_free.argtypes = [P]
    return L


def test_product_intersect_wedge_matches_reference_kats():
    """The kernels' intersect_wedge (irt_common.h), host-compiled, vs UElems.h's answers."""
    import ctypes as C
    npz = np.load(os.path.join(os.path.dirname(__file__), "golden", "kats_wedge.npz"))
    z = {k: npz[k] for k in npz.files}  # NpzFile re-reads on every access
    L = _wedge_lib()
    for k in range(len(z["wedge_p"])):
        v = C.c_float(0)
        V = np.ascontiguousarray(z["wedge_v"][k])
        h = L.irt_debug_intersect_wedge(V.ctypes.data, irt.Vec3(*z["wedge_p"][k].tolist()),
                                        C.byref(v))
        assert h == z["wedge_hit"][k], k
        if h:
            assert np.float32(v.value).view(np.uint32) == z["wedge_value"][k].view(np.uint32), k


def test_wedge_locator_matches_reference_scan():
    """The wedge locator irt_build_wedge_accel uploads (cube map of record wedge boxes)
    finds exactly the reference's wedge (first in index order) at the fixture points."""
    import ctypes as C
    npz = np.load(os.path.join(os.path.dirname(__file__), "golden", "kats_wedge.npz"))
    z = {k: npz[k] for k in npz.files}
    cells = np.ascontiguousarray(z["scene_cells"]).view(irt.CELL_DTYPE).ravel()
    L = _wedge_lib()
    h = C.c_void_p()
    assert L.irt_debug_scene_build(cells.ctypes.data, cells.size, C.byref(h)) == 0
    assert L.irt_debug_scene_build_wedges(h, cells.ctypes.data, cells.size) == 0
    for k, p in enumerate(z["scene_points"]):
        v = C.c_float(0)
        hit = L.irt_debug_scene_locate_wedge(h, irt.Vec3(*p.tolist()), C.byref(v))
        assert hit == z["scene_hit"][k], k
        if hit:
            assert np.float32(v.value).view(np.uint32) == z["scene_value"][k].view(np.uint32), k
    L.irt_debug_scene_free(h)


def test_wedge_locator_matches_oracle_on_coarse_and_fine_grids():
    """Locator vs the oracle's brute-force wedge scan, incl. the 20-face icosahedron (boxes
    spanning whole cube faces) and points outside every column."""
    import ctypes as C
    import oracle as O
    L = _wedge_lib()
    rng = np.random.default_rng(4)
    for rn, bis, lev in ((1, 0, 4), (2, 0, 9), (2, 3, 47)):
        cells = irt.synth_grid(rn, bis, lev, noise=0.3)
        h = C.c_void_p()
        assert L.irt_debug_scene_build(cells.ctypes.data, cells.size, C.byref(h)) == 0
        assert L.irt_debug_scene_build_wedges(h, cells.ctypes.data, cells.size) == 0
        for _ in range(400):
            c = cells[rng.integers(cells.size)]
            lat, lon = c["lat"].astype(np.float64), c["lon"].astype(np.float64)
            d = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
            w = rng.dirichlet([1, 1, 1]) * 1.6 - 0.2
            r = rng.uniform(c["height"][0] - 3000, c["height"][c["numLayers"]] + 3000)
            v = w @ d
            p = (v / np.linalg.norm(v) * r).astype(np.float32)
            a, b = C.c_float(0), C.c_float(0)
            h1 = L.irt_debug_scene_locate_wedge(h, irt.Vec3(*p.tolist()), C.byref(a))
            h2 = O.olib().oracle_wedge_sample(O._p(cells), cells.size, O.v3(p), C.byref(b))
            assert h1 == h2
            if h1:
                assert np.float32(a.value).view(np.uint32) == np.float32(b.value).view(np.uint32)
        L.irt_debug_scene_free(h)


# ------------------------------------------------------------------ TRIANGLE_MODE
def test_triangle_locator_matches_oracle_and_cell_sampler():
    """TRIANGLE_MODE (deviceCode.cu:61-76) through the locator vs the oracle's scan over
    every bottom triangle (the same ray_triangle definition; OptiX's test is not available,
    parity unpinned), and against the cell sampler, which it matches away from record
    boundaries."""
    import ctypes as C
    import oracle as O
    L = _wedge_lib()
    L.irt_debug_scene_locate_triangle.argtypes = [C.c_void_p, irt.Vec3, C.POINTER(C.c_float),
                                                  C.POINTER(C.c_uint32)]
    L.irt_debug_scene_locate.argtypes = [C.c_void_p, irt.Vec3, C.POINTER(C.c_float),
                                         C.POINTER(C.c_uint32)]
    rng = np.random.default_rng(8)
    for rn, bis, lev in ((1, 0, 4), (2, 0, 9), (2, 3, 47)):
        cells = irt.synth_grid(rn, bis, lev, noise=0.3)
        h = C.c_void_p()
        assert L.irt_debug_scene_build(cells.ctypes.data, cells.size, C.byref(h)) == 0
        assert L.irt_debug_scene_build_wedges(h, cells.ctypes.data, cells.size) == 0
        same_as_cells = 0
        for _ in range(300):
            c = cells[rng.integers(cells.size)]
            lat, lon = c["lat"].astype(np.float64), c["lon"].astype(np.float64)
            d = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
            w = rng.dirichlet([1, 1, 1]) * 1.4 - 0.13
            r = rng.uniform(c["height"][0] - 3000, c["height"][c["numLayers"]] + 3000)
            v = w @ d
            p = (v / np.linalg.norm(v) * r).astype(np.float32)
            a, b, e = C.c_float(0), C.c_float(0), C.c_float(0)
            rec = C.c_uint32(0)
            h1 = L.irt_debug_scene_locate_triangle(h, irt.Vec3(*p.tolist()), C.byref(a), C.byref(rec))
            h2 = O.olib().oracle_triangle_sample(O._p(cells), cells.size, O.v3(p), C.byref(b))
            assert h1 == h2
            if h1:
                assert np.float32(a.value).view(np.uint32) == np.float32(b.value).view(np.uint32)
            rc = C.c_uint32(0)
            h3 = L.irt_debug_scene_locate(h, irt.Vec3(*p.tolist()), C.byref(e), C.byref(rc))
            if h3 == h1 and (not h1 or e.value == a.value):
                same_as_cells += 1
        assert same_as_cells >= 0.8 * 300, same_as_cells  # chord vs sphere bands differ
        L.irt_debug_scene_free(h)


def test_lcg_jump_equals_sequential_steps():
    """The cooperative Woodcock loop places sample k with the LCG state 2k+1 (or k+1) draws
    ahead through one affine map (irt_common.h lcg_jump); that map must be the n-fold LCG
    step (dvr_course-common-both.h:41-86) for every n the kernel tabulates, on any state."""
    L = irt.lib()
    L.irt_debug_lcg_jump.argtypes = [C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.irt_debug_lcg_jump.restype = None
    rng = np.random.default_rng(3)
    states = [int(v) for v in rng.integers(0, 2**32, 16)] + [0, 1, 2**32 - 1]
    for n in range(256):
        m, a = C.c_uint32(), C.c_uint32()
        L.irt_debug_lcg_jump(n, C.byref(m), C.byref(a))
        for s0 in states:
            s = s0
            for _ in range(n):
                s = (1664525 * s + 1013904223) & 0xFFFFFFFF
            assert (m.value * s0 + a.value) & 0xFFFFFFFF == s, (n, s0)


def test_division_by_a_launch_constant_as_one_double_product():
    """irt_device.h div_uniform: a / b correctly rounded to float equals the float rounding of
    (double)a * (1 / (double)b) -- the kernel's form for the per-launch divisors (transfer
    function and shell-grid scale).  Random operands over many binades, the kernel's
    operand ranges, and special values."""
    rng = np.random.default_rng(7)
    n = 4_000_000
    a = (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-60, 60, n)).astype(np.float32)
    b = (rng.uniform(0.5, 1, n) * 2.0 ** rng.integers(-60, 60, n)).astype(np.float32)
    b[::3] = -b[::3]
    # the kernel's cases: (value - tfLo) / (tfHi - tfLo) and (lat - lo) / (hi - lo)
    a2 = (rng.uniform(-0.1, 1.1, n).astype(np.float32) - np.float32(0.0123))
    b2 = np.full(n, np.float32(np.float32(0.987) - np.float32(0.0123)), np.float32)
    a3 = (rng.uniform(-1.6, 1.6, n).astype(np.float32) - np.float32(-1.5707964))
    b3 = np.full(n, np.float32(np.float32(1.5707964) - np.float32(-1.5707964)), np.float32)
    sp = np.float32([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, 3.0, 1e-30, 7e30])
    a4, b4 = np.meshgrid(sp, sp)
    with np.errstate(all="ignore"):
        for x, y in ((a, b), (a2, b2), (a3, b3), (a4.ravel(), b4.ravel())):
            ref = x / y  # float32 IEEE division
            got = (x.astype(np.float64) * (1.0 / y.astype(np.float64))).astype(np.float32)
            same = (ref.view(np.uint32) == got.view(np.uint32)) | (np.isnan(ref) & np.isnan(got))
            assert same.all(), (x[~same][:4], y[~same][:4])


_RECIP_C = r"""
#include <math.h>
#include <stdint.h>
/* irt_device.h recip_d / div_recip with the hardware estimate of 1/b replaced by the float
   k ulps away from RN(1/b) (v_rcp_f32 is within 1 ulp); returns the mismatches vs a / b. */
long check(const float *a, const float *b, long n, int k) {
  long bad = 0;
  for (long i = 0; i < n; ++i) {
    float r0f = 1.0f / b[i];
    for (int s = 0; s < (k < 0 ? -k : k); ++s) r0f = nextafterf(r0f, k < 0 ? 0.0f : INFINITY);
    const double r0 = (double)r0f;
    const double e = fma(-(double)b[i], r0, 1.0);
    const double r = fma(r0, fma(e, e, e), r0);
    const float got = (float)((double)a[i] * r);
    const float ref = a[i] / b[i];
    if (!(got == ref || (isnan(got) && isnan(ref))) || signbit(got) != signbit(ref)) ++bad;
  }
  return bad;
}
"""


def test_division_through_a_refined_reciprocal(tmp_path):
    """irt_device.h recip_d / div_recip (gen_ray's normalize, boxTest, intersectSphere): a / b
    correctly rounded equals (float)((double)a * r) with r the hardware reciprocal estimate
    refined once cubically in double -- for every estimate within 2 ulps of 1/b, random
    operands over the divisor range recip_ok admits (2^-100..2^100), the kernel's operand
    shapes, quotients that overflow or land in the float subnormal range, and signed zeros."""
    import ctypes
    import subprocess
    src = tmp_path / "recip.c"
    so = tmp_path / "librecip.so"
    src.write_text(_RECIP_C)
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC", "-o", str(so),
                    str(src), "-lm"], check=True)
    lib = ctypes.CDLL(str(so))
    lib.check.restype = ctypes.c_long
    fp = ctypes.POINTER(ctypes.c_float)
    lib.check.argtypes = [fp, fp, ctypes.c_long, ctypes.c_int]
    rng = np.random.default_rng(11)
    n = 1_000_000
    a = (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-126, 127, n)).astype(np.float32)
    b = (rng.uniform(0.5, 1, n) * 2.0 ** rng.integers(-99, 101, n)).astype(np.float32)
    b[::3] = -b[::3]
    # the kernel's shapes: direction components / length, box slabs / direction, sphere roots
    d = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    ln = np.sqrt((d * d).sum(1, dtype=np.float32)).astype(np.float32)
    a2, b2 = d[:, 0].copy(), ln
    a3 = (rng.uniform(-7e6, 7e6, n).astype(np.float32) - np.float32(1.4e7))
    b3 = np.where(np.abs(d[:, 1]) < 1e-5, np.float32(1e-5), d[:, 1]).astype(np.float32)
    a4 = rng.uniform(-1e14, 1e14, n).astype(np.float32)
    b4 = rng.uniform(-2e7, 2e7, n).astype(np.float32)
    a5 = np.float32([0.0, -0.0, 3.4e38, -3.4e38, 1e-45, 1e-38, 1.0, np.inf, np.nan])
    b5 = np.float32([1.0, 1.0, 2.0 ** -99, 2.0 ** -99, 2.0 ** 99, 2.0 ** 90, -(2.0 ** -100), 3.0, 3.0])
    for x, y in ((a, b), (a2, b2), (a3, b3), (a4, b4), (a5, b5)):
        x = np.ascontiguousarray(x, np.float32)
        y = np.ascontiguousarray(y, np.float32)
        for k in (-2, -1, 0, 1, 2):
            assert lib.check(x.ctypes.data_as(fp), y.ctypes.data_as(fp), x.size, k) == 0, (k, x[:3], y[:3])


_ATAN_C = r"""
#include <math.h>
#include <stdint.h>
#include <string.h>
#include "irt_common.h"
static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float bf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
/* irt_common.h glibc_atanf over every stride-th float, glibc_atan2f over n xorshift pairs
   (a quarter with x == 1.0, a quarter of moderate integers): mismatches vs the host glibc */
extern "C" long check(uint32_t stride, long n) {
  long bad = 0;
  for (uint64_t u = 0; u < 0x100000000ull; u += stride) {
    const float x = bf((uint32_t)u), a = irt::glibc_atanf(x), b = atanf(x);
    if (fb(a) != fb(b) && !(isnan(a) && isnan(b))) ++bad;
  }
  uint64_t s = 88172645463325252ull;
  for (long i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    float y = bf((uint32_t)s), x = bf((uint32_t)(s >> 32));
    if (i % 4 == 1) x = 1.0f;
    if (i % 4 == 2) { y = (float)((int32_t)(s & 0xffffff) - 0x800000) * 1.3f; x = (float)((int32_t)(s >> 40) - 0x800000) * 0.7f; }
    const float a = irt::glibc_atan2f(y, x), b = atan2f(y, x);
    if (fb(a) != fb(b) && !(isnan(a) && isnan(b))) ++bad;
  }
  return bad;
}
"""


def test_atanf_reduction_as_one_division_matches_glibc(tmp_path):
    """irt_common.h glibc_atanf reduces its argument with ONE division of selected operands
    (fdlibm's four interval formulas as written) and glibc_atan2f drops fdlibm's x == 1
    shortcut: both still round exactly as the host glibc -- atanf on every 61st float
    (checked once on all 2^32), atan2f on 4 M pairs including x == 1 (once on 2e8)."""
    import ctypes
    import subprocess
    src = tmp_path / "atan.cpp"
    so = tmp_path / "libatan.so"
    src.write_text(_ATAN_C)
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "icon-ray-tracing_amd", "csrc")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC", "-I", csrc,
                    "-o", str(so), str(src), "-lm"], check=True)
    lib = ctypes.CDLL(str(so))
    lib.check.restype = ctypes.c_long
    lib.check.argtypes = [ctypes.c_uint32, ctypes.c_long]
    assert lib.check(61, 4_000_000) == 0
