"""Pin the oracle: its restatement must reproduce the reference's own outputs
(tests/golden, generated from /root/reference headers via oracle/_ref) bit for bit."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from golden_util import FRAME_FIXTURES, load, oracle_scene, params
from helpers import bits


@pytest.mark.parametrize("locator", [1, 2], ids=["scan", "dirgrid"])
@pytest.mark.parametrize("name", FRAME_FIXTURES)
def test_frame_fixture(name, locator):
    """Both oracle locators: the reference's scan over precomputed planes (1) and the
    direction-voxel locator of the CPU baseline (2)."""
    d = load(name)
    S = oracle_scene(d)
    # host setup: bounds, shell accelerator, majorants (hostCode.cu:792-808, 299-397)
    assert np.array_equal(bits([S.sb.lower.x, S.sb.lower.y, S.sb.lower.z, S.sb.upper.x,
                                S.sb.upper.y, S.sb.upper.z]), bits(d["spherical_bounds"]))
    assert np.array_equal(bits([S.vb.lower.x, S.vb.lower.y, S.vb.lower.z, S.vb.upper.x,
                                S.vb.upper.y, S.vb.upper.z]), bits(d["volume_bounds"]))
    if "value_ranges" in d:  # shell-mode fixtures carry the shell accelerator
        assert np.array_equal(S.value_ranges, d["value_ranges"])
        assert np.array_equal(bits(S.max_op), bits(d["max_opacities"]))
    assert np.float32(S.unit_distance) == d["unit_distance"]
    W, H = int(d["width"]), int(d["height"])
    accum = np.zeros((H, W, 4), np.float32)
    fb = np.zeros((H, W), np.uint32)
    for k, aid in enumerate(d["accum_ids"]):
        _, _, st = S.render(params(S, d, aid), W, H, accum=accum, fb=fb, threads=4, fast=locator)
        assert st.locate_calls == d["counts"][k][0] and st.samples_found == d["counts"][k][1]
    assert np.array_equal(bits(accum), bits(d["accum"]))
    assert np.array_equal(fb, d["fb"])


@pytest.mark.parametrize("name", ["f2_r2b02_l90"])
def test_literal_sample_mode_matches_fixture(name):
    """The literal sample() (toSpherical incl. the dead asinf/atan2f, corners rebuilt per
    call) gives the same frame as the fast mode the other tests use."""
    d = load(name)
    S = oracle_scene(d)
    W, H = int(d["width"]), int(d["height"])
    a, f, _ = S.render(params(S, d, 0), W, H, rect=(32, 32, 96, 96), threads=8, fast=False)
    assert np.array_equal(bits(a[32:96, 32:96]), bits(d["accum"][32:96, 32:96]))
    assert np.array_equal(f[32:96, 32:96], d["fb"][32:96, 32:96])


@pytest.fixture(scope="module")
def kats():
    return load_kats()


def load_kats():
    z = np.load(O.os.path.join(O.os.path.dirname(O.HERE), "tests", "golden", "kats.npz"))
    d = {k: z[k] for k in z.files}
    d["cells"] = np.ascontiguousarray(d["cells"]).view(O.CELL_DTYPE).ravel()
    return d


def test_kat_lcg(kats):
    L = O.olib()
    for (a, b), ref in zip(kats["lcg_seeds"], kats["lcg"]):
        out = np.zeros(16, np.float32)
        L.oracle_lcg(int(a), int(b), 16, out.ctypes.data)
        assert np.array_equal(bits(out), bits(ref))


def test_kat_sample_and_find_height(kats):
    L = O.olib()
    cells = kats["cells"]
    for p, i, hit, val in zip(kats["sample_points"], kats["sample_cell"], kats["sample_hit"],
                              kats["sample_value"]):
        v = C.c_float(0)
        h = L.oracle_sample(cells[i:i + 1].ctypes.data, O.v3(p), C.byref(v))
        assert h == hit and (not hit or np.float32(v.value) == val)
    assert kats["sample_hit"].sum() > 100
    for i, h, r in zip(kats["fh_cell"], kats["fh_h"], kats["fh_result"]):
        assert L.oracle_find_height(cells[i:i + 1].ctypes.data, float(h)) == r
    for i in range(cells.size):
        b = O.OBox3()
        L.oracle_get_bounds(cells[i:i + 1].ctypes.data, C.byref(b))
        got = [b.lower.x, b.lower.y, b.lower.z, b.upper.x, b.upper.y, b.upper.z]
        assert np.array_equal(bits(got), bits(kats["get_bounds"][i]))


def test_kat_rays_and_sdda(kats):
    L = O.olib()
    dims = kats["sdda_dims"]
    sb6 = kats["sdda_sb6"]
    sb = O.b3(sb6[:3], sb6[3:])
    box = O.b3(kats["box6"][:3], kats["box6"][3:])
    for k, (o, dr) in enumerate(zip(kats["ray_org"], kats["ray_dir"])):
        tn, tf = C.c_float(), C.c_float()
        h = L.oracle_intersect_sphere(O.v3(o), O.v3(dr), 6.4e6, C.byref(tn), C.byref(tf))
        ref = kats["sphere"][k]
        assert h == ref[0] and (not h or (np.float32(tn.value) == ref[1] and np.float32(tf.value) == ref[2]))
        t0, t1 = C.c_float(), C.c_float()
        h = L.oracle_box_test(O.v3(o), O.v3(dr), 0.0, 1e10, box, C.byref(t0), C.byref(t1))
        ref = kats["box_test"][k]
        assert h == ref[0] and np.float32(t0.value) == ref[1] and np.float32(t1.value) == ref[2]
        leaf = np.full(2048, -1, np.int32)
        a0 = np.zeros(2048, np.float32)
        a1 = np.zeros(2048, np.float32)
        n = L.oracle_sdda_trace(O.v3(o), O.v3(dr), 0.0, 1e10, dims.ctypes.data, sb, 2048,
                                leaf.ctypes.data, a0.ctypes.data, a1.ctypes.data)
        assert n == kats["sdda_count"][k]
        m = min(n, 2048)
        assert np.array_equal(leaf[:m], kats["sdda_leaf"][k][:m])
        assert np.array_equal(bits(a0[:m]), bits(kats["sdda_t0"][k][:m]))
        assert np.array_equal(bits(a1[:m]), bits(kats["sdda_t1"][k][:m]))
    assert (kats["sdda_count"] > 0).sum() > 50


def test_kat_shading_and_spherical(kats):
    L = O.olib()
    srgb = np.array([L.oracle_linear_to_srgb(float(x)) for x in kats["srgb_x"]], np.float32)
    assert np.array_equal(bits(srgb), bits(kats["srgb"]))
    rgba = np.array([L.oracle_make_rgba(c.ctypes.data) for c in kats["rgba_in"]], np.uint32)
    assert np.array_equal(rgba, kats["rgba"])
    for c, ref in zip(kats["cart"], kats["to_spherical"]):
        o = O.OVec3()
        L.oracle_to_spherical(O.v3(c), C.byref(o))
        assert np.array_equal(bits([o.x, o.y, o.z]), bits(ref))
    for s, ref in zip(kats["sph"], kats["to_cartesian"]):
        o = O.OVec3()
        L.oracle_to_cartesian(O.v3(s), C.byref(o))
        assert np.array_equal(bits([o.x, o.y, o.z]), bits(ref))


def test_kat_lut_and_camera(kats):
    L = O.olib()
    src = kats["lut_src"]
    dst = np.zeros((300, 4), np.float32)
    L.oracle_resample_lut(src.ctypes.data, src.shape[0], dst.ctypes.data, 300)
    assert np.array_equal(bits(dst), bits(kats["lut_300"]))
    box = O.b3(kats["camera_box6"][:3], kats["camera_box6"][3:])
    out = (O.OVec3 * 4)()
    L.oracle_camera_view_all(box, 90.0, 1.0, C.cast(out, C.c_void_p))
    got = [v for o in out for v in (o.x, o.y, o.z)]
    assert np.array_equal(bits(got), bits(kats["cameras"][0]))
    for spec, ref in zip(kats["camera_specs"], kats["cameras"][1:]):
        L.oracle_camera_orient(O.v3(spec[0:3]), O.v3(spec[3:6]), O.v3(spec[6:9]), float(spec[9]),
                               1.0, C.cast(out, C.c_void_p))
        got = [v for o in out for v in (o.x, o.y, o.z)]
        assert np.array_equal(bits(got), bits(ref))


# ------------------------------------------------------------------ GRID_ACCEL_MODE
@pytest.fixture(scope="module")
def kats_grid():
    z = np.load(O.os.path.join(O.os.path.dirname(O.HERE), "tests", "golden", "kats_grid.npz"))
    d = {k: z[k] for k in z.files}
    d["grid_cells"] = np.ascontiguousarray(d["grid_cells"]).view(O.CELL_DTYPE).ravel()
    return d


def test_kat_dda3(kats_grid):
    """dda3 (DDA.h:35-136) leaf sequences, incl. the g++ `int min(int, int)` resolution of
    `min(reduce_min(tnext), ray.tmax)`, ragged grids and tmin > 0."""
    d = kats_grid
    L = O.olib()
    maxo = d["dda3_leaf"].shape[1]
    for k in range(len(d["dda3_org"])):
        leaf = np.full(maxo, -1, np.int32)
        t0 = np.zeros(maxo, np.float32)
        t1 = np.zeros(maxo, np.float32)
        wb = d["dda3_wb6"]
        n = L.oracle_dda3_trace(O.v3(d["dda3_org"][k]), O.v3(d["dda3_dir"][k]),
                                float(d["dda3_tmin"][k]), float(d["dda3_tmax"][k]),
                                O._p(np.ascontiguousarray(d["dda3_dims"][k])), O.b3(wb[:3], wb[3:]),
                                maxo, O._p(leaf), O._p(t0), O._p(t1))
        assert n == d["dda3_count"][k], k
        m = min(n, maxo)
        assert np.array_equal(leaf[:m], d["dda3_leaf"][k][:m]), k
        assert np.array_equal(bits(t0[:m]), bits(d["dda3_t0"][k][:m])), k
        assert np.array_equal(bits(t1[:m]), bits(d["dda3_t1"][k][:m])), k


def test_kat_grid_build_and_majorants(kats_grid):
    """buildGrid_ICON + computeMaxOpacities(Grid) (hostCode.cu:205-297, 398-432) over the
    256^3 grid: full digest plus sampled entries."""
    import hashlib
    d = kats_grid
    S = O.OracleScene(d["grid_cells"])
    assert np.array_equal(bits([S.vb.lower.x, S.vb.lower.y, S.vb.lower.z, S.vb.upper.x,
                                S.vb.upper.y, S.vb.upper.z]), bits(d["grid_vb6"]))
    vr = S.build_grid()
    assert np.array_equal(bits(vr[d["grid_pick"]]), bits(d["grid_pick_vr"]))
    assert int((vr[:, 1] >= vr[:, 0]).sum()) == int(d["grid_nonempty"])
    assert hashlib.sha256(vr.tobytes()).digest() == d["grid_sha256"].tobytes()
    S.set_transfunc(d["grid_lut"], tuple(float(v) for v in d["grid_value_range"]), 1.0)
    assert np.array_equal(bits(S.grid_max_op[d["grid_pick"]]), bits(d["grid_pick_maxop"]))
    assert hashlib.sha256(S.grid_max_op.tobytes()).digest() == d["grid_maxop_sha256"].tobytes()


# ------------------------------------------------------------------ CUBQL_MODE wedges
@pytest.fixture(scope="module")
def kats_wedge():
    z = np.load(O.os.path.join(O.os.path.dirname(O.HERE), "tests", "golden", "kats_wedge.npz"))
    d = {k: z[k] for k in z.files}
    d["scene_cells"] = np.ascontiguousarray(d["scene_cells"]).view(O.CELL_DTYPE).ravel()
    return d


def test_kat_intersect_wedge(kats_wedge):
    """intersectWedgeEXT (UElems.h:214-311): hit and interpolated value, bit for bit, for
    unit-scale prisms and Earth-scale ICON wedges (where the float Newton often fails to
    converge -- the reference's behaviour, kept)."""
    d = kats_wedge
    L = O.olib()
    for k in range(len(d["wedge_p"])):
        v = C.c_float(0)
        V = np.ascontiguousarray(d["wedge_v"][k])
        h = L.oracle_intersect_wedge(O._p(V), O.v3(d["wedge_p"][k]), C.byref(v))
        assert h == d["wedge_hit"][k], k
        if h:
            assert bits([v.value])[0] == bits([d["wedge_value"][k]])[0], k


def test_kat_wedge_sample_volume(kats_wedge):
    """CUBQL_MODE sampleVolume (deviceCode.cu:90-115) over buildCuBQLAccel's wedges."""
    d = kats_wedge
    L = O.olib()
    cells = d["scene_cells"]
    for k in range(0, len(d["scene_points"]), 4):
        v = C.c_float(0)
        h = L.oracle_wedge_sample(O._p(cells), cells.size, O.v3(d["scene_points"][k]), C.byref(v))
        assert h == d["scene_hit"][k], k
        if h:
            assert bits([v.value])[0] == bits([d["scene_value"][k]])[0], k


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref not built (needs /root/reference)")
def test_reference_pixel_list_render_matches_oracle():
    """bench.py's CPU baseline runs the reference's own raygen (oracle/_ref) over a strided
    pixel list on several threads; it must equal the oracle pixel for pixel."""
    import irt
    cells = irt.synth_grid(2, 2, 30)
    S = O.OracleScene(cells)
    lut, vr = S.default_lut()
    S.set_transfunc(lut, vr)
    W = 64
    p = S.params(S.camera(W, W, irt.FRAMING_CAMERA))
    ys, xs = np.mgrid[0:W:3, 1:W:3]
    xy = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    a1, f1, cnt = O.ref_render_pixels(S, p, W, W, xy, threads=4)
    a2, f2, st = S.render_pixels(p, W, W, xy, threads=4, fast=False)
    assert np.array_equal(bits(a1), bits(a2)) and np.array_equal(f1, f2)
    assert int(cnt[0]) == st.locate_calls and int(cnt[1]) == st.samples_found


def test_dirgrid_locator_matches_scan_on_degenerate_scenes():
    """The CPU baseline's locator (oracle fast=2) == the reference's scan on scenes with
    cone-mode triangles, terrain, unsorted/zero-thickness/inverted records."""
    import irt
    from helpers import FRAMING, terrain_cells
    for cells, W in ((irt.synth_grid(1, 0, 4), 64), (terrain_cells(11), 80),
                     (irt.synth_grid(2, 3, 47, noise=0.2), 64)):
        S = O.OracleScene(cells)
        lut, vr = S.default_lut()
        S.set_transfunc(lut, vr)
        for cam in (FRAMING, None):
            p = S.params(S.camera(W, W, cam))
            a1, f1, s1 = S.render(p, W, W, threads=4, fast=1)
            a2, f2, s2 = S.render(p, W, W, threads=4, fast=2)
            assert np.array_equal(bits(a1), bits(a2)) and np.array_equal(f1, f2)
            assert (s1.locate_calls, s1.samples_found) == (s2.locate_calls, s2.samples_found)
