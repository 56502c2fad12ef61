"""oracle.py -- Python binding of the CPU ORACLE (TEST INFRASTRUCTURE ONLY).

Loads oracle/liboracle.so (the C++ restatement, icon_oracle.cpp) and, when present,
oracle/_ref/libiconref.so (built from the reference's own headers, ref_harness.cpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libiconref.so")

CELL_DTYPE = np.dtype(
    [("lat", "<f4", (3,)), ("lon", "<f4", (3,)), ("numLayers", "<i4"),
     ("height", "<f4", (32,)), ("value", "<f4", (32,))], align=False)


class OVec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class OBox3(C.Structure):
    _fields_ = [("lower", OVec3), ("upper", OVec3)]


class OParams(C.Structure):
    _fields_ = [("org", OVec3), ("dir_00", OVec3), ("dir_du", OVec3), ("dir_dv", OVec3),
                ("accumID", C.c_int32), ("ambientColor", OVec3), ("ambientRadiance", C.c_float),
                ("unitDistance", C.c_float), ("raygen", C.c_int32), ("bounds", OBox3),
                ("dims", C.c_int32 * 3), ("sphericalBounds", OBox3),
                ("maxOpacities", C.c_void_p), ("tf_lower", C.c_float), ("tf_upper", C.c_float),
                ("opacityScale", C.c_float), ("lut", C.c_void_p), ("lut_size", C.c_int32),
                ("accelMode", C.c_int32), ("gridDims", C.c_int32 * 3), ("gridBounds", OBox3),
                ("gridMaxOpacities", C.c_void_p), ("mode", C.c_int32)]


class OStats(C.Structure):
    _fields_ = [("rays_launched", C.c_uint64), ("rays_in_box", C.c_uint64),
                ("locate_calls", C.c_uint64), ("samples_found", C.c_uint64),
                ("rng_draws", C.c_uint64), ("leaves", C.c_uint64)]

    def asdict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


def v3(a) -> OVec3:
    return OVec3(float(a[0]), float(a[1]), float(a[2]))


def b3(lo, hi) -> OBox3:
    return OBox3(v3(lo), v3(hi))


def build(ref: bool = False):
    subprocess.check_call(["make", "-s", "-C", HERE] + (["ref"] if ref else []))


_O = None
_R = None


def olib() -> C.CDLL:
    global _O
    if _O is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = C.CDLL(ORACLE_SO)
        P, I, F, S = C.c_void_p, C.c_int, C.c_float, C.c_size_t
        L.oracle_filter_cells.argtypes = [P, S, F, F, F, F]
        L.oracle_filter_cells.restype = S
        L.oracle_compute_bounds.argtypes = [P, S, C.POINTER(OBox3), C.POINTER(OBox3), P]
        L.oracle_unit_distance.argtypes = [F]
        L.oracle_unit_distance.restype = F
        L.oracle_default_lut5.argtypes = [P]
        L.oracle_resample_lut.argtypes = [P, I, P, I]
        L.oracle_camera_view_all.argtypes = [OBox3, F, F, P]
        L.oracle_camera_orient.argtypes = [OVec3, OVec3, OVec3, F, F, P]
        L.oracle_build_shell.argtypes = [P, S, P, OBox3, P]
        L.oracle_max_opacities.argtypes = [P, S, P, I, F, F, P]
        L.oracle_clear.argtypes = [P, P, S]
        L.oracle_render.argtypes = [P, S, C.POINTER(OParams), I, I, I, I, I, I, P, P, I, I,
                                    C.POINTER(OStats)]
        L.oracle_render.restype = I
        L.oracle_render_pixels.argtypes = [P, S, C.POINTER(OParams), I, I, P, I, P, P, I, I,
                                           C.POINTER(OStats)]
        L.oracle_render_pixels.restype = I
        L.oracle_lcg.argtypes = [C.c_uint32, C.c_uint32, I, P]
        L.oracle_sample.argtypes = [P, OVec3, C.POINTER(C.c_float)]
        L.oracle_find_height.argtypes = [P, F]
        L.oracle_intersect_sphere.argtypes = [OVec3, OVec3, F, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.oracle_box_test.argtypes = [OVec3, OVec3, F, F, OBox3, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.oracle_sdda_trace.argtypes = [OVec3, OVec3, F, F, P, OBox3, I, P, P, P]
        L.oracle_dda3_trace.argtypes = [OVec3, OVec3, F, F, P, OBox3, I, P, P, P]
        L.oracle_build_grid.argtypes = [P, S, P, OBox3, P]
        L.oracle_intersect_wedge.argtypes = [P, OVec3, C.POINTER(C.c_float)]
        L.oracle_wedge_sample.argtypes = [P, S, OVec3, C.POINTER(C.c_float)]
        L.oracle_triangle_sample.argtypes = [P, S, OVec3, C.POINTER(C.c_float)]
        L.oracle_linear_to_srgb.argtypes = [F]
        L.oracle_linear_to_srgb.restype = F
        L.oracle_make_rgba.argtypes = [P]
        L.oracle_make_rgba.restype = C.c_uint32
        L.oracle_to_spherical.argtypes = [OVec3, C.POINTER(OVec3)]
        L.oracle_to_cartesian.argtypes = [OVec3, C.POINTER(OVec3)]
        L.oracle_get_bounds.argtypes = [P, C.POINTER(OBox3)]
        L.oracle_post_classify.argtypes = [P, I, F, F, F, F, P]
        _O = L
    return _O


def have_ref() -> bool:
    return os.path.exists(REF_SO)


def rlib() -> C.CDLL:
    global _R
    if _R is None:
        L = C.CDLL(REF_SO)
        P, I, F = C.c_void_p, C.c_int, C.c_float
        L.ref_render.argtypes = [P, I, P, I, P, F, I, P, P, P, P, P, P, I, I, I, I, I, I, I, P, P,
                                 I, P]
        L.ref_render_pixels.argtypes = [P, I, P, I, P, F, I, P, P, P, P, P, P, I, I, I, P, I,
                                        P, P, P]
        L.ref_compute_bounds.argtypes = [P, I, P, P, P]
        L.ref_build_shell.argtypes = [P, I, P, P, P]
        L.ref_max_opacities.argtypes = [P, C.c_long, P, I, F, F, P]
        L.ref_resample_lut.argtypes = [P, I, P, I]
        L.ref_camera.argtypes = [I, P, P, F, P]
        L.ref_lcg.argtypes = [C.c_uint, C.c_uint, I, P]
        L.ref_sample.argtypes = [P, P, C.POINTER(C.c_float)]
        L.ref_find_height.argtypes = [P, F]
        L.ref_intersect_sphere.argtypes = [P, P, F, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.ref_box_test.argtypes = [P, P, F, F, P, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.ref_sdda_trace.argtypes = [P, P, F, F, P, P, I, P, P, P]
        L.ref_dda3_trace.argtypes = [P, P, F, F, P, P, I, P, P, P]
        L.ref_build_grid.argtypes = [P, I, P, P, P]
        L.ref_set_accel.argtypes = [I, P, P, P]
        L.ref_set_sampler.argtypes = [I, P, I]
        L.ref_intersect_wedge.argtypes = [P, P, C.POINTER(C.c_float)]
        L.ref_wedge_sample.argtypes = [P, I, P, C.POINTER(C.c_float)]
        L.ref_linear_to_srgb.argtypes = [F]
        L.ref_linear_to_srgb.restype = F
        L.ref_make_rgba.argtypes = [P]
        L.ref_make_rgba.restype = C.c_uint
        L.ref_to_spherical.argtypes = [P, P]
        L.ref_to_cartesian.argtypes = [P, P]
        L.ref_get_bounds.argtypes = [P, P]
        L.ref_generate_ray.argtypes = [P, I, I, C.c_uint, C.c_uint, P]
        _R = L
    return _R


def _p(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


# ----------------------------------------------------------------------- scene setup
class OracleScene:
    """Host setup of hostCode.cu:792-840 + shell accelerator, on the oracle."""

    DIMS = (1, 1024, 1024)

    def __init__(self, cells: np.ndarray):
        self.cells = np.ascontiguousarray(cells, dtype=CELL_DTYPE)
        L = olib()
        sb, vb = OBox3(), OBox3()
        dr = np.zeros(2, dtype=np.float32)
        L.oracle_compute_bounds(_p(self.cells), self.cells.size, C.byref(sb), C.byref(vb), _p(dr))
        self.sb, self.vb, self.data_range = sb, vb, (float(dr[0]), float(dr[1]))
        self.unit_distance = L.oracle_unit_distance(sb.lower.x)
        self.dims = np.array(self.DIMS, dtype=np.int32)
        self.num_mcs = int(np.prod(self.DIMS))
        self.value_ranges = np.zeros((self.num_mcs, 2), dtype=np.float32)
        L.oracle_build_shell(_p(self.cells), self.cells.size, _p(self.dims), sb,
                             _p(self.value_ranges))
        self.max_op = np.zeros(self.num_mcs, dtype=np.float32)
        self.lut = None
        self.grid_vr = None  # GRID_ACCEL_MODE grid, built on demand (build_grid)
        self.grid_max_op = None

    GRID_DIMS = (256, 256, 256)  # Grid{nullptr, vec3i(256), volbounds} (hostCode.cu:670)

    def build_grid(self):
        """buildICONGrid (hostCode.cu:668-682) over the volume bounds; majorants follow the TF."""
        if self.grid_vr is None:
            n = int(np.prod(self.GRID_DIMS))
            self.grid_dims = np.array(self.GRID_DIMS, dtype=np.int32)
            self.grid_vr = np.zeros((n, 2), dtype=np.float32)
            olib().oracle_build_grid(_p(self.cells), self.cells.size, _p(self.grid_dims), self.vb,
                                     _p(self.grid_vr))
            self.grid_max_op = np.zeros(n, dtype=np.float32)
            if self.lut is not None:
                self._grid_max_opacities()
        return self.grid_vr

    def _grid_max_opacities(self):
        olib().oracle_max_opacities(_p(self.grid_vr), self.grid_vr.shape[0], _p(self.lut),
                                    self.lut.shape[0], self.value_range[0], self.value_range[1],
                                    _p(self.grid_max_op))

    def default_lut(self):
        L = olib()
        lut5 = np.zeros((5, 4), dtype=np.float32)
        L.oracle_default_lut5(_p(lut5))
        lut = np.zeros((300, 4), dtype=np.float32)
        L.oracle_resample_lut(_p(lut5), 5, _p(lut), 300)
        vr = self.data_range if self.data_range[1] > self.data_range[0] else (0.0, 1.0)
        return lut, vr

    def set_transfunc(self, lut: np.ndarray, value_range, opacity_scale=1.0):
        self.lut = np.ascontiguousarray(lut, dtype=np.float32).reshape(-1, 4)
        self.value_range = (float(value_range[0]), float(value_range[1]))
        self.opacity_scale = float(opacity_scale)
        olib().oracle_max_opacities(_p(self.value_ranges), self.num_mcs, _p(self.lut),
                                    self.lut.shape[0], self.value_range[0], self.value_range[1],
                                    _p(self.max_op))
        if self.grid_vr is not None:
            self._grid_max_opacities()

    def camera(self, width, height, camera=None, camera_div=None):
        """(org, dir_00, dir_du, dir_dv) as hostCode.cu:939-945."""
        out = (OVec3 * 4)()
        if camera is None:
            olib().oracle_camera_view_all(self.vb, 90.0, 1.0, C.cast(out, C.c_void_p))
        else:
            vp, vi, vu, fovy = camera
            olib().oracle_camera_orient(v3(vp), v3(vi), v3(vu), fovy, 1.0, C.cast(out, C.c_void_p))
        dw, dh = camera_div if camera_div is not None else (width, height)
        org = [out[0].x, out[0].y, out[0].z]
        ll = [out[1].x, out[1].y, out[1].z]
        h = np.array([out[2].x, out[2].y, out[2].z], dtype=np.float32) / np.float32(dw)
        v = np.array([out[3].x, out[3].y, out[3].z], dtype=np.float32) / np.float32(dh)
        return (np.array(org, np.float32), np.array(ll, np.float32), h, v)

    def params(self, cam, accum_id=0, raygen=0, unit_distance=None, accel_mode=0,
               mode=0) -> OParams:
        org, ll, du, dv = cam
        p = OParams()
        p.org, p.dir_00, p.dir_du, p.dir_dv = v3(org), v3(ll), v3(du), v3(dv)
        p.accumID = accum_id
        p.ambientColor = OVec3(1.0, 1.0, 1.0)
        p.ambientRadiance = 1.0
        p.unitDistance = self.unit_distance if unit_distance is None else unit_distance
        p.raygen = raygen
        p.bounds = self.vb
        for i in range(3):
            p.dims[i] = int(self.dims[i])
        p.sphericalBounds = self.sb
        p.maxOpacities = self.max_op.ctypes.data
        p.tf_lower, p.tf_upper = self.value_range
        p.opacityScale = self.opacity_scale
        p.lut = self.lut.ctypes.data
        p.lut_size = self.lut.shape[0]
        p.accelMode = accel_mode
        p.mode = mode
        if accel_mode == 1:
            self.build_grid()
            for i in range(3):
                p.gridDims[i] = int(self.grid_dims[i])
            p.gridBounds = self.vb
            p.gridMaxOpacities = self.grid_max_op.ctypes.data
        return p

    def render(self, params: OParams, width, height, rect=None, accum=None, fb=None,
               threads=0, fast=True):
        """One frame (crop `rect`=(x0,y0,x1,y1)); returns accum (H,W,4), fb (H,W), stats."""
        if accum is None:
            accum = np.zeros((height, width, 4), dtype=np.float32)
        if fb is None:
            fb = np.zeros((height, width), dtype=np.uint32)
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, width, height)
        st = OStats()
        rc = olib().oracle_render(_p(self.cells), self.cells.size, C.byref(params), width, height,
                                  x0, y0, x1, y1, _p(accum), _p(fb), threads, int(fast),
                                  C.byref(st))
        assert rc == 0
        return accum, fb, st

    def render_pixels(self, params: OParams, width, height, xy: np.ndarray, threads=0,
                      fast=False):
        """Raygen over an explicit pixel list (n,2) int32; returns (accum, fb, stats)."""
        xy = np.ascontiguousarray(xy, dtype=np.int32).reshape(-1, 2)
        accum = np.zeros((height, width, 4), dtype=np.float32)
        fb = np.zeros((height, width), dtype=np.uint32)
        st = OStats()
        rc = olib().oracle_render_pixels(_p(self.cells), self.cells.size, C.byref(params), width,
                                         height, _p(xy), xy.shape[0], _p(accum), _p(fb), threads,
                                         int(fast), C.byref(st))
        assert rc == 0
        return accum, fb, st


class TimedScene:
    """An oracle scene whose locator is built once (oracle_scene_new), so that frames can
    be timed without the build -- bench.py's CPU baseline."""

    def __init__(self, scene: "OracleScene", fast: int = 2, threads: int = 0):
        L = olib()
        L.oracle_scene_new.restype = C.c_void_p
        L.oracle_scene_new.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int]
        L.oracle_scene_render.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                          C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                          C.c_int, C.c_void_p]
        L.oracle_scene_free.argtypes = [C.c_void_p]
        self.scene = scene
        self._h = L.oracle_scene_new(_p(scene.cells), scene.cells.size, fast, threads)

    def render(self, params, width, height, rect=None, threads=0):
        accum = np.zeros((height, width, 4), dtype=np.float32)
        fb = np.zeros((height, width), dtype=np.uint32)
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, width, height)
        st = OStats()
        rc = olib().oracle_scene_render(self._h, C.byref(params), width, height, x0, y0, x1, y1,
                                        _p(accum), _p(fb), threads, C.byref(st))
        assert rc == 0
        return accum, fb, st

    def close(self):
        if self._h:
            olib().oracle_scene_free(self._h)
            self._h = None


def ref_render(scene: OracleScene, params: OParams, width, height, rect=None, accum=None,
               fb=None, threads=0):
    """Same frame on the reference's own code (oracle/_ref)."""
    R = rlib()
    if accum is None:
        accum = np.zeros((height, width, 4), dtype=np.float32)
    if fb is None:
        fb = np.zeros((height, width), dtype=np.uint32)
    x0, y0, x1, y1 = rect if rect is not None else (0, 0, width, height)
    cam = np.array([params.org.x, params.org.y, params.org.z, params.dir_00.x, params.dir_00.y,
                    params.dir_00.z, params.dir_du.x, params.dir_du.y, params.dir_du.z,
                    params.dir_dv.x, params.dir_dv.y, params.dir_dv.z], dtype=np.float32)
    amb = np.array([1, 1, 1, 1], dtype=np.float32)
    bounds6 = np.array([scene.vb.lower.x, scene.vb.lower.y, scene.vb.lower.z, scene.vb.upper.x,
                        scene.vb.upper.y, scene.vb.upper.z], dtype=np.float32)
    sb6 = np.array([scene.sb.lower.x, scene.sb.lower.y, scene.sb.lower.z, scene.sb.upper.x,
                    scene.sb.upper.y, scene.sb.upper.z], dtype=np.float32)
    tf3 = np.array([params.tf_lower, params.tf_upper, params.opacityScale], dtype=np.float32)
    counters = np.zeros(2, dtype=np.uint64)
    if params.accelMode == 1:
        gd = np.array(list(params.gridDims), dtype=np.int32)
        wb6 = np.array([params.gridBounds.lower.x, params.gridBounds.lower.y,
                        params.gridBounds.lower.z, params.gridBounds.upper.x,
                        params.gridBounds.upper.y, params.gridBounds.upper.z], dtype=np.float32)
        R.ref_set_accel(1, _p(gd), _p(wb6), C.c_void_p(params.gridMaxOpacities))
    else:
        R.ref_set_accel(0, None, None, None)
    R.ref_set_sampler(params.mode, _p(scene.cells), scene.cells.size)
    R.ref_render(_p(scene.cells), scene.cells.size, _p(cam), params.accumID, _p(amb),
                 params.unitDistance, params.raygen, _p(bounds6), _p(scene.dims), _p(sb6),
                 _p(scene.max_op), _p(tf3), _p(scene.lut), scene.lut.shape[0], width, height,
                 x0, y0, x1, y1, _p(accum), _p(fb), threads, _p(counters))
    return accum, fb, counters


def ref_render_pixels(scene: OracleScene, params: OParams, width, height, xy: np.ndarray,
                      threads=1):
    """The reference's own raygen (oracle/_ref, compiled from /root/reference headers) over
    a pixel list, split over `threads` host threads (ctypes releases the GIL); returns
    (accum, fb, [sampleVolume calls, found])."""
    import threading
    R = rlib()
    xy = np.ascontiguousarray(xy, dtype=np.int32).reshape(-1, 2)
    accum = np.zeros((height, width, 4), dtype=np.float32)
    fb = np.zeros((height, width), dtype=np.uint32)
    cam = np.array([params.org.x, params.org.y, params.org.z, params.dir_00.x, params.dir_00.y,
                    params.dir_00.z, params.dir_du.x, params.dir_du.y, params.dir_du.z,
                    params.dir_dv.x, params.dir_dv.y, params.dir_dv.z], dtype=np.float32)
    amb = np.array([1, 1, 1, 1], dtype=np.float32)
    bounds6 = np.array([scene.vb.lower.x, scene.vb.lower.y, scene.vb.lower.z, scene.vb.upper.x,
                        scene.vb.upper.y, scene.vb.upper.z], dtype=np.float32)
    sb6 = np.array([scene.sb.lower.x, scene.sb.lower.y, scene.sb.lower.z, scene.sb.upper.x,
                    scene.sb.upper.y, scene.sb.upper.z], dtype=np.float32)
    tf3 = np.array([params.tf_lower, params.tf_upper, params.opacityScale], dtype=np.float32)
    R.ref_set_accel(0, None, None, None)
    R.ref_set_sampler(0, None, 0)
    chunks = np.array_split(np.arange(xy.shape[0]), max(1, threads))
    counts = np.zeros((len(chunks), 2), dtype=np.uint64)
    parts = [np.ascontiguousarray(xy[c]) for c in chunks]

    def run(k):
        R.ref_render_pixels(_p(scene.cells), scene.cells.size, _p(cam), params.accumID, _p(amb),
                            params.unitDistance, params.raygen, _p(bounds6), _p(scene.dims),
                            _p(sb6), _p(scene.max_op), _p(tf3), _p(scene.lut),
                            scene.lut.shape[0], width, height, _p(parts[k]), parts[k].shape[0],
                            _p(accum), _p(fb), _p(counts[k]))

    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(chunks))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return accum, fb, counts.sum(axis=0)
