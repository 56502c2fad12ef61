"""irt -- Python binding of the MI355X ICON renderer's C ABI (include/icon_rt_hip.h).

Thin ctypes layer over ``icon-ray-tracing_amd/libicon_rt_hip.so`` (built in-tree by
``make -C icon-ray-tracing_amd``).  It mirrors the host flow of the reference app
``icon_rt`` (szellmann/icon-ray-tracing, icon_rt/hostCode.cu:703-968): load ``.ic``
records, lat/lon filter, volume facts, default transfer function, camera, then frame
launches on the GPU.  There is no CPU fallback: without the library or a HIP device the
calls raise ``IrtError``.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# IRT_LIB_PATH: another build of the same library (profiles/ A/B runs only)
LIB_PATH = os.environ.get("IRT_LIB_PATH") or os.path.join(PKG_DIR, "libicon_rt_hip.so")

# icon_rt::ICONCell (icon_rt/ICONGrid.h:59-76), 284 bytes, the `.ic` record
CELL_DTYPE = np.dtype(
    [("lat", "<f4", (3,)), ("lon", "<f4", (3,)), ("numLayers", "<i4"),
     ("height", "<f4", (32,)), ("value", "<f4", (32,))], align=False)
assert CELL_DTYPE.itemsize == 284

RAYGEN_WITH_ACCEL = 0  # woodcockTrackingWithAccel (deviceCode.cu:281-341)
RAYGEN_AE = 1          # woodcockTrackingAE (deviceCode.cu:239-275)
ACCEL_SPHERE = 0       # SPHERE_ACCEL_MODE (Params.h:33): sdda over the shell grid
ACCEL_GRID = 1         # GRID_ACCEL_MODE (Params.h:34): dda3 over the 256^3 grid
MODE_USER_GEOM = 0     # Volume::mode (Params.h:29-31): sample() on the cells (default)
MODE_TRIANGLES = 1     # closest bottom triangle toward the centre (deviceCode.cu:61-76)
MODE_CUBQL = 2         # wedges + intersectWedgeEXT (deviceCode.cu:90-115)
# The raygen's render variants (irt_render.hip OPT_* bits), all bit-identical: the product
# library compiles 73405728 (the default: one-wave workgroups since round 4, 5 waves/SIMD; since
# round 5 with the miss mode, the LDS-DMA prologue tables and the DPP prefix, and 73667872 its
# form without the miss mode, which hole-free scenes run),
# 5376 (256-thread workgroups; the persistent launch's base) and 36864 (per-wave statistics);
# libicon_rt_hip_all.so (`make VARIANTS=all`) adds the A/B variants: 4096 no waves-per-SIMD
# floor, 5120 at 4 waves/SIMD, 70656 the one-lane-per-ray Woodcock loop, 136192 per-lane
# candidate scans, 529408 per-region shader-clock timing (profiles/probe.py), 1053696
# LDS-staged cell headers, 2102272 / 2102528 less LDS per workgroup, 8393728 / 8393984
# every candidate dealt out, 6296576 / 6296832 one-wave workgroups (6558976 the latter without
# the miss mode: round 4's and early round 5's defaults), 529664 the timing variant
# at 5 waves/SIMD, 2102784 the lean-LDS build at 6 waves/SIMD, 33559808 the certified fast
# lat/lon for the sdda cells (OPT_FASTSPH).
ALL_LIB_PATH = os.path.join(PKG_DIR, "libicon_rt_hip_all.so")


def compiled_variants() -> tuple:
    """The render variants the loaded library compiled (irt_debug_variants)."""
    L = lib()
    n = L.irt_debug_variants(None, 0)
    out = (C.c_int * n)()
    L.irt_debug_variants(out, n)
    return tuple(out)


E_INVALID, E_HIP, E_DATA, E_IO, E_CHAIN = -1, -2, -3, -4, -5  # IRT_E_* (icon_rt_hip.h)


class IrtError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]

    def tolist(self):
        return [self.x, self.y, self.z]


class Vec4(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("w", C.c_float)]


class Box1(C.Structure):
    _fields_ = [("lower", C.c_float), ("upper", C.c_float)]


class Box3(C.Structure):
    _fields_ = [("lower", Vec3), ("upper", Vec3)]


class LaunchParams(C.Structure):
    """Per-frame part of icon_rt::LaunchParams (icon_rt/Params.h:92-119)."""
    _fields_ = [("org", Vec3), ("dir_00", Vec3), ("dir_du", Vec3), ("dir_dv", Vec3),
                ("accumID", C.c_int32), ("ambientColor", Vec3), ("ambientRadiance", C.c_float),
                ("unitDistance", C.c_float), ("raygen", C.c_int32), ("accelMode", C.c_int32),
                ("mode", C.c_int32)]

    def camera12(self) -> np.ndarray:
        return np.array(self.org.tolist() + self.dir_00.tolist() + self.dir_du.tolist()
                        + self.dir_dv.tolist(), dtype=np.float32)


class VolumeInfo(C.Structure):
    _fields_ = [("numCells", C.c_uint64), ("bounds", Box3), ("sphericalBounds", Box3),
                ("dataRange", Box1), ("unitDistance", C.c_float), ("shellDims", C.c_int32 * 3),
                ("locatorFaceRes", C.c_int32), ("locatorEntries", C.c_uint64),
                ("deviceBytes", C.c_uint64)]


class RenderStats(C.Structure):
    _fields_ = [("raysLaunched", C.c_uint64), ("raysInBox", C.c_uint64),
                ("locateCalls", C.c_uint64), ("samplesFound", C.c_uint64),
                ("candidatesTested", C.c_uint64), ("kernelMs", C.c_float)]

    def asdict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None


def lib() -> C.CDLL:
    """Load the in-tree product library (fails loudly if it was not built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 (soname
        # libamdhip64.so.7, like /opt/rocm's).  Loading torch first makes the dynamic
        # linker bind our library to that same runtime, so torch tensors' device pointers,
        # streams and RCCL are shared with the kernels.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise IrtError(f"{LIB_PATH} not built; run `make -C icon-ray-tracing_amd` "
                           "(or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        P, I, F, S = C.c_void_p, C.c_int, C.c_float, C.c_size_t
        L.irt_last_error.restype = C.c_char_p
        sig = {
            "irt_create": [P, S, I, C.POINTER(P)],
            "irt_create_begin": [S, I, C.POINTER(P)],
            "irt_create_append": [P, P, S],
            "irt_create_end": [P],
            "irt_create_from_file": [C.c_char_p, C.c_long, I, C.POINTER(P)],
            "irt_create_synth": [I, I, I, F, F, C.c_uint32, I, C.POINTER(P)],
            "irt_create_synth_terrain": [I, I, I, F, F, C.c_uint32, F, I, C.POINTER(P)],
            "irt_debug_context_array": [P, I, P, S, C.POINTER(S)],
            "irt_debug_scene_array": [P, I, P, S, C.POINTER(S)],
            "irt_destroy": [P],
            "irt_get_volume_info": [P, C.POINTER(VolumeInfo)],
            "irt_set_transfunc": [P, P, I, Box1, F],
            "irt_clear_frame": [P, P, P, S, P],
            "irt_render": [P, C.POINTER(LaunchParams), I, I, P, P, P],
            "irt_render_tiles": [P, C.POINTER(LaunchParams), I, I, I, I, P, P,
                                 C.POINTER(C.c_int), P],
            "irt_render_accumulate": [P, C.POINTER(LaunchParams), I, I, I, P, P, P],
            "irt_render_sequence": [P, C.POINTER(LaunchParams), I, I, I, P, P, P],
            "irt_render_tiles_accumulate": [P, C.POINTER(LaunchParams), I, I, I, I, I, P, P,
                                            C.POINTER(C.c_int), P],
            "irt_unpack_tiles": [P, P, I, I, I, I, P, P],
            "irt_deal_tiles": [C.POINTER(LaunchParams), C.POINTER(VolumeInfo), I, I, I, F, P, S,
                               C.POINTER(C.c_int)],
            "irt_render_tile_list": [P, C.POINTER(LaunchParams), I, I, P, I, I, P, P, P],
            "irt_unpack_tile_table": [P, P, I, I, P, I, I, P, P],
            "irt_get_render_stats": [P, C.POINTER(RenderStats)],
            "irt_get_render_stats_total": [P, C.POINTER(RenderStats), C.POINTER(C.c_longlong)],
            "irt_reset_render_stats_total": [P],
            "irt_set_timing_interval": [P, C.c_int],
            "irt_get_shell": [P, P, P],
            "irt_get_grid": [P, P, P],
            "irt_build_wedge_accel": [P, P, S],
            "irt_num_tiles": [I, I],
            "irt_load_ic": [C.c_char_p, C.c_long, P, S, C.POINTER(S)],
            "irt_save_ic": [C.c_char_p, P, S],
            "irt_convert_icon": [C.POINTER(ConvertOpts), P, S, C.POINTER(S)],
            "irt_convert_icon_umesh": [C.POINTER(ConvertOpts), C.c_char_p, C.POINTER(S), C.POINTER(S)],
            "irt_filter_cells": [P, S, Box1, Box1, C.POINTER(S)],
            "irt_compute_volume_info": [P, S, C.POINTER(VolumeInfo)],
            "irt_default_transfunc": [Box1, P, C.POINTER(Box1)],
            "irt_resample_lut": [P, I, P, I],
            "irt_camera_view_all": [Box3, F, I, I, C.POINTER(LaunchParams)],
            "irt_camera_look_at": [Vec3, Vec3, Vec3, F, I, I, C.POINTER(LaunchParams)],
            "irt_synth_grid": [I, I, I, F, F, C.c_uint32, P, S, C.POINTER(S)],
            "irt_synth_grid_terrain": [I, I, I, F, F, C.c_uint32, F, P, S, C.POINTER(S)],
            # host-only inspection (include/icon_rt_hip_debug.h)
            "irt_debug_asinf": [F],
            "irt_debug_atan2f": [F, F],
            "irt_debug_f2i": [F],
            "irt_debug_logf_entry": [C.c_uint32],
            "irt_debug_srgb_thresholds": [P],
            "irt_debug_scene_build": [P, S, C.POINTER(P)],
            "irt_debug_scene_info": [P, C.POINTER(VolumeInfo)],
            "irt_debug_scene_locate": [P, Vec3, C.POINTER(C.c_float), C.POINTER(C.c_uint32)],
            "irt_debug_scene_locate_binned": [P, Vec3, C.POINTER(C.c_float),
                                              C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)],
            "irt_debug_scene_candidates": [P, Vec3, P, I],
            "irt_debug_scene_planes": [P, C.c_uint32, P],
            "irt_debug_scene_values": [P, C.c_uint32, F, P],
            "irt_debug_logf_mismatches": [],
            "irt_debug_host_woodcock_log": [P],
            "irt_debug_device_woodcock_log": [I, P],
            "irt_debug_scene_free": [P],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            if name not in ("irt_last_error",):
                fn.restype = C.c_int
        L.irt_debug_asinf.restype = F
        L.irt_debug_atan2f.restype = F
        L.irt_debug_logf_entry.restype = F
        L.irt_destroy.restype = None
        L.irt_debug_scene_free.restype = None
        L.irt_debug_srgb_thresholds.restype = None
        _lib = L
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().irt_last_error().decode(errors="replace")
        raise IrtError(f"{what} failed ({rc}): {msg}", rc)


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def vec3(v) -> Vec3:
    return Vec3(float(v[0]), float(v[1]), float(v[2]))


def box1(lo, hi) -> Box1:
    return Box1(float(lo), float(hi))


# ----------------------------------------------------------------------- host helpers
def default_kernel_id(ctx=None) -> int:
    """Template id of the raygen kernel (k_render<id>, as rocprofv3 names it) that `ctx`
    launches -- the default variant, its hole-free form (bit 262144) on scenes without holes
    or its located-mode void walk (bit 1073741824) on scenes with holes, with bit 128 (OPT_SLOT)
    where the launches use the slot table (irt_debug_slot_use) -- or, without a context,
    that of the default variant."""
    L = lib()
    if ctx is not None:
        L.irt_debug_get_variant.argtypes = [C.c_void_p]
        v = int(L.irt_debug_get_variant(ctx._h)) & ~4096
        d = int(L.irt_debug_default_variant())
        L.irt_debug_slot_use.argtypes = [C.c_void_p, C.c_void_p]
        if v in ((d & ~4096), (d | 262144) & ~4096, (d | 1073741824) & ~4096) and L.irt_debug_slot_use(ctx._h, None) == 1:
            v |= 128  # kernel_for: the default kernels' OPT_SLOT form
        return v
    return int(L.irt_debug_default_variant()) & ~4096  # OPT_MONO: one kernel per frame


def synth_grid(root_n: int, bisections: int, levels: int, top_height: float = 75e3,
               noise: float = 0.0, seed: int = 1234, terrain: float = 0.0) -> np.ndarray:
    """Synthetic RnBk ICON grid as `.ic` records (host/irt_synth.cpp); terrain > 0: over
    terrain up to `terrain` metres, as convert_icon writes it (irt_synth_grid_terrain)."""
    n = C.c_size_t()
    _check(lib().irt_synth_grid_terrain(root_n, bisections, levels, top_height, noise, seed, terrain,
                                        None, 0, C.byref(n)), "irt_synth_grid")
    cells = np.zeros(n.value, dtype=CELL_DTYPE)
    _check(lib().irt_synth_grid_terrain(root_n, bisections, levels, top_height, noise, seed, terrain,
                                        _ptr(cells), n.value, C.byref(n)), "irt_synth_grid")
    return cells


def load_ic(path: str, max_num_cells: int = -1) -> np.ndarray:
    n = C.c_size_t()
    _check(lib().irt_load_ic(path.encode(), max_num_cells, None, 0, C.byref(n)), "irt_load_ic")
    cells = np.zeros(n.value, dtype=CELL_DTYPE)
    _check(lib().irt_load_ic(path.encode(), max_num_cells, _ptr(cells), n.value, C.byref(n)),
           "irt_load_ic")
    return cells


class ConvertOpts(C.Structure):
    """irt_convert_opts: convert_icon's command line (convert_icon.cpp:121-161)."""
    _fields_ = [("hgridFile", C.c_char_p), ("hsurfFile", C.c_char_p),
                ("hhlFiles", C.POINTER(C.c_char_p)), ("numHhlFiles", C.c_int),
                ("dataFiles", C.POINTER(C.c_char_p)), ("numDataFiles", C.c_int),
                ("varName", C.c_char_p), ("maxLayers", C.c_int)]


def convert_icon(hgrid: str, hsurf: str, hhl: list, data: list, var: str = "pres",
                 max_layers: int = 5) -> np.ndarray:
    """tools/convert_icon (convert_icon.cpp:168-391): DWD ICON netCDF files -> .ic records."""
    hp = (C.c_char_p * max(len(hhl), 1))(*[f.encode() for f in hhl])
    dp = (C.c_char_p * max(len(data), 1))(*[f.encode() for f in data])
    o = ConvertOpts(hgrid.encode(), hsurf.encode(), hp, len(hhl), dp, len(data), var.encode(),
                    max_layers)
    n = C.c_size_t()
    _check(lib().irt_convert_icon(C.byref(o), None, 0, C.byref(n)), "irt_convert_icon")
    cells = np.zeros(n.value, dtype=CELL_DTYPE)
    _check(lib().irt_convert_icon(C.byref(o), _ptr(cells), n.value, C.byref(n)),
           "irt_convert_icon")
    return cells


def convert_icon_umesh(hgrid: str, hsurf: str, hhl: list, data: list, path: str,
                       var: str = "pres", max_layers: int = 5):
    """convert_icon's UMesh branch (convert_icon.cpp:393-452): writes `path` in umesh's
    binary layout; returns (vertices, wedges) written."""
    hp = (C.c_char_p * max(len(hhl), 1))(*[f.encode() for f in hhl])
    dp = (C.c_char_p * max(len(data), 1))(*[f.encode() for f in data])
    o = ConvertOpts(hgrid.encode(), hsurf.encode(), hp, len(hhl), dp, len(data), var.encode(),
                    max_layers)
    nv, nw = C.c_size_t(), C.c_size_t()
    _check(lib().irt_convert_icon_umesh(C.byref(o), path.encode(), C.byref(nv), C.byref(nw)),
           "irt_convert_icon_umesh")
    return nv.value, nw.value


def read_umesh(path: str) -> dict:
    """The arrays of a .umesh file as irt_convert_icon_umesh writes it (u64-counted)."""
    raw = open(path, "rb").read()
    pos = 0

    def u64():
        nonlocal pos
        v = int(np.frombuffer(raw, np.uint64, 1, pos)[0])
        pos += 8
        return v

    def arr(dtype, width):
        nonlocal pos
        n = u64()
        a = np.frombuffer(raw, dtype, n * width, pos).reshape(n, width) if width > 1 else \
            np.frombuffer(raw, dtype, n, pos)
        pos += a.nbytes
        return a

    out = {"magic": u64(), "vertices": arr(np.float32, 3), "scalars": arr(np.float32, 1)}
    for name, w in (("triangles", 3), ("quads", 4), ("tets", 4), ("pyrs", 5),
                    ("wedges", 6), ("hexes", 8)):
        out[name] = arr(np.int32, w)
    if pos != len(raw):
        raise ValueError(f"{path}: {len(raw) - pos} trailing bytes")
    return out


def save_ic(path: str, cells: np.ndarray):
    cells = np.ascontiguousarray(cells, dtype=CELL_DTYPE)
    _check(lib().irt_save_ic(path.encode(), _ptr(cells), cells.size), "irt_save_ic")


def filter_cells(cells: np.ndarray, lat_range=(-np.inf, np.inf), lon_range=(-np.inf, np.inf)):
    """--lat-range / --lon-range filter in degrees (hostCode.cu:736-758); returns a copy."""
    out = np.array(cells, dtype=CELL_DTYPE, copy=True)
    n = C.c_size_t()
    _check(lib().irt_filter_cells(_ptr(out), out.size, box1(*lat_range), box1(*lon_range),
                                  C.byref(n)), "irt_filter_cells")
    return out[: n.value].copy()


def volume_info(cells: np.ndarray) -> VolumeInfo:
    cells = np.ascontiguousarray(cells, dtype=CELL_DTYPE)
    info = VolumeInfo()
    _check(lib().irt_compute_volume_info(_ptr(cells), cells.size, C.byref(info)),
           "irt_compute_volume_info")
    return info


def default_transfunc(data_range) -> tuple[np.ndarray, tuple[float, float]]:
    """hostCode.cu:823-836 + Pipeline::setTransfunc resampling (pipeline.cu:469-473)."""
    lut = np.zeros((300, 4), dtype=np.float32)
    vr = Box1()
    _check(lib().irt_default_transfunc(box1(*data_range), _ptr(lut), C.byref(vr)),
           "irt_default_transfunc")
    return lut, (vr.lower, vr.upper)


def resample_lut(src: np.ndarray, n: int) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.float32).reshape(-1, 4)
    dst = np.zeros((n, 4), dtype=np.float32)
    _check(lib().irt_resample_lut(_ptr(src), src.shape[0], _ptr(dst), n), "irt_resample_lut")
    return dst


def camera_view_all(bounds: Box3, img_w: int, img_h: int, fovy_deg: float = 90.0) -> LaunchParams:
    lp = LaunchParams()
    _check(lib().irt_camera_view_all(bounds, fovy_deg, img_w, img_h, C.byref(lp)),
           "irt_camera_view_all")
    return lp


def camera_look_at(vp, vi, vu, fovy_deg: float, img_w: int, img_h: int) -> LaunchParams:
    lp = LaunchParams()
    _check(lib().irt_camera_look_at(vec3(vp), vec3(vi), vec3(vu), fovy_deg, img_w, img_h,
                                    C.byref(lp)), "irt_camera_look_at")
    return lp


def num_tiles(w: int, h: int) -> int:
    return lib().irt_num_tiles(w, h)


def deal_tiles(lp: LaunchParams, info: VolumeInfo, w: int, h: int, ranks: int,
               rank0_extra: float = 0.0) -> np.ndarray:
    """irt_deal_tiles: the cost-balanced deal of the frame's 64x64 tiles over `ranks` ranks,
    (ranks, max_tiles) int32, row r = rank r's tiles in render order, -1 padding; rank 0
    carries rank0_extra x a frame's cost besides its tiles."""
    m = C.c_int()
    _check(lib().irt_deal_tiles(C.byref(lp), C.byref(info), w, h, ranks, rank0_extra, None, 0,
                                C.byref(m)), "irt_deal_tiles")
    table = np.full((ranks, m.value), -1, np.int32)
    _check(lib().irt_deal_tiles(C.byref(lp), C.byref(info), w, h, ranks, rank0_extra,
                                _ptr(table), table.size, C.byref(m)), "irt_deal_tiles")
    return table


@dataclass
class FrameSetup:
    """What icon_rt's main() derives before the first launch (hostCode.cu:736-958)."""
    lp: LaunchParams
    lut: np.ndarray
    value_range: tuple[float, float]
    opacity_scale: float
    info: VolumeInfo


# The survey's framing camera: --camera 0 0 1.4e7 0 0 0 0 1 0 -fovy 60
FRAMING_CAMERA = ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)


def setup_frame(cells: np.ndarray, width: int, height: int, camera=None,
                camera_div=None, raygen: int = RAYGEN_WITH_ACCEL, info: VolumeInfo = None) -> FrameSetup:
    """Mirror hostCode.cu main(): volume facts, default TF, unitDistance, camera.

    info: the volume facts when already known (Context.info: a streamed context never
          holds the whole cell array on the host); otherwise computed from `cells`.

    camera: None -> Camera::viewAll(volbounds) with fovy 90 (hostCode.cu:819-821);
            (vp, vi, vu, fovyDeg) -> Pipeline --camera/-fovy (pipeline.cu:444-454).
    camera_div: the image size dir_du/dir_dv are divided by; the reference hard-codes
            512 (hostCode.cu:815,944-945); default: the real (width, height).
    """
    if info is None:
        info = volume_info(cells)
    lut, vr = default_transfunc((info.dataRange.lower, info.dataRange.upper))
    dw, dh = camera_div if camera_div is not None else (width, height)
    if camera is None:
        lp = camera_view_all(info.bounds, dw, dh)
    else:
        vp, vi, vu, fovy = camera
        lp = camera_look_at(vp, vi, vu, fovy, dw, dh)
    lp.accumID = 0
    lp.ambientColor = Vec3(1.0, 1.0, 1.0)
    lp.ambientRadiance = 1.0
    lp.unitDistance = info.unitDistance
    lp.raygen = raygen
    return FrameSetup(lp=lp, lut=lut, value_range=vr, opacity_scale=1.0, info=info)


# scene arrays the render kernel reads (irt_debug_context_array / irt_debug_scene_array)
SCENE_ARRAYS = {"bin_hdr": 0, "fat": 1, "blocks": 2, "sph_r": 3, "sph_off": 4, "sph_rec": 5,
                "sph_bits": 6}
# ... and those only a context holds: the slot table (irt_common.h kSlot4; empty when the
# scene's cells do not share their radial edges, or with IRT_SLOTS=0)
CONTEXT_ARRAYS = {"slots": 7}


def _array(fn, h, name):
    which = SCENE_ARRAYS[name] if name in SCENE_ARRAYS else CONTEXT_ARRAYS[name]
    n = C.c_size_t()
    _check(fn(h, which, None, 0, C.byref(n)), "scene array")
    out = np.zeros(max(n.value, 1), np.uint8)
    _check(fn(h, which, _ptr(out), n.value, C.byref(n)), "scene array")
    return out[:n.value]


# ----------------------------------------------------------------------- GPU context
class Context:
    """One renderer context on one HIP device (irt_create ... irt_destroy).

    Context(cells) uploads a host array; Context.synth / Context.from_file /
    Context.streamed feed the cells to HBM chunk by chunk (irt_create_begin / _append /
    _end), so host memory stays at one chunk."""

    def __init__(self, cells: np.ndarray = None, device: int = 0, _handle=None):
        if _handle is None:
            cells = np.ascontiguousarray(cells, dtype=CELL_DTYPE)
            _handle = C.c_void_p()
            _check(lib().irt_create(_ptr(cells), cells.size, device, C.byref(_handle)),
                   "irt_create")
        self._h = _handle
        self.device = device
        self.info = VolumeInfo()
        _check(lib().irt_get_volume_info(self._h, C.byref(self.info)), "irt_get_volume_info")

    @classmethod
    def synth(cls, root_n: int, bisections: int, levels: int, device: int = 0,
              top_height: float = 75e3, noise: float = 0.0, seed: int = 1234,
              terrain: float = 0.0) -> "Context":
        """The grid of synth_grid(...), generated straight into HBM (irt_create_synth /
        irt_create_synth_terrain)."""
        h = C.c_void_p()
        _check(lib().irt_create_synth_terrain(root_n, bisections, levels, top_height, noise, seed,
                                              terrain, device, C.byref(h)), "irt_create_synth")
        return cls(device=device, _handle=h)

    @classmethod
    def from_file(cls, path: str, max_num_cells: int = -1, device: int = 0) -> "Context":
        """A `.ic` file streamed into HBM (irt_create_from_file, hostCode.cu:717-734)."""
        h = C.c_void_p()
        _check(lib().irt_create_from_file(path.encode(), max_num_cells, device, C.byref(h)),
               "irt_create_from_file")
        return cls(device=device, _handle=h)

    @classmethod
    def streamed(cls, chunks, num_cells: int, device: int = 0) -> "Context":
        """`num_cells` records from an iterable of record arrays, in order."""
        h = C.c_void_p()
        _check(lib().irt_create_begin(num_cells, device, C.byref(h)), "irt_create_begin")
        try:
            for ch in chunks:
                ch = np.ascontiguousarray(ch, dtype=CELL_DTYPE)
                _check(lib().irt_create_append(h, _ptr(ch), ch.size), "irt_create_append")
            _check(lib().irt_create_end(h), "irt_create_end")
        except Exception:
            lib().irt_destroy(h)
            raise
        return cls(device=device, _handle=h)

    def array(self, name: str) -> np.ndarray:
        """A scene array as the device built it (bytes; irt_debug_context_array)."""
        return _array(lib().irt_debug_context_array, self._h, name)

    def array_bytes(self, name: str) -> int:
        """The size of a scene array, without copying it."""
        which = SCENE_ARRAYS[name] if name in SCENE_ARRAYS else CONTEXT_ARRAYS[name]
        n = C.c_size_t()
        _check(lib().irt_debug_context_array(self._h, which, None, 0, C.byref(n)), "scene array")
        return n.value

    def close(self):
        if getattr(self, "_h", None):
            lib().irt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_transfunc(self, lut: np.ndarray, value_range, opacity_scale: float = 1.0):
        lut = np.ascontiguousarray(lut, dtype=np.float32).reshape(-1, 4)
        _check(lib().irt_set_transfunc(self._h, _ptr(lut), lut.shape[0], box1(*value_range),
                                       float(opacity_scale)), "irt_set_transfunc")

    def set_statistics(self, on: bool):
        """Per-launch event counts on (default) or off (irt_set_statistics); frames are
        identical either way, the counts read 0 while off."""
        L = lib()
        L.irt_set_statistics.argtypes = [C.c_void_p, C.c_int]
        _check(L.irt_set_statistics(self._h, 1 if on else 0), "irt_set_statistics")

    def set_queue(self, on: bool):
        """Persistent launches (every resident wave pulls 8x8 packets from a per-launch
        counter) on or off for this context; frames are identical either way."""
        L = lib()
        L.irt_debug_set_queue.argtypes = [C.c_void_p, C.c_int]
        _check(L.irt_debug_set_queue(self._h, 1 if on else 0), "irt_debug_set_queue")

    def set_wg_trace(self, ptr: int):
        """Measurement only: the next renders' workgroups write {start, end, HW_ID, XCC_ID}
        to the device buffer at `ptr` (4 u32 per workgroup; 0: off)."""
        L = lib()
        L.irt_debug_set_wg_trace.argtypes = [C.c_void_p, C.c_void_p]
        _check(L.irt_debug_set_wg_trace(self._h, C.c_void_p(ptr or None)), "irt_debug_set_wg_trace")

    def set_chain(self, on: bool):
        """Chained progressive frames (default on): a multi-frame launch lerps each frame
        straight into accum/fb instead of through the sample buffer + k_accumulate; frames are
        identical either way."""
        L = lib()
        L.irt_debug_set_chain.argtypes = [C.c_void_p, C.c_int]
        _check(L.irt_debug_set_chain(self._h, 1 if on else 0), "irt_debug_set_chain")

    def chain_errors(self) -> int:
        """Launches whose chained-frame waits timed out (0 in every correct run); retires
        every launch in flight (waits for the device)."""
        L = lib()
        L.irt_debug_chain_errors.argtypes = [C.c_void_p]
        n = L.irt_debug_chain_errors(self._h)
        if n < 0:
            raise IrtError("irt_debug_chain_errors failed")
        return n

    def set_chain_fault(self, spins: int, withhold_frame: int = -1):
        """Test hook: chained waits give up after `spins` polls (0: default) and frame
        `withhold_frame`'s waves never publish (-1: none) -- the IRT_E_CHAIN path."""
        L = lib()
        L.irt_debug_set_chain_fault.argtypes = [C.c_void_p, C.c_uint32, C.c_int]
        _check(L.irt_debug_set_chain_fault(self._h, spins, withhold_frame), "irt_debug_set_chain_fault")

    def sched_split(self):
        """(split work items of the last launch -- parts x split packets, padded with empty items to
        a multiple of 8 -- and log2 of the parts per packet): measured-cost scheduling."""
        L = lib()
        L.irt_debug_sched_split.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        n, lg = C.c_int(), C.c_int()
        _check(L.irt_debug_sched_split(self._h, C.byref(n), C.byref(lg)), "irt_debug_sched_split")
        return n.value, lg.value

    def launch_workgroups(self, num_tiles: int, frames: int = 1) -> int:
        """Workgroups of one launch of num_tiles tiles x frames (the wg-trace buffer needs 4
        u32 per workgroup)."""
        L = lib()
        L.irt_debug_launch_workgroups.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.irt_debug_launch_workgroups.restype = C.c_longlong
        n = L.irt_debug_launch_workgroups(self._h, num_tiles, frames)
        if n < 0:
            raise IrtError("irt_debug_launch_workgroups failed")
        return n

    def queue(self) -> bool:
        L = lib()
        L.irt_debug_get_queue.argtypes = [C.c_void_p]
        return L.irt_debug_get_queue(self._h) == 1

    def clear(self, fb_ptr: int, accum_ptr: int, num_pixels: int, stream: int = 0):
        _check(lib().irt_clear_frame(self._h, C.c_void_p(fb_ptr), C.c_void_p(accum_ptr),
                                     num_pixels, C.c_void_p(stream)), "irt_clear_frame")

    def render(self, lp: LaunchParams, width: int, height: int, fb_ptr: int, accum_ptr: int,
               stream: int = 0):
        _check(lib().irt_render(self._h, C.byref(lp), width, height, C.c_void_p(fb_ptr),
                                C.c_void_p(accum_ptr), C.c_void_p(stream)), "irt_render")

    def render_tiles(self, lp: LaunchParams, width: int, height: int, tile_begin: int,
                     tile_stride: int, fb_ptr: int, accum_ptr: int, stream: int = 0) -> int:
        n = C.c_int()
        _check(lib().irt_render_tiles(self._h, C.byref(lp), width, height, tile_begin,
                                      tile_stride, C.c_void_p(fb_ptr), C.c_void_p(accum_ptr),
                                      C.byref(n), C.c_void_p(stream)), "irt_render_tiles")
        return n.value

    def render_sequence(self, lps, width: int, height: int, fb_ptr: int, accum_ptr: int,
                        stream: int = 0):
        """irt_render_sequence: lps[k] (camera and accumID per frame) in one launch."""
        arr = (LaunchParams * len(lps))(*lps)
        _check(lib().irt_render_sequence(self._h, arr, len(lps), width, height, C.c_void_p(fb_ptr),
                                         C.c_void_p(accum_ptr), C.c_void_p(stream)),
               "irt_render_sequence")

    def render_tile_list_sequence(self, lps, width: int, height: int, tiles, fb_tiles_ptr: int,
                                  accum_tiles_ptr: int, stream: int = 0):
        """irt_render_tile_list_sequence: lps[k] over the listed tiles, packed in list order."""
        arr = (LaunchParams * len(lps))(*lps)
        t = np.ascontiguousarray(tiles, dtype=np.int32)
        L = lib()
        L.irt_render_tile_list_sequence.argtypes = [C.c_void_p, C.POINTER(LaunchParams), C.c_int, C.c_int, C.c_int,
                                                    C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        _check(L.irt_render_tile_list_sequence(self._h, arr, len(lps), width, height, _ptr(t), t.size,
                                               C.c_void_p(fb_tiles_ptr), C.c_void_p(accum_tiles_ptr),
                                               C.c_void_p(stream)), "irt_render_tile_list_sequence")

    def render_accumulate(self, lp: LaunchParams, width: int, height: int, num_frames: int,
                          fb_ptr: int, accum_ptr: int, stream: int = 0):
        """Frames lp.accumID .. lp.accumID+num_frames-1 of the progressive accumulation in
        one launch (irt_render_accumulate)."""
        _check(lib().irt_render_accumulate(self._h, C.byref(lp), width, height, num_frames,
                                           C.c_void_p(fb_ptr), C.c_void_p(accum_ptr),
                                           C.c_void_p(stream)), "irt_render_accumulate")

    def render_tiles_accumulate(self, lp: LaunchParams, width: int, height: int, tile_begin: int,
                                tile_stride: int, num_frames: int, fb_ptr: int, accum_ptr: int,
                                stream: int = 0) -> int:
        n = C.c_int()
        _check(lib().irt_render_tiles_accumulate(self._h, C.byref(lp), width, height, tile_begin,
                                                 tile_stride, num_frames, C.c_void_p(fb_ptr),
                                                 C.c_void_p(accum_ptr), C.byref(n),
                                                 C.c_void_p(stream)), "irt_render_tiles_accumulate")
        return n.value

    def render_tile_list(self, lp: LaunchParams, width: int, height: int, tiles, num_frames: int,
                         fb_tiles_ptr: int, accum_tiles_ptr: int, stream: int = 0):
        """irt_render_tile_list: the listed tiles (row-major ids), packed in list order."""
        t = np.ascontiguousarray(tiles, dtype=np.int32)
        _check(lib().irt_render_tile_list(self._h, C.byref(lp), width, height, _ptr(t), t.size,
                                          num_frames, C.c_void_p(fb_tiles_ptr),
                                          C.c_void_p(accum_tiles_ptr), C.c_void_p(stream)),
               "irt_render_tile_list")

    def unpack_tile_table(self, gathered_ptr: int, table: np.ndarray, width: int, height: int,
                          fb_ptr: int, stream: int = 0):
        """irt_unpack_tile_table: rank-major packed tiles whose ids are table[rank, k]."""
        t = np.ascontiguousarray(table, dtype=np.int32)
        _check(lib().irt_unpack_tile_table(self._h, C.c_void_p(gathered_ptr), t.shape[0], t.shape[1],
                                           _ptr(t), width, height, C.c_void_p(fb_ptr),
                                           C.c_void_p(stream)), "irt_unpack_tile_table")

    def unpack_tiles(self, gathered_ptr: int, num_ranks: int, max_tiles: int, width: int,
                     height: int, fb_ptr: int, stream: int = 0):
        _check(lib().irt_unpack_tiles(self._h, C.c_void_p(gathered_ptr), num_ranks, max_tiles,
                                      width, height, C.c_void_p(fb_ptr), C.c_void_p(stream)),
               "irt_unpack_tiles")

    def stats(self) -> RenderStats:
        st = RenderStats()
        _check(lib().irt_get_render_stats(self._h, C.byref(st)), "irt_get_render_stats")
        return st

    def stats_total(self) -> tuple[RenderStats, int]:
        """Sums of the statistics of every launch since reset_stats_total()."""
        st = RenderStats()
        n = C.c_longlong()
        _check(lib().irt_get_render_stats_total(self._h, C.byref(st), C.byref(n)),
               "irt_get_render_stats_total")
        return st, n.value

    def reset_stats_total(self):
        _check(lib().irt_reset_render_stats_total(self._h), "irt_reset_render_stats_total")

    def set_timing_interval(self, every: int):
        """Kernel-timing events on every `every`-th launch only (default 8)."""
        _check(lib().irt_set_timing_interval(self._h, int(every)), "irt_set_timing_interval")

    def build_wedge_accel(self, cells: np.ndarray):
        """buildCuBQLAccel (hostCode.cu:557-649): enables LaunchParams.mode = MODE_CUBQL."""
        cells = np.ascontiguousarray(cells, dtype=CELL_DTYPE)
        _check(lib().irt_build_wedge_accel(self._h, _ptr(cells), cells.size),
               "irt_build_wedge_accel")

    def grid(self) -> tuple[np.ndarray, np.ndarray]:
        """GRID_ACCEL_MODE grid: (valueRanges (256^3, 2), maxOpacities (256^3,))."""
        n = 256 ** 3
        vr = np.zeros((n, 2), np.float32)
        mo = np.zeros(n, np.float32)
        _check(lib().irt_get_grid(self._h, _ptr(vr), _ptr(mo)), "irt_get_grid")
        return vr, mo

    def shell(self) -> tuple[np.ndarray, np.ndarray]:
        n = int(np.prod(list(self.info.shellDims)))
        vr = np.zeros((n, 2), dtype=np.float32)
        mo = np.zeros(n, dtype=np.float32)
        _check(lib().irt_get_shell(self._h, _ptr(vr), _ptr(mo)), "irt_get_shell")
        return vr, mo


class DebugScene:
    """Host-side locator (include/icon_rt_hip_debug.h), for CPU checks."""

    def __init__(self, cells: np.ndarray):
        cells = np.ascontiguousarray(cells, dtype=CELL_DTYPE)
        h = C.c_void_p()
        _check(lib().irt_debug_scene_build(_ptr(cells), cells.size, C.byref(h)),
               "irt_debug_scene_build")
        self._h = h
        self.info = VolumeInfo()
        lib().irt_debug_scene_info(self._h, C.byref(self.info))

    def locate(self, p):
        v = C.c_float()
        r = C.c_uint32()
        hit = lib().irt_debug_scene_locate(self._h, vec3(p), C.byref(v), C.byref(r))
        return (True, v.value, r.value) if hit == 1 else (False, 0.0, None)

    def locate_binned(self, p):
        """locate() through the binned locator of the render kernel; also returns the
        number of candidate entries examined."""
        v = C.c_float()
        r = C.c_uint32()
        t = C.c_uint32()
        hit = lib().irt_debug_scene_locate_binned(self._h, vec3(p), C.byref(v), C.byref(r),
                                                  C.byref(t))
        return (True, v.value, r.value, t.value) if hit == 1 else (False, 0.0, None, t.value)

    def candidates(self, p):
        n = lib().irt_debug_scene_candidates(self._h, vec3(p), None, 0)
        out = np.zeros(max(n, 1), dtype=np.uint32)
        lib().irt_debug_scene_candidates(self._h, vec3(p), _ptr(out), n)
        return out[:n]

    def values(self, rec: int, r: float):
        """(literal findHeight value, render-record value) of record `rec` at radius r."""
        out = np.zeros(2, dtype=np.float32)
        _check(lib().irt_debug_scene_values(self._h, rec, C.c_float(r), _ptr(out)),
               "irt_debug_scene_values")
        return out

    def array(self, name: str) -> np.ndarray:
        """A scene array as the host restatement built it (bytes)."""
        return _array(lib().irt_debug_scene_array, self._h, name)

    def planes(self, rec: int) -> np.ndarray:
        out = np.zeros(12, dtype=np.float32)
        _check(lib().irt_debug_scene_planes(self._h, rec, _ptr(out)), "irt_debug_scene_planes")
        return out.reshape(3, 4)

    def close(self):
        if getattr(self, "_h", None):
            lib().irt_debug_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
