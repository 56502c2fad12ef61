#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE's own code (oracle/_ref/libiconref.so,
compiled from /root/reference headers by oracle/Makefile `ref`).

Run in the build container (the only place /root/reference exists):
    make -C oracle ref && python tests/golden/make_golden.py

Each frame fixture holds its inputs (the `.ic` records, the LUT/value range, the camera
LaunchParams, accumIDs) and the reference outputs (accumBuffer float32 RGBA, fbPointer
RGBA8, sampleVolume call counts).  kats.npz holds single-function known answers from the
reference functions (LCG, sample, findHeight, intersectSphere, boxTest, sdda,
linear_to_srgb/make_rgba, toSpherical/toCartesian, getBounds, resampleLUT, Camera);
kats_grid.npz + f6_*_grid.npz the GRID_ACCEL_MODE path (dda3, buildGrid_ICON, a frame);
kats_wedge.npz + f7_*_wedge.npz the CUBQL_MODE sampler (intersectWedgeEXT, the wedge
sampleVolume, a frame).
The `.ic` inputs are synthetic grids from icon-ray-tracing_amd's generator (real DWD data
is not available offline); they are stored verbatim, so the fixtures do not depend on it.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "icon-ray-tracing_amd", "python"), os.path.join(ROOT, "oracle")]

import irt  # noqa: E402  (grid generator only)
import oracle as O  # noqa: E402

FRAMING = irt.FRAMING_CAMERA

FRAMES = {
    # name: (rootN, bisections, levels, numCells cap, W, H, camera, accumIDs, raygen, tf)
    "f1_ico12_viewall": (1, 0, 4, 12, 256, 256, None, (0,), 0, "default"),
    "f1_ico12_framing": (1, 0, 4, 12, 256, 256, FRAMING, (0,), 0, "default"),
    "f2_r2b02_l90": (2, 2, 90, -1, 128, 128, FRAMING, (0,), 0, "default"),
    "f3_r2b00_l10_ae": (2, 0, 10, -1, 64, 64, FRAMING, (0,), 1, "default"),
    "f4_r2b01_l31_progressive": (2, 1, 31, -1, 64, 64, FRAMING, (0, 2, 3), 0, "default"),
    "f5_r2b01_l40_sparse": (2, 1, 40, -1, 64, 64, FRAMING, (0,), 0, "sparse"),
}

SPARSE_LUT5 = np.array([[0.1, 0.2, 0.9, 0.05], [0.9, 0.9, 0.2, 0.02], [0.8, 0.1, 0.1, 0.3]],
                       np.float32)


def make_frame(name, spec, mode=0):
    rn, bis, L, cap, W, H, cam, ids, raygen, tf = spec
    cells = irt.synth_grid(rn, bis, L, noise=0.1 if tf == "sparse" else 0.0)
    if cap >= 0:
        cells = cells[:cap].copy()  # --num-cells (hostCode.cu:112-113,728-730)
    S = O.OracleScene(cells)
    # host setup restated with the reference's types (oracle/_ref)
    R = O.rlib()
    sb6, vb6, dr = np.zeros(6, np.float32), np.zeros(6, np.float32), np.zeros(2, np.float32)
    R.ref_compute_bounds(cells.ctypes.data, cells.size, sb6.ctypes.data, vb6.ctypes.data,
                         dr.ctypes.data)
    vr_ref = np.zeros((S.num_mcs, 2), np.float32)
    R.ref_build_shell(cells.ctypes.data, cells.size, S.dims.ctypes.data, sb6.ctypes.data,
                      vr_ref.ctypes.data)
    if tf == "sparse":
        lut = np.zeros((300, 4), np.float32)
        R.ref_resample_lut(SPARSE_LUT5.ctypes.data, 3, lut.ctypes.data, 300)
        vrange, opacity = (float(dr[0]), float(dr[1])), 0.5
    else:
        lut5 = np.array([[0.149, 0.015, 0.705, 1.0], [0.486, 0.603, 0.956, 0.75],
                         [0.866, 0.866, 0.866, 0.5], [0.996, 0.690, 0.552, 0.25],
                         [0.752, 0.298, 0.231, 0.0]], np.float32)
        lut = np.zeros((300, 4), np.float32)
        R.ref_resample_lut(lut5.ctypes.data, 5, lut.ctypes.data, 300)
        vrange = (float(dr[0]), float(dr[1])) if dr[1] > dr[0] else (0.0, 1.0)
        opacity = 1.0
    maxop = np.zeros(S.num_mcs, np.float32)
    R.ref_max_opacities(vr_ref.ctypes.data, S.num_mcs, lut.ctypes.data, 300, vrange[0],
                        vrange[1], maxop.ctypes.data)
    cam12 = np.zeros(12, np.float32)
    if cam is None:
        R.ref_camera(1, vb6.ctypes.data, np.zeros(9, np.float32).ctypes.data, 90.0,
                     cam12.ctypes.data)
    else:
        vp9 = np.array(list(cam[0]) + list(cam[1]) + list(cam[2]), np.float32)
        R.ref_camera(0, vb6.ctypes.data, vp9.ctypes.data, cam[3], cam12.ctypes.data)
    # hostCode.cu:944-945 divides by the image size
    cam12[6:9] = cam12[6:9] / np.float32(W)
    cam12[9:12] = cam12[9:12] / np.float32(H)
    # unitDistance = powf(10, floorf(log10f(R_inner)) - 3) (hostCode.cu:838-840)
    unit_c = C.c_float(O.olib().oracle_unit_distance(float(sb6[0]))).value
    S.set_transfunc(lut, vrange, opacity)
    S.max_op[:] = maxop
    S.value_ranges[:] = vr_ref
    accum = np.zeros((H, W, 4), np.float32)
    fb = np.zeros((H, W), np.uint32)
    counts = []
    p = S.params((cam12[0:3], cam12[3:6], cam12[6:9], cam12[9:12]), raygen=raygen,
                 unit_distance=unit_c, mode=mode)
    for aid in ids:
        p.accumID = aid
        _, _, c = O.ref_render(S, p, W, H, accum=accum, fb=fb, threads=1)
        counts.append(c.copy())
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"), cells=cells.view(np.uint8).reshape(cells.size, 284),
        width=W, height=H, camera12=cam12, accum_ids=np.array(ids, np.int32), raygen=raygen,
        lut=lut, value_range=np.array(vrange, np.float32), opacity_scale=np.float32(opacity),
        unit_distance=np.float32(unit_c), spherical_bounds=sb6, volume_bounds=vb6,
        data_range=dr, value_ranges=vr_ref, max_opacities=maxop, accum=accum, fb=fb,
        counts=np.array(counts, np.uint64), mode=mode)
    print(f"{name}: {cells.size} records {W}x{H}, hit {(accum[..., 3] > 0).mean():.3f}, "
          f"samples {counts}")


def make_kats():
    R = O.rlib()
    rng = np.random.default_rng(20261015)
    out = {}
    # LCG (dvr_course-common-both.h:41-86)
    seeds = np.array([[0, 0], [1, 0], [12345, 678], [0xFFFFFFFF, 7], [1048576 * 3 + 17, 511]],
                     np.uint32)
    lcg = np.zeros((len(seeds), 16), np.float32)
    for i, (a, b) in enumerate(seeds):
        R.ref_lcg(int(a), int(b), 16, lcg[i].ctypes.data)
    out["lcg_seeds"], out["lcg"] = seeds, lcg
    # cells for sample / findHeight / getBounds
    cells = irt.synth_grid(2, 1, 45, noise=0.3)[:200].copy()
    out["cells"] = cells.view(np.uint8).reshape(cells.size, 284)
    pts, idx = [], []
    for i in range(cells.size):
        c = cells[i]
        lat, lon = c["lat"].astype(np.float64), c["lon"].astype(np.float64)
        d = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
        for _ in range(6):
            w = rng.dirichlet([1, 1, 1]) * 1.3 - 0.1  # some outside the triangle
            r = rng.uniform(c["height"][0] - 500, c["height"][c["numLayers"]] + 500)
            v = (w @ d)
            pts.append((v / np.linalg.norm(v) * r).astype(np.float32))
            idx.append(i)
        # exactly on layer boundary heights
        v = d.mean(0)
        for j in (0, 1, c["numLayers"]):
            pts.append((v / np.linalg.norm(v) * np.float64(c["height"][j])).astype(np.float32))
            idx.append(i)
    pts, idx = np.array(pts, np.float32), np.array(idx, np.int32)
    hit, val = np.zeros(len(pts), np.int32), np.zeros(len(pts), np.float32)
    for k, (p, i) in enumerate(zip(pts, idx)):
        v = C.c_float(0)
        hit[k] = R.ref_sample(cells[i:i + 1].ctypes.data, p.ctypes.data, C.byref(v))
        val[k] = v.value
    out["sample_points"], out["sample_cell"], out["sample_hit"], out["sample_value"] = pts, idx, hit, val
    fh_h = np.concatenate([cells[i]["height"][:cells[i]["numLayers"] + 1] for i in range(20)])
    fh_i = np.concatenate([[i] * (cells[i]["numLayers"] + 1) for i in range(20)]).astype(np.int32)
    fh_h = np.concatenate([fh_h, fh_h + 0.25, fh_h - 0.25]).astype(np.float32)
    fh_i = np.concatenate([fh_i, fh_i, fh_i])
    out["fh_cell"], out["fh_h"] = fh_i, fh_h
    out["fh_result"] = np.array([R.ref_find_height(cells[i:i + 1].ctypes.data, float(h))
                                 for i, h in zip(fh_i, fh_h)], np.int32)
    gb = np.zeros((cells.size, 6), np.float32)
    for i in range(cells.size):
        R.ref_get_bounds(cells[i:i + 1].ctypes.data, gb[i].ctypes.data)
    out["get_bounds"] = gb
    # rays: intersectSphere, boxTest, sdda
    n = 300
    org = np.zeros((n, 3), np.float32)
    org[:] = (rng.normal(size=(n, 3)) * 1e7).astype(np.float32)
    org[:20] = (rng.normal(size=(20, 3)) * 2e6).astype(np.float32)  # inside the inner sphere
    tgt = (rng.normal(size=(n, 3)) * 5e6).astype(np.float32)
    dirs = (tgt - org)
    dirs = (dirs / np.linalg.norm(dirs, axis=1, keepdims=True)).astype(np.float32)
    out["ray_org"], out["ray_dir"] = org, dirs
    sph = np.zeros((n, 4), np.float32)
    for k in range(n):
        tn, tf = C.c_float(), C.c_float()
        h = R.ref_intersect_sphere(org[k].ctypes.data, dirs[k].ctypes.data, 6.4e6, C.byref(tn), C.byref(tf))
        sph[k] = [h, tn.value, tf.value, 0]
    out["sphere"] = sph
    box6 = np.array([-6.5e6, -6.4e6, -6.3e6, 6.5e6, 6.4e6, 6.3e6], np.float32)
    bt = np.zeros((n, 3), np.float32)
    for k in range(n):
        t0, t1 = C.c_float(), C.c_float()
        h = R.ref_box_test(org[k].ctypes.data, dirs[k].ctypes.data, 0.0, 1e10, box6.ctypes.data,
                           C.byref(t0), C.byref(t1))
        bt[k] = [h, t0.value, t1.value]
    out["box6"], out["box_test"] = box6, bt
    dims = np.array([1, 1024, 1024], np.int32)
    sb6 = np.array([6.371229e6, -1.5707964, -3.1415927, 6.446229e6, 1.5707964, 3.1415927], np.float32)
    maxo = 2048
    leaves = np.full((n, maxo), -1, np.int32)
    lt0 = np.zeros((n, maxo), np.float32)
    lt1 = np.zeros((n, maxo), np.float32)
    cnt = np.zeros(n, np.int32)
    for k in range(n):
        cnt[k] = R.ref_sdda_trace(org[k].ctypes.data, dirs[k].ctypes.data, 0.0, 1e10,
                                  dims.ctypes.data, sb6.ctypes.data, maxo, leaves[k].ctypes.data,
                                  lt0[k].ctypes.data, lt1[k].ctypes.data)
    out["sdda_dims"], out["sdda_sb6"], out["sdda_count"] = dims, sb6, cnt
    out["sdda_leaf"], out["sdda_t0"], out["sdda_t1"] = leaves, lt0, lt1
    # shading
    xs = np.concatenate([rng.uniform(-0.1, 1.2, 4000), np.linspace(0, 0.01, 500),
                         [0.0031308, 0.0031309, 1.0, 0.0]]).astype(np.float32)
    out["srgb_x"] = xs
    out["srgb"] = np.array([R.ref_linear_to_srgb(float(x)) for x in xs], np.float32)
    cols = rng.uniform(-0.2, 1.2, (1000, 4)).astype(np.float32)
    out["rgba_in"] = cols
    out["rgba"] = np.array([R.ref_make_rgba(c.ctypes.data) for c in cols], np.uint32)
    # toSpherical / toCartesian
    cart = (rng.normal(size=(2000, 3)) * 6.4e6).astype(np.float32)
    out["cart"], out["to_spherical"] = cart, np.zeros_like(cart)
    for k in range(len(cart)):
        R.ref_to_spherical(cart[k].ctypes.data, out["to_spherical"][k].ctypes.data)
    sp = np.stack([rng.uniform(6.3e6, 6.5e6, 2000), rng.uniform(-1.6, 1.6, 2000),
                   rng.uniform(-3.2, 3.2, 2000)], 1).astype(np.float32)
    out["sph"], out["to_cartesian"] = sp, np.zeros_like(sp)
    for k in range(len(sp)):
        R.ref_to_cartesian(sp[k].ctypes.data, out["to_cartesian"][k].ctypes.data)
    # resampleLUT + Camera
    src = rng.uniform(0, 1, (7, 4)).astype(np.float32)
    dst = np.zeros((300, 4), np.float32)
    R.ref_resample_lut(src.ctypes.data, 7, dst.ctypes.data, 300)
    out["lut_src"], out["lut_300"] = src, dst
    cams = []
    vb6 = np.array([-6.4e6, -6.4e6, -6.4e6, 6.4e6, 6.4e6, 6.4e6], np.float32)
    c12 = np.zeros(12, np.float32)
    R.ref_camera(1, vb6.ctypes.data, np.zeros(9, np.float32).ctypes.data, 90.0, c12.ctypes.data)
    cams.append(c12.copy())
    for vp9, fov in [([0, 0, 1.4e7, 0, 0, 0, 0, 1, 0], 60.0), ([3e6, -2e7, 1e6, 1e5, 0, -2e5, 0, 0, 1], 35.0),
                     ([1e7, 1e7, 1e7, 0, 0, 0, 0, 1, 0], 0.0)]:
        v = np.array(vp9, np.float32)
        R.ref_camera(0, vb6.ctypes.data, v.ctypes.data, fov, c12.ctypes.data)
        cams.append(c12.copy())
    out["camera_box6"], out["cameras"] = vb6, np.array(cams)
    out["camera_specs"] = np.array([[0, 0, 1.4e7, 0, 0, 0, 0, 1, 0, 60.0],
                                    [3e6, -2e7, 1e6, 1e5, 0, -2e5, 0, 0, 1, 35.0],
                                    [1e7, 1e7, 1e7, 0, 0, 0, 0, 1, 0, 0.0]], np.float32)
    np.savez_compressed(os.path.join(HERE, "kats.npz"), **out)
    print("kats:", {k: v.shape for k, v in out.items()})


def make_grid_fixtures(frame=True):
    """GRID_ACCEL_MODE (Params.h:34): dda3 known answers from DDA.h itself, the 256^3
    buildGrid_ICON value ranges (hostCode.cu:205-297) as a digest plus sampled entries, and
    one frame of woodcockTrackingWithAccel with accelMode = GRID_ACCEL_MODE."""
    import hashlib
    R = O.rlib()
    rng = np.random.default_rng(20261016)
    out = {}
    n = 400
    org = (rng.normal(size=(n, 3)) * 1.4e7).astype(np.float32)
    org[:30] = (rng.normal(size=(30, 3)) * 2e6).astype(np.float32)  # starting inside the grid
    tgt = (rng.normal(size=(n, 3)) * 3e6).astype(np.float32)
    dirs = tgt - org
    dirs = (dirs / np.linalg.norm(dirs, axis=1, keepdims=True)).astype(np.float32)
    dirs[:10, 0] = np.float32(1e-5)  # generateRay's clamped components
    tmin = rng.uniform(0, 1e7, n).astype(np.float32)
    tmin[:100] = 0.0
    tmax = (tmin + rng.uniform(1e3, 3e7, n)).astype(np.float32)
    dims_all = np.zeros((n, 3), np.int32)
    dims_all[:] = (256, 256, 256)
    dims_all[300:] = rng.integers(1, 40, (n - 300, 3))  # ragged grids
    wb6 = np.array([-6.45e6, -6.44e6, -6.43e6, 6.45e6, 6.44e6, 6.43e6], np.float32)
    maxo = 2048
    leaves = np.full((n, maxo), -1, np.int32)
    lt0 = np.zeros((n, maxo), np.float32)
    lt1 = np.zeros((n, maxo), np.float32)
    cnt = np.zeros(n, np.int32)
    for k in range(n):
        cnt[k] = R.ref_dda3_trace(org[k].ctypes.data, dirs[k].ctypes.data, float(tmin[k]),
                                  float(tmax[k]), dims_all[k].ctypes.data, wb6.ctypes.data, maxo,
                                  leaves[k].ctypes.data, lt0[k].ctypes.data, lt1[k].ctypes.data)
    out.update(dda3_org=org, dda3_dir=dirs, dda3_tmin=tmin, dda3_tmax=tmax, dda3_dims=dims_all,
               dda3_wb6=wb6, dda3_count=cnt, dda3_leaf=leaves, dda3_t0=lt0, dda3_t1=lt1)
    # buildGrid_ICON over a synthetic R2B02 x 60 scene
    cells = irt.synth_grid(2, 2, 60, noise=0.2)
    sb6, vb6, dr = np.zeros(6, np.float32), np.zeros(6, np.float32), np.zeros(2, np.float32)
    R.ref_compute_bounds(cells.ctypes.data, cells.size, sb6.ctypes.data, vb6.ctypes.data,
                         dr.ctypes.data)
    gdims = np.array([256, 256, 256], np.int32)
    gvr = np.zeros((256 ** 3, 2), np.float32)
    R.ref_build_grid(cells.ctypes.data, cells.size, gdims.ctypes.data, vb6.ctypes.data,
                     gvr.ctypes.data)
    pick = np.sort(np.concatenate([rng.choice(256 ** 3, 20000, replace=False),
                                   rng.choice(np.flatnonzero(gvr[:, 1] >= gvr[:, 0]), 20000,
                                              replace=False)]))
    out.update(grid_cells=cells.view(np.uint8).reshape(cells.size, 284), grid_vb6=vb6,
               grid_sha256=np.frombuffer(hashlib.sha256(gvr.tobytes()).digest(), np.uint8),
               grid_nonempty=np.int64((gvr[:, 1] >= gvr[:, 0]).sum()), grid_pick=pick,
               grid_pick_vr=gvr[pick])
    lut5 = np.array([[0.149, 0.015, 0.705, 1.0], [0.486, 0.603, 0.956, 0.75],
                     [0.866, 0.866, 0.866, 0.5], [0.996, 0.690, 0.552, 0.25],
                     [0.752, 0.298, 0.231, 0.0]], np.float32)
    lut = np.zeros((300, 4), np.float32)
    R.ref_resample_lut(lut5.ctypes.data, 5, lut.ctypes.data, 300)
    gmo = np.zeros(256 ** 3, np.float32)
    R.ref_max_opacities(gvr.ctypes.data, 256 ** 3, lut.ctypes.data, 300, float(dr[0]),
                        float(dr[1]), gmo.ctypes.data)
    out.update(grid_lut=lut, grid_value_range=dr.copy(),
               grid_maxop_sha256=np.frombuffer(hashlib.sha256(gmo.tobytes()).digest(), np.uint8),
               grid_pick_maxop=gmo[pick])
    np.savez_compressed(os.path.join(HERE, "kats_grid.npz"), **out)
    print("kats_grid:", cnt.sum(), "dda3 leaves;", int(out["grid_nonempty"]), "non-empty MCs")
    if not frame:
        return
    # one GRID_ACCEL_MODE frame (the sphere-mode machinery of make_frame, accelMode 1)
    W = H = 80
    S = O.OracleScene(cells)
    vr_ref = np.zeros((S.num_mcs, 2), np.float32)
    R.ref_build_shell(cells.ctypes.data, cells.size, S.dims.ctypes.data, sb6.ctypes.data,
                      vr_ref.ctypes.data)
    S.value_ranges[:] = vr_ref
    S.set_transfunc(lut, (float(dr[0]), float(dr[1])), 1.0)
    S.build_grid()
    S.grid_vr[:] = gvr
    S.grid_max_op[:] = gmo
    cam12 = np.zeros(12, np.float32)
    vp9 = np.array(list(FRAMING[0]) + list(FRAMING[1]) + list(FRAMING[2]), np.float32)
    R.ref_camera(0, vb6.ctypes.data, vp9.ctypes.data, FRAMING[3], cam12.ctypes.data)
    cam12[6:9] = cam12[6:9] / np.float32(W)
    cam12[9:12] = cam12[9:12] / np.float32(H)
    unit_c = C.c_float(O.olib().oracle_unit_distance(float(sb6[0]))).value
    p = S.params((cam12[0:3], cam12[3:6], cam12[6:9], cam12[9:12]), raygen=0,
                 unit_distance=unit_c, accel_mode=1)
    accum = np.zeros((H, W, 4), np.float32)
    fb = np.zeros((H, W), np.uint32)
    _, _, c = O.ref_render(S, p, W, H, accum=accum, fb=fb, threads=1)
    np.savez_compressed(
        os.path.join(HERE, "f6_r2b02_l60_grid.npz"),
        cells=cells.view(np.uint8).reshape(cells.size, 284), width=W, height=H, camera12=cam12,
        accum_ids=np.array([0], np.int32), raygen=0, accel_mode=1, lut=lut,
        value_range=dr.copy(), opacity_scale=np.float32(1.0), unit_distance=np.float32(unit_c),
        spherical_bounds=sb6, volume_bounds=vb6, data_range=dr, accum=accum, fb=fb,
        counts=np.array([c.copy()], np.uint64))
    print(f"f6_r2b02_l60_grid: {cells.size} records {W}x{H}, "
          f"hit {(accum[..., 3] > 0).mean():.3f}, samples {c}")


def make_wedge_fixtures():
    """CUBQL_MODE (Params.h:31): intersectWedgeEXT known answers from UElems.h itself, the
    wedge sampleVolume of deviceCode.cu:90-115 over buildCuBQLAccel's wedges (hostCode.cu:
    557-600) at points around a scene, and one frame with volume.mode = CUBQL_MODE."""
    R = O.rlib()
    rng = np.random.default_rng(20261017)
    out = {}
    # single wedges: random prisms (general, thin/flat, and Earth-scale ICON-like)
    nW = 600
    V = np.zeros((nW, 6, 4), np.float32)
    P = np.zeros((nW, 3), np.float32)
    for k in range(nW):
        if k < 200:
            tri = rng.normal(size=(3, 3))
            off = rng.normal(size=3) * 0.3 + np.array([0, 0, 1.0])
            V[k, :3, :3] = tri
            V[k, 3:, :3] = tri + off
            scale = 1.0
        else:
            lat = rng.uniform(-1.5, 1.5) + rng.normal(size=3) * (0.02 if k < 400 else 0.2)
            lon = rng.uniform(-3.1, 3.1) + rng.normal(size=3) * (0.02 if k < 400 else 0.2)
            h0 = 6.371229e6 + rng.uniform(0, 7e4)
            h1 = h0 + rng.uniform(10, 3000)
            d = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
            V[k, :3, :3] = d * h0
            V[k, 3:, :3] = d * h1
            scale = 0.0
        V[k, :, 3] = rng.uniform(0, 1)
        w = rng.dirichlet([1, 1, 1]) * 1.3 - 0.1
        tt = rng.uniform(-0.2, 1.2)
        P[k] = ((1 - tt) * (w @ V[k, :3, :3]) + tt * (w @ V[k, 3:, :3])).astype(np.float32)
        del scale
    hit = np.zeros(nW, np.int32)
    val = np.zeros(nW, np.float32)
    for k in range(nW):
        v = C.c_float(0)
        hit[k] = R.ref_intersect_wedge(V[k].ctypes.data, P[k].ctypes.data, C.byref(v))
        val[k] = v.value
    out.update(wedge_v=V, wedge_p=P, wedge_hit=hit, wedge_value=val)
    # sampleVolume in CUBQL_MODE over a scene's wedges
    cells = irt.synth_grid(2, 2, 20, noise=0.3)
    pts = []
    for _ in range(4000):
        c = cells[rng.integers(cells.size)]
        lat, lon = c["lat"].astype(np.float64), c["lon"].astype(np.float64)
        d = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
        w = rng.dirichlet([1, 1, 1]) * 1.4 - 0.13
        r = rng.uniform(c["height"][0] - 2000, c["height"][c["numLayers"]] + 2000)
        v = w @ d
        pts.append((v / np.linalg.norm(v) * r).astype(np.float32))
    pts = np.array(pts, np.float32)
    shit = np.zeros(len(pts), np.int32)
    sval = np.zeros(len(pts), np.float32)
    for k in range(len(pts)):
        v = C.c_float(0)
        shit[k] = R.ref_wedge_sample(cells.ctypes.data, cells.size, pts[k].ctypes.data, C.byref(v))
        sval[k] = v.value
    out.update(scene_cells=cells.view(np.uint8).reshape(cells.size, 284), scene_points=pts,
               scene_hit=shit, scene_value=sval)
    np.savez_compressed(os.path.join(HERE, "kats_wedge.npz"), **out)
    print("kats_wedge:", int(hit.sum()), "of", nW, "wedge hits;", int(shit.sum()), "of",
          len(pts), "scene hits")
    # one CUBQL_MODE frame
    make_frame("f7_r2b02_l20_wedge", (2, 2, 20, -1, 64, 64, FRAMING, (0,), 0, "default"),
               mode=2)


if __name__ == "__main__":
    if not O.have_ref():
        sys.exit("oracle/_ref/libiconref.so missing: make -C oracle ref (needs /root/reference)")
    if len(sys.argv) > 1 and sys.argv[1] == "grid":
        make_grid_fixtures()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "wedge":
        make_wedge_fixtures()
        sys.exit(0)
    for name, spec in FRAMES.items():
        make_frame(name, spec)
    make_kats()
    make_grid_fixtures()
    make_wedge_fixtures()
