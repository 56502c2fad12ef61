"""GPU parity: the MI355X raygen (through the C ABI) against the CPU oracle.

The bar is bit-exactness: accumBuffer (float32 RGBA) and fbPointer (RGBA8) identical for
every pixel, plus identical per-frame sample counts (the oracle counts sampleVolume calls
exactly like the reference raygen makes them).  Sizes are those the oracle finishes in
seconds; full BASELINE sizes are covered by tests/test_gpu_scale.py through
size-independent properties.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

import irt
from helpers import FRAMING, GpuFrame, bits, gpu_frame, oracle_frame, terrain_cells

pytestmark = pytest.mark.gpu


def assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, label=""):
    diff = np.any(bits(a_gpu) != bits(a_ref), axis=-1) | (f_gpu != f_ref)
    n = int(diff.sum())
    if n:
        ys, xs = np.nonzero(diff)
        y, x = ys[0], xs[0]
        raise AssertionError(f"{label}: {n} of {diff.size} pixels differ; first ({x},{y}): "
                             f"gpu {a_gpu[y, x]} {f_gpu[y, x]:08x} vs ref {a_ref[y, x]} {f_ref[y, x]:08x}")


def test_device_woodcock_log_matches_glibc_everywhere():
    """logf(1.f - rnd()) on the device (glibc's algorithm, irt_common.h) == the host glibc
    logf for every one of the 2^24 values rnd() can return."""
    dev = np.zeros(1 << 24, np.float32)
    host = np.zeros(1 << 24, np.float32)
    L = irt.lib()
    assert L.irt_debug_device_woodcock_log(0, dev.ctypes.data) == 0, L.L.irt_last_error()
    L.irt_debug_host_woodcock_log(host.ctypes.data)  # glibc logf, evaluated here
    assert np.array_equal(bits(dev), bits(host))


def test_device_math_matches_glibc():
    """glibc_asinf / glibc_atan2f on the device round exactly as the host glibc."""
    rng = np.random.default_rng(5)
    n = 1 << 21
    a = np.concatenate([rng.uniform(-1, 1, n - 8).astype(np.float32),
                        np.float32([0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 1e-30, 0.975])])
    y = (rng.normal(size=n) * 7e6).astype(np.float32)
    x = (rng.normal(size=n) * 7e6).astype(np.float32)
    x[:1000] = 0.0
    y[1000:2000] = 0.0
    oa = np.zeros(n, np.float32)
    ot = np.zeros(n, np.float32)
    L = irt.lib()
    L.irt_debug_device_math.argtypes = [C.c_int] + [C.c_void_p] * 3 + [C.c_int] + [C.c_void_p] * 2
    rc = L.irt_debug_device_math(0, a.ctypes.data, y.ctypes.data, x.ctypes.data, n,
                                 oa.ctypes.data, ot.ctypes.data)
    assert rc == 0, L.L.irt_last_error()
    libm = C.CDLL("libm.so.6")
    libm.asinf.restype = C.c_float
    libm.asinf.argtypes = [C.c_float]
    libm.atan2f.restype = C.c_float
    libm.atan2f.argtypes = [C.c_float, C.c_float]
    idx = np.arange(0, n, 97)
    ga = np.array([libm.asinf(float(a[i])) for i in idx], np.float32)
    gt = np.array([libm.atan2f(float(y[i]), float(x[i])) for i in idx], np.float32)
    assert np.array_equal(bits(oa[idx]), bits(ga))
    assert np.array_equal(bits(ot[idx]), bits(gt))
    # and every element against the host compile of the same restatement
    ha = np.array([L.irt_debug_asinf(float(v)) for v in a[:200000]], np.float32)
    assert np.array_equal(bits(oa[:200000]), bits(ha))


def test_fast_spherical_bounds():
    """The sdda entry/exit cells use fast asin/atan2 certified against glibc's
    (irt_device.h): a cell or step sign is taken from the fast value only when every value
    within kLatErr / kLonErr of it gives the same.  This proves those bounds exhaustively on
    the device: every float asin argument, every float atan argument, every reciprocal."""
    L = irt.lib()
    L.irt_debug_fast_math_bounds.argtypes = [C.c_int, C.c_void_p]
    L.irt_debug_fast_spherical_consts.argtypes = [C.c_void_p]
    L.irt_debug_fast_spherical_consts.restype = None
    out = np.zeros(4, np.float64)
    assert L.irt_debug_fast_math_bounds(0, out.ctypes.data) == 0, L.irt_last_error()
    e_asin, e_fatan, e_gatan, e_rcp = (float(v) for v in out)
    assert all(np.isfinite(out)), out
    consts = np.zeros(2, np.float32)
    L.irt_debug_fast_spherical_consts(consts.ctypes.data)
    lat_err, lon_err = (float(v) for v in consts)
    pad = 2.0 ** -23  # rounding of v -+ E (ulp(pi) / 2 ~ 1.19e-7)
    # asin: both paths evaluate glibc's argument z / r exactly; the bound is direct
    assert e_asin + pad <= lat_err, (e_asin, lat_err)
    # atan2: fast q = |y| rcp(|x|) (relative error <= e_rcp + 2^-24), glibc q = fl(|y/x|)
    # (2^-24); atan's relative slope q / (1 + q^2) <= 1/2; two quadrant-step roundings per
    # evaluation (<= ulp(pi/2)/2 + ulp(pi)/2)
    quad = 2 * (2.0 ** -24 + 2.0 ** -23)
    e_lon = e_fatan + e_gatan + 0.5005 * (e_rcp + 2.0 ** -24) + 0.5005 * 2.0 ** -24 + quad
    assert e_lon + pad <= lon_err, (e_fatan, e_gatan, e_rcp, e_lon, lon_err)
    assert e_rcp <= 2.0 ** -22


CASES = [
    # (rootN, bisections, levels, W, camera, raygen)
    (1, 0, 4, 128, None, 0),        # C1-class: 20-face icosahedron, viewAll camera
    (1, 0, 4, 128, FRAMING, 0),
    (2, 0, 10, 96, FRAMING, 1),     # woodcockTrackingAE
    (2, 2, 90, 96, FRAMING, 0),     # R2B02 x 90 levels (3 records per column)
    (2, 3, 47, 80, FRAMING, 0),
    (2, 2, 90, 64, None, 0),
]


@pytest.mark.parametrize("rn,bis,L,W,cam,raygen", CASES)
def test_frame_bit_exact(rn, bis, L, W, cam, raygen):
    cells = irt.synth_grid(rn, bis, L)
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, W, W, camera=cam, raygen=raygen)
    a_gpu, f_gpu, st_gpu, ctx = gpu_frame(cells, W, W, camera=cam, raygen=raygen)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, f"R{rn}B{bis:02d}L{L}")
    g, o = st_gpu[0], st_ref[0]
    assert g.raysLaunched == o.rays_launched
    assert g.raysInBox == o.rays_in_box
    assert g.locateCalls == o.locate_calls
    assert g.samplesFound == o.samples_found


def test_progressive_accumulation_bit_exact():
    cells = irt.synth_grid(2, 1, 31)
    ids = (0, 2, 3, 4)  # the frame IDs icon_rt actually renders with --sample-limit 5
    a_ref, f_ref, _, _ = oracle_frame(cells, 72, 72, camera=FRAMING, accum_ids=ids)
    a_gpu, f_gpu, _, _ = gpu_frame(cells, 72, 72, camera=FRAMING, accum_ids=ids)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, "progressive")


def test_sparse_transfunc_and_opacity_scale():
    """A sample-heavy TF (low opacity) and opacityScale != 1 (postClassify quirk)."""
    cells = irt.synth_grid(2, 2, 40, noise=0.2)
    lut5 = np.array([[0.1, 0.2, 0.9, 0.05], [0.9, 0.9, 0.2, 0.02], [0.8, 0.1, 0.1, 0.3]],
                    np.float32)
    lut = irt.resample_lut(lut5, 300)
    info = irt.volume_info(cells)
    vr = (info.dataRange.lower, info.dataRange.upper)
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, 64, 64, camera=FRAMING, lut=lut, value_range=vr,
                                           opacity_scale=0.5)
    a_gpu, f_gpu, st_gpu, _ = gpu_frame(cells, 64, 64, camera=FRAMING, lut=lut, value_range=vr,
                                        opacity_scale=0.5)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, "sparse TF")
    assert st_gpu[0].locateCalls == st_ref[0].locate_calls


def test_shell_accelerator_matches_oracle():
    cells = irt.synth_grid(2, 3, 47, noise=0.1)
    _, _, _, S = oracle_frame(cells, 8, 8, camera=FRAMING)
    setup = irt.setup_frame(cells, 8, 8)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    vr, mo = ctx.shell()
    # value ranges: equal as numbers (the sign of a zero bound depends on atomic arrival
    # order in the reference too and never changes a majorant)
    assert np.array_equal(vr, S.value_ranges)
    assert np.array_equal(bits(mo), bits(S.max_op))


def test_tiles_match_full_frame():
    """Frame-tile subsets (the multi-GPU split) reproduce the full launch bit for bit."""
    import torch
    cells = irt.synth_grid(2, 2, 90)
    W, H = 200, 136  # ragged: partial tiles on both edges
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    dev = "cuda:0"
    fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    ctx.render(setup.lp, W, H, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    full = fb.cpu().numpy()
    for ranks in (2, 3, 8):
        ntot = irt.num_tiles(W, H)
        maxt = (ntot + ranks - 1) // ranks
        gathered = torch.zeros(ranks * maxt * 4096, dtype=torch.int32, device=dev)
        for r in range(ranks):
            tacc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)
            view = gathered[r * maxt * 4096:(r + 1) * maxt * 4096]
            n = ctx.render_tiles(setup.lp, W, H, r, ranks, view.data_ptr(), tacc.data_ptr())
            assert n == len(range(r, ntot, ranks))
        out = torch.zeros(W * H, dtype=torch.int32, device=dev)
        ctx.unpack_tiles(gathered.data_ptr(), ranks, maxt, W, H, out.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), full), f"{ranks} ranks"


def test_dealt_tile_lists_match_full_frame():
    """The cost-balanced deal (irt_deal_tiles -> irt_render_tile_list, packed in list order ->
    irt_unpack_tile_table) reproduces the full launch bit for bit, single frames and
    progressive batches, ragged frames, 1..8 ranks (8 > tiles: empty ranks)."""
    import torch
    import irt_dist
    cells = irt.synth_grid(2, 2, 90)
    W, H = 200, 136  # 4 x 3 tiles, ragged on both edges
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    lp = setup.lp
    dev = "cuda:0"
    for k in (1, 3):
        fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
        acc = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
        if k == 1:
            ctx.render(lp, W, H, fb.data_ptr(), acc.data_ptr())
        else:
            ctx.render_accumulate(lp, W, H, k, fb.data_ptr(), acc.data_ptr())
        torch.cuda.synchronize()
        full = fb.cpu().numpy()
        for ranks in (1, 2, 3, 8, 16):
            splits = [irt_dist.TileSplit.dealt(W, H, r, ranks, lp, ctx.info) for r in range(ranks)]
            maxt = splits[0].max_tiles
            gathered = torch.zeros(ranks * maxt * 4096, dtype=torch.int32, device=dev)
            for r, sp in enumerate(splits):
                tacc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)
                sp.render(ctx, lp, k, gathered[r * maxt * 4096:].data_ptr(), tacc.data_ptr())
                if sp.tiles():  # the launch's rays: this rank's in-frame pixels, k frames
                    assert ctx.stats().raysLaunched == k * sum(
                        int((sp.tile_pixels(t)[:, 0] >= 0).sum()) for t in sp.tiles())
            out = torch.zeros(W * H, dtype=torch.int32, device=dev)
            splits[0].unpack(ctx, gathered.data_ptr(), out.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), full), f"{ranks} ranks, {k} frames"
    # bad tile ids are rejected before any launch
    with pytest.raises(irt.IrtError, match="tile id"):
        ctx.render_tile_list(lp, W, H, [0, 12], 1, fb.data_ptr(), acc.data_ptr())
    with pytest.raises(irt.IrtError, match="tile id"):
        ctx.unpack_tile_table(fb.data_ptr(), np.array([[0, -2]], np.int32), W, H, out.data_ptr())
    ctx.close()


@pytest.mark.parametrize("W,H,ranks", [(203, 71, 3), (1024, 1024, 8), (64, 200, 5)])
def test_unpack_tile_table_equals_host_twin(W, H, ranks):
    """irt_unpack_tile_table scatters slot k of rank r to tile table[r, k] (a random
    permutation dealt into rows with -1 padding) exactly as irt_dist.unpack_host does."""
    import torch
    import irt_dist
    ctx = irt.Context(irt.synth_grid(2, 1, 4), 0)
    T = irt.num_tiles(W, H)
    maxt = -(-T // ranks)
    rng = np.random.default_rng(W + 3 * H)
    table = np.full(ranks * maxt, -1, np.int32)
    slots = rng.permutation(ranks * maxt)[:T]
    table[slots] = rng.permutation(T)
    table = table.reshape(ranks, maxt)
    split = irt_dist.TileSplit(W, H, 0, ranks, table)
    g = rng.integers(0, 2**32, ranks * maxt * 4096, dtype=np.uint32)
    gathered = torch.from_numpy(g.view(np.int32)).to("cuda:0")
    out = torch.full((W * H + 64,), -1, dtype=torch.int32, device="cuda:0")
    split.unpack(ctx, gathered.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    # the host twin reads rank r's tiles in table order, skipping -1 slots: compact the rows
    compact = np.zeros_like(g).reshape(ranks, maxt, 4096)
    for r in range(ranks):
        keep = np.nonzero(table[r] >= 0)[0]
        compact[r, :len(keep)] = g.reshape(ranks, maxt, 4096)[r, keep]
    ctable = np.full_like(table, -1)
    for r in range(ranks):
        row = table[r][table[r] >= 0]
        ctable[r, :len(row)] = row
    assert np.array_equal(got[:W * H].reshape(H, W),
                          irt_dist.unpack_host(compact.ravel(), irt_dist.TileSplit(W, H, 0, ranks, ctable)))
    assert (got[W * H:] == 0xFFFFFFFF).all()
    ctx.close()


@pytest.mark.parametrize("W,H,ranks", [(203, 71, 3), (130, 64, 1), (64, 200, 5), (1024, 1024, 8)])
def test_unpack_tiles_equals_host_twin(W, H, ranks):
    """irt_unpack_tiles (16-byte rows where W % 4 == 0, pixel by pixel on ragged edges) equals
    irt_dist.unpack_host on random packed tiles; pixels outside the frame are never written."""
    import torch
    import irt_dist
    ctx = irt.Context(irt.synth_grid(2, 1, 4), 0)
    split = irt_dist.TileSplit(W, H, 0, ranks)
    rng = np.random.default_rng(W * 7 + H)
    g = rng.integers(0, 2**32, ranks * split.max_tiles * 4096, dtype=np.uint32)
    dev = "cuda:0"
    gathered = torch.from_numpy(g.view(np.int32)).to(dev)
    out = torch.full((W * H + 64,), -1, dtype=torch.int32, device=dev)  # guard words past the end
    ctx.unpack_tiles(gathered.data_ptr(), ranks, split.max_tiles, W, H, out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got[:W * H].reshape(H, W), irt_dist.unpack_host(g, split))
    assert (got[W * H:] == 0xFFFFFFFF).all()
    ctx.close()


def test_lat_lon_filtered_and_truncated_scenes():
    """--lat-range/--lon-range filter and --num-cells truncation (hostCode.cu:728-758)."""
    cells = irt.synth_grid(2, 2, 20)
    sub = irt.filter_cells(cells, (-30, 60), (-90, 45))
    assert 0 < sub.size < cells.size
    for c in (sub, cells[:12]):
        a_ref, f_ref, _, _ = oracle_frame(c, 64, 64, camera=FRAMING)
        a_gpu, f_gpu, _, _ = gpu_frame(c, 64, 64, camera=FRAMING)
        assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, f"subset {c.size}")


def test_empty_scene_matches_reference_semantics():
    """Zero cells: volbounds stays (+inf,-inf), for which the reference's boxTest
    (vecmath.h:1926-1937) reports a hit for every ray (t0=0 < t1=1e10), and sdda then
    runs on infinite sphere radii; the frame must still match the oracle."""
    cells = irt.synth_grid(1, 0, 4)[:0]
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, 32, 32, camera=FRAMING)
    a_gpu, f_gpu, st_gpu, _ = gpu_frame(cells, 32, 32, camera=FRAMING)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, "empty")
    assert st_gpu[0].raysInBox == st_ref[0].rays_in_box


@pytest.mark.parametrize("name", __import__("golden_util").FRAME_FIXTURES)
def test_gpu_matches_reference_golden(name):
    """Straight against the reference's own outputs (tests/golden, from oracle/_ref), with
    the fixture's own LaunchParams, LUT and value range fed through the C ABI."""
    from golden_util import load
    from helpers import GpuFrame
    d = load(name)
    W, H = int(d["width"]), int(d["height"])
    ctx = irt.Context(d["cells"], 0)
    ctx.set_transfunc(d["lut"], tuple(float(v) for v in d["value_range"]), float(d["opacity_scale"]))
    if "value_ranges" in d:
        vr, mo = ctx.shell()
        assert np.array_equal(vr, d["value_ranges"])
        assert np.array_equal(bits(mo), bits(d["max_opacities"]))
    fr = GpuFrame(ctx, W, H)
    c = d["camera12"]
    lp = irt.LaunchParams()
    lp.org, lp.dir_00, lp.dir_du, lp.dir_dv = (irt.vec3(c[i:i + 3]) for i in (0, 3, 6, 9))
    lp.ambientColor = irt.Vec3(1, 1, 1)
    lp.ambientRadiance = 1.0
    lp.unitDistance = float(d["unit_distance"])
    lp.raygen = int(d["raygen"])
    lp.accelMode = int(d.get("accel_mode", 0))
    lp.mode = int(d.get("mode", 0))
    if lp.mode == irt.MODE_CUBQL:
        ctx.build_wedge_accel(d["cells"])
    for k, aid in enumerate(d["accum_ids"]):
        lp.accumID = int(aid)
        st = fr.render(lp)
        assert (st.locateCalls, st.samplesFound) == tuple(int(v) for v in d["counts"][k])
    a, f = fr.host()
    assert_same_frame(a, f, d["accum"], d["fb"], name)
    ctx.close()


def test_terrain_and_degenerate_records_bit_exact():
    """Terrain-following record boundaries (per-cell radial bin edges differ), unsorted
    heights, zero-thickness records (spheres) and inverted records."""
    cells = terrain_cells(11)
    for cam in (FRAMING, None):
        a_ref, f_ref, st_ref, _ = oracle_frame(cells, 80, 80, camera=cam)
        a_gpu, f_gpu, st_gpu, _ = gpu_frame(cells, 80, 80, camera=cam)
        assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, "terrain")
        assert st_gpu[0].locateCalls == st_ref[0].locate_calls
        assert st_gpu[0].samplesFound == st_ref[0].samples_found


@pytest.mark.parametrize("levels", [90, 65])
def test_convert_icon_terrain_bit_exact_with_and_without_miss_mode(levels):
    """The terrain grid as convert_icon writes it (irt_synth_grid_terrain: voids under land,
    the inverted first layer over land, coarse blocks whose keys fall below height[0]; 65
    levels: zero-thickness top records) against the oracle, counts included, with the raygen's
    miss mode (the variant such a scene runs) and without it (the hole-free variant forced)."""
    cells = irt.synth_grid(2, 3, levels, terrain=4000.0)
    W = 160
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, W, W, camera=FRAMING)
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    L = irt.lib()
    L.irt_debug_set_variant.argtypes = [C.c_void_p, C.c_int]
    L.irt_debug_get_variant.argtypes = [C.c_void_p]
    d = L.irt_debug_default_variant()
    VOIDLOC = 1073741824
    if os.environ.get("IRT_RENDER_VARIANT"):  # a forced variant (A/B runs of the suite)
        d = int(os.environ["IRT_RENDER_VARIANT"]) & ~(262144 | VOIDLOC)
    # holes: the miss mode with the located-mode void walk (scene_variant), unless forced
    assert L.irt_debug_get_variant(ctx._h) in (d, d | 262144, d | VOIDLOC)
    if not os.environ.get("IRT_RENDER_VARIANT"):
        assert L.irt_debug_get_variant(ctx._h) == d | VOIDLOC
    for v in (d | VOIDLOC, d, d | 262144):
        assert L.irt_debug_set_variant(ctx._h, v) == 0
        fr = GpuFrame(ctx, W, W)
        st = fr.render(setup.lp)
        a, f = fr.host()
        assert_same_frame(a, f, a_ref, f_ref, f"terrain L{levels} variant {v}")
        assert (st.locateCalls, st.samplesFound) == (st_ref[0].locate_calls, st_ref[0].samples_found)
        assert st.locateCalls > st.samplesFound  # the voids: samples outside every cell
    ctx.close()


@pytest.mark.skipif(not os.path.exists(irt.ALL_LIB_PATH), reason="make VARIANTS=all not built")
def test_ab_library_variants_identical():
    """test_all_render_variants_identical on the A/B library (every variant), in a child
    process: one HIP library per process (IRT_LIB_PATH selects it at load)."""
    env = dict(os.environ, IRT_LIB_PATH=irt.ALL_LIB_PATH)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        f"{__file__}::test_all_render_variants_identical",
                        f"{__file__}::test_persistent_launch_identical"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "2 passed" in r.stdout


def _hole_skip(v):
    """Whether render variant v has the quad-bound miss test (irt_render.hip Tracer::locate_wave
    kHoleSkip: the wave-wide scan of the miss-mode kernels, from headers)."""
    SERIAL, WEDGE, GRID, SCAN1, NOMISS, HDRLDS, NOHOLESKIP, SLOT = (65536, 16384, 8192, 131072, 262144,
                                                                  1048576, 4, 128)
    wave_scan = not v & (SERIAL | WEDGE | GRID | SCAN1)
    return wave_scan and not v & (NOMISS | SLOT | HDRLDS | NOHOLESKIP)


def test_all_render_variants_identical():
    """Every compiled variant of the binned raygen (batching, occupancy bounds, LUT in LDS)
    renders the same frame and counts as the default.  The product library compiles the
    default and the statistics variant; test_ab_library_variants_identical runs this test
    again on libicon_rt_hip_all.so (`make VARIANTS=all`) with every A/B variant."""
    L = irt.lib()
    L.irt_debug_set_variant.argtypes = [C.c_void_p, C.c_int]
    cells = irt.synth_grid(2, 3, 90)
    W = 128
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    import torch
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    ref = None
    variants = irt.compiled_variants()
    assert irt.lib().irt_debug_default_variant() in variants
    for v in variants:
        assert L.irt_debug_set_variant(ctx._h, v) == 0
        acc.zero_()
        ctx.render(setup.lp, W, W, fb.data_ptr(), acc.data_ptr())
        st = ctx.stats()
        out = (fb.cpu().numpy().copy(), bits(acc.cpu().numpy()), st.locateCalls, st.samplesFound,
               st.candidatesTested)
        # and a progressive batch (per-frame sample buffer + k_accumulate) on top of it
        ctx.render_accumulate(setup.lp, W, W, 3, fb.data_ptr(), acc.data_ptr())
        st = ctx.stats()
        out += (fb.cpu().numpy().copy(), bits(acc.cpu().numpy()), st.locateCalls, st.samplesFound)
        if ref is None:
            ref = out
            continue
        assert np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]), v
        assert out[2:4] == ref[2:4], v
        # candidate tests are the locator's own count: the quad-bound miss test (round 6) skips
        # a void's candidates, so only kernels of the same class test the same number
        if _hole_skip(v) == _hole_skip(variants[0]):
            assert out[4] == ref[4], v
        else:
            assert out[4] <= ref[4] if _hole_skip(v) else out[4] >= ref[4], v
        assert np.array_equal(out[5], ref[5]) and np.array_equal(out[6], ref[6]), v
        assert out[7:] == ref[7:], v
    ctx.close()


def _batch_frame(cells, W, camera, first, k, prior=()):
    """GPU frames: `prior` single-frame launches, then one progressive batch of k frames
    starting at accumID `first` (irt_render_accumulate)."""
    import torch
    setup = irt.setup_frame(cells, W, W, camera=camera)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    lp = setup.lp
    for aid in prior:
        lp.accumID = aid
        ctx.render(lp, W, W, fb.data_ptr(), acc.data_ptr())
    lp.accumID = first
    ctx.render_accumulate(lp, W, W, k, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    st = ctx.stats()
    a = acc.cpu().numpy().reshape(W, W, 4)
    f = fb.cpu().numpy().view(np.uint32).reshape(W, W)
    ctx.close()
    return a, f, st


@pytest.mark.parametrize("cam", [FRAMING, None])
def test_progressive_batch_equals_sequential_frames(cam):
    """irt_render_accumulate (k frames in one launch) == k reference frames in sequence,
    including pixels whose jittered ray hits the box in some frames only (viewAll)."""
    cells = irt.synth_grid(2, 1, 31)
    W = 72
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, W, W, camera=cam, accum_ids=(0, 1, 2, 3, 4))
    a_gpu, f_gpu, st = _batch_frame(cells, W, cam, 0, 5)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, "batch of 5")
    assert st.locateCalls == sum(s.locate_calls for s in st_ref)
    assert st.raysLaunched == 5 * W * W
    # a batch continuing an accumulation (frames 0,1 single, then 2..6 batched)
    a_ref, f_ref, _, _ = oracle_frame(cells, W, W, camera=cam, accum_ids=tuple(range(7)))
    a_gpu, f_gpu, _ = _batch_frame(cells, W, cam, 2, 5, prior=(0, 1))
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, "frames 0,1 + batch 2..6")


def test_tiles_accumulate_match_full_batch():
    """The weak-scaling split: every rank renders its interleaved tiles for k frames;
    unpacked, the ranks' tiles equal the full-frame batch."""
    import torch
    cells = irt.synth_grid(2, 2, 47)
    W, H, k, ranks = 200, 136, 3, 3
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    lp = setup.lp
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    ctx.render_accumulate(lp, W, H, k, fb.data_ptr(), acc.data_ptr())
    ntiles = irt.num_tiles(W, H)
    maxt = (ntiles + ranks - 1) // ranks
    g = torch.zeros(ranks * maxt * 4096, dtype=torch.int32, device="cuda")
    for r in range(ranks):
        tacc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device="cuda")
        ctx.render_tiles_accumulate(lp, W, H, r, ranks, k, g[r * maxt * 4096:].data_ptr(),
                                    tacc.data_ptr())
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    ctx.unpack_tiles(g.data_ptr(), ranks, maxt, W, H, out.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), fb.cpu().numpy())
    ctx.close()


def test_converted_icon_files_render_bit_exact(tmp_path):
    """convert_icon output (netCDF -> .ic, with the reference's HSURF/HHL mixing and its
    numLayers % 32 - 1 record quirk) through irt_load_ic and the raygen, vs the oracle."""
    from icon_nc import write_icon_set
    hg, hs, hhl, data = write_icon_set(str(tmp_path), bisections=2, levels=40)
    irt.save_ic(str(tmp_path / "c.ic"), irt.convert_icon(hg, hs, hhl, data, max_layers=40))
    cells = irt.load_ic(str(tmp_path / "c.ic"))
    for accel in (0, 1):
        a_ref, f_ref, st_ref, _ = oracle_frame(cells, 64, 64, camera=FRAMING, accel_mode=accel)
        a_gpu, f_gpu, st_gpu, ctx = gpu_frame(cells, 64, 64, camera=FRAMING, accel_mode=accel)
        assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, f"converted accel={accel}")
        assert st_gpu[0].locateCalls == st_ref[0].locate_calls
        ctx.close()


def test_measured_cost_scheduling_keeps_frames_identical(monkeypatch):
    """Repeated launches on one context with IRT_SCHED=2 (off by default): after the first
    few the workgroups run in the measured-cost (longest-first) tile order; every frame must
    stay bit-identical to the oracle's, counters included."""
    from helpers import GpuFrame
    monkeypatch.setenv("IRT_SCHED", "2")
    cells = irt.synth_grid(2, 3, 47)
    W = 160
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, W, W, camera=FRAMING)
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    fr = GpuFrame(ctx, W, W)
    applied = 0
    for k in range(24):
        fr.accum.zero_()
        fr.fb.zero_()
        st = fr.render(setup.lp)
        a, f = fr.host()
        assert_same_frame(a, f, a_ref, f_ref, f"launch {k}")
        assert (st.locateCalls, st.samplesFound) == (st_ref[0].locate_calls, st_ref[0].samples_found)
        applied += _sched_state(ctx)[1]
    policy, last, total = _sched_state(ctx)
    assert policy == 2 and last == 1 and total == applied > 0  # the order was in effect
    ctx.close()


def _sched_state(ctx):
    L = irt.lib()
    L.irt_debug_sched.argtypes = [C.c_void_p] + [C.c_void_p] * 3
    p, a, n = C.c_int(), C.c_int(), C.c_longlong()
    assert L.irt_debug_sched(ctx._h, C.byref(p), C.byref(a), C.byref(n)) == 0
    return p.value, a.value, n.value


def test_measured_cost_scheduling_on_a_rank_tile_subset(monkeypatch):
    """the scheduled path with tileStride > 1 (one rank's interleaved tiles, where
    the policy-2 band is tilesX/tileStride tiles): repeated launches run in a measured-cost
    order and every launch's tiles equal the full frame's."""
    import torch
    monkeypatch.setenv("IRT_SCHED", "2")
    cells = irt.synth_grid(2, 3, 47)
    W, H = 328, 200  # 6 x 4 tiles, the last column and row ragged
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    dev = "cuda:0"
    fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    ctx.render(setup.lp, W, H, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    full = fb.cpu().numpy()
    ranks, rank = 3, 1
    ntot = irt.num_tiles(W, H)
    maxt = (ntot + ranks - 1) // ranks
    gathered = torch.zeros(ranks * maxt * 4096, dtype=torch.int32, device=dev)
    mine = gathered[rank * maxt * 4096:(rank + 1) * maxt * 4096]
    seen = 0
    tiles_x = (W + 63) // 64
    tile = ((np.arange(H) // 64)[:, None] * tiles_x + (np.arange(W) // 64)[None, :]).reshape(-1)
    sel = tile % ranks == rank  # this rank's pixels
    for k in range(24):
        tacc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)
        mine.zero_()
        ctx.render_tiles(setup.lp, W, H, rank, ranks, mine.data_ptr(), tacc.data_ptr())
        seen += _sched_state(ctx)[1]
        out = torch.zeros(W * H, dtype=torch.int32, device=dev)
        ctx.unpack_tiles(gathered.data_ptr(), ranks, maxt, W, H, out.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy()[sel], full[sel]), f"launch {k}"
    assert seen > 0 and _sched_state(ctx)[1] == 1
    ctx.close()


@pytest.mark.parametrize("mode", ["device", "off"])
def test_counter_probe_modes_survive_growing_launches(monkeypatch, mode):
    """the IRT_COUNTERS=device probe buffer grows with the launch (a frame with
    more workgroups than the first), and IRT_COUNTERS=off keeps the counter block the
    statistics variant adds into.  Frames stay bit-identical to the default context's."""
    from helpers import GpuFrame
    cells = irt.synth_grid(2, 2, 47)
    ref = {}
    for W in (64, 200):
        setup = irt.setup_frame(cells, W, W, camera=FRAMING)
        ctx = irt.Context(cells, 0)
        ctx.set_transfunc(setup.lut, setup.value_range)
        fr = GpuFrame(ctx, W, W)
        fr.render(setup.lp)
        ref[W] = fr.host()
        ctx.close()
    monkeypatch.setenv("IRT_COUNTERS", mode)
    ctx = irt.Context(cells, 0)
    L = irt.lib()
    L.irt_debug_set_variant.argtypes = [C.c_void_p, C.c_int]
    for variant in ((0, 36864) if mode == "off" else (0,)):  # 36864: the statistics variant
        if variant:
            assert L.irt_debug_set_variant(ctx._h, variant) == 0
        for W in (64, 200):  # 16 then 64 workgroups
            setup = irt.setup_frame(cells, W, W, camera=FRAMING)
            ctx.set_transfunc(setup.lut, setup.value_range)
            fr = GpuFrame(ctx, W, W)
            fr.render(setup.lp)
            a, f = fr.host()
            assert_same_frame(a, f, *ref[W], f"IRT_COUNTERS={mode} variant {variant} W={W}")
    ctx.close()


def test_grid_is_built_on_first_use():
    """GRID_ACCEL_MODE's 256^3 grid is built lazily (ensure_grid): a sphere-mode context holds
    no grid; the first grid render or irt_get_grid builds it from the scene's blocks, and a
    transfer function set before or after gives the same majorants as the oracle's."""
    cells = irt.synth_grid(2, 2, 31)
    setup = irt.setup_frame(cells, 8, 8)
    S = oracle_frame(cells, 8, 8)[3]
    S.build_grid()
    ctx = irt.Context(cells, 0)
    before = ctx.info.deviceBytes
    ctx.set_transfunc(setup.lut, setup.value_range)  # before the grid exists
    vr, mo = ctx.grid()
    assert np.array_equal(vr, S.grid_vr) and np.array_equal(bits(mo), bits(S.grid_max_op))
    info = irt.VolumeInfo()
    assert irt.lib().irt_get_volume_info(ctx._h, C.byref(info)) == 0
    assert info.deviceBytes - before >= 256 ** 3 * 12  # the grid arrived with its first use
    ctx.close()


def test_null_stream_is_ordered_with_torch_default_stream():
    """irt_render with stream NULL runs on HIP's null stream, ordered with torch's default
    stream: a zero_() of the buffers enqueued just before must land before the kernel reads
    them, and a read-back enqueued just after must see the finished frame (no host sync in
    between)."""
    import torch
    cells = irt.synth_grid(2, 2, 90)
    W = 96
    a_ref, f_ref, _, _ = oracle_frame(cells, W, W, camera=FRAMING)
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    fb = torch.full((W * W,), 12345, dtype=torch.int32, device="cuda")
    acc = torch.full((W * W * 4,), 7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        acc.fill_(7.0)   # garbage the previous frame...
        fb.fill_(12345)
        acc.zero_()      # ...then clear: both on torch's default stream
        fb.zero_()
        ctx.render(setup.lp, W, W, fb.data_ptr(), acc.data_ptr())  # stream NULL
        a = acc.cpu().numpy().reshape(W, W, 4)  # default-stream copy, no explicit sync
        f = fb.cpu().numpy().view(np.uint32).reshape(W, W)
        assert_same_frame(a, f, a_ref, f_ref, "null stream")
    ctx.close()


def test_comb_transfunc_sample_heavy():
    """bench.py's C3s transfer function (alpha 0.01 except every 50th LUT entry 1.0): the
    majorants stay 1 while almost every tentative collision is rejected -- many samples
    per ray, the long Woodcock chains -- still bit-exact, counts included."""
    cells = irt.synth_grid(2, 3, 90)
    setup = irt.setup_frame(cells, 8, 8)
    lut = setup.lut.copy()
    lut[:, 3] = 0.01
    lut[::50, 3] = 1.0
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, 80, 80, camera=FRAMING, lut=lut,
                                           value_range=setup.value_range)
    a_gpu, f_gpu, st_gpu, _ = gpu_frame(cells, 80, 80, camera=FRAMING, lut=lut,
                                        value_range=setup.value_range)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, "comb TF")
    assert st_gpu[0].locateCalls == st_ref[0].locate_calls
    assert st_ref[0].samples_found > 4 * 80 * 80  # sample-heavy indeed


@pytest.mark.parametrize("raygen", [0, 1])
def test_cooperative_woodcock_holes_and_long_chains(raygen):
    """The wave-cooperative Woodcock loop (irt_render.hip woodcock_wave) at its edges: a
    lat/lon-filtered scene, so samples fall in holes between cells (not located: the ray
    resumes from that sample's step draw, inside a group of speculative lanes), under the
    comb TF (long chains: few rays left per wave, up to 64 lanes on one ray), in both
    raygens.  Frame, locate and found counts as the oracle's."""
    cells = irt.filter_cells(irt.synth_grid(2, 3, 60), (-40, 50), (-100, 70))
    setup = irt.setup_frame(cells, 8, 8)
    lut = setup.lut.copy()
    lut[:, 3] = 0.01
    lut[::50, 3] = 1.0
    kw = dict(camera=FRAMING, lut=lut, value_range=setup.value_range, raygen=raygen)
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, 72, 72, **kw)
    a_gpu, f_gpu, st_gpu, ctx = gpu_frame(cells, 72, 72, **kw)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, f"coop raygen {raygen}")
    assert st_gpu[0].locateCalls == st_ref[0].locate_calls
    assert st_gpu[0].samplesFound == st_ref[0].samples_found
    assert st_ref[0].locate_calls > st_ref[0].samples_found  # holes were sampled


@pytest.mark.parametrize("maxlg,ramp", [("6", "0"), ("0", "0"), ("3", "0"), ("2", "1")])
def test_cooperative_group_caps(monkeypatch, maxlg, ramp):
    """The speculation cap of the cooperative loop (IRT_COOP_MAXLG / IRT_COOP_RAMP; the
    default ramps from one lane per ray) changes only how many samples a round evaluates:
    whole-wave groups, solo rounds only, a fixed cap, another ramp -- each the oracle's
    frame and counts, over holes and long chains."""
    monkeypatch.setenv("IRT_COOP_MAXLG", maxlg)
    monkeypatch.setenv("IRT_COOP_RAMP", ramp)
    cells = irt.filter_cells(irt.synth_grid(2, 3, 60), (-40, 50), (-100, 70))
    setup = irt.setup_frame(cells, 8, 8)
    lut = setup.lut.copy()
    lut[:, 3] = 0.01
    lut[::50, 3] = 1.0
    kw = dict(camera=FRAMING, lut=lut, value_range=setup.value_range)
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, 64, 64, **kw)
    a_gpu, f_gpu, st_gpu, _ = gpu_frame(cells, 64, 64, **kw)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, f"maxlg {maxlg} ramp {ramp}")
    assert st_gpu[0].locateCalls == st_ref[0].locate_calls
    assert st_gpu[0].samplesFound == st_ref[0].samples_found


def test_device_srgb_byte_equals_threshold_count():
    """csrc/irt_device.h srgb_byte (hardware log2/exp2 estimate, then settled on the host
    thresholds) == the number of thresholds <= x, which test_host_logic pins to the
    reference's make_8bit(linear_to_srgb(x)): every threshold and its float neighbours,
    a dense sweep, random values, specials."""
    L = irt.lib()
    L.irt_debug_device_srgb.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int]
    th = np.zeros(256, np.float32)
    L.irt_debug_srgb_thresholds(th.ctypes.data)
    t = th[1:]
    near = np.concatenate([t, np.nextafter(t, np.float32(-np.inf)), np.nextafter(t, np.float32(np.inf)),
                           np.nextafter(np.nextafter(t, np.float32(-np.inf)), np.float32(-np.inf))])
    rng = np.random.default_rng(7)
    x = np.concatenate([near, np.linspace(-0.05, 1.05, 1 << 20, dtype=np.float32),
                        rng.random(1 << 20, dtype=np.float32),
                        rng.random(1 << 16, dtype=np.float32) * np.float32(1e-3),
                        np.float32([0.0, -0.0, 0.0031308, 1.0, 2.0, -1.0, 1e-30, np.nan, np.inf, -np.inf])])
    x = x.astype(np.float32)
    out = np.zeros(x.size, np.uint32)
    assert L.irt_debug_device_srgb(0, x.ctypes.data, out.ctypes.data, x.size) == 0, L.irt_last_error()
    want = np.searchsorted(t, x, side="right").astype(np.uint32)
    want[np.isnan(x)] = 0
    bad = np.nonzero(out != want)[0]
    assert bad.size == 0, (x[bad[:5]], out[bad[:5]], want[bad[:5]])


@pytest.mark.parametrize("entry", ["irt_debug_locate", "irt_debug_locate_wave"])
@pytest.mark.parametrize("scene", ["r2b03_l90", "terrain", "filtered"])
def test_device_locator_matches_host_restatement(scene, entry):
    """The kernel's point location == the host restatement of the binned lists (which
    tests/test_host_logic.py pins to the reference's brute-force first hit), point for
    point: found flag and value bits, including points exactly on record boundaries =
    radial bin edges (the second-bin pass), their float neighbours, shared triangle edges
    and zero-thickness records.  Two device paths: Tracer::locate (one lane per point,
    irt_debug_locate) and the cooperative kernel's wave-wide scan Tracer::locate_wave
    (irt_debug_locate_wave: dealt-out candidates and the bin-edge pass, many of them in
    one wave here)."""
    _locator_check(scene, entry)


@pytest.mark.parametrize("subs", [4, 1])
@pytest.mark.parametrize("scene", ["r2b03_l90", "filtered"])
def test_device_locator_slot_table(monkeypatch, scene, subs):
    """The same points through the wave-wide scan started from the slot table (OPT_SLOT,
    irt_common.h kSlot4; forced on these small scenes with IRT_SLOTS=1), with quads (the
    default) and one sub-cell per slot unit."""
    monkeypatch.setenv("IRT_SLOTS", "1")
    monkeypatch.setenv("IRT_SLOT_SUBS", str(subs))
    _locator_check(scene, "irt_debug_locate_wave", slots=True)


def _locator_check(scene, entry, slots=False):
    from helpers import locator_points, terrain_cells
    cells = {"r2b03_l90": lambda: irt.synth_grid(2, 3, 90),
             "terrain": lambda: terrain_cells(11),
             "filtered": lambda: irt.filter_cells(irt.synth_grid(2, 3, 40), (-30, 60), (-90, 45))}[scene]()
    pts = locator_points(cells, 5)
    ctx = irt.Context(cells, 0)
    assert (ctx.array("slots").size > 0) == slots
    D = irt.DebugScene(cells)
    L = irt.lib()
    fn = getattr(L, entry)
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    found = np.zeros(len(pts), np.int32)
    value = np.zeros(len(pts), np.float32)
    assert fn(ctx._h, pts.ctypes.data, len(pts), found.ctypes.data, value.ctypes.data) == 0, \
        L.irt_last_error()
    n_hit = 0
    for k, p in enumerate(pts):
        hb, vb, _, _ = D.locate_binned(p)
        assert bool(found[k]) == bool(hb), (k, p)
        if hb:
            n_hit += 1
            assert np.float32(vb).view(np.uint32) == value[k].view(np.uint32), (k, p)
    assert n_hit > len(pts) // 3
    ctx.close()
    D.close()


def test_counts_past_the_workgroup_ring_cap(monkeypatch):
    """a launch with more workgroups (x frames) than the per-workgroup count ring
    allows (IRT_WG_COUNTS_MAX; 2^18 by default) counts through the device-atomic block for that
    launch only; launches on either side of it keep the ring.  Statistics and frames equal a
    default context's, launch by launch (single frames and progressive batches)."""
    import torch
    cells = irt.synth_grid(2, 2, 47)

    def run():
        ctx = irt.Context(cells, 0)
        out = []
        for W, frames in ((64, 1), (200, 1), (64, 1), (64, 3), (200, 2), (64, 1)):  # 16/64/16/48/128/16 WGs
            setup = irt.setup_frame(cells, W, W, camera=FRAMING)
            ctx.set_transfunc(setup.lut, setup.value_range)
            fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
            acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
            if frames == 1:
                ctx.render(setup.lp, W, W, fb.data_ptr(), acc.data_ptr())
            else:
                ctx.render_accumulate(setup.lp, W, W, frames, fb.data_ptr(), acc.data_ptr())
            st = ctx.stats()
            out.append((fb.cpu().numpy().copy(), bits(acc.cpu().numpy()), st.raysLaunched, st.raysInBox,
                        st.locateCalls, st.samplesFound, st.candidatesTested))
        tot = ctx.stats_total()
        ctx.close()
        return out, (tot[0].locateCalls, tot[0].samplesFound, tot[1])

    ref, ref_tot = run()
    assert ref[1][4] > 0 and ref[4][4] > 0
    monkeypatch.setenv("IRT_WG_COUNTS_MAX", "20")
    got, got_tot = run()
    for k, (a, b) in enumerate(zip(ref, got)):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), k
        assert a[2:] == b[2:], (k, a[2:], b[2:])
    assert got_tot == ref_tot


def test_persistent_launch_identical():
    """Persistent launches (RenderArgs::queue: every resident wave pulls 8x8-pixel packets
    from the launch's counter, as the reference's thread pool pulls tiles,
    common/thread_pool.h:146-161) render every frame, count and progressive batch exactly as
    the grid launch: single frames at ragged sizes (partial packets), progressive batches,
    tile lists and strided tile splits, many launches in a row (the counter pair is reset by
    each launch's last wave), and two streams.  The persistent kernels live in the A/B library
    only (test_ab_library_variants_identical runs this there); the product library refuses
    them."""
    import torch
    cells = irt.synth_grid(2, 3, 90)
    S = irt.setup_frame(cells, 8, 8, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(S.lut, S.value_range)
    if irt.LIB_PATH != irt.ALL_LIB_PATH:
        with pytest.raises(irt.IrtError):
            ctx.set_queue(True)
        ctx.close()
        return
    # the persistent launch runs the 256-thread-workgroup kernel (5376), not the default's
    # one-wave workgroups
    L = irt.lib()
    L.irt_debug_set_variant.argtypes = [C.c_void_p, C.c_int]
    assert L.irt_debug_set_variant(ctx._h, 5376) == 0

    def run(on, fn):
        ctx.set_queue(on)
        return fn()

    def frame(W, H, acc_id=0, frames=1, stream=0):
        setup = irt.setup_frame(cells, W, H, camera=FRAMING)
        setup.lp.accumID = acc_id
        fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
        if frames == 1:
            ctx.render(setup.lp, W, H, fb.data_ptr(), acc.data_ptr(), stream)
        else:
            ctx.render_accumulate(setup.lp, W, H, frames, fb.data_ptr(), acc.data_ptr(), stream)
        torch.cuda.synchronize()
        st = ctx.stats()
        return (fb.cpu().numpy(), bits(acc.cpu().numpy()),
                (st.raysLaunched, st.raysInBox, st.locateCalls, st.samplesFound, st.candidatesTested))

    def same(a, b, what):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), what
        assert a[2] == b[2], (what, a[2], b[2])

    for W, H in ((128, 128), (131, 77), (9, 300), (64, 64)):
        same(run(True, lambda: frame(W, H)), run(False, lambda: frame(W, H)), f"{W}x{H}")
    same(run(True, lambda: frame(96, 80, 3, 4)), run(False, lambda: frame(96, 80, 3, 4)), "batch")
    # many launches back to back through the ring of counter pairs (kSlots = 32)
    ctx.set_queue(True)
    first = frame(100, 100)
    L.irt_debug_queue_wgs.argtypes = [C.c_void_p]
    assert L.irt_debug_queue_wgs(ctx._h) > 0  # the launches above were persistent ones
    for k in range(40):
        same(frame(100, 100), first, f"launch {k}")
    s2 = torch.cuda.Stream()
    same(frame(100, 100, stream=s2.cuda_stream), first, "side stream")
    # tile lists (multi-GPU rows) and strided tiles
    W = H = 200
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)

    def tiles(on):
        ctx.set_queue(on)
        out = []
        fbt = torch.zeros(16 * 4096, dtype=torch.int32, device="cuda")
        act = torch.zeros(16 * 4096 * 4, dtype=torch.float32, device="cuda")
        ctx.render_tile_list(setup.lp, W, H, [15, 2, 7, 0, 9], 2, fbt.data_ptr(), act.data_ptr())
        torch.cuda.synchronize()
        out.append((fbt.cpu().numpy(), bits(act.cpu().numpy())))
        fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
        ctx.render_tiles(setup.lp, W, H, 1, 3, fb.data_ptr(), acc.data_ptr())
        torch.cuda.synchronize()
        out.append((fb.cpu().numpy(), bits(acc.cpu().numpy())))
        return out

    for (a0, a1), (b0, b1) in zip(tiles(True), tiles(False)):
        assert np.array_equal(a0, b0) and np.array_equal(a1, b1)
    ctx.close()


def test_statistics_off_renders_the_same_frames():
    """irt_set_statistics(ctx, 0): no per-workgroup count stores -- the same pixels, the
    counts read 0; back on, the counts are the oracle's again.  Also many launches in a row
    with the done markers recorded only every 8th launch (the ring's covering events)."""
    import torch
    cells = irt.synth_grid(2, 3, 90)
    W = 96
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, W, W, camera=FRAMING)
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    for on in (False, True, False, True):
        ctx.set_statistics(on)
        for _ in range(11):  # past a done-marker boundary each time
            acc.zero_()
            fb.zero_()
            ctx.render(setup.lp, W, W, fb.data_ptr(), acc.data_ptr())
        st = ctx.stats()
        a = acc.cpu().numpy().reshape(W, W, 4)
        f = fb.cpu().numpy().reshape(W, W).view(np.uint32)
        assert_same_frame(a, f, a_ref, f_ref, f"statistics {'on' if on else 'off'}")
        if on:
            assert (st.locateCalls, st.samplesFound) == (st_ref[0].locate_calls, st_ref[0].samples_found)
        else:
            assert (st.raysLaunched, st.locateCalls, st.samplesFound) == (0, 0, 0)
    ctx.close()
