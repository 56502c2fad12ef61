"""GPU parity of GRID_ACCEL_MODE (Params.h:34): the raygen woodcockTrackingWithAccel with
dda3 (DDA.h:35-136) over the 256^3 Cartesian macrocell grid built by buildGrid_ICON
(hostCode.cu:205-297, 668-682), against the oracle and the reference's own outputs
(tests/golden/kats_grid.npz, made from oracle/_ref).  Bar: bit-exact."""
import hashlib

import numpy as np
import pytest

import irt
from golden_util import GOLDEN, load
from helpers import FRAMING, bits, gpu_frame, oracle_frame
from test_gpu_parity import assert_same_frame

pytestmark = pytest.mark.gpu


def test_grid_build_matches_reference_kats():
    z = np.load(f"{GOLDEN}/kats_grid.npz")
    cells = np.ascontiguousarray(z["grid_cells"]).view(irt.CELL_DTYPE).ravel()
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(z["grid_lut"], tuple(float(v) for v in z["grid_value_range"]), 1.0)
    vr, mo = ctx.grid()
    pick = z["grid_pick"]
    # value ranges equal as numbers (the sign of a zero bound follows atomic arrival order)
    assert np.array_equal(vr[pick], z["grid_pick_vr"])
    assert int((vr[:, 1] >= vr[:, 0]).sum()) == int(z["grid_nonempty"])
    assert np.array_equal(bits(mo[pick]), bits(z["grid_pick_maxop"]))
    assert hashlib.sha256(mo.tobytes()).digest() == z["grid_maxop_sha256"].tobytes()
    ctx.close()


def test_grid_build_matches_oracle():
    cells = irt.synth_grid(2, 3, 47, noise=0.1)
    _, _, _, S = oracle_frame(cells, 8, 8, camera=FRAMING, accel_mode=1)
    setup = irt.setup_frame(cells, 8, 8)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    vr, mo = ctx.grid()
    assert np.array_equal(vr, S.grid_vr)
    assert np.array_equal(bits(mo), bits(S.grid_max_op))
    ctx.close()


def test_grid_build_reads_value31_of_unsorted_records():
    """getValue at a record's own heights (buildGrid_ICON, hostCode.cu:245-250) can reach
    index numLayers = 31 when the heights are not sorted (findHeight, ICONGrid.h:117-145),
    and then reads value[31].  Records of 31 layers whose low heights exceed height[31] --
    the last record among them -- must give the oracle's value ranges and majorants."""
    cells = irt.synth_grid(2, 2, 62)  # two 31-layer records per column
    assert (cells["numLayers"] == 31).all()
    rng = np.random.default_rng(31)
    pick = np.concatenate([rng.choice(cells.size - 1, 40, replace=False), [cells.size - 1]])
    for i in pick:
        h = cells["height"][i].copy()
        h[0] = h[31] + (h[31] - h[0])  # height[0] above every other: findHeight(height[0]) = 31
        cells["height"][i] = h
        cells["value"][i, 31] = 1e3 + i  # outside every other value: a wrong slot shows
    _, _, _, S = oracle_frame(cells, 8, 8, camera=FRAMING, accel_mode=1)
    setup = irt.setup_frame(cells, 8, 8)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    vr, mo = ctx.grid()
    assert (S.grid_vr[:, 1] >= 1e3).any()  # value[31] does reach the grid
    assert np.array_equal(vr, S.grid_vr)
    assert np.array_equal(bits(mo), bits(S.grid_max_op))
    ctx.close()


GRID_CASES = [
    # (rootN, bisections, levels, W, camera, raygen, accumIDs)
    (1, 0, 4, 96, None, 0, (0,)),      # C1-class, viewAll camera
    (2, 2, 60, 80, FRAMING, 0, (0,)),
    (2, 3, 47, 64, FRAMING, 0, (0, 2, 3)),  # progressive accumulation
    (2, 2, 30, 64, FRAMING, 1, (0,)),  # AE raygen ignores the accel mode
]


@pytest.mark.parametrize("rn,bis,L,W,cam,raygen,ids", GRID_CASES)
def test_grid_frame_bit_exact(rn, bis, L, W, cam, raygen, ids):
    cells = irt.synth_grid(rn, bis, L)
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, W, W, camera=cam, raygen=raygen,
                                           accum_ids=ids, accel_mode=1)
    a_gpu, f_gpu, st_gpu, ctx = gpu_frame(cells, W, W, camera=cam, raygen=raygen,
                                          accum_ids=ids, accel_mode=1)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, f"grid R{rn}B{bis:02d}L{L}")
    for g, o in zip(st_gpu, st_ref):
        assert (g.locateCalls, g.samplesFound) == (o.locate_calls, o.samples_found)
    ctx.close()


def test_grid_golden_frame():
    """f6: the reference's own GRID_ACCEL_MODE frame (also covered by the generic golden
    test); here with the mode switched back and forth on one context."""
    d = load("f6_r2b02_l60_grid")
    W, H = int(d["width"]), int(d["height"])
    from helpers import GpuFrame
    ctx = irt.Context(d["cells"], 0)
    ctx.set_transfunc(d["lut"], tuple(float(v) for v in d["value_range"]), 1.0)
    fr = GpuFrame(ctx, W, H)
    c = d["camera12"]
    lp = irt.LaunchParams()
    lp.org, lp.dir_00, lp.dir_du, lp.dir_dv = (irt.vec3(c[i:i + 3]) for i in (0, 3, 6, 9))
    lp.ambientColor = irt.Vec3(1, 1, 1)
    lp.ambientRadiance = 1.0
    lp.unitDistance = float(d["unit_distance"])
    lp.accelMode = irt.ACCEL_SPHERE
    fr.render(lp)  # a sphere-mode frame first: the grid path must not depend on it
    fr.accum.zero_()
    fr.fb.zero_()
    lp.accelMode = irt.ACCEL_GRID
    st = fr.render(lp)
    assert (st.locateCalls, st.samplesFound) == tuple(int(v) for v in d["counts"][0])
    a, f = fr.host()
    assert_same_frame(a, f, d["accum"], d["fb"], "f6 grid")
    ctx.close()


def test_unknown_accel_mode_is_rejected():
    cells = irt.synth_grid(1, 0, 4)
    setup = irt.setup_frame(cells, 16, 16)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    from helpers import GpuFrame
    fr = GpuFrame(ctx, 16, 16)
    setup.lp.accelMode = 7
    with pytest.raises(irt.IrtError):
        fr.render(setup.lp)
    ctx.close()


@pytest.mark.slow
def test_grid_c2_strided_pixels_match_oracle():
    """C2 (R2B05 x 47 levels, 512^2) in GRID_ACCEL_MODE: a strided pixel sample against the
    oracle (the raygen is per-pixel independent), plus determinism of the full frame."""
    import oracle as O
    from helpers import GpuFrame
    W = 512
    cells = irt.synth_grid(2, 5, 47)
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    setup.lp.accelMode = irt.ACCEL_GRID
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    fr = GpuFrame(ctx, W, W)
    st = fr.render(setup.lp)
    a, f = fr.host()
    S = O.OracleScene(cells)
    S.set_transfunc(setup.lut, setup.value_range)
    lp = setup.lp
    cam = tuple(np.array(v.tolist(), np.float32) for v in (lp.org, lp.dir_00, lp.dir_du, lp.dir_dv))
    p = S.params(cam, accum_id=0, raygen=0, unit_distance=lp.unitDistance, accel_mode=1)
    ys, xs = np.mgrid[3:W:16, 5:W:16]
    xy = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    a_ref, f_ref, _ = S.render_pixels(p, W, W, xy, threads=16, fast=True)
    xs, ys = xy[:, 0], xy[:, 1]
    bad = np.any(bits(a[ys, xs]) != bits(a_ref[ys, xs]), axis=-1) | (f[ys, xs] != f_ref[ys, xs])
    assert not bad.any(), f"{int(bad.sum())} of {len(xy)} sampled pixels differ"
    assert (a_ref[ys, xs, 3] > 0).sum() > len(xy) // 3
    fr.accum.zero_()
    fr.fb.zero_()
    st2 = fr.render(lp)
    a2, f2 = fr.host()
    assert np.array_equal(bits(a2), bits(a)) and np.array_equal(f2, f)
    assert st2.samplesFound == st.samplesFound
    ctx.close()
