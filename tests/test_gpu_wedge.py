"""GPU parity of the unstructured samplers: TRIANGLE_MODE (deviceCode.cu:61-76; the
product's ray_triangle definition, parity unpinned) and the CUBQL_MODE sampler
(Params.h:31; deviceCode.cu:90-115): sampleVolume
through the wedges of buildCuBQLAccel (hostCode.cu:557-600) and intersectWedgeEXT
(UElems.h:214-311), against the oracle's brute-force wedge scan and the reference's own
outputs (tests/golden/kats_wedge.npz, f7_*_wedge.npz).  Bar: bit-exact.

Parity note: cuBQL's BVH traversal order is not reproducible (the submodule is not
vendored); both sides take the first accepting wedge in (cell, layer) order."""
import numpy as np
import pytest

import irt
from helpers import FRAMING, GpuFrame, bits, gpu_frame, oracle_frame
from test_gpu_parity import assert_same_frame

pytestmark = pytest.mark.gpu

WEDGE_CASES = [
    # (rootN, bisections, levels, W, camera, accelMode, accumIDs)
    (2, 1, 12, 48, FRAMING, 0, (0,)),
    (2, 2, 20, 64, FRAMING, 0, (0, 2)),
    (2, 3, 47, 48, FRAMING, 0, (0,)),
    (2, 2, 20, 48, None, 0, (0,)),
    (2, 2, 20, 48, FRAMING, 1, (0,)),  # with GRID_ACCEL_MODE traversal
    (1, 0, 4, 48, FRAMING, 0, (0,)),   # 20 faces: Newton rarely converges (reference)
]


@pytest.mark.parametrize("rn,bis,L,W,cam,accel,ids", WEDGE_CASES)
def test_wedge_frame_bit_exact(rn, bis, L, W, cam, accel, ids):
    cells = irt.synth_grid(rn, bis, L, noise=0.2)
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, W, W, camera=cam, accum_ids=ids,
                                           accel_mode=accel, mode=2, threads=16)
    a_gpu, f_gpu, st_gpu, ctx = gpu_frame(cells, W, W, camera=cam, accum_ids=ids,
                                          accel_mode=accel, mode=2)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, f"wedge R{rn}B{bis:02d}L{L}")
    for g, o in zip(st_gpu, st_ref):
        assert (g.locateCalls, g.samplesFound) == (o.locate_calls, o.samples_found)
    ctx.close()


def test_wedge_mode_needs_its_accel():
    cells = irt.synth_grid(2, 0, 4)
    setup = irt.setup_frame(cells, 16, 16)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    fr = GpuFrame(ctx, 16, 16)
    setup.lp.mode = irt.MODE_CUBQL
    with pytest.raises(irt.IrtError, match="irt_build_wedge_accel"):
        fr.render(setup.lp)
    setup.lp.mode = irt.MODE_TRIANGLES  # needs the same accel
    with pytest.raises(irt.IrtError, match="irt_build_wedge_accel"):
        fr.render(setup.lp)
    setup.lp.mode = 7
    with pytest.raises(irt.IrtError, match="unknown sampler"):
        fr.render(setup.lp)
    with pytest.raises(irt.IrtError):
        ctx.build_wedge_accel(cells[:-1])
    ctx.build_wedge_accel(cells)
    setup.lp.mode = irt.MODE_CUBQL
    fr.render(setup.lp)
    ctx.close()


@pytest.mark.slow
def test_wedge_c2_strided_pixels_match_oracle():
    """C2 (R2B05 x 47, 512^2) in CUBQL_MODE: a strided pixel sample against the oracle's
    brute-force wedge scan (3.85 M wedges)."""
    import oracle as O
    W = 512
    cells = irt.synth_grid(2, 5, 47)
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    setup.lp.mode = irt.MODE_CUBQL
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    ctx.build_wedge_accel(cells)
    fr = GpuFrame(ctx, W, W)
    fr.render(setup.lp)
    a, f = fr.host()
    S = O.OracleScene(cells)
    S.set_transfunc(setup.lut, setup.value_range)
    lp = setup.lp
    cam = tuple(np.array(v.tolist(), np.float32) for v in (lp.org, lp.dir_00, lp.dir_du, lp.dir_dv))
    p = S.params(cam, accum_id=0, raygen=0, unit_distance=lp.unitDistance, mode=2)
    ys, xs = np.mgrid[7:W:40, 9:W:40]
    xy = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    a_ref, f_ref, _ = S.render_pixels(p, W, W, xy, threads=16, fast=True)
    xs, ys = xy[:, 0], xy[:, 1]
    bad = np.any(bits(a[ys, xs]) != bits(a_ref[ys, xs]), axis=-1) | (f[ys, xs] != f_ref[ys, xs])
    assert not bad.any(), f"{int(bad.sum())} of {len(xy)} sampled pixels differ"
    assert (a_ref[ys, xs, 3] > 0).sum() > len(xy) // 3
    ctx.close()


TRI_CASES = [
    # (rootN, bisections, levels, W, camera, accelMode)
    (2, 2, 30, 64, FRAMING, 0),
    (2, 3, 47, 64, None, 0),
    (2, 2, 20, 48, FRAMING, 1),  # with GRID_ACCEL_MODE traversal
    (1, 0, 4, 48, FRAMING, 0),
]


@pytest.mark.parametrize("rn,bis,L,W,cam,accel", TRI_CASES)
def test_triangle_frame_bit_exact(rn, bis, L, W, cam, accel):
    cells = irt.synth_grid(rn, bis, L, noise=0.2)
    a_ref, f_ref, st_ref, _ = oracle_frame(cells, W, W, camera=cam, accel_mode=accel, mode=1,
                                           threads=16)
    a_gpu, f_gpu, st_gpu, ctx = gpu_frame(cells, W, W, camera=cam, accel_mode=accel,
                                          mode=irt.MODE_TRIANGLES)
    assert_same_frame(a_gpu, f_gpu, a_ref, f_ref, f"triangles R{rn}B{bis:02d}L{L}")
    assert (st_gpu[0].locateCalls, st_gpu[0].samplesFound) == (st_ref[0].locate_calls,
                                                               st_ref[0].samples_found)
    ctx.close()
