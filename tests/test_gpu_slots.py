"""The slot table (irt_common.h kSlot4, csrc/irt_build.hip k_slot_fill; Tracer::locate_wave's
OPT_SLOT form): per (cube-map cell, slot unit of 4 sub-cells -- 2 or 1 with IRT_SLOT_SUBS --,
radial bin) of a scene whose cells share their radial edges, the first candidate the unit's
sub-cell masks admit, the masks and the list's position, so that a sample's scan starts with one
gather (the slot's copy, when it is the sample's own first admitted candidate).

Pinned here: the table the device builds equals a numpy restatement from the headers and fat
entries byte for byte; frames, accumulators and every count equal a context without the table
(IRT_SLOTS=0); scenes whose cells' edges are more than three distinct values (terrain) get no
table; by default only
scenes whose headers outgrow the last-level cache get one.  The small scenes here force it
(IRT_SLOTS=1); tests/test_gpu_parity.py::test_device_locator_slot_table runs the wave-wide
locate through it against the host restatement, test_gpu_scale.py's C5 frames run through it.
"""
import numpy as np
import pytest

import irt
from helpers import FRAMING, bits, restate_slots

pytestmark = pytest.mark.gpu

@pytest.mark.parametrize("subs", [4, 2, 1])
@pytest.mark.parametrize("scene", ["r2b02_l90", "r2b03_l47_noise", "r2b03_l20", "filtered"])
def test_slot_table_restated(monkeypatch, scene, subs):
    """(filtered: cells at the region's border hold fewer records and fewer edges, a subset of
    the others')"""
    monkeypatch.setenv("IRT_SLOTS", "1")
    monkeypatch.setenv("IRT_SLOT_SUBS", str(subs))
    cells = {"r2b02_l90": lambda: irt.synth_grid(2, 2, 90),
             "r2b03_l47_noise": lambda: irt.synth_grid(2, 3, 47, noise=0.2),
             "r2b03_l20": lambda: irt.synth_grid(2, 3, 20),
             "filtered": lambda: irt.filter_cells(irt.synth_grid(2, 3, 40), (-30, 60), (-90, 45))}[scene]()
    ctx = irt.Context(cells, 0)
    slots = ctx.array("slots")
    assert slots.size > 0, "a flat grid's cells share their edges"
    want = restate_slots(ctx.array("bin_hdr"), ctx.array("fat"), subs)
    got = slots.view(np.uint32)
    assert want is not None and got.size == want.size
    if not np.array_equal(got, want):
        w = np.nonzero(got != want)[0]
        raise AssertionError(f"{w.size} words differ, first at {w[0]}")
    ctx.close()


@pytest.mark.parametrize("bis", [3, 4])
def test_default_unit_fits_the_scene(monkeypatch, bis):
    """Without IRT_SLOT_SUBS the context takes the finest slot unit (1, 2, then 4 sub-cells)
    whose table is at most the scene's own bytes -- its headers, fat entries and blocks -- and
    quads otherwise: the table equals that unit's restatement."""
    monkeypatch.setenv("IRT_SLOTS", "1")
    monkeypatch.delenv("IRT_SLOT_SUBS", raising=False)
    ctx = irt.Context(irt.synth_grid(2, bis, 90), 0)
    got = ctx.array("slots").view(np.uint32)
    hdr, fat = ctx.array("bin_hdr"), ctx.array("fat")
    tables = {u: restate_slots(hdr, fat, u) for u in (1, 2, 4)}
    scene = sum(ctx.array_bytes(a) for a in ("bin_hdr", "fat", "blocks"))
    sizes = {u: t.nbytes for u, t in tables.items()}
    if any(abs(sizes[u] - scene) < 0.05 * scene for u in (1, 2)):
        pytest.skip("a unit's table is within 5 % of the scene's bytes")
    want = next((u for u in (1, 2) if sizes[u] <= scene), 4)
    assert got.size == tables[want].size and np.array_equal(got, tables[want]), (want, sizes, scene)
    ctx.close()


def test_cells_with_own_edges_have_no_table(monkeypatch):
    monkeypatch.setenv("IRT_SLOTS", "1")
    ctx = irt.Context(irt.synth_grid(2, 3, 90, terrain=4000.0), 0)
    assert ctx.array("slots").size == 0
    assert restate_slots(ctx.array("bin_hdr"), ctx.array("fat")) is None  # > 3 distinct edges
    ctx.close()


def test_slots_off_and_auto(monkeypatch):
    cells = irt.synth_grid(2, 3, 90)
    monkeypatch.setenv("IRT_SLOTS", "0")
    ctx = irt.Context(cells, 0)
    assert ctx.array("slots").size == 0
    ctx.close()
    monkeypatch.delenv("IRT_SLOTS")
    ctx = irt.Context(cells, 0)  # 1,350 cells of headers: no table by default
    assert ctx.array("slots").size == 0
    ctx.close()


def _frames(ctx, lp, W, n, batch):
    import torch
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    out = []
    for aid in range(0, n, batch):
        lp.accumID = aid
        if batch == 1:
            ctx.render(lp, W, W, fb.data_ptr(), acc.data_ptr())
        else:
            ctx.render_accumulate(lp, W, W, batch, fb.data_ptr(), acc.data_ptr())
        torch.cuda.synchronize()
        st = ctx.stats()
        out.append((fb.cpu().numpy().copy(), bits(acc.cpu().numpy()),
                    (st.raysLaunched, st.raysInBox, st.locateCalls, st.samplesFound, st.candidatesTested)))
    return out


@pytest.mark.parametrize("bis,levels,batch,subs", [(4, 90, 1, 4), (4, 90, 4, 4), (3, 47, 1, 4), (4, 90, 1, 2),
                                                   (3, 47, 1, 1)])
def test_frames_equal_without_table(monkeypatch, bis, levels, batch, subs):
    cells = irt.synth_grid(2, bis, levels, noise=0.1 if levels == 47 else 0.0)
    W = 320
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    monkeypatch.setenv("IRT_SLOTS", "0")
    ref_ctx = irt.Context(cells, 0)
    monkeypatch.setenv("IRT_SLOTS", "1")
    monkeypatch.setenv("IRT_SLOT_SUBS", str(subs))
    ctx = irt.Context(cells, 0)
    assert ctx.array("slots").size > 0 and ref_ctx.array("slots").size == 0
    for c in (ref_ctx, ctx):
        c.set_transfunc(setup.lut, setup.value_range)
    n = 8
    ref = _frames(ref_ctx, setup.lp, W, n, batch)
    got = _frames(ctx, setup.lp, W, n, batch)
    for k in range(len(ref)):
        assert np.array_equal(got[k][0], ref[k][0]) and np.array_equal(got[k][1], ref[k][1]), k
        assert got[k][2] == ref[k][2], k
    ref_ctx.close()
    ctx.close()


def _comb(lut):
    """bench.py's sparse "comb" TF: alpha 0.01, every 50th entry 1.0"""
    lut = np.array(lut, dtype=np.float32, copy=True)
    lut[:, 3] = 0.01
    lut[::50, 3] = 1.0
    return lut


def test_sparse_transfer_function_uses_the_table(monkeypatch):
    """A scene whose headers fit the last-level cache builds the table on its first sparse TF
    (mean Woodcock samples per acceptance >= 8) and its launches start from it while that TF is
    set; the dense default TF does not use it.  Frames and counts equal a context without the
    table either way."""
    import ctypes as C
    monkeypatch.delenv("IRT_SLOTS", raising=False)
    monkeypatch.delenv("IRT_SLOT_SUBS", raising=False)
    cells = irt.synth_grid(2, 4, 90)
    W = 256
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    L = irt.lib()
    L.irt_debug_slot_use.argtypes = [C.c_void_p, C.c_void_p]
    ctx = irt.Context(cells, 0)
    monkeypatch.setenv("IRT_SLOTS", "0")
    ref = irt.Context(cells, 0)
    monkeypatch.delenv("IRT_SLOTS")
    samples = C.c_double()
    ctx.set_transfunc(setup.lut, setup.value_range)
    assert L.irt_debug_slot_use(ctx._h, C.byref(samples)) == 0 and 0 < samples.value < 8
    assert ctx.array("slots").size == 0  # not built for a dense TF
    comb = _comb(setup.lut)
    for c in (ctx, ref):
        c.set_transfunc(comb, setup.value_range)
    assert L.irt_debug_slot_use(ctx._h, C.byref(samples)) == 1 and samples.value >= 8
    assert ctx.array("slots").size > 0 and L.irt_debug_slot_use(ref._h, None) == 0
    a, b = _frames(ctx, setup.lp, W, 4, 2), _frames(ref, setup.lp, W, 4, 2)
    for k in range(len(a)):
        assert np.array_equal(a[k][0], b[k][0]) and np.array_equal(a[k][1], b[k][1]) and a[k][2] == b[k][2], k
    ctx.set_transfunc(setup.lut, setup.value_range)  # dense again: the table stays, unused
    assert L.irt_debug_slot_use(ctx._h, None) == 0 and ctx.array("slots").size > 0
    ctx.close()
    ref.close()

