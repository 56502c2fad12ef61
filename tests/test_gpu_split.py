"""Measured-cost scheduling with split packets (irt_context.hip sched_prepare, RenderArgs::splitList).

Single frames of a scene with holes run in measured-cost order by default: every 8th launch
records each packet's duration, and later launches start the costliest 64x64 tiles first and
render the packets longer than IRT_SPLIT_FACTOR x the frame's ideal span ahead of the rest, in
2^splitLg parts of 64 >> splitLg rays, one one-wave workgroup each.  Only the lane layout
changes, so every frame and every count must equal an unscheduled context's.  A tiny
IRT_SPLIT_FACTOR splits the costliest tenth of the packets whatever their cost.
"""
import numpy as np
import pytest

import irt
from helpers import FRAMING, bits

pytestmark = pytest.mark.gpu


def _frames(ctx, lp, W, n):
    import torch
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    out = []
    for aid in range(n):
        lp.accumID = aid
        ctx.render(lp, W, W, fb.data_ptr(), acc.data_ptr())
        torch.cuda.synchronize()
        st = ctx.stats()
        out.append((fb.cpu().numpy().copy(), bits(acc.cpu().numpy()),
                    (st.raysLaunched, st.raysInBox, st.locateCalls, st.samplesFound, st.candidatesTested),
                    ctx.sched_split()[0]))
    return out


@pytest.mark.parametrize("terrain,lg", [(4000.0, 1), (4000.0, 2), (0.0, 1)])
def test_split_packets_equal_unscheduled(monkeypatch, terrain, lg):
    cells = irt.synth_grid(2, 4, 90, terrain=terrain)
    W = 384
    setup = irt.setup_frame(cells, W, W, camera=FRAMING)
    monkeypatch.setenv("IRT_SCHED", "0")
    ref_ctx = irt.Context(cells, 0)
    monkeypatch.setenv("IRT_SCHED", "1")  # the default for terrain; forced on the flat grid
    monkeypatch.setenv("IRT_SPLIT_FACTOR", "1e-6")
    monkeypatch.setenv("IRT_SPLIT_LG", str(lg))
    ctx = irt.Context(cells, 0)
    for c in (ref_ctx, ctx):
        c.set_transfunc(setup.lut, setup.value_range)
    n = 24
    ref = _frames(ref_ctx, setup.lp, W, n)
    got = _frames(ctx, setup.lp, W, n)
    for k in range(n):
        assert np.array_equal(got[k][0], ref[k][0]) and np.array_equal(got[k][1], ref[k][1]), k
        assert got[k][2] == ref[k][2], k
    assert all(r[3] == 0 for r in ref)
    splits = [g[3] for g in got]
    assert max(splits) >= 8 and max(splits) % 8 == 0, splits  # the later launches did split
    ref_ctx.close()
    ctx.close()


def test_scenes_with_holes_schedule_by_default():
    import ctypes as C
    cells = irt.synth_grid(2, 3, 90, terrain=4000.0)
    ctx = irt.Context(cells, 0)
    L = irt.lib()
    L.irt_debug_sched.argtypes = [C.c_void_p] + [C.c_void_p] * 3
    p, a, n = C.c_int(), C.c_int(), C.c_longlong()
    assert L.irt_debug_sched(ctx._h, C.byref(p), C.byref(a), C.byref(n)) == 0
    import os
    if not os.environ.get("IRT_SCHED"):
        assert p.value == 1
    flat = irt.Context(irt.synth_grid(2, 3, 90), 0)
    assert L.irt_debug_sched(flat._h, C.byref(p), C.byref(a), C.byref(n)) == 0
    if not os.environ.get("IRT_SCHED"):
        assert p.value == 0
    ctx.close()
    flat.close()
