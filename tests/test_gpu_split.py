"""A single frame's tail in half packets (RenderArgs::splitFrom, irt_debug_set_split_tail).

A one-frame launch of the one-wave-workgroup kernel may render its last packets with two
workgroups of 32 rays each (rows 0-3 and 4-7 of the 8x8 packet) instead of one of 64, so that
the launch's last waves are shorter.  Every ray is computed as before (its seed, draws and
locate are the lane layout's business only), so frames and counts must be bit-identical to the
unsplit launch, for full frames, ragged frames and tile lists, and for every split size.
"""
import numpy as np
import pytest

import irt
from helpers import FRAMING, bits

pytestmark = pytest.mark.gpu


def _frame(ctx, lp, W, H, split, tiles=None):
    import torch
    ctx.set_split_tail(split)
    n = W * H if tiles is None else len(tiles) * 4096
    fb = torch.zeros(n, dtype=torch.int32, device="cuda")
    acc = torch.zeros(n * 4, dtype=torch.float32, device="cuda")
    if tiles is None:
        ctx.render(lp, W, H, fb.data_ptr(), acc.data_ptr())
    else:
        ctx.render_tile_list(lp, W, H, tiles, 1, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    st = ctx.stats()
    return (fb.cpu().numpy().copy(), bits(acc.cpu().numpy()),
            (st.raysLaunched, st.raysInBox, st.locateCalls, st.samplesFound, st.candidatesTested))


@pytest.mark.parametrize("rn,bis,L,W,H,cam", [
    (2, 2, 47, 200, 136, None),        # ragged: partial tiles, rays outside the box
    (2, 3, 90, 512, 512, FRAMING),     # 4,096 one-wave workgroups
    (2, 5, 90, 1024, 1024, FRAMING),   # 16,384: more than the chip holds
])
def test_split_tail_equals_unsplit(rn, bis, L, W, H, cam):
    cells = irt.synth_grid(rn, bis, L)
    setup = irt.setup_frame(cells, W, H, camera=cam)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    setup.lp.accumID = 3
    ref = _frame(ctx, setup.lp, W, H, 0)
    nwg = ctx.launch_workgroups(((W + 63) // 64) * ((H + 63) // 64), 1)
    for split in (8, 1000, 1 << 30):
        got = _frame(ctx, setup.lp, W, H, split)
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), split
        assert got[2] == ref[2], split
        # the launch has one more workgroup per split packet
        assert ctx.launch_workgroups(((W + 63) // 64) * ((H + 63) // 64), 1) == nwg + min(split, nwg) // 8 * 8
    ctx.set_split_tail(0)
    ctx.close()


def test_split_tail_tile_list_and_progressive():
    """A rank's tile list (packed output) split, and multi-frame launches (chained: never split)
    unchanged."""
    cells = irt.synth_grid(2, 2, 47)
    W, H = 320, 256
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    tiles = np.array([5, 0, 19, 7, 6, 12], dtype=np.int32)
    ref = _frame(ctx, setup.lp, W, H, 0, tiles)
    got = _frame(ctx, setup.lp, W, H, 200, tiles)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    assert got[2] == ref[2]
    assert ctx.launch_workgroups(6, 4) == 6 * 64 * 4  # a chained launch is not split
    ctx.set_split_tail(0)
    ctx.close()
