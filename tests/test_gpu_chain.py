"""Chained progressive frames (RenderArgs::chain, the default for multi-frame launches).

irt_render_accumulate / irt_render_tile_list with k frames: workgroup (b, f) lerps frame f of
block b straight into accum/fb once frame f - 1's wave of the same pixels has published them
(write-through stores + a per-(block, wave) epoch word), instead of the per-frame sample buffer
and the k_accumulate pass.  Bit-identical to the sample-buffer batch and to k single-frame
launches (which the oracle pins in test_gpu_parity.py), counts included; no wait may time out.
Frames small enough that all k frames' workgroups are resident at once exercise real waits;
large ones (more workgroups than the chip holds) the normal case of an already-published word.
"""
import numpy as np
import pytest

import irt
from helpers import FRAMING, bits

pytestmark = pytest.mark.gpu


def _batch(ctx, lp, W, H, k, first, chain, prior=0):
    import torch
    ctx.set_chain(chain)
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    for aid in range(prior):
        lp.accumID = aid
        ctx.render(lp, W, H, fb.data_ptr(), acc.data_ptr())
    lp.accumID = first
    ctx.render_accumulate(lp, W, H, k, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    st = ctx.stats()
    return (fb.cpu().numpy().copy(), bits(acc.cpu().numpy()),
            (st.raysLaunched, st.raysInBox, st.locateCalls, st.samplesFound, st.candidatesTested))


@pytest.mark.parametrize("rn,bis,L,W,H,k,cam", [
    (2, 2, 47, 96, 80, 2, FRAMING),      # 4 tiles: every frame resident at once
    (2, 2, 47, 200, 136, 5, None),       # viewAll: rays that hit the box in some frames only
    (2, 3, 90, 512, 512, 9, FRAMING),    # 1,024 workgroups per frame
    (2, 3, 90, 1024, 1024, 3, FRAMING),  # 4,096 per frame: more than the chip holds
])
def test_chained_batch_equals_sample_buffer_batch(rn, bis, L, W, H, k, cam):
    cells = irt.synth_grid(rn, bis, L)
    setup = irt.setup_frame(cells, W, H, camera=cam)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    ref = _batch(ctx, setup.lp, W, H, k, 0, chain=False)
    got = _batch(ctx, setup.lp, W, H, k, 0, chain=True)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    assert got[2] == ref[2]
    # continuing an accumulation: two single frames, then a chained batch from accumID 2
    ref = _batch(ctx, setup.lp, W, H, k, 2, chain=False, prior=2)
    got = _batch(ctx, setup.lp, W, H, k, 2, chain=True, prior=2)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    assert ctx.chain_errors() == 0
    ctx.close()


def test_chained_tile_lists_equal_sample_buffer_tile_lists():
    """A rank's tile list (the multi-GPU progressive mode) over k chained frames, repeated
    (the epochs advance from launch to launch on the same publish words)."""
    import torch
    cells = irt.synth_grid(2, 2, 47)
    W, H, k = 320, 256, 4
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    tiles = np.array([5, 0, 19, 7, 6, 12], dtype=np.int32)
    out = {}
    for chain in (False, True):
        ctx.set_chain(chain)
        fbt = torch.zeros(len(tiles) * 4096, dtype=torch.int32, device="cuda")
        acct = torch.zeros(len(tiles) * 4096 * 4, dtype=torch.float32, device="cuda")
        res = []
        for rep in range(3):
            setup.lp.accumID = rep * k
            ctx.render_tile_list(setup.lp, W, H, tiles, k, fbt.data_ptr(), acct.data_ptr())
            torch.cuda.synchronize()
            res.append((fbt.cpu().numpy().copy(), bits(acct.cpu().numpy())))
        out[chain] = res
    for (fa, aa), (fb_, ab) in zip(out[False], out[True]):
        assert np.array_equal(fa, fb_) and np.array_equal(aa, ab)
    assert ctx.chain_errors() == 0
    ctx.close()


@pytest.mark.parametrize("accel,sampler", [(irt.ACCEL_GRID, irt.MODE_USER_GEOM),
                                           (0, irt.MODE_CUBQL)])
def test_chained_batch_other_kernels(accel, sampler):
    """The grid-accel and wedge-sampler kernels run the same chained epilogue."""
    cells = irt.synth_grid(2, 0, 12)
    W, H, k = 128, 128, 3
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    if sampler != irt.MODE_USER_GEOM:
        ctx.build_wedge_accel(cells)
    setup.lp.accelMode = accel
    setup.lp.mode = sampler
    ref = _batch(ctx, setup.lp, W, H, k, 0, chain=False)
    got = _batch(ctx, setup.lp, W, H, k, 0, chain=True)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    assert got[2] == ref[2]
    assert ctx.chain_errors() == 0
    ctx.close()


def _views(setup, W, H, n, first=0, accum=None):
    """n orbit views around the globe (a new view per frame, accumID 0 unless `accum`)."""
    out = []
    for k in range(n):
        th = 2.0 * np.pi * (first + k) / 60.0
        c = irt.camera_look_at((1.4e7 * np.sin(th), 0.0, 1.4e7 * np.cos(th)), (0.0, 0.0, 0.0),
                               (0.0, 1.0, 0.0), 60.0, W, H)
        q = irt.LaunchParams.from_buffer_copy(setup.lp)
        q.org, q.dir_00, q.dir_du, q.dir_dv = c.org, c.dir_00, c.dir_du, c.dir_dv
        q.accumID = 0 if accum is None else accum + k
        out.append(q)
    return out


@pytest.mark.parametrize("W,H,n,accum", [(96, 80, 5, None), (512, 512, 7, None), (200, 136, 4, 3)])
def test_sequence_equals_single_launches(W, H, n, accum):
    """irt_render_sequence (an orbit: camera and accumID per frame, chained in one launch) ==
    the same views rendered one launch each, counts included; a moving camera that keeps
    accumulating (accumID 3, 4, ...) too."""
    import torch
    cells = irt.synth_grid(2, 3, 90)
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    lps = _views(setup, W, H, n, accum=accum)
    out = []
    for seq in (False, True):
        fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
        if seq:
            ctx.render_sequence(lps, W, H, fb.data_ptr(), acc.data_ptr())
        else:
            for q in lps:
                ctx.render(q, W, H, fb.data_ptr(), acc.data_ptr())
        torch.cuda.synchronize()
        out.append((fb.cpu().numpy().copy(), bits(acc.cpu().numpy())))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    # counts: the sequence's launch against the sum of the single launches
    ctx.reset_stats_total()
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    for q in lps:
        ctx.render(q, W, H, fb.data_ptr(), acc.data_ptr())
    ref, _ = ctx.stats_total()
    ctx.reset_stats_total()
    ctx.render_sequence(lps, W, H, fb.data_ptr(), acc.data_ptr())
    got, _ = ctx.stats_total()
    for f in ("raysLaunched", "raysInBox", "locateCalls", "samplesFound", "candidatesTested"):
        assert getattr(got, f) == getattr(ref, f), f
    assert ctx.chain_errors() == 0
    # without chaining the sequence is one launch per view (the host loop): the same frames
    ctx.set_chain(False)
    fb2 = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    acc2 = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    ctx.render_sequence(lps, W, H, fb2.data_ptr(), acc2.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(fb2.cpu().numpy(), out[0][0]) and np.array_equal(bits(acc2.cpu().numpy()), out[0][1])
    ctx.set_chain(True)
    # only the camera and accumID may differ between frames
    bad = _views(setup, W, H, 2)
    bad[1].ambientRadiance = bad[0].ambientRadiance * 2.0
    with pytest.raises(irt.IrtError):
        ctx.render_sequence(bad, W, H, fb.data_ptr(), acc.data_ptr())
    ctx.close()


def test_tile_list_sequence_split_equals_full_sequence():
    """irt_render_tile_list_sequence on every rank's tiles (the multi-GPU split of an orbit,
    both deals), unpacked, equals the full-frame sequence."""
    import torch
    import irt_dist
    cells = irt.synth_grid(2, 3, 90)
    W, H, n = 320, 200, 5
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    lps = _views(setup, W, H, n)
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    ctx.render_sequence(lps, W, H, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    ref = fb.cpu().numpy().copy()
    for ranks in (2, 3):
        for dealt in (False, True):
            splits = [irt_dist.TileSplit.dealt(W, H, r, ranks, lps[0], ctx.info, n) if dealt
                      else irt_dist.TileSplit(W, H, r, ranks) for r in range(ranks)]
            maxt = max(sp.max_tiles for sp in splits)
            g = torch.zeros(ranks * maxt * 4096, dtype=torch.int32, device="cuda")
            for r, sp in enumerate(splits):
                tacc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device="cuda")
                sp.render_sequence(ctx, lps, g[r * maxt * 4096:].data_ptr(), tacc.data_ptr())
            out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            splits[0].unpack(ctx, g.data_ptr(), out.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), ref), (ranks, dealt)
    assert ctx.chain_errors() == 0
    ctx.close()


def _sequential(ctx, lp, W, H, k):
    """k single-frame launches (accumID 0 .. k-1): the frames a chained batch must equal."""
    import torch
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    for aid in range(k):
        lp.accumID = aid
        ctx.render(lp, W, H, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    return fb.cpu().numpy().copy(), bits(acc.cpu().numpy())


def test_chained_launches_on_two_streams_equal_sequential_frames():
    """Two chained launches of one context in flight on two streams at once (two images, two
    cameras): a spin kernel holds the first stream, so without ordering the second launch
    would run while the first still polls the same (block, wave) publish words.  Launches of a
    context run in call order across streams (the second stream waits for the first launch),
    so both images equal their sequential frames and no wait times out."""
    import torch
    cells = irt.synth_grid(2, 3, 90)
    W, H, k = 256, 192, 4
    sa = irt.setup_frame(cells, W, H, camera=FRAMING)
    sb = irt.setup_frame(cells, W, H, camera=None)  # viewAll: another image
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(sa.lut, sa.value_range)
    ref_a = _sequential(ctx, sa.lp, W, H, k)
    ref_b = _sequential(ctx, sb.lp, W, H, k)
    assert not np.array_equal(ref_a[0], ref_b[0])
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for rep in range(3):
        bufs = [(torch.zeros(W * H, dtype=torch.int32, device="cuda"),
                 torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")) for _ in range(2)]
        torch.cuda.synchronize()
        with torch.cuda.stream(s1):
            torch.cuda._sleep(20_000_000)  # ~10 ms: launch A queues behind it
        sa.lp.accumID = 0
        ctx.render_accumulate(sa.lp, W, H, k, bufs[0][0].data_ptr(), bufs[0][1].data_ptr(), s1.cuda_stream)
        sb.lp.accumID = 0
        ctx.render_accumulate(sb.lp, W, H, k, bufs[1][0].data_ptr(), bufs[1][1].data_ptr(), s2.cuda_stream)
        torch.cuda.synchronize()
        for (fb, acc), (rf, ra) in zip(bufs, (ref_a, ref_b)):
            assert np.array_equal(fb.cpu().numpy(), rf), rep
            assert np.array_equal(bits(acc.cpu().numpy()), ra), rep
    assert ctx.chain_errors() == 0
    ctx.close()


def test_chain_timeout_fails_loudly():
    """The failure path of the hand-off: frame 0's waves withhold their publish and a wait gives
    up after one poll, so frame 1 is lerped against an unpublished accum.  The library must not
    return those pixels silently: the next call that sees the launch -- here a render, then
    (for a second faulty launch) irt_get_render_stats -- returns IRT_E_CHAIN, and the context
    then renders multi-frame launches unchained, equal to the sequential frames again."""
    import torch
    cells = irt.synth_grid(2, 2, 47)
    W, H, k = 96, 80, 3
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    ref = _sequential(ctx, setup.lp, W, H, k)
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    ctx.set_chain_fault(1, 0)
    setup.lp.accumID = 0
    ctx.render_accumulate(setup.lp, W, H, k, fb.data_ptr(), acc.data_ptr())  # queued: IRT_OK
    torch.cuda.synchronize()
    with pytest.raises(irt.IrtError) as e:  # the next call reports it
        ctx.render_accumulate(setup.lp, W, H, k, fb.data_ptr(), acc.data_ptr())
    assert e.value.code == irt.E_CHAIN and "timed out" in str(e.value)
    # chaining is off now: the same batch renders through the sample buffer, correctly
    fb.zero_()
    acc.zero_()
    ctx.render_accumulate(setup.lp, W, H, k, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    ctx.stats()  # no error
    assert np.array_equal(fb.cpu().numpy(), ref[0]) and np.array_equal(bits(acc.cpu().numpy()), ref[1])
    # a second faulty launch, reported by irt_get_render_stats
    ctx.set_chain(True)
    ctx.render_accumulate(setup.lp, W, H, k, fb.data_ptr(), acc.data_ptr())
    with pytest.raises(irt.IrtError) as e:
        ctx.stats()
    assert e.value.code == irt.E_CHAIN
    assert ctx.chain_errors() == 2
    ctx.set_chain_fault(0, -1)
    ctx.set_chain(True)
    _batch(ctx, setup.lp, W, H, k, 0, chain=True)
    assert ctx.chain_errors() == 2  # no new failure
    ctx.close()


def test_chained_frames_stay_on_one_xcd():
    """Where chained workgroups run (measurement, not a correctness condition: the hand-off
    stores and loads every byte sc1): frame f's workgroup of a block and frame f - 1's, one frame
    of workgroups apart, land on the same XCD under the dispatcher's round-robin deal -- the L2
    locality the kernel's block-to-workgroup mapping was chosen for.  Reported, and asserted
    only for the hand-off's frames, which must also equal the sequential frames."""
    import torch
    cells = irt.synth_grid(2, 3, 90)
    W, H, k = 512, 512, 3
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    nt = irt.num_tiles(W, H)
    nwg = ctx.launch_workgroups(nt, k)
    per = nwg // k
    trace = torch.zeros(4 * nwg, dtype=torch.int32, device="cuda")
    ctx.set_wg_trace(trace.data_ptr())
    got = _batch(ctx, setup.lp, W, H, k, 0, chain=True)
    ctx.set_wg_trace(0)
    t = trace.cpu().numpy().view(np.uint32).reshape(k, per, 4)
    xcc = t[:, :, 3] & 0xF
    same = float(np.mean(xcc[1:] == xcc[:-1]))
    print(f"chained predecessor on the same XCD: {same:.4f} of {per * (k - 1)} workgroups")
    ref = _sequential(ctx, setup.lp, W, H, k)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    assert ctx.chain_errors() == 0
    ctx.close()
