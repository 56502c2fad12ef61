"""The N>1 frame split on CPU: world_size-2 gloo processes render their tiles (the
cost-balanced deal of irt_deal_tiles, or round-robin) with the oracle, gather the packed
RGBA8 tiles to rank 0 through torch.distributed with two frames in flight
(irt_dist.FrameGather, the code path bench.py runs over RCCL), and rank 0's assembled frames
must equal the single-process frames bit for bit.  The deal itself: every tile exactly once,
ceil/floor(T/N) tiles per rank, deterministic, and balanced under its own cost estimate."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, out_path, deal):
    sys.path[:0] = [os.path.join(HERE, "..", "icon-ray-tracing_amd", "python"),
                    os.path.join(HERE, "..", "oracle"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import irt
    import irt_dist
    from helpers import FRAMING
    import oracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    cells = irt.synth_grid(2, 1, 31)
    S = O.OracleScene(cells)
    lut, vr = S.default_lut()
    S.set_transfunc(lut, vr)
    cam = S.camera(W, H, FRAMING)
    if deal == "dealt":  # every rank computes the same table from the same camera
        setup = irt.setup_frame(cells, W, H, camera=FRAMING)
        split = irt_dist.TileSplit.dealt(W, H, rank, world, setup.lp, setup.info)
    else:
        split = irt_dist.TileSplit(W, H, rank, world)
    # two frames in flight, as bench.py runs them: render frame s into buffer s % 2, start
    # its gather asynchronously, finish it only when the buffer is needed again
    fg = irt_dist.FrameGather(split, "cpu", buffers=2)
    works = []
    for s in (0, 1):
        p = S.params(cam, accum_id=s)
        # this rank's tiles (the oracle stands in for irt_render_tiles) into the packed buffer
        packed = np.zeros((split.max_tiles, irt_dist.TILE_PIX), np.uint32)
        for k, t in enumerate(split.tiles()):
            xy = split.tile_pixels(t)
            ok = xy[:, 0] >= 0
            _, fb, _ = S.render_pixels(p, W, H, xy[ok].astype(np.int32), threads=2)
            packed[k, ok] = fb[xy[ok, 1], xy[ok, 0]]
        fg.bufs[s].copy_(torch.from_numpy(packed.view(np.int32).ravel()))
        works.append(fg.gather_async(s))
    for s in (0, 1):
        g = fg.finish(works[s], s)
        if rank == 0:
            frame = irt_dist.unpack_host(g.numpy().view(np.uint32), split)
            np.save(out_path.replace(".npy", f"{s}.npy"), frame)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,deal", [(2, "dealt"), (2, "mod"), (4, "dealt")])
def test_two_rank_gloo_frame_split(tmp_path, world, deal):
    import torch.multiprocessing as mp

    import irt
    from helpers import FRAMING, oracle_frame

    W, H = 136, 72  # ragged: partial tiles on the right and bottom
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, out, deal), nprocs=world,
                       join=True, start_method="spawn")
    cells = irt.synth_grid(2, 1, 31)
    for s in (0, 1):
        frame = np.load(out.replace(".npy", f"{s}.npy"))
        _, fb_ref, _, _ = oracle_frame(cells, W, H, camera=FRAMING, accum_ids=(s,))
        assert np.array_equal(frame, fb_ref), s
        assert (fb_ref != 0).mean() > 0.3


def test_tile_split_covers_every_pixel_once():
    import irt_dist
    for (W, H, world) in [(1024, 1024, 8), (200, 136, 3), (64, 64, 4), (2048, 2048, 8)]:
        seen = np.zeros((H, W), np.int32)
        for r in range(world):
            s = irt_dist.TileSplit(W, H, r, world)
            assert len(s.tiles()) <= s.max_tiles
            for t in s.tiles():
                xy = s.tile_pixels(t)
                ok = xy[:, 0] >= 0
                seen[xy[ok, 1], xy[ok, 0]] += 1
        assert (seen == 1).all()


def _dealt_splits(W, H, world, frames=1):
    import irt
    import irt_dist
    from helpers import FRAMING
    cells = irt.synth_grid(2, 2, 47)
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    return [irt_dist.TileSplit.dealt(W, H, r, world, setup.lp, setup.info, frames)
            for r in range(world)]


def test_dealt_split_covers_every_pixel_once():
    import irt
    for (W, H, world) in [(1024, 1024, 8), (200, 136, 3), (64, 64, 4), (2048, 2048, 8),
                          (1024, 1024, 7), (96, 64, 8)]:
        splits = _dealt_splits(W, H, world)
        seen = np.zeros((H, W), np.int32)
        T = irt.num_tiles(W, H)
        for r, s in enumerate(splits):
            assert np.array_equal(s.table, splits[0].table)  # deterministic
            n = len(s.tiles())
            assert n <= s.max_tiles and n >= T // world - 2 - T // (4 * world)
            for t in s.tiles():
                xy = s.tile_pixels(t)
                ok = xy[:, 0] >= 0
                seen[xy[ok, 1], xy[ok, 0]] += 1
        assert (seen == 1).all()
        assert max(len(s.tiles()) for s in splits) == splits[0].max_tiles


def test_dealt_split_balances_the_globe():
    """Under the frame's own per-pixel shell coverage (the framing camera's centred globe),
    the cost-balanced deal (whose own estimate also weighs limb chords and off-globe rays)
    spreads the shell pixels within 3 % across 8 ranks at 1024^2;
    the round-robin deal hands whole tile columns to ranks (rank 0 the outermost)."""
    import irt_dist
    W = H = 1024
    y, x = np.mgrid[0:H, 0:W]
    u, v = (x + .5) / W * 2 - 1, (y + .5) / H * 2 - 1
    disk = (u * u + v * v < 0.898 ** 2).astype(np.float64)  # 63 % of the frame
    tile = disk.reshape(16, 64, 16, 64).sum(axis=(1, 3)).ravel()
    dealt = [sum(tile[t] for t in s.tiles()) for s in _dealt_splits(W, H, 8, frames=10**6)]
    mod = [sum(tile[t] for t in irt_dist.TileSplit(W, H, r, 8).tiles()) for r in range(8)]
    assert max(dealt) / np.mean(dealt) < 1.03, dealt
    assert max(mod) / np.mean(mod) > 1.15 and np.argmin(mod) == 0, mod
    # one frame per step: rank 0 also unpacks the frame (irt_dist.UNPACK_COST of a frame's
    # render), so it gets correspondingly fewer shell pixels, the others stay balanced
    one = [sum(tile[t] for t in s.tiles()) for s in _dealt_splits(W, H, 8, frames=1)]
    assert one[0] < 0.85 * np.mean(one[1:])
    assert max(one[1:]) / np.mean(one[1:]) < 1.03, one
