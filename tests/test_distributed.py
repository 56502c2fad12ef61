"""The N>1 frame split on CPU: world_size-2 gloo processes render their interleaved tiles
with the oracle, gather the packed RGBA8 tiles to rank 0 through torch.distributed with
two frames in flight (irt_dist.FrameGather, the code path bench.py runs over RCCL), and
rank 0's assembled frames must equal the single-process frames bit for bit."""
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


def _worker(rank, world, port, W, H, out_path):
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


@pytest.mark.parametrize("world", [2])
def test_two_rank_gloo_frame_split(tmp_path, world):
    import torch.multiprocessing as mp

    import irt
    from helpers import FRAMING, oracle_frame

    W, H = 136, 72  # ragged: partial tiles on the right and bottom
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, out), nprocs=world,
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
