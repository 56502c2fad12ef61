"""The multi-GPU frame split with the HIP renderer: world-size-2 processes (gloo,
host-staged collectives, both ranks on cuda:0) render their 64x64 tiles -- the
cost-balanced deal (irt_deal_tiles, irt_render_tile_list) or round-robin (irt_render_tiles /
irt_render_tiles_accumulate) -- on torch's default stream, gather them to rank 0 with
irt_dist.FrameGather (two frames in flight, rank-major receive buffers), and rank 0 unpacks
them (irt_unpack_tile_table / irt_unpack_tiles) on a side stream
(irt_dist.FramePipeline, the loop bench.py runs) -- bench.py's two multi-GPU modes:
  * frame       one frame per step split over the ranks (strong scaling),
  * progressive N progressive frames per step, each rank rendering its tiles of all N
                (weak scaling).
Rank 0's framebuffer must equal a single-process render bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GRID = (2, 3, 47)
W, H = 200, 136  # ragged: partial tiles on the right and bottom
STEPS = 11  # past two reuse cycles of the 8 packed buffers (FramePipeline batch 4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, out_path, deal, backend="gloo"):
    sys.path[:0] = [os.path.join(HERE, "..", "icon-ray-tracing_amd", "python"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import irt
    import irt_dist
    from helpers import FRAMING

    torch.cuda.set_device(0)
    if backend == "nccl":  # RCCL: its communicator, stream and Work.wait() semantics
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = irt.Context.synth(*GRID, 0)
    setup = irt.setup_frame(None, W, H, camera=FRAMING, info=ctx.info)
    ctx.set_transfunc(setup.lut, setup.value_range)
    lp = setup.lp
    split = (irt_dist.TileSplit.dealt(W, H, rank, world, lp, ctx.info) if deal == "dealt"
             else irt_dist.TileSplit(W, H, rank, world))
    fg = irt_dist.FrameGather(split, "cuda:0", buffers=8, stage_cpu=backend == "gloo")
    acc = torch.zeros(split.max_tiles * 4096 * 4, dtype=torch.float32, device="cuda:0")
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda:0")
    frames = 1 if mode == "frame" else world
    pipe = irt_dist.FramePipeline(ctx, fg, fb)  # bench.py's loop: rank 0 unpacks on a side stream
    for s in range(STEPS):
        lp.accumID = s * frames
        pipe.step(s, lambda buf: split.render(ctx, lp, frames, buf.data_ptr(), acc.data_ptr()))
    pipe.drain()
    if rank == 0:
        torch.cuda.synchronize()
        np.save(out_path, fb.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


def _reference_frame(mode, world):
    import torch

    import irt
    from helpers import FRAMING
    ctx = irt.Context.synth(*GRID, 0)
    setup = irt.setup_frame(None, W, H, camera=FRAMING, info=ctx.info)
    ctx.set_transfunc(setup.lut, setup.value_range)
    lp = setup.lp
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda:0")
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
    frames = 1 if mode == "frame" else world
    for s in range(STEPS):
        lp.accumID = s * frames
        if frames == 1:
            ctx.render(lp, W, H, fb.data_ptr(), acc.data_ptr())
        else:
            ctx.render_accumulate(lp, W, H, frames, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    ref = fb.cpu().numpy()
    ctx.close()
    return ref


@pytest.mark.parametrize("deal", ["dealt", "mod"])
@pytest.mark.parametrize("mode", ["frame", "progressive"])
def test_two_rank_hip_frame_split(tmp_path, mode, deal):
    import torch.multiprocessing as mp

    world = 2
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), mode, out, deal), nprocs=world, join=True,
                       start_method="spawn")
    ref = _reference_frame(mode, world)
    got = np.load(out)
    assert (ref != 0).mean() > 0.3
    assert np.array_equal(got, ref), int((got != ref).sum())


@pytest.mark.parametrize("deal", ["dealt", "mod"])
@pytest.mark.parametrize("mode", ["frame", "progressive"])
def test_rccl_process_group_frame_pipeline(tmp_path, mode, deal):
    """The measured multi-GPU path on RCCL itself: a process group on backend "nccl" (one rank:
    the GPU box has one GPU, and RCCL refuses two ranks on one device) runs FramePipeline --
    tile render on a high-priority stream, dist.gather of the packed RGBA8 tiles on RCCL's own
    stream (no host staging), Work.wait() before buffer reuse, rank 0's unpack on a side
    stream -- for STEPS steps; the assembled frame must equal irt_render's bit for bit."""
    import torch.multiprocessing as mp

    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(1, _free_port(), mode, out, deal, "nccl"), nprocs=1, join=True,
                       start_method="spawn")
    ref = _reference_frame(mode, 1)
    got = np.load(out)
    assert (ref != 0).mean() > 0.3
    assert np.array_equal(got, ref), int((got != ref).sum())
