"""irt_dist.FramePipeline's buffer reuse under real stream semantics.

bench.py's multi-GPU step loop renders step s into packed buffer s mod 2K and starts an
asynchronous gather of it; the render stream waits only once per K steps, on the newest
gather of the previous half-cycle, trusting that the gathers run in issue order (RCCL runs a
process group's collectives in order on one stream).  Here one process drives the real
FramePipeline with an in-process stand-in for torch.distributed.gather that has RCCL's
stream semantics: the "collective" waits for the issuing stream, runs on a stream of its
own, and its work's wait() makes the CURRENT stream wait for it (never the host).  Each
stand-in gather first spins on the GPU for ~1 ms (a slow link), then snapshots the packed
buffer it reads.  Every snapshot must equal that step's tiles rendered in isolation -- over
three reuse cycles of the 8 buffers, as rank 0 (side-stream gathers and unpacks) and as a
non-zero rank -- and a pipeline with the reuse wait removed must be caught tearing frames
(the negative control proves the check can fail).
"""
import numpy as np
import pytest

import irt
from helpers import FRAMING

pytestmark = pytest.mark.gpu

GRID = (2, 2, 47)
W, H = 200, 136
STEPS = 3 * 8 + 2  # three reuse cycles of the 8 packed buffers (batch K = 4)


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        import torch
        torch.cuda.current_stream().wait_event(self.ev)


def _spin_cycles(torch):
    """torch.cuda._sleep cycles for ~1 ms on this device (calibrated with events)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 1 << 20
    torch.cuda._sleep(n)  # warm
    s.record()
    torch.cuda._sleep(n)
    e.record()
    torch.cuda.synchronize()
    ms = max(s.elapsed_time(e), 1e-3)
    return int(n / ms)


def _make_gather_class():
    import torch
    import irt_dist

    class LocalGather(irt_dist.FrameGather):
        """dist.gather stand-in (world of one process): RCCL's stream semantics, a slow link."""

        def __init__(self, split, device, buffers, spin):
            super().__init__(split, device, buffers=buffers)
            self.cstream = torch.cuda.Stream()
            self.spin = spin
            self.snaps = []  # per gather, in issue (= step) order: the buffer as it was read

        def gather_async(self, b):
            self.cstream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.cstream):
                torch.cuda._sleep(self.spin)
                snap = self.bufs[b].clone()
                if self.parts:
                    self.parts[b][self.split.rank].copy_(snap)
                ev = torch.cuda.Event()
                ev.record(self.cstream)
            self.snaps.append(snap)
            return _Work(ev)

    return LocalGather


def _run(role, broken):
    import torch
    import irt_dist
    ctx = irt.Context.synth(*GRID, 0)
    setup = irt.setup_frame(None, W, H, camera=FRAMING, info=ctx.info)
    ctx.set_transfunc(setup.lut, setup.value_range)
    lp = setup.lp
    rank, world = (0, 1) if role == "rank0" else (1, 2)
    split = irt_dist.TileSplit.dealt(W, H, rank, world, lp, ctx.info)
    dev = torch.device("cuda:0")
    render_stream = torch.cuda.Stream(dev, priority=-1)  # bench.py's render stream
    torch.cuda.set_stream(render_stream)
    stream = render_stream.cuda_stream
    maxt = split.max_tiles
    # the reference: each step's packed tiles rendered in isolation, in the same order
    ref = []
    acc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)
    buf = torch.zeros(maxt * 4096, dtype=torch.int32, device=dev)
    for s in range(STEPS):
        lp.accumID = s
        split.render(ctx, lp, 1, buf.data_ptr(), acc.data_ptr(), stream)
        torch.cuda.synchronize()
        ref.append(buf.cpu().numpy().copy())
    assert not np.array_equal(ref[0], ref[8])  # the reuse partner differs: tearing is visible
    # the pipeline
    fg = _make_gather_class()(split, dev, 8, _spin_cycles(torch))
    fb = torch.zeros(W * H, dtype=torch.int32, device=dev) if rank == 0 else None
    Pipe = irt_dist.FramePipeline
    if broken:
        class Pipe(irt_dist.FramePipeline):  # noqa: F811 -- the reuse wait removed
            def _wait_reuse(self, t):
                pass
    pipe = Pipe(ctx, fg, fb)
    acc.zero_()
    for s in range(STEPS):
        lp.accumID = s
        pipe.step(s, lambda b: split.render(ctx, lp, 1, b.data_ptr(), acc.data_ptr(), stream))
    pipe.drain()
    torch.cuda.synchronize()
    torn = [s for s in range(STEPS) if not np.array_equal(fg.snaps[s].cpu().numpy(), ref[s])]
    out = None
    if rank == 0:  # the unpacked framebuffer holds the newest frame
        out = fb.cpu().numpy()
        whole = torch.zeros(W * H, dtype=torch.int32, device=dev)
        a = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
        for s in range(STEPS):
            lp.accumID = s
            ctx.render(lp, W, H, whole.data_ptr(), a.data_ptr(), stream)
        torch.cuda.synchronize()
        out = (out, whole.cpu().numpy())
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    ctx.close()
    return torn, len(fg.snaps), out


@pytest.mark.parametrize("role", ["rank0", "rank1"])
def test_pipeline_buffer_reuse_waits_for_the_gather(role):
    torn, n, out = _run(role, broken=False)
    assert n == STEPS
    assert not torn, f"steps {torn} gathered a buffer already overwritten"
    if out is not None:
        assert np.array_equal(out[0], out[1])


@pytest.mark.parametrize("role", ["rank0", "rank1"])
def test_pipeline_without_the_reuse_wait_is_caught(role):
    torn, n, _ = _run(role, broken=True)
    assert n == STEPS
    assert torn, "removing the reuse wait went unnoticed: the check cannot fail"
