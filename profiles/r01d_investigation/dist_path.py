"""One rank's share of a multi-GPU bench step, timed on one GPU (C3, framing camera).

For world N, bench.py's step on each rank is irt_render_tiles_accumulate over the rank's
interleaved 64x64 tiles (t = rank mod N) of N consecutive progressive frames: one frame's
worth of rays per rank.  This times rank 0's launch for N = 1, 2, 4, 8 against the
single-frame irt_render path bench.py uses at N = 1, to show what the driver's scaling run
pays per GPU before the RCCL gather (not measurable on a one-GPU box).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "icon-ray-tracing_amd", "python"))
import torch  # noqa: E402
import irt  # noqa: E402

FRAMING = ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)
W = H = 1024
STEPS = int(os.environ.get("STEPS", "200"))
cells = irt.synth_grid(2, 7, 90)
setup = irt.setup_frame(cells, W, H, camera=FRAMING)
ctx = irt.Context(cells, 0)
ctx.set_transfunc(setup.lut, setup.value_range, setup.opacity_scale)
lp = setup.lp
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev).cuda_stream
fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
accum = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
ntiles = irt.num_tiles(W, H)


def timed(fn):
    for s in range(5):
        fn(s)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for s in range(STEPS):
        fn(5 + s)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / STEPS * 1e3


def single(s):
    lp.accumID = s
    ctx.render(lp, W, H, fb.data_ptr(), accum.data_ptr(), stream)


res = {"single_frame_ms": timed(single)}
for world in (1, 2, 4, 8):
    maxt = (ntiles + world - 1) // world
    out = torch.zeros(maxt * 4096, dtype=torch.int32, device=dev)
    acc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)

    def step(s, world=world, out=out, acc=acc):
        lp.accumID = s * world
        ctx.render_tiles_accumulate(lp, W, H, 0, world, world, out.data_ptr(), acc.data_ptr(),
                                    stream)
    res[f"rank0_world{world}_ms"] = timed(step)
print(json.dumps({k: round(v, 4) for k, v in res.items()}))
