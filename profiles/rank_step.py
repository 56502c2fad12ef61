#!/usr/bin/env python3
"""One rank's share of an N-GPU bench step, on one GPU, without the collective.

bench.py on N GPUs: each rank renders its interleaved 64x64 tiles
(irt_render_tiles_accumulate: N progressive frames per step in --mode progressive, one
frame in --mode frame), RCCL gathers the packed tiles, and rank 0 unpacks them.  This
script times rank 0's GPU work per step for N = 1, 2, 4, 8 (render, plus the unpack of a
gathered buffer of the right size) back to back on one stream, and the single-GPU path for
reference.  It projects the step time the driver's multi-GPU runs can reach, apart from the
exchange itself.

    python profiles/rank_step.py [--config c3] [--steps 100]
Prints one JSON line per (mode, N).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "icon-ray-tracing_amd", "python"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402  (CONFIGS, FRAMING, make_lut)
import irt  # noqa: E402
import irt_dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=100)
    args = ap.parse_args()
    rn, bis, L, W, H, tf, _, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    ctx = irt.Context.synth(rn, bis, L, 0)
    setup = irt.setup_frame(None, W, H, camera=bench.FRAMING, info=ctx.info)
    ctx.set_transfunc(bench.make_lut(tf, setup.lut), setup.value_range)
    lp = setup.lp
    stream = torch.cuda.current_stream(dev).cuda_stream
    fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)

    def timed(fn):
        for s in range(3):
            fn(s)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for s in range(args.steps):
            fn(3 + s)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / args.steps * 1e3

    def single(s):
        lp.accumID = s
        ctx.render(lp, W, H, fb.data_ptr(), acc.data_ptr(), stream)

    ms = timed(single)
    print(json.dumps({"config": args.config, "mode": "single", "n": 1, "ms_per_step": round(ms, 4),
                      "mray_s": round(W * H / ms / 1e3, 1)}), flush=True)
    for mode in ("progressive", "frame"):
        for n in (1, 2, 4, 8):
            split = irt_dist.TileSplit(W, H, 0, n)
            maxt = split.max_tiles
            tiles = torch.zeros(maxt * 4096, dtype=torch.int32, device=dev)
            tacc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)
            gathered = torch.zeros(n * maxt * 4096, dtype=torch.int32, device=dev)
            frames = 1 if mode == "frame" else n

            def step(s):
                lp.accumID = s * frames
                if frames == 1:
                    ctx.render_tiles(lp, W, H, 0, n, tiles.data_ptr(), tacc.data_ptr(), stream)
                else:
                    ctx.render_tiles_accumulate(lp, W, H, 0, n, frames, tiles.data_ptr(),
                                                tacc.data_ptr(), stream)
                ctx.unpack_tiles(gathered.data_ptr(), n, maxt, W, H, fb.data_ptr(), stream)

            ms = timed(step)
            print(json.dumps({"config": args.config, "mode": mode, "n": n,
                              "ms_per_step": round(ms, 4),
                              # all ranks' rays per step: W*H*frames (frames = n or 1)
                              "projected_mray_s": round(W * H * frames / ms / 1e3, 1)}),
                  flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
