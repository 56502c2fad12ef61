#!/usr/bin/env python3
"""Every rank's share of an N-GPU bench step, timed on one GPU, without the collective.

bench.py on N GPUs: each rank renders its 64x64 tiles (N progressive frames per step in
--mode progressive, one frame in --mode frame) into a packed buffer, RCCL gathers the packed
tiles and rank 0 unpacks them.  The step time of the job is the SLOWEST rank's, so this
script times the share of EVERY rank r = 0..N-1 (render; with N > 1 rank 0 also the unpack
of a gathered buffer of the right size), back to back on one stream, for both deals:
  * "mod":   tile t -> rank t mod N (rounds 1-2; whole tile columns per rank when N divides
             the tile row),
  * "dealt": irt_deal_tiles' cost-balanced deal (round 3, bench.py's: longest-processing-
             time first on an estimate of each tile's cost, rank 0 lighter by the unpack).
It prints one JSON line per (deal, mode, N) with the per-rank times, max/mean, and the
projected whole-job rate from the max rank (the exchange itself left out).

    python profiles/rank_step.py [--config c3] [--steps 50]

The C5 orbit renders its consecutive views (irt_render_sequence on one GPU,
irt_render_tile_list_sequence per rank).
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
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--modes", default="progressive,frame")
    ap.add_argument("--deals", default="mod,dealt")
    ap.add_argument("--batch", type=int, default=1,
                    help="frames per launch (bench.py --batch): the single-GPU step renders B "
                         "chained frames, a rank's step B (frame mode) or N*B (progressive)")
    args = ap.parse_args()
    rn, bis, L, W, H, tf, orbit, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    ctx = irt.Context.synth(rn, bis, L, 0)
    cam = bench.orbit_camera(0) if orbit else bench.FRAMING
    setup = irt.setup_frame(None, W, H, camera=cam, info=ctx.info)
    ctx.set_transfunc(bench.make_lut(tf, setup.lut), setup.value_range)
    ctx.set_statistics(False)  # as bench.py's timed loop
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

    B = max(1, args.batch)
    views = None
    if orbit:  # the orbit's views as whole launch-parameter records (bench.py's orbit_lps)
        views = []
        for k in range(bench.ORBIT_FRAMES):
            c = irt.camera_look_at(*bench.orbit_camera(k), W, H)
            q = irt.LaunchParams.from_buffer_copy(lp)
            q.org, q.dir_00, q.dir_du, q.dir_dv = c.org, c.dir_00, c.dir_du, c.dir_dv
            q.accumID = 0
            views.append(q)

    def seq(s, n):  # the step's n consecutive orbit views
        return [views[(s * n + k) % bench.ORBIT_FRAMES] for k in range(n)]

    def single(s):
        lp.accumID = s * B
        if views is not None:
            ctx.render_sequence(seq(s, B), W, H, fb.data_ptr(), acc.data_ptr(), stream)
        elif B > 1:
            ctx.render_accumulate(lp, W, H, B, fb.data_ptr(), acc.data_ptr(), stream)
        else:
            ctx.render(lp, W, H, fb.data_ptr(), acc.data_ptr(), stream)

    ms1 = timed(single) / B  # per frame
    print(json.dumps({"config": args.config, "mode": "single", "n": 1, "batch": B,
                      "ms_per_frame": round(ms1, 4), "mray_s": round(W * H / ms1 / 1e3, 1)}), flush=True)
    for deal in args.deals.split(","):
        for mode in args.modes.split(","):
            for n in (int(v) for v in args.ranks.split(",")):
                frames = B if mode == "frame" else n * B
                steps = []
                for r in range(n):
                    split = (irt_dist.TileSplit.dealt(W, H, r, n, lp, ctx.info, frames) if deal == "dealt"
                             else irt_dist.TileSplit(W, H, r, n))
                    maxt = split.max_tiles
                    tiles = torch.zeros(maxt * 4096, dtype=torch.int32, device=dev)
                    tacc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)
                    gathered = torch.zeros(n * maxt * 4096, dtype=torch.int32, device=dev)

                    def step(s, split=split, tiles=tiles, tacc=tacc, gathered=gathered, r=r):
                        lp.accumID = s * frames
                        if views is not None:  # irt_render_tile_list_sequence
                            split.render_sequence(ctx, seq(s, frames), tiles.data_ptr(), tacc.data_ptr(), stream)
                        else:
                            split.render(ctx, lp, frames, tiles.data_ptr(), tacc.data_ptr(), stream)
                        if r == 0 and n > 1:
                            split.unpack(ctx, gathered.data_ptr(), fb.data_ptr(), stream)

                    steps.append(step)
                # the ranks timed in turn, three passes; each rank's fastest pass (the box's
                # run-to-run noise is ~3 %, more than the imbalance being measured)
                per_rank = [min(v) for v in zip(*[[timed(f) for f in steps] for _ in range(3)])]
                mx, mean = max(per_rank), sum(per_rank) / n
                print(json.dumps({"config": args.config, "deal": deal, "mode": mode, "n": n, "batch": B,
                                  "ms_per_rank": [round(v, 4) for v in per_rank],
                                  "max_over_mean": round(mx / mean, 4),
                                  "ms_per_step_max": round(mx, 4),
                                  # all ranks' rays per step: W*H*frames, over the slowest rank
                                  "projected_mray_s": round(W * H * frames / mx / 1e3, 1),
                                  "speedup_vs_single": round(ms1 * frames / mx, 3)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
