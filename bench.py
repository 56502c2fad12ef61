#!/usr/bin/env python3
"""bench.py -- Mray/s + ms/frame of the MI355X ICON renderer (BASELINE.json metric).

The hot path is the raygen woodcockTrackingWithAccel (icon_rt/deviceCode.cu:281-341) over
every pixel of a 1024x1024 frame.  Inputs (cells, locator, shell accelerator, transfer
function) are resident in HBM before the timed region.

Default workload (configs[2] of BASELINE.json, C3): synthetic R2B07 ICON grid (1,310,720
cells) x 90 levels (3,932,160 `.ic` records), 1024x1024, framing camera
`--camera 0 0 1.4e7 0 0 0 0 1 0 -fovy 60`, the reference's default transfer function.

One step:
  * 1 GPU: one frame (one launch of the raygen over the 1024x1024 frame);
  * N GPUs (weak scaling, one process per GPU under torchrun): N consecutive frames of the
    reference's progressive accumulation (--sample-limit, accumID = step*N + k), tile-split:
    every rank renders its interleaved 64x64 tiles of all N frames in ONE launch
    (irt_render_tiles_accumulate), and rank 0 gathers the final RGBA8 tiles over RCCL
    (torch.distributed "nccl") and unpacks the framebuffer.  The gather of step s runs on
    the collective's stream while step s+1 renders (double-buffered tiles).  Per-GPU work
    is one frame's rays per step at every N; `value` counts all ranks' rays.
Frames are enqueued back to back: per-launch statistics come back through a ring, never
stalling the host between launches.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "icon-ray-tracing_amd", "python"))

METRIC = "Mray/s + ms/frame at 1024², R2B07 ICON grid, 1/2/4/8 MI355X vs host CPU"
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E (MI355X_MICROARCH.md)
BYTES_PER_SAMPLE = 92  # geometry 36 + findHeight 20 + value 4 + 2 LUT entries 32
BYTES_PER_RAY = 44     # accum read 16 + write 16 + RGBA8 4 + 2 majorants 8

CONFIGS = {
    # name: (rootN, bisections, levels, W, H, description)
    "c2": (2, 5, 47, 512, 512, "C2: R2B05 (81,920 cells) x 47 levels, 512x512"),
    "c3": (2, 7, 90, 1024, 1024, "C3: R2B07 (1,310,720 cells) x 90 levels, 1024x1024"),
    "c4": (2, 7, 90, 2048, 2048, "C4: R2B07 (1,310,720 cells) x 90 levels, 2048x2048"),
    "c5": (2, 9, 90, 1024, 1024, "C5: R2B09 (20,971,520 cells) x 90 levels, 1024x1024, "
                                 "60-frame orbit"),
}
ORBIT_FRAMES = 60  # C5: eye = 1.4e7 (sin t, 0, cos t), t = 2 pi k / 60, looking at the origin
FRAMING = ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(cells, setup, W, H, budget_s=15.0):
    """The reference's CPU path (brute-force sampleVolume, deviceCode.cu:116-123) on the
    host cores, on a bounded strided sample of the same frame's pixels: the reference's own
    raygen compiled from /root/reference headers (oracle/_ref, built by __graft_entry__.build)
    when present ("reference"), else the oracle's restatement ("port")."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    use_ref = O.have_ref()
    threads = max(1, min(16, os.cpu_count() or 1))
    S = O.OracleScene(cells)
    S.set_transfunc(setup.lut, setup.value_range, setup.opacity_scale)
    lp = setup.lp
    cam = (np.array(lp.org.tolist(), np.float32), np.array(lp.dir_00.tolist(), np.float32),
           np.array(lp.dir_du.tolist(), np.float32), np.array(lp.dir_dv.tolist(), np.float32))
    params = S.params(cam, accum_id=0, raygen=lp.raygen, unit_distance=lp.unitDistance)
    # An unbiased bounded sample: a regular sub-grid of the frame's pixels, refined until
    # the run takes about budget_s/2 .. 2 budget_s of CPU time.
    stride, elapsed, pix, st = 128, 0.0, 0, None
    while True:
        ys, xs = np.mgrid[stride // 2:H:stride, stride // 2:W:stride]
        xy = np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.int32)
        t = time.perf_counter()
        if use_ref:
            _, _, cnt = O.ref_render_pixels(S, params, W, H, xy, threads=threads)
            locate = int(cnt[0])
        else:
            _, _, st = S.render_pixels(params, W, H, xy, threads=threads, fast=False)
            locate = st.locate_calls
        elapsed = time.perf_counter() - t
        pix = xy.shape[0]
        log(f"[cpu baseline] stride {stride}: {pix} rays in {elapsed:.2f} s")
        if elapsed > budget_s / 2 or stride <= 8:
            break
        stride //= 2
    mray = pix / elapsed / 1e6
    sample = (f"every {stride}th pixel in x and y of the {W}x{H} frame ({pix} rays, "
              f"{locate} sampleVolume calls, {elapsed:.1f} s on {threads} threads): "
              f"the reference's CPU raygen with its brute-force first-hit cell scan over "
              f"{cells.size} records (deviceCode.cu:116-123), " +
              ("compiled from the reference's own headers (oracle/_ref: ICONGrid.h sample(), "
               "ShellAccel.h sdda, vecmath), one host thread per pixel chunk"
               if use_ref else "oracle restatement, literal sample() incl. toSpherical"))
    kind = "reference" if use_ref else "port"
    return {"value": mray, "unit": "Mray/s", "cores": threads, "kind": kind, "sample": sample,
            "ms_per_frame_extrapolated": W * H / (mray * 1e6) * 1e3}


def profiled_traffic(kernel, records, width):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 summary of the
    same workload (profiles/*/summary.json: FETCH_SIZE x 2 + WRITE_SIZE, per the gfx950
    correction of MI355X_MICROARCH.md), or None."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary.json"))):
        try:
            s = json.load(open(p))
        except (OSError, ValueError):
            continue
        b = s.get("bench") or {}
        if not any(k.endswith(kernel) for k in s.get("kernels", {})):
            continue
        if s.get("records") != records or s.get("width") != width:
            continue
        if "traffic_bytes_per_launch_fetch_x2" in s and b:
            best = (s["traffic_bytes_per_launch_fetch_x2"], os.path.relpath(p, ROOT))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the multi-rank path with host-staged collectives "
                         "(ranks may share a GPU); nccl (RCCL) is the measured path")
    args = ap.parse_args()

    import torch
    import irt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = local % max(torch.cuda.device_count(), 1) if world > 1 else 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{device}"))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(device)
    dev = torch.device(f"cuda:{device}")

    rn, bis, L, W, H, desc = CONFIGS[args.config]
    t0 = time.time()
    cells = irt.synth_grid(rn, bis, L)
    log(f"[rank {rank}] grid: {cells.size} records ({time.time() - t0:.1f} s)")
    setup = irt.setup_frame(cells, W, H, camera=FRAMING)
    t0 = time.time()
    ctx = irt.Context(cells, device)
    ctx.set_transfunc(setup.lut, setup.value_range, setup.opacity_scale)
    log(f"[rank {rank}] context: {ctx.info.deviceBytes / 2**30:.2f} GiB HBM, locator G="
        f"{ctx.info.locatorFaceRes} entries={ctx.info.locatorEntries} ({time.time() - t0:.1f} s)")

    lp = setup.lp
    orbit = None
    if args.config == "c5":  # one orbit frame per step (a new view: accumID 0)
        orbit = []
        for k in range(ORBIT_FRAMES):
            th = 2.0 * np.pi * k / ORBIT_FRAMES
            orbit.append(irt.camera_look_at((1.4e7 * np.sin(th), 0.0, 1.4e7 * np.cos(th)),
                                            (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0, W, H))
    ntiles = irt.num_tiles(W, H)
    stream = torch.cuda.current_stream(device).cuda_stream
    # frames per step: 1 on one GPU; N on N GPUs (weak scaling: N frames of the
    # progressive accumulation per step, each rank rendering its interleaved 64x64 tiles of
    # all N frames in one launch, rank 0 gathering the final RGBA8 tiles over RCCL)
    frames = world
    if world == 1:
        fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
        accum = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
        ctx.clear(fb.data_ptr(), accum.data_ptr(), W * H, stream)
    else:
        import irt_dist
        split = irt_dist.TileSplit(W, H, rank, world)
        assert split.num_tiles == ntiles
        maxt = split.max_tiles
        fg = irt_dist.FrameGather(split, dev, buffers=2, stage_cpu=args.dist_backend == "gloo")
        tiles_acc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)
        fb = torch.zeros(W * H, dtype=torch.int32, device=dev) if rank == 0 else None
    inflight = {}

    def step(s):
        lp.accumID = s * frames
        if orbit is not None:
            c = orbit[s % ORBIT_FRAMES]
            lp.org, lp.dir_00, lp.dir_du, lp.dir_dv = c.org, c.dir_00, c.dir_du, c.dir_dv
            lp.accumID = 0
        if world == 1:
            ctx.render(lp, W, H, fb.data_ptr(), accum.data_ptr(), stream)
            return
        b = s % 2
        if b in inflight:  # the gather that last read this buffer must be done
            finish(inflight.pop(b), b)
        ctx.render_tiles_accumulate(lp, W, H, rank, world, frames, fg.bufs[b].data_ptr(),
                                    tiles_acc.data_ptr(), stream)
        inflight[b] = fg.gather_async(b)  # RCCL gather of this step's frame, overlapped

    def finish(work, b):
        g = fg.finish(work, b)
        if rank == 0:
            ctx.unpack_tiles(g.data_ptr(), world, maxt, W, H, fb.data_ptr(), stream)

    def drain():
        for b in sorted(inflight):
            finish(inflight.pop(b), b)

    for f in range(args.warmup):
        step(f)
    drain()
    st = ctx.stats()
    log(f"[rank {rank}] warmup: last launch kernel {st.kernelMs:.3f} ms, {st.samplesFound} "
        f"samples, {st.candidatesTested} candidates")
    ctx.reset_stats_total()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    if world > 1:
        drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    tot, launches = ctx.stats_total()
    import resource
    log(f"[rank {rank}] timed {args.steps} steps ({launches} launches) in {elapsed:.3f} s; "
        f"peak host RSS {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20:.1f} GiB")
    samples, in_box = tot.samplesFound, tot.raysInBox
    if world > 1:
        rdev = dev if args.dist_backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        agg = torch.tensor([samples, in_box, tot.raysLaunched], dtype=torch.float64, device=rdev)
        dist.all_reduce(agg)
        samples_all, in_box_all, launched_all = (int(v) for v in agg.tolist())
    else:
        samples_all, in_box_all, launched_all = samples, in_box, tot.raysLaunched

    ms_per_step = elapsed / args.steps * 1e3
    mray = W * H * frames * args.steps / elapsed / 1e6  # all ranks' rays
    # roofline of the dominant kernel on this rank: algorithmic bytes per launch over its
    # HIP-event-timed average duration (events on the stream the kernel runs on)
    avg_kernel_s = tot.kernelMs / 1e3 / max(launches, 1)
    bytes_per_launch = (BYTES_PER_SAMPLE * samples + BYTES_PER_RAY * in_box) / max(launches, 1)
    achieved = bytes_per_launch / avg_kernel_s if avg_kernel_s > 0 else float("nan")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(mray, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": desc + (", orbit camera (eye 1.4e7 (sin t, 0, cos t), -fovy 60), "
                                    "one orbit frame per step"
                                    if orbit is not None else
                                    ", framing camera --camera 0 0 1.4e7 0 0 0 0 1 0 -fovy 60, "
                                    "one frame per step") +
                           ", woodcockTrackingWithAccel, default TF",
                "records": int(cells.size), "width": W, "height": H,
                "parallelism": (f"{world} GPUs x 64x64 interleaved frame tiles, {frames} progressive "
                                f"frames per step in one launch per rank, RCCL gather of the "
                                f"final RGBA8 tiles to rank 0 overlapped with the next step")
                if world > 1 else "single GPU",
                "frames_per_step": frames,
                "ms_per_frame": round(elapsed / (args.steps * frames) * 1e3, 4),
                "samples_per_frame": samples_all / args.steps / frames,
                "rays_in_box_per_frame": in_box_all / args.steps / frames,
                "kernel_ms_rank0": round(avg_kernel_s * 1e3, 4),
                "bytes_per_launch_rank0": bytes_per_launch,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved / 1e9, 3),
                "peak": HBM_PEAK / 1e9,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK,
                "traffic": None,
            },
        }
        prof = profiled_traffic(f"k_render<{irt.default_kernel_id()}>", int(cells.size), W)
        if prof and world == 1:
            out["roofline"]["traffic"] = prof[0]
            out["roofline"]["traffic_source"] = (
                f"{prof[1]}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch "
                f"of the same kernel and workload")
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cells, setup, W, H, args.cpu_budget)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
