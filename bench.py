#!/usr/bin/env python3
"""bench.py -- Mray/s + ms/frame of the MI355X ICON renderer (BASELINE.json metric).

The hot path is the raygen woodcockTrackingWithAccel (icon_rt/deviceCode.cu:281-341) over
every pixel of a frame.  Inputs (cells, locator, shell accelerator, transfer function) are
resident in HBM before the timed region; the grid is streamed into HBM and the scene built
on the device (irt_create_synth), so host memory stays at one chunk at any size.

Default workload (BASELINE.json configs[2], C3): synthetic R2B07 ICON grid (1,310,720
cells) x 90 levels (3,932,160 `.ic` records), 1024x1024, framing camera
`--camera 0 0 1.4e7 0 0 0 0 1 0 -fovy 60`, the reference's default transfer function.
Other configs (--config): c2 (R2B05 x 47, 512^2), c3t (C3's grid over terrain, as convert_icon
writes it: per-column HSURF/HHL offsets and the inverted first layer), c3s (C3 with a sparse "comb" transfer
function: alpha 0.01 except every 50th LUT entry at 1.0, so every macrocell's majorant stays
1 while ~95 % of tentative collisions are rejected -- ~13x C3's samples, the sample-heavy
regime where HBM bandwidth matters), c4 (C3's grid at 2048^2), c5 (R2B09 x 90 = 62.9 M
records, one of 60 orbit cameras per step).

One step (--mode):
  * progressive (default; "weak"): N consecutive frames of the reference's progressive
    accumulation (--sample-limit, accumID = step*N + k); with N GPUs (one process per GPU
    under torchrun) every rank renders its interleaved 64x64 tiles of all N frames in ONE
    launch (irt_render_tiles_accumulate) and rank 0 gathers the final RGBA8 tiles over RCCL
    (torch.distributed "nccl") into rank-major storage and unpacks the framebuffer.  The
    gather of step s runs on the collective's stream while step s+1 renders
    (double-buffered tiles).  Per-GPU work is one frame's rays per step at every N.
  * frame ("strong"): ONE frame per step, its 64x64 tiles dealt round-robin to the N ranks
    (irt_render_tiles), gathered and unpacked the same way: single-frame latency, the
    BASELINE's C4 "frame-tile split with RCCL framebuffer gather".
Frames are enqueued back to back: per-launch statistics come back through a ring, never
stalling the host between launches.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c3s|c3t|c2|c4|c5]
       [--mode progressive|frame] [--dist-backend nccl|gloo] [--verify] [--secondary LIST]
       torchrun --nproc-per-node N bench.py --gpus N ...
With --gpus N > 1 and no launcher (WORLD_SIZE unset) bench.py starts the N ranks itself
(torch.distributed.run as a child process, before this process touches a GPU) and relays rank
0's JSON line; under a launcher --gpus must equal WORLD_SIZE.  On one GPU with the default c3,
the line also carries "secondary": C3t, C3s and C5 measured the same way with a few steps each.
"""
import argparse
import glob
import json
import os
import re
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
    # name: (rootN, bisections, levels, W, H, transfer function, orbit, description)
    "c2": (2, 5, 47, 512, 512, "default", False, "C2: R2B05 (81,920 cells) x 47 levels, 512x512"),
    "c3": (2, 7, 90, 1024, 1024, "default", False,
           "C3: R2B07 (1,310,720 cells) x 90 levels, 1024x1024"),
    "c3s": (2, 7, 90, 1024, 1024, "comb", False,
            "C3s: R2B07 (1,310,720 cells) x 90 levels, 1024x1024, sparse comb TF (alpha 0.01, "
            "every 50th of the 300 LUT entries 1.0: sample-heavy)"),
    "c3t": (2, 7, 90, 1024, 1024, "default", False,
            "C3t: R2B07 (1,310,720 cells) x 90 levels over terrain (HSURF up to 4 km, "
            "terrain-following HHL) as convert_icon writes it (inverted first layer over land, "
            "last record 25 layers), 1024x1024"),
    "c4": (2, 7, 90, 2048, 2048, "default", False,
           "C4: R2B07 (1,310,720 cells) x 90 levels, 2048x2048"),
    "c5": (2, 9, 90, 1024, 1024, "default", True,
           "C5: R2B09 (20,971,520 cells) x 90 levels, 1024x1024, 60-frame orbit"),
}


# configs over terrain (irt_synth_grid_terrain): the maximum HSURF in metres
TERRAIN = {"c3t": 4000.0}


def make_lut(kind, lut):
    """The config's LUT from the reference's default (hostCode.cu:823-836, resampled to 300
    entries): "default" as is; "comb" with alpha 0.01 except every 50th entry 1.0."""
    lut = np.array(lut, dtype=np.float32, copy=True)
    if kind == "comb":
        lut[:, 3] = 0.01
        lut[::50, 3] = 1.0
    return lut
ORBIT_FRAMES = 60  # C5: eye = 1.4e7 (sin t, 0, cos t), t = 2 pi k / 60, looking at the origin
FRAMING = ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def available_cores():
    """CPUs this process may use: os.cpu_count() capped by the affinity mask and the
    cgroup CPU quota (a GPU box shows the whole machine's CPUs, of which it gets a share)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(rn, bis, L, W, H, camera, tf, budget_s=15.0, terrain=0.0):
    """The reference's CPU path on the host cores, two ways (test-infrastructure oracle,
    oracle/; only this leg of bench.py touches it):
      * "port" (the primary number): the oracle's restatement of the reference raygen with
        a direction-voxel cell locator in place of the brute-force scan (same first-index
        answer, pinned against the reference's fixtures), 64x64 tiles pulled from an atomic
        counter by one thread per available core (common/pipeline.cu:767,
        thread_pool.h:146-161); whole frames, render time only (pipeline.cu:1062-1073);
      * "reference": the reference's own raygen and brute-force first-hit scan
        (deviceCode.cu:116-123), compiled from its headers (oracle/_ref), on a strided pixel
        sample of the frame (a whole frame would take hours)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import irt
    import oracle as O
    cores = available_cores()
    cells = irt.synth_grid(rn, bis, L, terrain=terrain)
    S = O.OracleScene(cells)
    lut, vr = S.default_lut()
    S.set_transfunc(make_lut(tf, lut), vr)
    cam = S.camera(W, H, camera)
    params = S.params(cam, accum_id=0, raygen=0)
    T = O.TimedScene(S, 2, cores)
    T.render(params, W, H, rect=(0, 0, 64, 64), threads=cores)  # build + warm
    frames, elapsed = 0, 0.0
    while elapsed < budget_s / 2 or frames < 1:
        t = time.perf_counter()
        _, _, st = T.render(params, W, H, threads=cores)
        elapsed += time.perf_counter() - t
        frames += 1
        if frames >= 200:
            break
    T.close()
    port_mray = W * H * frames / elapsed / 1e6
    out = {"value": port_mray, "unit": "Mray/s", "cores": cores, "kind": "port",
           "nproc": os.cpu_count(), "cpu_model": cpu_model(),
           "sample": (f"{frames} whole {W}x{H} frames ({elapsed:.1f} s of render time on "
                      f"{cores} threads, 64x64 tiles from an atomic counter): the oracle's "
                      f"restatement of woodcockTrackingWithAccel over {cells.size} records, "
                      f"cells located through a direction-voxel locator (first index wins, "
                      f"as the reference's scan; oracle/icon_oracle.cpp DirGrid)"),
           "ms_per_frame": elapsed / frames * 1e3,
           "samples_per_frame": int(st.samples_found)}
    # the reference's own code and brute-force scan, on a strided pixel sample
    if O.have_ref():
        stride, t_ref, pix, locate = 128, 0.0, 0, 0
        while True:
            ys, xs = np.mgrid[stride // 2:H:stride, stride // 2:W:stride]
            xy = np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.int32)
            t = time.perf_counter()
            _, _, cnt = O.ref_render_pixels(S, params, W, H, xy, threads=cores)
            t_ref = time.perf_counter() - t
            pix, locate = xy.shape[0], int(cnt[0])
            log(f"[cpu baseline] reference stride {stride}: {pix} rays in {t_ref:.2f} s")
            if t_ref > budget_s / 4 or stride <= 8:
                break
            stride //= 2
        ref = pix / t_ref / 1e6
        out["brute_force_reference"] = {
            "value": ref, "unit": "Mray/s", "cores": cores, "kind": "reference",
            "sample": (f"every {stride}th pixel in x and y ({pix} rays, {locate} sampleVolume "
                       f"calls, {t_ref:.1f} s on {cores} threads): the reference's CPU raygen "
                       f"with its brute-force first-hit cell scan (deviceCode.cu:116-123), "
                       f"compiled from its own headers (oracle/_ref)"),
            "ms_per_frame_extrapolated": W * H / (ref * 1e6) * 1e3}
    return out


def profiled_traffic(kernel, config, frames=1):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 summary of the
    same workload (profiles/*/summary.json: FETCH_SIZE x 2 + WRITE_SIZE, per the gfx950
    correction of MI355X_MICROARCH.md), or None."""
    def tag_order(p):  # profiles/rNN<tag>_*: tags run a..z, then aa..az (r05q before r05an)
        m = re.match(r"r(\d+)([a-z]*)", os.path.basename(os.path.dirname(p)))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")

    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary.json")), key=tag_order):
        try:
            s = json.load(open(p))
        except (OSError, ValueError):
            continue
        if s.get("config_name") != config or s.get("frames_per_launch", 1) != frames:
            continue
        # the profiled launches (not a context's one-workgroup prewarm dispatches of other forms)
        if not any(k.endswith(kernel) and v.get("calls", 0) > 1 for k, v in s.get("kernels", {}).items()):
            continue
        if "traffic_bytes_per_launch_fetch_x2" in s:
            best = (s["traffic_bytes_per_launch_fetch_x2"], os.path.relpath(p, ROOT))
    return best


def orbit_camera(k):
    th = 2.0 * np.pi * k / ORBIT_FRAMES
    return ((1.4e7 * np.sin(th), 0.0, 1.4e7 * np.cos(th)), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)


# the configs whose numbers DESIGN.md quotes besides the headline C3, measured in the same
# run (a few steps each, after the primary line's timed region) so that they come under the
# driver's clock too: terrain (the realistic-data layout), the sample-heavy TF and R2B09
SECONDARY = ("c3t", "c3s", "c5")


def spawn_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) started as a plain program: one rank per GPU, launched as
    the driver's own `torch.distributed.run --nproc-per-node N` form does, from this process
    before it imports torch or touches a GPU (it never execs: the launcher is a child).  The
    children's stderr passes through; of their stdout only rank 0's JSON line is relayed to
    ours, everything else goes to stderr.  Returns the launcher's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"[launcher] {n} ranks: {' '.join(cmd)}")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    for line in p.stdout:
        s = line.strip()
        is_json = False
        if s.startswith("{"):
            try:
                is_json = isinstance(json.loads(s), dict) and "metric" in json.loads(s)
            except ValueError:
                pass
        (sys.stdout if is_json else sys.stderr).write(line)
        (sys.stdout if is_json else sys.stderr).flush()
    return p.wait()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU).  Under torch.distributed.run it must equal "
                         "WORLD_SIZE; started directly with N > 1, bench.py launches the N ranks "
                         "itself")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="progressive", choices=["progressive", "frame"],
                    help="progressive: N frames per step (weak); frame: one frame per step "
                         "split over the N ranks (strong)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--sampler", default="user", choices=["user", "tri", "cubql"],
                    help="Volume::mode (Params.h:29-31): sample() on the cells (default), "
                         "TRIANGLE_MODE, CUBQL_MODE wedges")
    ap.add_argument("--accel", default="sphere", choices=["sphere", "grid"],
                    help="Volume::accelMode (Params.h:33-34): the spherical shell (sdda, "
                         "default) or the 256^3 grid (dda3)")
    ap.add_argument("--force-dist", action="store_true",
                    help="(overhead check) run the multi-rank path -- tile render, RCCL gather, "
                         "unpack -- even with one rank (under torchrun)")
    ap.add_argument("--stats", default="off", choices=["on", "off"],
                    help="per-launch event counts (irt_set_statistics) inside the timed loop.  "
                         "off (default): the product renders without them, as the reference "
                         "does; the counts the roofline needs come from rendering the same "
                         "steps again afterwards with counting on (untimed, identical frames)")
    ap.add_argument("--batch", type=int, default=8,
                    help="progressive frames per launch on one GPU (irt_render_accumulate: the "
                         "reference's accumulation loop over accumID, frames chained in one "
                         "launch; every frame's accum and fb are written). 1: one launch per frame")
    ap.add_argument("--no-single-compare", action="store_true",
                    help="skip timing the same frames at one launch per frame after the timed "
                         "region (profiling runs: one launch shape per kernel trace)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the multi-rank path with host-staged collectives "
                         "(ranks may share a GPU); nccl (RCCL) is the measured path")
    ap.add_argument("--verify", action="store_true",
                    help="multi-rank: after the timed region rank 0 renders the same accumID "
                         "sequence on its own context with irt_render_accumulate and compares "
                         "the assembled framebuffer pixel for pixel (exit 3 on a mismatch)")
    ap.add_argument("--secondary", default="auto",
                    help="comma-separated configs measured after the primary line on one GPU "
                         "(a few steps each, reported under \"secondary\"); auto: "
                         + ",".join(SECONDARY) + " when the primary config is c3; none: skip")
    ap.add_argument("--secondary-steps", type=int, default=10)
    return ap.parse_args(argv)


def run_config(args, config, steps, warmup, rank, world, dist_path, primary=True):
    """Build `config`'s scene on this rank's GPU, render `warmup` + `steps` steps (timed
    between barriers + synchronize), and return the result dict on rank 0 (None elsewhere)."""
    import torch
    import irt
    import resource
    if dist_path:
        import torch.distributed as dist
    device = torch.cuda.current_device()
    dev = torch.device(f"cuda:{device}")

    rn, bis, L, W, H, tf, orbit_cfg, desc = CONFIGS[config]
    t0 = time.time()
    terrain = TERRAIN.get(config, 0.0)
    # streamed into HBM, built on the device
    ctx = irt.Context.synth(rn, bis, L, device, terrain=terrain)
    info = ctx.info
    setup = irt.setup_frame(None, W, H, camera=FRAMING, info=info)
    ctx.set_transfunc(make_lut(tf, setup.lut), setup.value_range)
    # HIP events around every k-th launch of the timed region (the roofline's kernel
    # duration): each timed launch adds ~4.7 us of event packets to its step (every launch
    # timed: +8 us per C3 step), so k = steps/4 (at most 32; four timed launches per run, one
    # at least when steps < 4) keeps them to ~1 % of the region
    ctx.set_timing_interval(max(1, min(32, steps // 4)))
    create_s = time.time() - t0
    log(f"[rank {rank}] {config} context: {info.numCells} records, {info.deviceBytes / 2**30:.2f} GiB HBM, "
        f"locator G={info.locatorFaceRes} entries={info.locatorEntries} ({create_s:.1f} s, "
        f"peak host RSS {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20:.2f} GiB)")

    lp = setup.lp
    lp.mode = {"user": irt.MODE_USER_GEOM, "tri": irt.MODE_TRIANGLES, "cubql": irt.MODE_CUBQL}[args.sampler]
    lp.accelMode = irt.ACCEL_GRID if args.accel == "grid" else 0
    if args.sampler != "user":  # buildTriangleAccel / buildCuBQLAccel (hostCode.cu:440-649)
        ctx.build_wedge_accel(irt.synth_grid(rn, bis, L, terrain=terrain))
    orbit = None
    if orbit_cfg:  # one orbit frame per step (a new view: accumID 0)
        orbit = [irt.camera_look_at(*orbit_camera(k), W, H) for k in range(ORBIT_FRAMES)]
    ntiles = irt.num_tiles(W, H)
    if dist_path:
        # render on a high-priority stream: its hardware queue comes from another pool than
        # RCCL's normal-priority stream.  Sharing one queue (measured: torch's default stream
        # and the gather's stream on the same queue) puts step s's gather in front of step
        # s+1's unpack and render, ~20 us of barrier latency per step.
        torch.cuda.set_stream(torch.cuda.Stream(dev, priority=-1))
    stream = torch.cuda.current_stream(device).cuda_stream
    # frames per step: --batch consecutive progressive frames (chained in one launch; the
    # orbit's frames are new views, one per step), times N in progressive mode on N GPUs
    # (per-GPU work fixed as N grows); in frame mode the same --batch frames split over the
    # N GPUs (total work fixed)
    strong = args.mode == "frame"
    batch = max(1, args.batch)
    frames = batch * (world if dist_path and not strong else 1)
    orbit_lps = None
    if orbit is not None:  # each orbit view as a whole launch-parameter record (accumID 0)
        orbit_lps = []
        for c in orbit:
            q = irt.LaunchParams.from_buffer_copy(lp)
            q.org, q.dir_00, q.dir_du, q.dir_dv = c.org, c.dir_00, c.dir_du, c.dir_dv
            q.accumID = 0
            orbit_lps.append(q)
    if not dist_path:
        fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
        accum = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
        ctx.clear(fb.data_ptr(), accum.data_ptr(), W * H, stream)
    else:
        import irt_dist
        # the cost-balanced deal (irt_deal_tiles) for the first camera: the orbit keeps the
        # globe centred at the same size, so one deal serves every step
        split = irt_dist.TileSplit.dealt(W, H, rank, world, orbit[0] if orbit else setup.lp, info,
                                         frames)
        assert split.num_tiles == ntiles
        maxt = split.max_tiles
        fg = irt_dist.FrameGather(split, dev, buffers=8, stage_cpu=args.dist_backend == "gloo")
        tiles_acc = torch.zeros(maxt * 4096 * 4, dtype=torch.float32, device=dev)
        fb = torch.zeros(W * H, dtype=torch.int32, device=dev) if rank == 0 else None
    pipe = None
    if dist_path:
        pipe = irt_dist.FramePipeline(ctx, fg, fb)

    def step(s):
        lp.accumID = s * frames
        if orbit is not None and frames > 1:
            # `frames` consecutive orbit views in one launch (irt_render_sequence; on N GPUs
            # every rank its tiles of them, irt_render_tile_list_sequence)
            seq = [orbit_lps[(s * frames + k) % ORBIT_FRAMES] for k in range(frames)]
            if not dist_path:
                ctx.render_sequence(seq, W, H, fb.data_ptr(), accum.data_ptr(), stream)
            else:
                pipe.step(s, lambda buf: split.render_sequence(ctx, seq, buf.data_ptr(), tiles_acc.data_ptr(),
                                                              stream))
            return
        if orbit is not None:
            c = orbit[s % ORBIT_FRAMES]
            lp.org, lp.dir_00, lp.dir_du, lp.dir_dv = c.org, c.dir_00, c.dir_du, c.dir_dv
            lp.accumID = 0
        if not dist_path:
            if frames > 1:  # `frames` consecutive progressive frames in one launch
                ctx.render_accumulate(lp, W, H, frames, fb.data_ptr(), accum.data_ptr(), stream)
            else:
                ctx.render(lp, W, H, fb.data_ptr(), accum.data_ptr(), stream)
            return
        pipe.step(s, lambda buf: split.render(ctx, lp, frames, buf.data_ptr(),
                                              tiles_acc.data_ptr(), stream))

    for f in range(warmup):
        step(f)
    if dist_path:
        pipe.drain()
    st = ctx.stats()
    log(f"[rank {rank}] {config} warmup: last launch kernel {st.kernelMs:.3f} ms, {st.samplesFound} "
        f"samples, {st.candidatesTested} candidates")
    ctx.reset_stats_total()
    ctx.set_statistics(args.stats == "on")
    torch.cuda.synchronize()
    if dist_path:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(steps):
        step(warmup + k)
    host_loop = time.perf_counter() - t_start  # host side of the loop (launches only)
    if dist_path:
        pipe.drain()  # the gathers and rank 0's unpacks are inside the timed region
    torch.cuda.synchronize()
    if dist_path:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    tot, launches = ctx.stats_total()  # kernel time of the timed launches (HIP events)
    if args.stats == "off":
        # the event counts of the same steps (same accumIDs and cameras: identical frames and
        # counts), rendered again with counting on, untimed
        ctx.reset_stats_total()
        ctx.set_statistics(True)
        for k in range(steps):
            step(warmup + k)
        if dist_path:
            pipe.drain()
        torch.cuda.synchronize()
        counted, _ = ctx.stats_total()
        counted.kernelMs = tot.kernelMs
        tot = counted
    verify = None
    if dist_path and args.verify and rank == 0:
        # rank 0's assembled frame against its own context rendering every frame of every
        # tile: the same accumID sequence (warmup + timed steps, then the counted re-run of the
        # timed steps) through irt_render_accumulate on a fresh framebuffer
        assert orbit is None, "--verify covers the progressive (non-orbit) configs"
        ref_fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
        ref_acc = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
        runs = [(0, (warmup + steps) * frames)]
        if args.stats == "off":
            runs.append((warmup * frames, steps * frames))
        q = irt.LaunchParams.from_buffer_copy(lp)
        for first, count in runs:
            for a in range(first, first + count, batch):
                q.accumID = a
                ctx.render_accumulate(q, W, H, min(batch, first + count - a), ref_fb.data_ptr(),
                                      ref_acc.data_ptr(), stream)
        torch.cuda.synchronize()
        bad = int((ref_fb != fb).sum().item())
        verify = {"pixels": W * H, "mismatches": bad, "frames_per_pixel": sum(c for _, c in runs),
                  "against": "irt_render_accumulate of the whole frame on rank 0's context, the "
                             "same accumID sequence"}
        log(f"[rank 0] verify: {bad} of {W * H} pixels differ from the single-context frame")
    single = None
    if not dist_path and frames > 1 and not args.no_single_compare:
        # the same workload at one launch per frame (irt_render), for comparison: the frames
        # that follow the timed steps' accumulation, statistics as in the timed loop
        ctx.set_statistics(args.stats == "on")
        n1 = steps * frames
        base = (warmup + steps) * frames
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for k in range(n1):
            if orbit is not None:
                ctx.render(orbit_lps[(base + k) % ORBIT_FRAMES], W, H, fb.data_ptr(), accum.data_ptr(), stream)
            else:
                lp.accumID = base + k
                ctx.render(lp, W, H, fb.data_ptr(), accum.data_ptr(), stream)
        torch.cuda.synchronize()
        e1 = time.perf_counter() - t1
        single = {"ms_per_frame": round(e1 / n1 * 1e3, 4), "value": round(W * H * n1 / e1 / 1e6, 3),
                  "frames": n1}
    log(f"[rank {rank}] {config} timed {steps} steps ({launches} launches) in {elapsed:.4f} s "
        f"(host loop {host_loop:.4f} s); peak host RSS {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20:.2f} GiB")
    samples, in_box = tot.samplesFound, tot.raysInBox
    if dist_path:
        rdev = dev if args.dist_backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        agg = torch.tensor([samples, in_box, tot.raysLaunched], dtype=torch.float64, device=rdev)
        dist.all_reduce(agg)
        samples_all, in_box_all, launched_all = (int(v) for v in agg.tolist())
    else:
        samples_all, in_box_all, launched_all = samples, in_box, tot.raysLaunched
    # chained-frame waits that gave up (0 in a correct run: every frame then equals one
    # launch per frame); counted over every launch of this context, all ranks summed
    chain_timeouts = ctx.chain_errors()
    if dist_path:
        ct = torch.tensor([chain_timeouts], dtype=torch.float64, device=rdev)
        dist.all_reduce(ct)
        chain_timeouts = int(ct.item())
    if chain_timeouts:
        log(f"[rank {rank}] WARNING: {chain_timeouts} chained-frame waits timed out; frames may be wrong")

    ms_per_step = elapsed / steps * 1e3
    mray = W * H * frames * steps / elapsed / 1e6  # all ranks' rays
    # roofline of the dominant kernel on this rank: algorithmic bytes per launch over its
    # HIP-event-timed average duration (events on the stream the kernel runs on)
    avg_kernel_s = tot.kernelMs / 1e3 / max(launches, 1)
    bytes_per_launch = (BYTES_PER_SAMPLE * samples + BYTES_PER_RAY * in_box) / max(launches, 1)
    achieved = bytes_per_launch / avg_kernel_s if avg_kernel_s > 0 else float("nan")

    out = None
    if rank == 0:
        if world == 1 and not dist_path:
            parallelism = "single GPU"
        elif strong:
            parallelism = (f"{world} GPUs x 64x64 cost-balanced tiles of the step's {frames} frame(s) "
                           f"(one launch per rank), RCCL "
                           f"gather of the RGBA8 tiles to rank 0 overlapped with the next step")
        else:
            parallelism = (f"{world} GPUs x 64x64 cost-balanced frame tiles, {frames} progressive "
                           f"frames per step in one launch per rank, RCCL gather of the final "
                           f"RGBA8 tiles to rank 0 overlapped with the next step")
        if dist_path and args.dist_backend == "gloo":
            parallelism += " (gloo rehearsal: host-staged gathers)"
        out = {
            "metric": METRIC,
            "value": round(mray, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": round(ms_per_step, 4),
            "frames_per_launch": frames,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "name": config,
                "workload": desc + (", orbit camera (eye 1.4e7 (sin t, 0, cos t), -fovy 60), " +
                                    ("one orbit frame per step" if frames == 1 else
                                     f"{frames} consecutive orbit views per step (one launch)")
                                    if orbit is not None else
                                    ", framing camera --camera 0 0 1.4e7 0 0 0 0 1 0 -fovy 60, " +
                                    ("one frame per step" if frames == 1 else
                                     f"{frames} consecutive progressive frames (accumID) per step")) +
                           ", woodcockTrackingWithAccel, " + ("sparse comb TF" if tf == "comb" else "default TF") +
                           ("" if args.sampler == "user" else
                            {"tri": ", TRIANGLE_MODE sampler", "cubql": ", CUBQL_MODE wedge sampler"}[args.sampler]) +
                           (", GRID_ACCEL_MODE (dda3 over the 256^3 grid)" if args.accel == "grid" else ""),
                "records": int(info.numCells), "width": W, "height": H,
                "transfer_function": tf,
                "sampler": args.sampler,
                "accel": args.accel,
                "parallelism": parallelism,
                "frames_per_step": frames,
                "ms_per_frame": round(elapsed / (steps * frames) * 1e3, 4),
                "samples_per_frame": samples_all / steps / frames,
                "rays_in_box_per_frame": in_box_all / steps / frames,
                "candidates_per_sample": tot.candidatesTested / max(samples, 1),
                "kernel_ms_rank0": round(avg_kernel_s * 1e3, 4),
                "statistics_in_timed_loop": args.stats,
                "frames_per_launch": frames,
                "bytes_per_launch_rank0": bytes_per_launch,
                "chain_timeouts": chain_timeouts,
                # the slot table (built when the headers outgrow the last-level cache)
                "slot_table_bytes": ctx.array_bytes("slots"),
                "context_create_s": round(create_s, 2),
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
        if single is not None:
            out["single_frame_launches"] = single  # the same frames, one launch each
        if verify is not None:
            out["verify"] = verify
        prof = profiled_traffic(f"k_render<{irt.default_kernel_id(ctx)}>", config, frames)
        if prof and world == 1:
            out["roofline"]["traffic"] = prof[0]
            out["roofline"]["traffic_source"] = (
                f"{prof[1]}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch "
                f"of the same kernel and workload")
        if primary and world == 1 and not args.no_cpu_baseline:
            cam = orbit_camera(0) if orbit is not None else FRAMING
            out["cpu_baseline"] = cpu_baseline(rn, bis, L, W, H, cam, tf, args.cpu_budget, terrain)
    if dist_path:
        dist.barrier()
    del fb
    if not dist_path:
        del accum
    ctx.close()
    torch.cuda.empty_cache()
    return out


def secondary_entry(out):
    """The fields of a secondary config's line that DESIGN.md quotes."""
    c, r = out["config"], out["roofline"]
    e = {"workload": c["workload"], "value": out["value"], "unit": out["unit"],
         "ms_per_step": out["ms_per_step"], "ms_per_frame": c["ms_per_frame"],
         "frames_per_launch": out["frames_per_launch"], "steps": out["steps"],
         "warmup": out["warmup"], "records": c["records"],
         "samples_per_frame": c["samples_per_frame"],
         "candidates_per_sample": c["candidates_per_sample"],
         "kernel_ms": c["kernel_ms_rank0"], "slot_table_bytes": c["slot_table_bytes"],
         "context_create_s": c["context_create_s"], "chain_timeouts": c["chain_timeouts"],
         "roofline": {k: r[k] for k in ("achieved", "unit", "frac", "traffic") if k in r}}
    if "traffic_source" in r:
        e["roofline"]["traffic_source"] = r["traffic_source"]
    if "bytes_per_launch_rank0" in c and r.get("traffic"):
        e["roofline"]["traffic_over_algorithmic"] = r["traffic"] / c["bytes_per_launch_rank0"]
    if "single_frame_launches" in out:
        e["single_frame_launches"] = out["single_frame_launches"]
    return e


def main():
    args = parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # no launcher: start the N ranks ourselves (before any GPU call in this process)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world} (one rank per GPU)")
        sys.exit(2)

    import torch

    dist_path = world > 1 or args.force_dist
    ndev = torch.cuda.device_count()  # counts without initialising the GPU on this image
    if dist_path and args.dist_backend == "nccl" and ndev < world:
        log(f"error: {world} RCCL ranks need {world} GPUs, {ndev} visible")
        sys.exit(2)
    device = local % max(ndev, 1) if dist_path else 0
    json_out = sys.stdout
    if dist_path:
        # RCCL (and the runtime under it) may print banners on fd 1: send everything
        # native to stderr and keep stdout for the one JSON line
        json_out = os.fdopen(os.dup(1), "w")
        sys.stdout.flush()
        os.dup2(2, 1)
        import torch.distributed as dist
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{device}"))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(device)

    out = run_config(args, args.config, args.steps, args.warmup, rank, world, dist_path)
    if out is not None and not dist_path:
        names = ([] if args.secondary == "none" else
                 list(SECONDARY) if args.secondary == "auto" and args.config == "c3" else
                 [] if args.secondary == "auto" else args.secondary.split(","))
        sec = {}
        for name in names:
            if name not in CONFIGS or name == args.config:
                continue
            t = time.time()
            try:
                o = run_config(args, name, args.secondary_steps, 2, rank, world, dist_path,
                               primary=False)
                sec[name] = secondary_entry(o)
                sec[name]["wall_s"] = round(time.time() - t, 1)
            except Exception as e:  # a secondary config never costs the primary line
                log(f"[rank 0] secondary {name} failed: {e!r}")
                sec[name] = {"error": repr(e)}
        if sec:
            out["secondary"] = sec
    if out is not None:
        print(json.dumps(out), file=json_out, flush=True)
    bad = out is not None and out.get("verify", {}).get("mismatches", 0) > 0
    if dist_path:
        dist.barrier()
        dist.destroy_process_group()
    if bad:
        sys.exit(3)


if __name__ == "__main__":
    main()
