#!/usr/bin/env python3
"""Where a launch's machine time goes: every workgroup's start and end (s_memrealtime,
100 MHz), the XCC it ran on, for several back-to-back launches of one bench config.

    python profiles/wg_trace.py [--config c3] [--launches 4] [--warmup 5]

Per launch it prints one JSON line: the span (first start -> last end), the gap to the
previous launch's last end, workgroup durations (median / p90 / max), the mean and peak
number of resident workgroups, the slot-time used against peak x span ("fill"), and the
ramp (time until 90 % of the peak is resident) and tail (time from the last moment 90 % of
the peak was resident to the end).  Measurement only: frames are unchanged by the trace.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "icon-ray-tracing_amd", "python"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import irt  # noqa: E402


def analyse(tr, prev_end):
    st = tr[:, 0].astype(np.int64)
    en = tr[:, 1].astype(np.int64)
    base = st.min()
    st = (st - base) & 0xFFFFFFFF
    en = (en - base) & 0xFFFFFFFF
    span = int(en.max())
    dur = en - st
    ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    t = ev[:, 0]
    peak = int(conc.max())
    # time-weighted residency
    dt = np.diff(t, append=t[-1])
    mean_res = float((conc * dt).sum() / max(span, 1))
    hi = conc >= 0.9 * peak
    ramp = int(t[np.argmax(hi)]) if hi.any() else span
    last_hi = int(t[len(hi) - 1 - np.argmax(hi[::-1])]) if hi.any() else 0
    tail = span - last_hi
    xcc = tr[:, 3] & 0xF
    per_xcc_end = [round(float(en[xcc == x].max()) / 100, 2) if (xcc == x).any() else None for x in range(8)]
    per_xcc_busy = [round(float(dur[xcc == x].sum()) / 100, 1) for x in range(8)]
    top = np.argsort(-dur)[:8]
    out = {
        "workgroups": int(len(tr)),
        "longest": [[int(i), round(float(dur[i]) / 100, 2), round(float(st[i]) / 100, 2)] for i in top],
        "span_us": span / 100,
        "gap_from_prev_us": None if prev_end is None else ((int(tr[:, 0].min()) - prev_end) & 0xFFFFFFFF) / 100
        if ((int(tr[:, 0].min()) - prev_end) & 0xFFFFFFFF) < 2**31 else -(((prev_end - int(tr[:, 0].min())) & 0xFFFFFFFF) / 100),
        "wg_us_median": float(np.median(dur)) / 100,
        "wg_us_p90": float(np.percentile(dur, 90)) / 100,
        "wg_us_max": float(dur.max()) / 100,
        "resident_peak": peak,
        "resident_mean": round(mean_res, 1),
        "fill": round(float(dur.sum()) / max(peak * span, 1), 3),
        "ramp_us": ramp / 100,
        "tail_us": tail / 100,
        "per_xcc_last_end_us": per_xcc_end,
        "per_xcc_busy_wg_us": per_xcc_busy,
    }
    return out, int(tr[:, 1].max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--launches", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1, help="chained frames per launch (bench.py --batch)")
    args = ap.parse_args()
    rn, bis, L, W, H, tf, orbit_cfg, desc = bench.CONFIGS[args.config]
    dev = torch.device("cuda:0")
    ctx = irt.Context.synth(rn, bis, L, 0, terrain=bench.TERRAIN.get(args.config, 0.0))
    setup = irt.setup_frame(None, W, H, camera=bench.FRAMING, info=ctx.info)
    ctx.set_transfunc(bench.make_lut(tf, setup.lut), setup.value_range)
    ctx.set_statistics(False)
    lp = setup.lp
    fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
    accum = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(0).cuda_stream
    ctx.clear(fb.data_ptr(), accum.data_ptr(), W * H, stream)
    orbit = None
    if orbit_cfg:
        orbit = [irt.camera_look_at(*bench.orbit_camera(k), W, H) for k in range(bench.ORBIT_FRAMES)]

    B = max(1, args.batch) if orbit is None else 1

    def step(s):
        lp.accumID = s * B
        if orbit is not None:
            c = orbit[s % bench.ORBIT_FRAMES]
            lp.org, lp.dir_00, lp.dir_du, lp.dir_dv = c.org, c.dir_00, c.dir_du, c.dir_dv
            lp.accumID = 0
        if B > 1:
            ctx.render_accumulate(lp, W, H, B, fb.data_ptr(), accum.data_ptr(), stream)
        else:
            ctx.render(lp, W, H, fb.data_ptr(), accum.data_ptr(), stream)

    for s in range(args.warmup):
        step(s)
    nwg = ctx.launch_workgroups(irt.num_tiles(W, H), B)  # incl. a single frame's split packets
    bufs = [torch.zeros(nwg * 4, dtype=torch.int32, device=dev) for _ in range(args.launches)]
    torch.cuda.synchronize()
    for k in range(args.launches):
        ctx.set_wg_trace(bufs[k].data_ptr())
        step(args.warmup + k)
    ctx.set_wg_trace(0)
    torch.cuda.synchronize()
    prev = None
    for k in range(args.launches):
        tr = bufs[k].cpu().numpy().view(np.uint32).reshape(-1, 4)
        L = irt.lib()
        L.irt_debug_get_variant.argtypes = [ctypes.c_void_p]
        # the rows this launch wrote (a split single frame has extra workgroups, first)
        tr = tr[tr[:, 1] != 0]
        out, prev = analyse(tr, prev)
        out.update({"config": args.config, "launch": k, "frames_per_launch": B})
        print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
