#!/usr/bin/env python3
"""In-process A/B probe of the render path on one GPU: for each case (context env
overrides, camera, kernel variant) the frame is checked bit for bit against the first case
and timed over interleaved rounds (kernel ms from HIP events, step ms from back-to-back
launches).  One JSON line per case.

    python profiles/probe.py --config c3 --cases 'base;IRT_COUNTERS=atomic;cam=away' [--rounds 5]

A case is `;`-separated; inside a case, `,`-separated KEY=VALUE items: environment
variables read at context creation (IRT_*), `cam=framing|viewall|away`, `variant=N`,
`tf=default|zero|dense|comb` (alpha 0: the full sdda walk without a sample; alpha 1: one
accepted sample per in-shell ray; comb: bench.py's C3s sparse comb), `mode=user|tri|cubql`
(sampler), `accel=sphere|grid`.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "icon-ray-tracing_amd", "python"))

CONFIGS = {"c2": (2, 5, 47, 512), "c3": (2, 7, 90, 1024), "c4": (2, 7, 90, 2048),
           "small": (2, 3, 90, 256), "c3t": (2, 7, 90, 1024), "smallt": (2, 3, 90, 256)}
TERRAIN = {"c3t": 4000.0, "smallt": 4000.0}  # bench.py's C3t grid (irt_synth_grid_terrain)
CAMS = {"framing": ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0),
        "away": ((0.0, 0.0, 1.4e7), (0.0, 0.0, 2.8e7), (0.0, 1.0, 0.0), 60.0),
        "viewall": None}


def parse(case):
    env, opt = {}, {"cam": "framing", "variant": None, "tf": "default", "mode": "user",
                    "accel": "sphere"}
    for item in filter(None, case.split(",")):
        if item == "base":
            continue
        k, v = item.split("=", 1)
        if k in opt:
            opt[k] = v
        else:
            env[k] = v
    return env, opt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--cases", default="base")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--frames", type=int, default=20)
    args = ap.parse_args()
    import torch
    import irt
    L = irt.lib()
    L.irt_debug_set_variant.argtypes = [C.c_void_p, C.c_int]
    L.irt_debug_counters.argtypes = [C.c_void_p, C.c_void_p]
    rn, bis, lev, W = CONFIGS[args.config]
    cells = irt.synth_grid(rn, bis, lev, terrain=TERRAIN.get(args.config, 0.0))
    cases = [parse(c) for c in args.cases.split(";")]
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    runs = []
    for env, opt in cases:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        t0 = time.time()
        ctx = irt.Context(cells, 0)
        t_create = time.time() - t0
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
        setup = irt.setup_frame(cells, W, W, camera=CAMS[opt["cam"]])
        setup.lp.mode = {"user": irt.MODE_USER_GEOM, "tri": irt.MODE_TRIANGLES,
                         "cubql": irt.MODE_CUBQL}[opt["mode"]]
        setup.lp.accelMode = irt.ACCEL_GRID if opt["accel"] == "grid" else 0
        if opt["mode"] != "user":
            ctx.build_wedge_accel(cells)
        lut = setup.lut.copy()
        if opt["tf"] == "zero":
            lut[:, 3] = 0.0
        elif opt["tf"] == "dense":
            lut[:, 3] = 1.0
        elif opt["tf"] == "comb":
            lut[:, 3] = 0.01
            lut[::50, 3] = 1.0
        ctx.set_transfunc(lut, setup.value_range)
        ctx.set_timing_interval(1)
        if opt["variant"]:
            assert L.irt_debug_set_variant(ctx._h, int(opt["variant"])) == 0, L.irt_last_error()
        acc.zero_()
        fb.zero_()
        ctx.render(setup.lp, W, W, fb.data_ptr(), acc.data_ptr(), stream)
        torch.cuda.synchronize()
        st = ctx.stats()
        cnt = np.zeros(16, np.uint64)
        L.irt_debug_counters(ctx._h, cnt.ctypes.data)
        out = (fb.cpu().numpy().copy(), acc.cpu().numpy().view(np.uint32).copy())
        runs.append(dict(env=env, opt=opt, ctx=ctx, setup=setup, out=out, st=st.asdict(),
                         counters=[int(v) for v in cnt], create_s=t_create, k=[], step=[]))
    ref = {}
    for r in runs:  # identical frames among cases sharing camera, TF, sampler and accel
        key = (r["opt"]["cam"], r["opt"]["tf"], r["opt"]["mode"], r["opt"]["accel"])
        if key not in ref:
            ref[key] = r["out"]
        r["identical"] = bool(np.array_equal(r["out"][0], ref[key][0]) and
                              np.array_equal(r["out"][1], ref[key][1]))
    for _ in range(args.rounds):
        for r in runs:
            ctx, lp = r["ctx"], r["setup"].lp
            ctx.reset_stats_total()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for f in range(args.frames):
                ctx.render(lp, W, W, fb.data_ptr(), acc.data_ptr(), stream)
            torch.cuda.synchronize()
            r["step"].append((time.perf_counter() - t) / args.frames * 1e3)
            tot, n = ctx.stats_total()
            r["k"].append(tot.kernelMs / max(n, 1))
    for r in runs:
        k = float(np.median(r["k"]))
        L.irt_debug_queue_wgs.argtypes = [C.c_void_p]
        qwg = int(L.irt_debug_queue_wgs(r["ctx"]._h))
        print(json.dumps({"config": args.config, "env": r["env"], **r["opt"], "queue_wgs": qwg,
                          "identical": r["identical"], "kernel_ms": round(k, 4),
                          "step_ms": round(float(np.median(r["step"])), 4),
                          "mray_s": round(W * W / (k * 1e-3) / 1e6, 1),
                          "create_s": round(r["create_s"], 2), "stats": r["st"],
                          "counters": r["counters"]}), flush=True)
        r["ctx"].close()


if __name__ == "__main__":
    main()
