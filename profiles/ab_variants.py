#!/usr/bin/env python3
"""In-process A/B timing of the render-kernel variants (irt_render.hip OPT_* bits).

All variants must give the same frame; this script checks that bit for bit against
variant 0, then times the variants interleaved over several rounds on one context
(cdna_hip_programming.md rule 24) and prints one JSON line per variant.

    python profiles/ab_variants.py [--config c3] [--rounds 5] [--frames 10] [--variants 0,1,...]
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

CONFIGS = {"c2": (2, 5, 47, 512), "c3": (2, 7, 90, 1024), "small": (2, 3, 90, 256)}
FRAMING = ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--variants", default="0,1,1536,2048,4096")
    ap.add_argument("--camera", default="framing", choices=["framing", "viewall"])
    ap.add_argument("--no-check", action="store_true",
                    help="report but do not stop on differences (counter-collection passes may "
                         "replay a dispatch, which doubles the in-kernel statistics)")
    args = ap.parse_args()
    import torch
    import irt
    L = irt.lib()
    L.irt_debug_set_variant.argtypes = [C.c_void_p, C.c_int]
    rn, bis, lev, W = CONFIGS[args.config]
    cells = irt.synth_grid(rn, bis, lev)
    setup = irt.setup_frame(cells, W, W, camera=FRAMING if args.camera == "framing" else None)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    variants = [int(v) for v in args.variants.split(",")]
    ref = None
    for v in variants:
        assert L.irt_debug_set_variant(ctx._h, v) == 0, L.irt_last_error()
        acc.zero_()
        ctx.render(setup.lp, W, W, fb.data_ptr(), acc.data_ptr())
        st = ctx.stats()
        out = (fb.cpu().numpy().copy(), acc.cpu().numpy().view(np.uint32).copy(), st.samplesFound)
        if ref is None:
            ref = out
        same = [np.array_equal(out[0], ref[0]), np.array_equal(out[1], ref[1]), out[2] == ref[2]]
        print(f"variant {v}: identical to {variants[0]} (fb, accum, samples): {same}",
              file=sys.stderr, flush=True)
        if not all(same) and not args.no_check:
            raise SystemExit(f"variant {v} differs")
    times = {v: [] for v in variants}
    for r in range(args.rounds):
        for v in variants:
            L.irt_debug_set_variant(ctx._h, v)
            ks = []
            for f in range(args.frames):
                ctx.render(setup.lp, W, W, fb.data_ptr(), acc.data_ptr())
                ks.append(ctx.stats().kernelMs)
            times[v].append(float(np.median(ks)))
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"variant": v, "config": args.config, "camera": args.camera,
                          "kernel_ms_median": float(np.median(t)), "kernel_ms_min": float(t.min()),
                          "mray_s": W * W / (np.median(t) * 1e-3) / 1e6}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
