#!/usr/bin/env python3
"""Per-frame wave statistics of the raygen (statistics variant, counters[5..9]): Woodcock
draws per ray and per wave (max over lanes), zero-length sdda leaves, range-1 rays.

    python profiles/wave_stats.py [--config c3] [--variants 49152,42496] [--camera framing]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "icon-ray-tracing_amd", "python"))
CONFIGS = {"c2": (2, 5, 47, 512), "c3": (2, 7, 90, 1024), "small": (2, 3, 90, 256)}
FRAMING = ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--variants", default="32768,36864")
    ap.add_argument("--camera", default="framing", choices=["framing", "viewall"])
    args = ap.parse_args()
    import torch
    import irt
    L = irt.lib()
    L.irt_debug_set_variant.argtypes = [C.c_void_p, C.c_int]
    L.irt_debug_counters.argtypes = [C.c_void_p, C.c_void_p]
    rn, bis, lev, W = CONFIGS[args.config]
    cells = irt.synth_grid(rn, bis, lev)
    setup = irt.setup_frame(cells, W, W, camera=FRAMING if args.camera == "framing" else None)
    ctx = irt.Context(cells, 0)
    ctx.set_transfunc(setup.lut, setup.value_range)
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    for v in (int(x) for x in args.variants.split(",")):
        assert L.irt_debug_set_variant(ctx._h, v) == 0, L.irt_last_error()
        ctx.render(setup.lp, W, W, fb.data_ptr(), acc.data_ptr())
        c = np.zeros(16, np.uint64)
        assert L.irt_debug_counters(ctx._h, c.ctypes.data) == 0
        waves = W * W // 64
        print(json.dumps({"variant": v, "config": args.config, "camera": args.camera,
                          "rays": int(c[0]), "in_box": int(c[1]), "locate": int(c[2]),
                          "found": int(c[3]), "candidates": int(c[4]), "draws": int(c[5]),
                          "draws_per_wave_max_avg": float(c[6]) / waves,
                          "draws_per_wave_sum_avg": float(c[5]) / waves,
                          "deg_leaves": int(c[7]), "deg_per_wave_max_avg": float(c[8]) / waves,
                          "range1_rays_or_max_draws": int(c[9]),
                          "march_draw_hist_le2_3to5_6to10_gt10": [int(v) for v in c[12:16]]}),
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
