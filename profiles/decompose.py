#!/usr/bin/env python3
"""Where a C3 frame's kernel time goes: the same 1024x1024 launch over workloads that stop
the raygen at different depths (all through the product path, default kernel variant).

  away     camera looking away from the globe: generateRay + boxTest + the pixel write
  empty    framing camera, all-zero TF alpha: no Woodcock sample anywhere (every majorant
           0), but the full sdda walk (entry/exit toSpherical, both ranges)
  dense    framing camera, TF alpha 1: the first sample that lands in a cell is accepted
  default  framing camera, the reference's default TF (the bench workload)
  viewall  the reference's default viewAll camera (globe covers ~7 % of pixels)

    python profiles/decompose.py [--frames 20]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "icon-ray-tracing_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--cases", default="away,empty,dense,default,viewall")
    args = ap.parse_args()
    import torch
    import irt
    rn, bis, lev, W = {"c3": (2, 7, 90, 1024), "c2": (2, 5, 47, 512)}[args.config]
    cells = irt.synth_grid(rn, bis, lev)
    ctx = irt.Context(cells, 0)
    fb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    acc = torch.zeros(W * W * 4, dtype=torch.float32, device="cuda")
    base = irt.setup_frame(cells, W, W, camera=irt.FRAMING_CAMERA)
    lut0 = base.lut.copy()
    cases = {
        "away": (irt.setup_frame(cells, W, W, camera=((0, 0, 1.4e7), (0, 0, 2.8e7), (0, 1, 0), 60.0)).lp, lut0),
        "empty": (base.lp, np.concatenate([lut0[:, :3], np.zeros((lut0.shape[0], 1), np.float32)], 1)),
        "dense": (base.lp, np.concatenate([lut0[:, :3], np.ones((lut0.shape[0], 1), np.float32)], 1)),
        "default": (base.lp, lut0),
        "viewall": (irt.setup_frame(cells, W, W).lp, lut0),
    }
    for name, (lp, lut) in cases.items():
        if name not in args.cases.split(","):
            continue
        ctx.set_transfunc(np.ascontiguousarray(lut, np.float32), base.value_range)
        ms = []
        for _ in range(args.frames):
            ctx.render(lp, W, W, fb.data_ptr(), acc.data_ptr())
            st = ctx.stats()
            ms.append(st.kernelMs)
        print(json.dumps({"case": name, "kernel_ms_median": float(np.median(ms)),
                          "kernel_ms_min": float(np.min(ms)), "rays_in_box": st.raysInBox,
                          "samples_found": st.samplesFound, "locate_calls": st.locateCalls,
                          "candidates": st.candidatesTested}), flush=True)


if __name__ == "__main__":
    main()
