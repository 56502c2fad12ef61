#!/usr/bin/env python3
"""C5 (R2B09 x 90 levels, 62.9 M records) context creation streamed into HBM
(irt_create_synth): wall time, per-stage build times (IRT_BUILD_VERBOSE=1), peak host RSS,
then a few orbit frames.  One JSON line."""
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "icon-ray-tracing_amd", "python"))


def main():
    import torch
    import irt
    rn, bis, lev = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (2, 9, 90)))
    t0 = time.time()
    ctx = irt.Context.synth(rn, bis, lev, 0)
    t_create = time.time() - t0
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20
    info = ctx.info
    setup_lp = irt.camera_look_at((0.0, 0.0, 1.4e7), (0, 0, 0), (0, 1, 0), 60.0, 1024, 1024)
    lut, vr = irt.default_transfunc((info.dataRange.lower, info.dataRange.upper))
    ctx.set_transfunc(lut, vr)
    lp = setup_lp
    lp.ambientColor = irt.Vec3(1, 1, 1)
    lp.ambientRadiance = 1.0
    lp.unitDistance = info.unitDistance
    fb = torch.zeros(1024 * 1024, dtype=torch.int32, device="cuda")
    acc = torch.zeros(1024 * 1024 * 4, dtype=torch.float32, device="cuda")
    for _ in range(3):
        ctx.render(lp, 1024, 1024, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    ctx.reset_stats_total()
    t = time.perf_counter()
    for _ in range(20):
        ctx.render(lp, 1024, 1024, fb.data_ptr(), acc.data_ptr())
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 20 * 1e3
    st = ctx.stats()
    print(json.dumps({"records": int(info.numCells), "create_s": round(t_create, 2),
                      "peak_rss_gib": round(rss, 2), "hbm_gib": round(info.deviceBytes / 2**30, 2),
                      "locator_G": info.locatorFaceRes, "locator_entries": int(info.locatorEntries),
                      "frame_ms": round(ms, 4), "candidates_per_sample":
                      st.candidatesTested / max(st.samplesFound, 1)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
