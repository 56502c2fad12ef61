#!/usr/bin/env python3
"""Where a frame's samples are: per 8x8 packet (the unit one wave renders) the oracle's
sampleVolume calls, hits and draws, and for the costliest packets the same per ray -- to tell
a packet whose rays are all busy from one that waits for a single long ray.  CPU only
(the oracle's direction-voxel locator; test infrastructure, measurement only).

    python profiles/ray_cost.py [--config c3t] [--top 12] [--threads 8]
"""
import argparse
import ctypes as C
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "icon-ray-tracing_amd", "python"), ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import bench  # noqa: E402
import irt  # noqa: E402
import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3t")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    rn, bis, L, W, H, tf, orbit_cfg, desc = bench.CONFIGS[args.config]
    cells = irt.synth_grid(rn, bis, L, terrain=bench.TERRAIN.get(args.config, 0.0))
    setup = irt.setup_frame(cells, W, H, camera=bench.FRAMING)
    S = O.OracleScene(cells)
    S.set_transfunc(bench.make_lut(tf, setup.lut), setup.value_range)
    lp = setup.lp
    cam = tuple(np.array(v.tolist(), np.float32) for v in (lp.org, lp.dir_00, lp.dir_du, lp.dir_dv))
    p = S.params(cam, accum_id=0, raygen=0, unit_distance=lp.unitDistance)
    T = O.TimedScene(S, 2, args.threads)
    lib = O.olib()
    T.render(p, W, H, rect=(0, 0, 8, 8), threads=1)  # builds the locator once
    bufs = [(np.zeros(W * H * 4, np.float32), np.zeros(W * H, np.uint32)) for _ in range(args.threads)]

    def rect_stats(k, rect):
        acc, fb = bufs[k % args.threads]
        st = O.OStats()
        rc = lib.oracle_scene_render(T._h, C.byref(p), W, H, *rect, O._p(acc), O._p(fb), 1, C.byref(st))
        assert rc == 0
        return st.locate_calls, st.samples_found, st.rng_draws

    def packets(k0):
        out = []
        for k in range(k0, k0 + 64):
            py, px = divmod(k, W // 8)
            out.append(rect_stats(k0 // 64, (8 * px, 8 * py, 8 * px + 8, 8 * py + 8)))
        return out

    n = (W // 8) * (H // 8)
    with ThreadPoolExecutor(args.threads) as ex:
        res = [s for part in ex.map(packets, range(0, n, 64)) for s in part]
    pk = np.array(res, dtype=np.int64).reshape(H // 8, W // 8, 3)
    loc = pk[..., 0].ravel()
    order = np.argsort(-loc)
    summary = {"config": args.config, "packets": int(n), "locate_total": int(loc.sum()),
               "found_total": int(pk[..., 1].sum()),
               "locate_per_packet_median": float(np.median(loc)), "p99": float(np.percentile(loc, 99)),
               "max": int(loc.max()), "top_share": float(loc[order[:args.top]].sum() / max(loc.sum(), 1))}
    print(json.dumps(summary), flush=True)
    for k in order[:args.top]:
        py, px = divmod(int(k), W // 8)
        rays = [rect_stats(0, (8 * px + i, 8 * py + j, 8 * px + i + 1, 8 * py + j + 1)) for j in range(8) for i in range(8)]
        r = np.array(rays, dtype=np.int64)
        print(json.dumps({"packet": [int(8 * px), int(8 * py)], "locate": int(r[:, 0].sum()),
                          "found": int(r[:, 1].sum()), "ray_locate_max": int(r[:, 0].max()),
                          "ray_locate_median": float(np.median(r[:, 0])),
                          "ray_miss_max": int((r[:, 0] - r[:, 1]).max()),
                          "rays_over_64": int((r[:, 0] > 64).sum())}), flush=True)
    T.close()


if __name__ == "__main__":
    main()
