#!/usr/bin/env python3
"""How many of a terrain frame's misses (samples outside every cell) the cell header's void
bound certifies (analysis only, CPU: the oracle's oracle_trace_misses hook and the host build's
headers; nothing here runs on the GPU or in the product).

For the traced rays' miss points, the cube-map cell and sub-cell (irt_common.h cubemap_cell_sub)
and three bounds of the radial range of the records that can reach the point:
  quad     the header's words 24..31 (irt_build.h cell_header): per 2 x 2 sub-cells
  sub      per sub-cell, from the header's masks (the first kMaskCand candidates of every bin by
           their sub-cell bits, the rest of a bin as reaching every sub-cell)
  none     no bound (every miss scans its candidates)
A miss is certain when its radius lies outside the bound: the kernel decides it without a
candidate test, and a solo lane walks on through it (Tracer::woodcock_wave's void walk).

    python profiles/void_bounds.py [--config c3t] [--step 4]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "icon-ray-tracing_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
CONFIGS = {"c3t": (2, 7, 90, 1024, 4000.0), "c2t": (2, 5, 47, 512, 4000.0)}
FRAMING = ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)
KSUB = 4


def cell_sub(p, G):
    """irt_common.h cubemap_cell_sub in float32 (division, not the kernel's reciprocal: the
    padded lists make either exact enough)."""
    p = p.astype(np.float32)
    a = np.abs(p)
    fx = (a[:, 0] >= a[:, 1]) & (a[:, 0] >= a[:, 2])
    fy = ~fx & (a[:, 1] >= a[:, 2])
    face = np.where(fx, np.where(p[:, 0] >= 0, 0, 1), np.where(fy, np.where(p[:, 1] >= 0, 2, 3),
                                                               np.where(p[:, 2] >= 0, 4, 5)))
    den = np.where(fx, a[:, 0], np.where(fy, a[:, 1], a[:, 2]))
    n0 = np.where(fx, p[:, 1], p[:, 0])
    n1 = np.where(fx | fy, p[:, 2], p[:, 1])
    GS = G * KSUB
    fg = np.float32(0.5) * np.float32(GS)
    i = np.clip(((n0 / den + np.float32(1)) * fg).astype(np.int64), 0, GS - 1)
    j = np.clip(((n1 / den + np.float32(1)) * fg).astype(np.int64), 0, GS - 1)
    sub = (j % KSUB) * KSUB + (i % KSUB)
    cell = face * G * G + (j // KSUB) * G + (i // KSUB)
    return cell, sub


def sub_bounds(H, F):
    """Per (cell, sub-cell): [lowest height[0], highest height[numLayers]] of the records the
    header admits there (every bin; candidates past kMaskCand admitted everywhere)."""
    nc = H.shape[0]
    lo = np.full((nc, 16), np.inf, np.float32)
    hi = np.full((nc, 16), -np.inf, np.float32)
    h0 = F[:, 12].view(np.float32)
    hN = F[:, 13].view(np.float32)
    base = H[:, 3].astype(np.int64)
    ends = H[:, 4:8].astype(np.int64)
    for k in range(4):
        beg = ends[:, k - 1] if k else np.zeros(nc, np.int64)
        n = ends[:, k] - beg
        for j in range(int(n.max()) if nc else 0):
            has = n > j
            e = base[has] + beg[has] + j
            a, b = h0[e], hN[e]
            rows = np.nonzero(has)[0]
            for s in range(16):
                if j < 8:
                    ok = ((H[rows, 8 + s] >> (8 * k + j)) & 1).astype(bool)
                else:
                    ok = np.ones(rows.size, bool)
                r = rows[ok]
                lo[r, s] = np.minimum(lo[r, s], a[ok])
                hi[r, s] = np.maximum(hi[r, s], b[ok])
    return lo, hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3t", choices=sorted(CONFIGS))
    ap.add_argument("--step", type=int, default=4, help="every step-th pixel in x and y")
    args = ap.parse_args()
    import irt
    import oracle as O
    rn, bis, L, W, terrain = CONFIGS[args.config]
    cells = irt.synth_grid(rn, bis, L, terrain=terrain)
    S = O.OracleScene(cells)
    lut, vr = S.default_lut()
    S.set_transfunc(lut, vr)
    params = S.params(S.camera(W, W, FRAMING), accum_id=0, raygen=0)
    ys, xs = np.mgrid[0:W:args.step, 0:W:args.step]
    xy = np.ascontiguousarray(np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32))
    lib = O.olib()
    lib.oracle_trace_misses.restype = C.c_long
    lib.oracle_trace_misses.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_int,
                                        C.c_void_p, C.c_int, C.c_void_p, C.c_long, C.c_int]
    cap = 20_000_000
    out = np.zeros(3 * cap, np.float32)
    n = lib.oracle_trace_misses(cells.ctypes.data, cells.size, C.byref(params), W, W,
                                xy.ctypes.data, xy.shape[0], out.ctypes.data, cap, 0)
    P = out[:3 * min(n, cap)].reshape(-1, 3)
    D = irt.DebugScene(cells)
    H = D.array("bin_hdr").view(np.uint32).reshape(-1, 32).astype(np.int64)
    F = D.array("fat").view(np.uint32).reshape(-1, 16)
    G = int(round((H.shape[0] / 6) ** 0.5))
    cell, sub = cell_sub(P, G)
    r = np.sqrt((P.astype(np.float32) ** 2).sum(1, dtype=np.float32))
    q = (sub // 8) * 2 + (sub % 4) // 2
    qhi = H[cell, 24 + 2 * q].astype(np.uint32).view(np.float32)
    qlo = H[cell, 25 + 2 * q].astype(np.uint32).view(np.float32)
    lo, hi = sub_bounds(H, F)
    slo, shi = lo[cell, sub], hi[cell, sub]
    quad = (r > qhi) | (r < qlo)
    subc = (r > shi) | (r < slo)
    res = {"config": args.config, "rays": int(xy.shape[0]), "misses": int(n),
           "certain_quad": float(quad.mean()), "certain_sub": float(subc.mean()),
           "sub_not_quad": float((subc & ~quad).mean()), "quad_not_sub": float((quad & ~subc).mean())}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
