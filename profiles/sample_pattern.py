#!/usr/bin/env python3
"""Sample-outcome patterns of a frame's rays and the Woodcock rounds they cost (analysis only,
CPU: the oracle's oracle_trace_pixels hook; nothing here runs on the GPU or in the product).

For a sample of 8x8 packets, each ray's counted sampleVolume calls are traced as letters ('m'
outside every cell, 'l' located and rejected, 'A' accepted, 'E' past tmax, '|' a woodcockFunc
call).  The script reports how the outcomes alternate and replays the wave-cooperative loop of
irt_render.hip (Tracer::woodcock_wave: lane caps 1, 2, 4, ... per call, groups of 64/R lanes,
located or miss mode) on the traces to count a wave's rounds, under the kernel's rule and under
alternative round rules.

    python profiles/sample_pattern.py [--config c3t] [--step 4] [--json out.json]
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

CONFIGS = {"c3": (2, 7, 90, 1024, 0.0), "c3t": (2, 7, 90, 1024, 4000.0),
           "c2t": (2, 5, 47, 512, 4000.0), "c2": (2, 5, 47, 512, 0.0)}
FRAMING = ((0.0, 0.0, 1.4e7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 60.0)


def traces(cfg, step, stride=8192, rows=None):
    import irt
    import oracle as O
    rn, bis, L, W, terrain = CONFIGS[cfg]
    cells = irt.synth_grid(rn, bis, L, terrain=terrain)
    S = O.OracleScene(cells)
    lut, vr = S.default_lut()
    S.set_transfunc(lut, vr)
    cam = S.camera(W, W, FRAMING)
    params = S.params(cam, accum_id=0, raygen=0)
    pk = []
    for py in (range(0, W // 8, step) if rows is None else rows):
        for px in range(0, W // 8, step):
            pk.append((px, py))
    xy = np.array([(8 * px + (l & 7), 8 * py + (l >> 3)) for px, py in pk for l in range(64)],
                  dtype=np.int32)
    out = np.zeros(xy.shape[0] * stride, dtype=np.uint8)
    lib = O.olib()
    lib.oracle_trace_pixels.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_int,
                                        C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
    rc = lib.oracle_trace_pixels(cells.ctypes.data, cells.size, C.byref(params), W, W,
                                 xy.ctypes.data, xy.shape[0], out.ctypes.data, stride, 0)
    assert rc == 0
    out = out.reshape(-1, stride)
    strs = [bytes(r[:np.argmin(r)] if r[-1] == 0 or 0 in r else r).decode() for r in out]
    return [strs[64 * i:64 * i + 64] for i in range(len(pk))]


def calls_of(s):
    """A ray's counted woodcockFunc calls, each a string of outcomes ('' for a call whose
    first sample is past tmax is 'E')."""
    return [c for c in s.split("|")[1:]]


def outcome_stats(packets):
    n = {"m": 0, "l": 0, "A": 0, "E": 0}
    switches = 0
    runs = {"m": [], "l": []}
    for P in packets:
        for s in P:
            for c in calls_of(s):
                prev, run = None, 0
                for ch in c:
                    n[ch] = n.get(ch, 0) + 1
                    kind = "m" if ch == "m" else ("l" if ch in "lA" else None)
                    if kind is None:
                        continue
                    if kind == prev:
                        run += 1
                    else:
                        if prev is not None:
                            switches += 1
                            runs[prev].append(run)
                        prev, run = kind, 1
                if prev is not None:
                    runs[prev].append(run)
    hist = {k: np.bincount(np.minimum(np.array(v, dtype=np.int64), 16), minlength=17).tolist()
            for k, v in runs.items() if v}
    return {"samples": n, "mode_switches": switches, "run_hist_capped16": hist}


def simulate(packets, rule="kernel", voidwalk=True, maxlg0=0, ramp=1, groupwalk=False, cap=32):
    """Rounds per wave of Tracer::woodcock_wave over the traced outcomes.  A wave runs its
    rays' counted calls in wave calls: every ray with a call pending joins; the wave call runs
    rounds until each joined ray's call is decided.  rule "kernel": a group's lanes assume all
    samples located (miss mode: all missing); the ray advances through its first event.
    voidwalk: a solo lane in miss mode crosses its run of misses in the same round (the kernel
    does so only for misses its quad-bound test certifies; this bounds it from below).
    rule "both": a group's lanes also speculate the other assumption (two half groups)."""
    per_wave, walks = [], []
    for P in packets:
        calls = [calls_of(s) for s in P]
        idx = [0] * 64
        rounds = 0
        walk_steps = 0
        while True:
            joined = [i for i in range(64) if idx[i] < len(calls[i])]
            if not joined:
                break
            pos = {i: 0 for i in joined}
            miss = {i: False for i in joined}
            live = set(joined)
            lg_cap = maxlg0
            while live:
                rounds += 1
                walk_round = 0
                R = len(live)
                lgR = 0 if R > 32 else 1 if R > 16 else 2 if R > 8 else 3 if R > 4 else 4 if R > 2 else 5 if R > 1 else 6
                lg = min(lg_cap, lgR)
                G = 1 << lg
                for i in list(live):
                    c = calls[i][idx[i]]
                    p = pos[i]
                    if rule == "both" and G >= 2:
                        # half the lanes under each assumption from the same (exact) position:
                        # the half whose assumption holds at sample p advances through its
                        # first event, the other breaks at once; the ray takes the longer
                        res = [(advance(c, p, G // 2, mm), mm) for mm in (miss[i], not miss[i])]
                        (adv, done, sw), mm = max(res, key=lambda r: (r[0][1], r[0][0]))
                        pos[i] = p + adv
                        if done:
                            live.discard(i)
                        else:
                            miss[i] = (not mm) if sw else mm
                        continue
                    if voidwalk and G == 1 and miss[i]:
                        p0 = p
                        while p < len(c) and c[p] == "m" and p - p0 < cap:
                            p += 1
                        walk_round = max(walk_round, p - p0)
                    adv, done, sw = advance(c, p, G, miss[i])
                    if groupwalk and G > 1 and miss[i] and adv == G and not done and not sw:
                        # the group's last lane walks on through the void (all G samples missed)
                        q0 = p + adv
                        q = q0
                        while q < len(c) and c[q] == "m" and q - q0 < cap:
                            q += 1
                        walk_round = max(walk_round, q - q0)
                        adv += q - q0
                    pos[i] = p + adv
                    if done:
                        live.discard(i)
                    elif sw:
                        miss[i] = not miss[i]
                walk_steps += walk_round
                lg_cap = min(lg_cap + ramp, 6)
            for i in joined:
                idx[i] += 1
        per_wave.append(rounds)
        walks.append(walk_steps)
    simulate.walk_steps = np.array(walks)
    return np.array(per_wave)


def advance(c, p, G, mm):
    """Samples taken from position p with G lanes under assumption mm (True: all miss);
    returns (samples consumed, call decided, assumption broke)."""
    for k in range(G):
        if p + k >= len(c):
            return k, True, False  # (a truncated trace: treat as decided)
        ch = c[p + k]
        if ch in "EA":
            return k + 1, True, False
        if (ch == "m") != mm:
            return k + 1, False, True
    return G, False, False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3t", choices=sorted(CONFIGS))
    ap.add_argument("--step", type=int, default=4, help="every step-th packet in x and y")
    ap.add_argument("--json")
    ap.add_argument("--stride", type=int, default=8192, help="trace letters per ray (cut)")
    ap.add_argument("--chunks", type=int, default=0,
                    help="all packets of every step-th packet row, this many rows per trace call")
    args = ap.parse_args()
    if args.chunks:
        # every packet row step-th, in chunks of packet rows (bounded memory), then pooled
        W = CONFIGS[args.config][3]
        packets = []
        rows = list(range(0, W // 8, args.step))
        for i in range(0, len(rows), args.chunks):
            packets += traces(args.config, 1, stride=args.stride, rows=rows[i:i + args.chunks])
    else:
        packets = traces(args.config, args.step, stride=args.stride)
    res = {"config": args.config, "packets": len(packets)}
    res.update(outcome_stats(packets))
    for name, kw in (("kernel", {}), ("kernel_novoid", {"voidwalk": False}), ("both", {"rule": "both"}),
                     ("groupwalk", {"groupwalk": True})):
        r = simulate(packets, **kw)
        res["rounds_" + name] = {"mean": float(r.mean()), "p50": float(np.median(r)),
                                 "p90": float(np.percentile(r, 90)), "max": int(r.max()),
                                 "sum": int(r.sum())}
        w = simulate.walk_steps  # the longest solo walk of each round, summed per wave
        res["walk_steps_" + name] = {"mean": float(w.mean()), "p90": float(np.percentile(w, 90)),
                                     "max": int(w.max())}
    print(json.dumps(res, indent=1))
    if args.json:
        json.dump(res, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
