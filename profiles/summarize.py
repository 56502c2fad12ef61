#!/usr/bin/env python3
"""Summarise one profiles/run_profiles.sh output directory into JSON: the k_render
kernel's rocprofv3 duration statistics and its per-dispatch PMC counters, next to the
bench's algorithmic byte model.

HBM traffic on gfx950 (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in
KiB; FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane) coalesced stream, other
access widths are uncalibrated.  Both the raw and the x2-corrected read figures are
reported; `traffic_bytes` uses raw FETCH_SIZE + WRITE_SIZE (a lower bound) unless the
caller decides otherwise.
"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_render"


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def col(r, *names):
    low = {k.lower(): v for k, v in r.items()}
    for n in names:
        if n.lower() in low:
            return low[n.lower()]
    raise KeyError(names)


def counters(d, name):
    vals = {}
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        if KERNEL not in col(r, "Kernel_Name") or col(r, "Counter_Name") != name:
            continue
        # the context's one-workgroup prewarm dispatch is not a render
        if int(float(col(r, "Grid_Size"))) <= int(float(col(r, "Workgroup_Size"))):
            continue
        key = col(r, "Dispatch_Id")
        vals[key] = vals.get(key, 0.0) + float(col(r, "Counter_Value"))
    return list(vals.values())


def main(d):
    out = {"dir": os.path.basename(d.rstrip("/"))}
    for r in rows(os.path.join(d, "stats", "**", "*kernel_stats.csv")):
        name = col(r, "Name")
        short = name.split("(")[0].replace("irt::", "")
        k = {"calls": int(col(r, "Calls")), "avg_ns": float(col(r, "AverageNs")),
             "total_ns": float(col(r, "TotalDurationNs")),
             "min_ns": float(col(r, "MinNs")), "max_ns": float(col(r, "MaxNs"))}
        out.setdefault("kernels", {})[short] = k
    # The context's prewarm dispatch (one workgroup returning at once, irt_render.hip
    # prewarm_render) runs the default kernel too: from the per-dispatch trace, the render
    # kernels' statistics without single-workgroup dispatches
    per = {}
    for r in rows(os.path.join(d, "stats", "**", "*kernel_trace.csv")):
        name = col(r, "Kernel_Name")
        if "k_render" not in name:
            continue
        grid = int(col(r, "Grid_Size_X")) * int(col(r, "Grid_Size_Y")) * int(col(r, "Grid_Size_Z"))
        wg = int(col(r, "Workgroup_Size_X")) * int(col(r, "Workgroup_Size_Y")) * int(col(r, "Workgroup_Size_Z"))
        if grid <= wg:
            continue
        short = name.split("(")[0].replace("irt::", "")
        per.setdefault(short, []).append(int(col(r, "End_Timestamp")) - int(col(r, "Start_Timestamp")))
    for short, v in per.items():
        k = out.setdefault("kernels", {}).setdefault(short, {})
        k.update({"calls": len(v), "avg_ns": sum(v) / len(v), "total_ns": float(sum(v)),
                  "min_ns": float(min(v)), "max_ns": float(max(v)), "single_workgroup_dispatches_excluded": True})
    try:
        bench = json.loads(open(os.path.join(d, "bench_stats.json")).read().strip().splitlines()[-1])
        cfg = bench["config"]
        out["bench"] = {"value": bench["value"], "ms_per_step": bench["ms_per_step"],
                        "kernel_ms_hip_events": cfg.get("kernel_ms_rank0"),
                        "samples_per_frame": cfg.get("samples_per_frame"),
                        "rays_in_box_per_frame": cfg.get("rays_in_box_per_frame"),
                        "frames_per_launch": cfg.get("frames_per_launch", 1),
                        "algorithmic_bytes_per_launch": (92 * cfg.get("samples_per_frame", 0)
                        + 44 * cfg.get("rays_in_box_per_frame", 0)) * cfg.get("frames_per_launch", 1)}
        out["records"], out["width"] = cfg.get("records"), cfg.get("width")
        out["config_name"] = cfg.get("name")
        out["frames_per_launch"] = cfg.get("frames_per_launch", 1)
    except Exception as e:  # noqa: BLE001
        out["bench_error"] = str(e)
    f = counters(os.path.join(d, "pmc_fetch"), "FETCH_SIZE")
    w = counters(os.path.join(d, "pmc_write"), "WRITE_SIZE")
    h = counters(os.path.join(d, "pmc_l2"), "TCC_HIT_sum")
    m = counters(os.path.join(d, "pmc_l2"), "TCC_MISS_sum")
    avg = lambda v: sum(v) / len(v) if v else None  # noqa: E731
    if f:
        out["fetch_kib_per_launch"] = avg(f)
    if w:
        out["write_kib_per_launch"] = avg(w)
    if f and w:
        out["traffic_bytes_per_launch_raw"] = (avg(f) + avg(w)) * 1024
        out["traffic_bytes_per_launch_fetch_x2"] = (2 * avg(f) + avg(w)) * 1024
    if h and m:
        out["l2_hit_rate"] = avg(h) / (avg(h) + avg(m))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
