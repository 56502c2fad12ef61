#!/usr/bin/env python3
"""Summarise profiles/ab_multi.sh output: per file, ms/frame of every round, the median,
candidates per sample and the HBM-roofline fraction (bench.py's HIP-event figure).
    python profiles/ab_summary.py DIR..."""
import glob
import json
import os
import statistics
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(os.path.join(d, "*.jsonl"))):
        rows = [json.loads(l) for l in open(f) if l.strip().startswith("{")]
        if not rows:
            print(f"{f}: no rows")
            continue
        ms = [r["config"]["ms_per_frame"] for r in rows]
        print(f"{os.path.relpath(f, d):55s} ms/frame {[round(m, 4) for m in ms]} median {statistics.median(ms):.4f} "
              f"cand/sample {rows[0]['config']['candidates_per_sample']:.3f} "
              f"frac {statistics.median([r['roofline']['frac'] for r in rows]):.4f}")
