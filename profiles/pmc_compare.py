#!/usr/bin/env python3
"""Per-wave side-by-side of a pmc_probe.sh table: python profiles/pmc_compare.py TABLE"""
import re
import sys

t = open(sys.argv[1]).read()
rows = []
for b in re.split(r"case \d+: ", t)[1:]:
    lines = b.strip().split("\n")
    d = {}
    for l in lines[2:]:
        k, v = l.split()
        d[k] = float(v)
    rows.append((lines[0], d))
keys = sorted(rows[0][1])
print("%-24s" % "per wave", " ".join("%14s" % n[:14] for n, _ in rows))
for k in keys:
    print("%-24s" % k, " ".join("%14.1f" % (d.get(k, 0) / d["SQ_WAVES"]) for _, d in rows))
