#!/usr/bin/env python3
"""Per-variant table of the counters collected by profiles/pmc_multi.sh (k_render dispatches,
averaged per dispatch)."""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
prefix = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, prefix + "*", "run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        m = re.search(r"irt::k_(render|setup|march)", r["Kernel_Name"])
        if not m:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for d, c in per.items():
        for k, v in c.items():
            acc[names[d]][k].append(v)
for name, c in sorted(acc.items()):
    print(name)
    for k, v in sorted(c.items()):
        print(f"   {k:32s} {sum(v) / len(v):16.1f}")
