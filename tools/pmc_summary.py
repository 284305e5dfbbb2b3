#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs under a directory: mean counter value per
(kernel, counter) over dispatches. usage: pmc_summary.py DIR [kernel-substring]"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        if sub and sub not in kn:
            continue
        m = re.search(r"(k_[a-z_]+<[^>]*>|k_[a-z_]+)", kn)
        short = m.group(1) if m else kn[:40]
        agg[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:40s} {c:34s} n={len(v):3d} mean={sum(v)/len(v):.6g}")
