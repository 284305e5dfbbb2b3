#!/usr/bin/env python3
"""Per-kernel mean of each PMC counter in a rocprofv3 --pmc output directory
(the profiles/rNN_pmc_*.txt summaries). usage: pmc_summary.py <dir>"""
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    k = k.replace("void ", "").replace("cgx::(anonymous namespace)::", "").replace("cgx::", "").split("(")[0]
    print(f"{k[:44]:44s} {c:34s} n={len(v):3d} mean={sum(v)/len(v):g}")
