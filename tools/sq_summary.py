#!/usr/bin/env python3
"""Per-kernel averages of a rocprofv3 --pmc counter collection (tools/sq_counters.sh output).
usage: tools/sq_summary.py DIR [kernel-substring ...]"""
import collections
import csv
import glob
import sys

files = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(files[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
want = sys.argv[2:]
for k in sorted(agg):
    if want and not any(w in k for w in want):
        continue
    n = len(disp[k])
    print("%-60s n=%d %s" % (k[-60:], n, {c: round(v / n) for c, v in sorted(agg[k].items())}))
