#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel over dispatches (diagnostic helper)."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(list)
for path in sys.argv[1:]:
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
by_k = collections.defaultdict(dict)
for (k, c), v in agg.items():
    by_k[k][c] = sum(v) / len(v)
for k, cs in by_k.items():
    if "owrx" not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-24s %16.1f" % (c, v))
