#!/usr/bin/env python3
"""Per-launch HBM traffic of the engine kernels from two rocprofv3 --pmc passes
(tools/gpu_steps.sh pmc): FETCH_SIZE and WRITE_SIZE (KB per dispatch), averaged over
dispatches.  gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half of
the bytes of wide coalesced streaming reads, so fetched bytes = 2 x FETCH_SIZE; WRITE_SIZE is
taken as is.  Writes profiles/<tag>_pmc_traffic_<config>.json, which bench.py reports as
roofline.traffic for the dominant kernel.

usage: tools/pmc_traffic.py TAG CONFIG FETCH_DIR WRITE_DIR"""
import collections
import csv
import glob
import json
import os
import sys

tag, config, fdir, wdir = sys.argv[1:5]
# per kernel and counter: (grid size, value) of every dispatch; a kernel's figure is the mean over
# its dispatches at its largest grid (full launches: a batched waterfall's owrx_sync flush is a
# smaller launch of the same kernel and would pull an all-dispatch mean down)
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in (fdir, wdir):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "owrx::" not in name:
                continue
            short = name.split("(")[0].replace("void ", "").replace("owrx::", "")
            vals[short][r["Counter_Name"]].append((int(r.get("Grid_Size") or 0), float(r["Counter_Value"])))


def full(pairs):
    if not pairs:
        return []
    g = max(p[0] for p in pairs)
    return [v for gs, v in pairs if gs == g]
out = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over "
                 "'python bench.py --config %s --steps 20 --warmup 5 --no-cpu-baseline --no-timing "
                 "--extra-block 0' (tools/gpu_steps.sh pmc); per kernel the dispatches at its largest "
                 "grid" % config,
       "config": config,
       "correction": "fetch_bytes = 2 x FETCH_SIZE (gfx950), write_bytes = WRITE_SIZE",
       "kernels": {}}
for k, cs in sorted(vals.items()):
    fv, wv = full(cs["FETCH_SIZE"]), full(cs["WRITE_SIZE"])
    f = sum(fv) / max(1, len(fv))
    w = sum(wv) / max(1, len(wv))
    out["kernels"][k] = {"fetch_size_kb": round(f, 1), "write_size_kb": round(w, 1),
                         "hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
                         "dispatches": [len(fv), len(wv)],
                         "grid": max(p[0] for p in cs["FETCH_SIZE"]) if cs["FETCH_SIZE"] else None}
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                    "%s_pmc_traffic_%s.json" % (tag, config))
json.dump(out, open(path, "w"), indent=1)
print(path)
for k, v in out["kernels"].items():
    print("%-28s %s" % (k, v))
