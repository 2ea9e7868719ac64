#!/usr/bin/env python3
"""Average PMC counters per dispatch of each kernel under a rocprofv3 output dir."""
import collections
import csv
import json
import sys
from pathlib import Path

root = Path(sys.argv[1])
out = {}
for f in sorted(root.rglob("*counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        if "k_render" not in k and "k_wf_level" not in k:  # k_render_tiles, k_render_refill, wavefront levels
            continue
        n = len(disp[k])
        out.setdefault(k, {}).update({c: x / n for c, x in v.items()})
print(json.dumps(out, indent=1))
