#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV, restricted to
the launches of the timed region: the last K dispatches of each kernel whose
name matches (bench.py renders `warmup + steps` frames after the scene's
one-time plan calibration, whose trial frames would otherwise dominate
rocprof's own --stats averages).

  python3 scripts/kernel_trace_summary.py TRACE.csv --match k_render_tiles --last 20 [--out f.json]
"""
import argparse
import csv
import json
import statistics
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--match", default="k_render_tiles")
    p.add_argument("--last", type=int, default=20)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    runs = defaultdict(list)
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            if a.match in r["Kernel_Name"]:
                runs[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                               int(r["VGPR_Count"]), int(r["SGPR_Count"]), int(r["Scratch_Size"])))
    out = {"trace": a.trace, "last": a.last, "kernels": {}}
    for name, v in runs.items():
        v.sort()
        sel = v[-a.last:]
        d = [(e - s) / 1e3 for s, e, *_ in sel]
        out["kernels"][name] = {"dispatches_total": len(v), "dispatches_used": len(sel),
                                "avg_us": round(statistics.mean(d), 3), "median_us": round(statistics.median(d), 3),
                                "min_us": round(min(d), 3), "max_us": round(max(d), 3),
                                "vgpr": sel[-1][2], "sgpr": sel[-1][3], "scratch_bytes": sel[-1][4]}
    js = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
