#!/usr/bin/env python3
"""Per-wave timeline of one C2 frame (crt_hip_profile_waves: s_memrealtime
stamps at wave start / end, 100 MHz) split by tile size of the measured-cost
plan (8x8 packet-walk tiles vs the window-walk tiles of <= 16 rays): how long
the waves of each class live, when the last ones end, and how many waves are
resident over time.

  python3 scripts/wave_timeline.py [scene] [--window 0|1] [--out file.json]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, os.environ.get("CRT_PKG") or str(ROOT / "chaos-ray-tracing-course-2025_amd"))   # CRT_PKG: another build
from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("scene", nargs="?", default="14-01-acceleration-tree__scene1")
    p.add_argument("--window", type=int, default=1)
    p.add_argument("--opt", action="append", default=[], help="NAME=V scene options (e.g. traversal=14)")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    g = N.HipScene(load_npz(ROOT / "tests/golden/scenes" / f"{a.scene}.npz"), window=a.window,
                   **{k: int(v) for k, v in (o.split("=") for o in a.opt)})
    st = N.RendererSettings.default()
    g.render(st)
    xywh, cost = g.plan_tiles(st)
    for _ in range(3):
        stamps, xy = g.profile_waves(st)
    t0 = stamps[:, 0].min()
    s = (stamps[:, 0] - t0).astype(np.float64) * 1e-2     # us
    e = (stamps[:, 1] - t0).astype(np.float64) * 1e-2
    dur = e - s
    npx = xywh[:, 2] * xywh[:, 3]
    out = {"scene": a.scene, "window": a.window, "span_us": float(e.max()), "waves": int(len(s))}
    for name, sel in [("small_le16", npx <= 16), ("tile_gt16", npx > 16)]:
        if not sel.any():
            continue
        d, ee = dur[sel], e[sel]
        out[name] = {"waves": int(sel.sum()), "sum_dur_us": float(d.sum()), "mean_dur_us": float(d.mean()),
                     "p50_dur": float(np.median(d)), "p90_dur": float(np.percentile(d, 90)),
                     "max_dur_us": float(d.max()), "last_end_us": float(ee.max()),
                     "p90_end_us": float(np.percentile(ee, 90)),
                     "cost_sum": float(cost[sel].sum()), "cost_max": float(cost[sel].max())}
    # resident waves over time (10 us bins)
    bins = np.arange(0.0, e.max() + 10.0, 10.0)
    res = [int(((s <= b) & (e > b)).sum()) for b in bins]
    out["resident_every_10us"] = res
    # longest waves with their tile
    top = np.argsort(-dur)[:12]
    out["longest"] = [[int(xywh[k, 0]), int(xywh[k, 1]), int(xywh[k, 2]), int(xywh[k, 3]), round(float(s[k]), 1),
                       round(float(dur[k]), 1), float(cost[k])] for k in top]
    js = json.dumps(out)
    if a.out:
        Path(a.out).write_text(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
