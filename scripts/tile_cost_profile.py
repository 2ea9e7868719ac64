#!/usr/bin/env python3
"""Per-tile measured walk cost (calibrated plan) next to per-wave durations of
one diagnostic frame: how long a wave takes per walk step, and which tiles
set the frame length."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "14-01-acceleration-tree__scene1"
g = N.HipScene(load_npz(ROOT / "tests/golden/scenes" / f"{scene}.npz"))
g.render()
xywh, cost = g.plan_tiles()
st, xy = g.profile_waves()
st, xy = g.profile_waves()
assert (xy == xywh[:, :2]).all()
t0 = st[:, 0].min()
s = (st[:, 0] - t0) * 0.01
e = (st[:, 1] - t0) * 0.01
dur = e - s
top = np.argsort(-dur)[:15]
heavy = cost > np.percentile(cost, 99)
out = {"tiles": int(len(cost)), "span_us": float(e.max()), "cost_total": float(cost.sum()),
       "cost_max": float(cost.max()), "cost_p50": float(np.median(cost)), "cost_p99": float(np.percentile(cost, 99)),
       "us_per_step_heavy": float(np.median(dur[heavy] / np.maximum(cost[heavy], 1))),
       "top_by_duration": [[int(xywh[k, 0]), int(xywh[k, 1]), int(xywh[k, 2]), int(xywh[k, 3]), float(cost[k]),
                            round(float(s[k]), 1), round(float(dur[k]), 1)] for k in top],
       "by_size": {f"{w}x{h}": [int(((xywh[:, 2] == w) & (xywh[:, 3] == h)).sum()),
                                round(float(dur[(xywh[:, 2] == w) & (xywh[:, 3] == h)].max()), 1)]
                   for w, h in sorted({(int(a), int(b)) for a, b in xywh[:, 2:4]})}}
np.savez_compressed(ROOT / "gpurun_out" / f"tilecost_{scene}.npz", xywh=xywh, cost=cost, stamps=st)
print(json.dumps(out))
