#!/usr/bin/env python3
"""Per-wave timeline of one frame (diagnostic build path): how long each 8x8
tile's wave lived and when it started, per traversal variant."""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "14-01-acceleration-tree__scene1"
variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["3"]
out = {}
for v in variants:
    g = N.HipScene(load_npz(ROOT / "tests/golden/scenes" / f"{scene}.npz"), traversal=int(v))
    g.render()
    st, xy = g.profile_waves()
    st, xy = g.profile_waves()
    t0 = st[:, 0].min()
    s = (st[:, 0] - t0).astype(np.float64) * 10e-3   # us
    e = (st[:, 1] - t0).astype(np.float64) * 10e-3
    dur = e - s
    top = np.argsort(-dur)[:10]
    out[v] = {"span_us": float(e.max()), "mean_dur_us": float(dur.mean()), "p50": float(np.median(dur)),
              "p99": float(np.percentile(dur, 99)), "max_dur_us": float(dur.max()),
              "last_end_start_us": float(s[np.argmax(e)]), "sum_dur_us": float(dur.sum()),
              "top": [[int(xy[k, 0]), int(xy[k, 1]), round(float(s[k]), 1), round(float(dur[k]), 1)] for k in top]}
    np.savez_compressed(ROOT / "gpurun_out" / f"waves_{scene}_{v}.npz", stamps=st, xy=xy)
print(json.dumps(out))
