#!/usr/bin/env python3
"""Diagnostic: per-wave timeline of the C2 camera-bins render, by the length of
the wave's cell list.  With the normal build the stamps are (wave start, wave
end); with a CRT_BINS_PHASE build (scripts/make_variant.sh phase
RENDER_FLAGS=-DCRT_BINS_PHASE) the start stamp is overwritten by the end of the
list walk, so end - stamp is the proof / fallback + shading + store part.
CRT_PKG selects the build."""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, os.environ.get("CRT_PKG") or str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

sc = load_npz(ROOT / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz")
g = N.HipScene(sc)
ln, _ = g.camera_bins()
tx = (1920 + 7) // 8
for _ in range(5):
    g.render()
res = []
for _ in range(3):
    st, xy = g.profile_waves()
    live = (st[:, 1] > 0) & (xy[:, 0] >= 0)
    s = st[live, 0].astype(np.int64)
    e = st[live, 1].astype(np.int64)
    cell = (xy[live, 1] // 8) * tx + xy[live, 0] // 8
    n = ln.reshape(-1)[cell]
    t0 = s.min()
    dur = (e - s) * 10e-3
    rec = {"waves": int(live.sum()), "idle_waves": int((~live).sum()), "span_us": float((e.max() - t0) * 10e-3)}
    for name, lo, hi in [("bvh", -1, -1), ("empty", 0, 0), ("1-15", 1, 15), ("16-47", 16, 47), ("48+", 48, 10**9)]:
        k = (n >= lo) & (n <= hi)
        if k.any():
            rec[name] = {"waves": int(k.sum()), "dur_mean": round(float(dur[k].mean()), 2),
                         "dur_p90": round(float(np.percentile(dur[k], 90)), 2),
                         "start_mean": round(float((s[k] - t0).mean() * 10e-3), 2),
                         "end_max": round(float((e[k] - t0).max() * 10e-3), 2)}
    res.append(rec)
print(json.dumps({"pkg": str(N.LIB_PATH), "build": N.build_id(), "runs": res}, indent=1))
