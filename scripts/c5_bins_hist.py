#!/usr/bin/env python3
"""Diagnostic: C5's camera-bins list lengths per 8x8 cell at 4K (mean cap
raised by CRT_BINS_MEAN_CAP, read by CRT_AB_OPTIONS builds only: run with
CRT_PKG=abtest/<variant built with HOST_AB_FLAGS=-DCRT_AB_OPTIONS>): how many cells are over the cell cap (they walk
the BVH) and the length distribution of the rest."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, os.environ.get("CRT_PKG") or str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.synthetic import c5_scene  # noqa: E402

os.environ.setdefault("CRT_BINS_MEAN_CAP", "1024")
g = N.HipScene(c5_scene(1_000_000, 3840, 2160))
i = g.info()
print("bins built:", i.get("bins_binnings"), "records", i.get("bins_records"))
ln, _ = g.camera_bins()
ln = np.asarray(ln)
print("cells", ln.size, "over cap", int((ln < 0).sum()), "empty", int((ln == 0).sum()))
ok = ln[ln >= 0]
for q in [50, 75, 90, 99, 100]:
    print(f"p{q}", np.percentile(ok, q))
print("mean", ok.mean())
