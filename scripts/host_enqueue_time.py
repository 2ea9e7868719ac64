#!/usr/bin/env python3
"""Diagnostic: host time of one crt_hip_render_device call (the enqueue) for
C2 frames issued back to back, against the GPU's frame period — whether the
pipelined camera-bins frames are host-bound."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
sys.path.insert(0, str(ROOT / "tests"))
from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402
from conftest import DeviceBuffers  # noqa: E402

sc = load_npz(ROOT / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz")
g = N.HipScene(sc)
st = N.RendererSettings.default()
db = DeviceBuffers()
d = db.alloc(1920 * 1080 * 12)
for _ in range(20):
    g.render_device(st, d)
db.sync()
for trial in range(3):
    n = 200
    ts = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        g.render_device(st, d)
        ts.append(time.perf_counter() - a)
    t_enq = time.perf_counter() - t0
    db.sync()
    t_all = time.perf_counter() - t0
    print(f"enqueue per call {np.median(ts)*1e6:.1f} us (mean {t_enq/n*1e6:.1f}), wall per frame {t_all/n*1e6:.1f} us")
