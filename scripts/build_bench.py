#!/usr/bin/env python3
"""Tree build time, C5 (1 M random triangles): host build (crt_scene_build.cpp,
the reference's algorithm on one core) vs the device build (crt_tree_build.hip),
and that both give the same tree."""
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.synthetic import c5_scene  # noqa: E402


def sha(arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


sc = c5_scene()
out = {}
for mode in ("device", "host", "device"):
    t0 = time.perf_counter()
    g = N.HipScene(sc, tree_build=mode)
    dt = time.perf_counter() - t0
    info = g.info()
    out.setdefault(mode, []).append({"create_s": round(dt, 3), "tree_build_ms": round(info["tree_build_ms"], 2),
                                     "nodes": info["node_count"], "refs": info["leaf_ref_count"],
                                     "tree_sha": sha(g.tree())[:16]})
    del g
print(json.dumps(out))
