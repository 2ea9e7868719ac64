#!/usr/bin/env python3
"""Diagnostic: the 333x200 compact-shard case of
tests/test_gpu_configs.py::test_compact_shards_lossless with camera-bins
options given on the command line (opt=v,...), in this process; prints OK or
the error."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, os.environ.get("CRT_PKG") or str(ROOT / "chaos-ray-tracing-course-2025_amd"))
sys.path.insert(0, str(ROOT / "tests"))
from crt_amd import native as N  # noqa: E402
from conftest import DeviceBuffers, scene_npz  # noqa: E402

opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in (sys.argv[1].split(",") if len(sys.argv) > 1 else []))
sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(333, 200)
sc.set_settings(bucket_size=20)
g = N.HipScene(sc, **opts)
st = N.RendererSettings.default()
full = g.render(st)
db = DeviceBuffers()
shards = 3
stride = g.compact_stride(shards)
gathered = db.alloc(4 * stride * shards)
for s in range(shards):
    g.render_shard_compact(st, s, shards, gathered + 4 * s * stride)
    db.sync()
    print("shard", s, "ok", flush=True)
print("OK", opts, flush=True)
