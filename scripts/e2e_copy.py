#!/usr/bin/env python3
"""A/B tool: crt_hip_render end to end (render + image into host memory, the
reference's render_image call, main.cpp:37-43) with the compact image copy
(option compact_copy 1, crt_api.hip image_to_host) against the whole-image
copy, into pinned and pageable memory; median of N blocking calls.

  python scripts/e2e_copy.py [--config c2|c3] [--frames 50]
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "chaos-ray-tracing-course-2025_amd"), str(ROOT)]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime shared with the library)

import bench  # noqa: E402
from crt_amd import native as N  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c2")
    p.add_argument("--frames", type=int, default=50)
    p.add_argument("--modes", default="1,0", help="compact_copy values to time")
    p.add_argument("--targets", default="pinned,pageable")
    a = p.parse_args()
    cfg = bench.CONFIGS[a.config]
    W, H = cfg["size"]
    sc = bench.make_scene(cfg, W, H)
    st = N.RendererSettings.default(**cfg["settings"])
    gpu = N.HipScene(sc, calibrate=1)
    pinned = torch.empty(W * H * 3, dtype=torch.float32, pin_memory=True)
    page = np.empty(W * H * 3, np.float32)
    want = gpu.render(st).view(np.uint32).ravel()
    out = {"config": a.config, "size": [W, H]}
    for mode in [int(m) for m in a.modes.split(",")]:
        gpu.set_option("compact_copy", mode)
        for name, ptr in (("pinned", pinned.data_ptr()), ("pageable", page.ctypes.data)):
            if name not in a.targets.split(","):
                continue
            for _ in range(5):
                gpu.render_host(st, ptr)
            ts = []
            for _ in range(a.frames):
                s = time.perf_counter()
                gpu.render_host(st, ptr)
                ts.append((time.perf_counter() - s) * 1e3)
            got = (pinned.numpy() if name == "pinned" else page).view(np.uint32)
            out[f"{'compact' if mode else 'full'}_{name}_ms"] = {
                "median": round(statistics.median(ts), 4), "min": round(min(ts), 4),
                "p90": round(sorted(ts)[int(0.9 * len(ts))], 4), "bit_identical": bool(np.array_equal(got, want))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
