#!/usr/bin/env python3
"""A/B tool: scene create costs in one process — the first create (HIP
start-up, code objects) and warm creates after it — with crt_scene_info's
parts; under a CRT_CREATE_TRACE variant (scripts/make_variant.sh ctrace
HOST_AB_FLAGS=-DCRT_CREATE_TRACE, CRT_PKG=abtest/ctrace) each step of the
upload is timed on stderr too.

  python scripts/create_times.py [--config c2] [--creates 3]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = Path(os.environ["CRT_PKG"]).resolve() if os.environ.get("CRT_PKG") else ROOT / "chaos-ray-tracing-course-2025_amd"
sys.path[:0] = [str(PKG), str(ROOT)]

import bench  # noqa: E402
from crt_amd import native as N  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c2")
    p.add_argument("--creates", type=int, default=3)
    a = p.parse_args()
    cfg = bench.CONFIGS[a.config]
    W, H = cfg["size"]
    sc = bench.make_scene(cfg, W, H)
    keep = []
    for k in range(a.creates):
        print(f"--- create {k}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        g = N.HipScene(sc)
        wall = (time.perf_counter() - t0) * 1e3
        info = {kk: round(v, 3) for kk, v in g.info().items()
                if kk in ("prep_ms", "tree_build_ms", "bvh_ms", "bins_ms", "upload_ms", "create_ms")}
        print(json.dumps({"create": k, "wall_ms": round(wall, 3), **info}), flush=True)
        keep.append(g)


if __name__ == "__main__":
    main()
