#!/usr/bin/env python3
"""Parts of the first crt_hip_render of a fresh process (C2 unless --scene):
first device-only frame (plan + code-object load), the same for a second
scene in the warm process (plan only), warm device frames, and the D2H of the
fp32 image into pageable vs pinned host memory.  Prints one JSON line.

  cold_parts.py [--scene 14-01-acceleration-tree__scene1] [--depth 3]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="14-01-acceleration-tree__scene1")
    p.add_argument("--depth", type=int, default=3)
    a = p.parse_args()
    import numpy as np
    import torch
    from crt_amd import native as N
    from crt_amd.scene_npz import load_npz
    sc = load_npz(ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.npz")
    st = N.RendererSettings.default(max_ray_depth=a.depth)
    torch.cuda.init()
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    npx = int(sc.a["cam_size"][0]) * int(sc.a["cam_size"][1])
    out = torch.empty(npx * 3, dtype=torch.float32, device="cuda")
    res = {}

    def dev_frame(g):
        torch.cuda.synchronize()
        t = time.perf_counter()
        g.render_device(st, out.data_ptr())
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    t = time.perf_counter()
    g1 = N.HipScene(sc, device=0)
    res["scene_create_ms"] = (time.perf_counter() - t) * 1e3
    res["first_device_frame_ms"] = dev_frame(g1)
    res["second_device_frame_ms"] = dev_frame(g1)
    res["warm_device_frame_ms"] = sorted(dev_frame(g1) for _ in range(10))[5]
    g2 = N.HipScene(sc, device=0)
    res["other_scene_first_device_frame_ms"] = dev_frame(g2)
    # D2H of the image: pageable (touched first) vs pinned
    page = np.ones(npx * 3, np.float32)
    pin = torch.empty(npx * 3, dtype=torch.float32, pin_memory=True)
    pt = torch.from_numpy(page)
    for name, dst in (("pageable", pt), ("pinned", pin)):
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            dst.copy_(out)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        res[f"d2h_{name}_ms"] = sorted(ts)[2]
    # crt_hip_render (render + D2H into the caller's pageable buffer) on a fresh scene and warm
    g3 = N.HipScene(sc, device=0)
    t = time.perf_counter()
    g3.render_host(st, page.ctypes.data)
    res["render_host_pageable_fresh_scene_ms"] = (time.perf_counter() - t) * 1e3
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        g3.render_host(st, page.ctypes.data)
        ts.append((time.perf_counter() - t) * 1e3)
    res["render_host_pageable_warm_ms"] = sorted(ts)[2]
    res["plan"] = g1.plan_info()
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
