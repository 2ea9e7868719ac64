#!/usr/bin/env python3
"""Render a scene K times through the C-ABI (no torch) — driver for rocprofv3
kernel traces / PMC passes and for in-process A/B of kernel variants.

  render_loop.py [--scene NAME] [--width W --height H] [--frames K] [--depth D]
                 [--ab VAR=a,b]   # A/B: one scene per env value, interleaved rounds
                 [--opt OPTION=a,b]   # A/B: one scene per set_option value
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, os.environ.get("CRT_PKG") or str(ROOT / "chaos-ray-tracing-course-2025_amd"))   # CRT_PKG: A/B of another build

from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="14-01-acceleration-tree__scene1")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--frames", type=int, default=5)
    p.add_argument("--depth", type=int, default=3)
    p.add_argument("--gi", type=int, default=4, help="diffuse_reflection_ray_count")
    p.add_argument("--ab", default=None, help="ENVVAR=v1,v2,... — build one scene per value")
    p.add_argument("--opt", default=None, help="OPTION=v1,v2,... — one scene per crt_hip_scene_set_option value")
    p.add_argument("--set", action="append", default=[], metavar="OPTION=V",
                   help="crt_hip_scene_set_option on every scene (repeatable), e.g. --set shadows=1")
    p.add_argument("--counts", action="store_true", help="print per-ray and per-wave work counts per variant")
    p.add_argument("--synthetic", type=int, default=0, help="C5: synthetic mesh of N triangles instead of --scene")
    a = p.parse_args()
    if a.synthetic:
        from crt_amd.synthetic import c5_scene
        sc = c5_scene(a.synthetic, width=a.width, height=a.height)
        a.scene = f"synthetic-{a.synthetic}"
    else:
        sc = load_npz(ROOT / "tests" / "golden" / "scenes" / f"{a.scene}.npz").set_resolution(a.width, a.height)
    st = N.RendererSettings.default(max_ray_depth=a.depth, diffuse_reflection_ray_count=a.gi)
    variants = [("default", None)]
    if a.ab:
        var, vals = a.ab.split("=", 1)
        sep = ";" if ";" in vals else ","
        variants = [(f"{var}={v}", (var, v)) for v in vals.split(sep)]
    if a.opt:
        opt, vals = a.opt.split("=", 1)
        variants = [(f"{opt}={v}", ("opt", opt, int(v))) for v in vals.split(",")]
    scenes = []
    for name, kv in variants:
        if kv and kv[0] == "opt":
            scenes.append((name, N.HipScene(sc).set_option(kv[1], kv[2])))
            continue
        if kv:
            os.environ[kv[0]] = kv[1]
        scenes.append((name, N.HipScene(sc)))
    for kv in a.set:
        k, v = kv.split("=", 1)
        for _, g in scenes:
            g.set_option(k, int(v))
    times = {name: [] for name, _ in scenes}
    ref = None
    for _ in range(a.frames):
        for name, g in scenes:
            img, stats = g.render(st, with_stats=True)
            times[name].append(stats["kernel_ms"])
            if ref is None:
                ref = img
            elif not np.array_equal(ref.view(np.uint32), img.view(np.uint32)):
                print(f"MISMATCH in variant {name}", flush=True)
    out = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)), "n": len(v)} for k, v in times.items()}
    if a.counts:
        for name, g in scenes:
            out[name]["work"] = g.count_work(st)
            out[name]["wave"] = g.wave_counts()
    import hashlib
    print(json.dumps({"scene": a.scene, "size": [a.width, a.height], "depth": a.depth, "kernel": out,
                      "image_sha1": hashlib.sha1(ref.tobytes()).hexdigest()[:16]}))


if __name__ == "__main__":
    main()
