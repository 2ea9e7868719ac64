#!/usr/bin/env python3
"""Where the first crt_hip_render of a fresh process spends its time
(the reference CLI's timed region, main.cpp:37-43) — VERDICT r02 item 5.

  cold_breakdown.py [--config c2] [--runs 3] [--out gpurun_out/cold.json]

1. bin/crt_renderer on the config's scene, `runs` fresh processes: the
   "Execution time" it prints (what bench.py's cold_cli reports);
2. one fresh Python process per plan mode (ctypes, no torch): scene creation,
   then the first, second and third crt_hip_render into a pageable numpy
   image, and one into pinned memory is not available without torch, so the
   steady-state device-only frame (crt_hip_render_device) is timed instead.
"""
import argparse
import json
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "chaos-ray-tracing-course-2025_amd"
sys.path.insert(0, str(PKG))
sys.path.insert(0, str(ROOT))

CHILD = r'''
import sys, time, json
sys.path.insert(0, sys.argv[1])
t0 = time.perf_counter()
from crt_amd import native as N
from crt_amd.scene_npz import load_npz
import numpy as np
lib = N.lib()
t_lib = time.perf_counter()
sc = load_npz(sys.argv[2]).set_resolution(int(sys.argv[3]), int(sys.argv[4]))
st = N.RendererSettings.default(max_ray_depth=int(sys.argv[5]))
opts = json.loads(sys.argv[6])
t1 = time.perf_counter()
g = N.HipScene(sc, device=0, **opts)
t2 = time.perf_counter()
ts = []
for _ in range(4):
    s = time.perf_counter()
    g.render(st)
    ts.append((time.perf_counter() - s) * 1e3)
print(json.dumps({"opts": opts, "import_ms": (t_lib - t0) * 1e3, "scene_create_ms": (t2 - t1) * 1e3,
                  "render_ms": ts, "plan": g.plan_info() if hasattr(g, "plan_info") else None}))
'''


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c2")
    p.add_argument("--runs", type=int, default=3)
    p.add_argument("--out", default=None)
    p.add_argument("--keep", default=None, help="also write the .crtscene here (for a traced CLI run)")
    a = p.parse_args()
    import bench
    from crt_amd.scene_json import arrays_to_crtscene
    cfg = bench.CONFIGS[a.config]
    w, h = cfg["size"]
    depth = cfg["settings"].get("max_ray_depth", 3)
    sc = bench.make_scene(cfg, w, h)
    res = {"config": a.config, "size": [w, h], "cli": [], "inproc": []}
    with tempfile.TemporaryDirectory() as td:
        doc = arrays_to_crtscene(sc.a, {})
        doc["settings"]["image_settings"].update(width=w, height=h)
        scene = Path(td) / "scene.crtscene"
        scene.write_text(json.dumps(doc))
        if a.keep:
            Path(a.keep).mkdir(parents=True, exist_ok=True)
            (Path(a.keep) / "scene.crtscene").write_text(json.dumps(doc))
        for _ in range(a.runs):
            t0 = time.perf_counter()
            r = subprocess.run([str(PKG / "bin" / "crt_renderer"), str(scene), str(Path(td) / "o.ppm"), "--gpus", "1",
                                "--max-depth", str(depth)], capture_output=True, text=True, timeout=300)
            wall = (time.perf_counter() - t0) * 1e3
            ex = float(r.stdout.split("Execution time: ", 1)[1].split()[0]) * 1e3 if r.returncode == 0 else None
            res["cli"].append({"execution_ms": ex, "process_ms": round(wall, 1), "rc": r.returncode})
            print(json.dumps(res["cli"][-1]), flush=True)
    npz = ROOT / "tests" / "golden" / "scenes" / f"{cfg['scene']}.npz"
    for opts in ({}, {"calibrate": 0}, {"calibrate": 1}):
        r = subprocess.run([sys.executable, "-c", CHILD, str(PKG), str(npz), str(w), str(h), str(depth), json.dumps(opts)],
                           capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else None
        res["inproc"].append(json.loads(line) if line else {"opts": opts, "error": r.stderr[-400:]})
        print(json.dumps(res["inproc"][-1]), flush=True)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
