"""Per-wave work of the BVH camera walk (crt_bvh.h trace_bvh_exact), on the CPU.

Runs the product's walk over every camera ray of a frame (tests/tools
prune_sim.cpp, bvh_sim_ray_stats) and groups the rays into the kernel's 8x8
tile waves: a per-lane walk costs each wave the MAX over its lanes of the
sequential steps, so the heaviest waves — not the mean — bound the frame tail.
    python3 scripts/bvh_wave_cost.py [--scene 14-01-acceleration-tree__scene1]
"""
import argparse
import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "chaos-ray-tracing-course-2025_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="14-01-acceleration-tree__scene1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    from conftest import scene_npz
    from oracle import pyoracle
    from crt_amd.native import _desc_ptr
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests/tools")], check=True)
    L = C.CDLL(str(ROOT / "tests/tools/_build/libprune_sim.so"))
    L.bvh_sim_ray_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    L.bvh_sim_ray_stats.restype = C.c_int
    w, h = a.width, a.height
    sc = scene_npz(a.scene).set_resolution(w, h)
    ys, xs = np.mgrid[0:h, 0:w]
    rays = np.ascontiguousarray(pyoracle.OracleScene(sc).camera_rays(np.stack([xs.ravel(), ys.ravel()], 1)),
                                np.float32)
    st = np.zeros((len(rays), 4), np.int32)
    assert L.bvh_sim_ray_stats(C.cast(_desc_ptr(sc), C.c_void_p), rays.ctypes.data, len(rays), st.ctypes.data) == 0
    st = st.reshape(h, w, 4)
    th, tw = (h + 7) // 8, (w + 7) // 8
    pad = np.zeros((th * 8, tw * 8, 4), np.int32)
    pad[:h, :w] = st
    waves = pad.reshape(th, 8, tw, 8, 4).transpose(0, 2, 1, 3, 4).reshape(th * tw, 64, 4)
    steps = waves[..., 0] + waves[..., 1] + waves[..., 2]      # one lane's sequential steps
    wmax = steps.max(1)
    order = np.argsort(-wmax)
    rep = {"scene": a.scene, "size": [w, h], "rays": int(w * h),
           "per_ray": {k: {"mean": float(st[..., i].mean()), "p99": float(np.percentile(st[..., i], 99)),
                           "max": int(st[..., i].max())}
                       for i, k in enumerate(["walk_nodes", "walk_tris", "proof_steps", "fallback"])},
           "wave_max_steps": {"mean": float(wmax.mean()), "p99": float(np.percentile(wmax, 99)),
                              "max": int(wmax.max())},
           "waves_with_fallback": int((waves[..., 3].max(1) > 0).sum()), "waves": int(len(wmax)),
           "heaviest": []}
    for k in order[:a.top]:
        lane = int(np.argmax(steps[k]))
        rep["heaviest"].append({"tile": [int(k % tw) * 8, int(k // tw) * 8], "max_steps": int(wmax[k]),
                                "lane": waves[k, lane].tolist(), "mean_steps": float(steps[k].mean()),
                                "fallback_lanes": int(waves[k, :, 3].sum())})
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
