#!/usr/bin/env python3
"""A/B of camera-bins plan options on C2: frames back to back with one camera
(lists reused), with the camera rebinned every frame, and the bench's orbit
(a new pose every frame).  usage: orbit_ab.py opt=v,opt=v [opt=v,...] ..."""
import os
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, os.environ.get("CRT_PKG") or str(ROOT / "chaos-ray-tracing-course-2025_amd"))   # CRT_PKG: A/B of another build
from crt_amd import native as N  # noqa: E402
from crt_amd.camera import orbit_poses  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

sc = load_npz(ROOT / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz")
st = N.RendererSettings.default()
fov = float(sc.a["cam_fov"][0])
out = torch.empty(1920 * 1080 * 3, dtype=torch.float32, device="cuda")
stream = torch.cuda.Stream()
sptr = stream.cuda_stream
cams = [N.CameraDesc(N.Vec3(*[float(v) for v in loc]), (N.C.c_float * 9)(*[float(v) for v in rot]), 1920, 1080, fov)
        for loc, rot in orbit_poses(sc.a, 60)]
home = N.CameraDesc(N.Vec3(*[float(v) for v in sc.a["cam_loc"]]),
                    (N.C.c_float * 9)(*[float(v) for v in sc.a["cam_rot"]]), 1920, 1080, fov)


def period(g, n, orbit):
    for k in range(20):
        if orbit:
            g.set_camera_desc(cams[k % len(cams)])
        g.render_device(st, out.data_ptr(), sptr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(n):
        if orbit:
            g.set_camera_desc(cams[k % len(cams)])
        g.render_device(st, out.data_ptr(), sptr)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    g.set_camera_desc(home)
    return ms


for spec in sys.argv[1:]:
    opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in spec.split(",") if kv)
    g = N.HipScene(sc, **opts)
    r = []
    for _ in range(3):
        fixed = period(g, 200, False)
        g.set_option("bins_reuse", 0)
        rebin = period(g, 200, False)
        g.set_option("bins_reuse", 1)
        orbit = period(g, 120, True)
        r.append((fixed, rebin, orbit))
    f, rb, o = (min(x[i] for x in r) for i in range(3))
    print(f"{spec:32s} fixed {f:.4f}  rebinned {rb:.4f}  orbit {o:.4f} ms  orbit/fixed {o / f:.3f}  "
          f"orbit/rebinned {o / rb:.3f}", flush=True)
    del g
