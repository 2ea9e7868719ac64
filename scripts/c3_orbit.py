"""C3 with a moving camera: frames back to back (a new pose before each,
device frames into one buffer) and one at a time (blocking), after a warm-up
long enough for every buffer set to be sized; options as OPT=name=v,..."""
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, os.environ.get("CRT_PKG") or str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.camera import orbit_poses  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

W, H = 1920, 1080
sc = load_npz(ROOT / "tests" / "golden" / "scenes" / "11-01-refractive__scene8.npz").set_resolution(W, H)
st = N.RendererSettings.default(max_ray_depth=8)
g = N.HipScene(sc)
for kv in os.environ.get("OPT", "").split(","):
    if kv:
        k, v = kv.split("=")
        g.set_option(k, int(v))
fov = float(sc.a["cam_fov"][0])
cams = [N.CameraDesc(N.Vec3(*[float(v) for v in loc]), (N.C.c_float * 9)(*[float(v) for v in rot]), W, H, fov)
        for loc, rot in orbit_poses(sc.a, 60)]
frame = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
s = torch.cuda.Stream()
sptr = s.cuda_stream


def step(k):
    g.set_camera_desc(cams[k % len(cams)])
    g.render_device(st, frame.data_ptr(), sptr)


res = {}
for name, steps in [("warm", 30), ("back_to_back", 40)]:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize()
    res[name] = (time.perf_counter() - t0) / steps * 1e3
one = []
for k in range(10):
    g.set_camera_desc(cams[k])
    t0 = time.perf_counter()
    g.render(st)
    one.append((time.perf_counter() - t0) * 1e3)
res["one_at_a_time_blocking"] = float(np.median(one))
fixed = []
for k in range(10):
    t0 = time.perf_counter()
    g.render(st)
    fixed.append((time.perf_counter() - t0) * 1e3)
res["fixed_blocking"] = float(np.median(fixed))
print({k: round(v, 4) for k, v in res.items()}, g.info()["wf_sets"], flush=True)
