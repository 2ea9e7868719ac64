#!/usr/bin/env python3
"""Diagnostic: C2 frames with a new camera pose each (bench --camera-orbit)
against the same frames rebinned with a fixed camera — host time of the
enqueue (set_camera + render_device) against the frame period, so an orbit
that is host-bound shows as host time ~ period."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
sys.path.insert(0, str(ROOT / "tests"))
from crt_amd import native as N  # noqa: E402
from crt_amd.camera import orbit_poses  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402
from conftest import DeviceBuffers  # noqa: E402

sc = load_npz(ROOT / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz")
g = N.HipScene(sc)
st = N.RendererSettings.default()
db = DeviceBuffers()
d = db.alloc(1920 * 1080 * 12)
fov = float(sc.a["cam_fov"][0])
cams = [N.CameraDesc(N.Vec3(*[float(v) for v in loc]), (N.C.c_float * 9)(*[float(v) for v in rot]), 1920, 1080, fov)
        for loc, rot in orbit_poses(sc.a, 60)]
home = N.CameraDesc(N.Vec3(*[float(v) for v in sc.a["cam_loc"]]),
                    (N.C.c_float * 9)(*[float(v) for v in sc.a["cam_rot"]]), 1920, 1080, fov)


def run(label, n, orbit, reuse):
    g.set_option("bins_reuse", reuse)
    for k in range(20):
        if orbit:
            g.set_camera_desc(cams[k % len(cams)])
        g.render_device(st, d)
    db.sync()
    hc = hr = 0.0
    t0 = time.perf_counter()
    for k in range(n):
        a = time.perf_counter()
        if orbit:
            g.set_camera_desc(cams[k % len(cams)])
        b = time.perf_counter()
        g.render_device(st, d)
        c = time.perf_counter()
        hc += b - a
        hr += c - b
    t1 = time.perf_counter()
    db.sync()
    t2 = time.perf_counter()
    print(f"{label:28s} period {(t2 - t0) / n * 1e3:.4f} ms  host set_camera {hc / n * 1e3:.4f} ms  "
          f"render_device {hr / n * 1e3:.4f} ms  enqueue total {(t1 - t0) / n * 1e3:.4f} ms", flush=True)
    g.set_camera_desc(home)


for _ in range(2):
    run("fixed camera, reuse", 200, False, 1)
    run("fixed camera, rebinned", 200, False, 0)
    run("orbit", 200, True, 1)
print("info", {k: v for k, v in g.info().items() if k in ("camera_moves", "view_rebuilds", "records_written",
                                                         "bins_binnings", "bins_reuses")})
