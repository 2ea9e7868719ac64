"""Diagnostic: bench.py's C3 sequence (fixed-camera frames, a blocking check
render, then a camera orbit) with per-call host times of the orbit frames, to
find what a moving-camera frame waits for after a blocking render."""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.camera import orbit_poses  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

W, H = 1920, 1080
sc = load_npz(ROOT / "tests" / "golden" / "scenes" / "11-01-refractive__scene8.npz").set_resolution(W, H)
st = N.RendererSettings.default(max_ray_depth=8)
g = N.HipScene(sc, events=0, calibrate=int(sys.argv[1]) if len(sys.argv) > 1 else 1)
if "--g2" in sys.argv:   # bench.py's second create (scene_create_ms_second), destroyed at once
    g2 = N.HipScene(sc, events=0, calibrate=1)
    del g2
if "--set-stream" in sys.argv:
    torch.cuda.set_stream(torch.cuda.Stream())
frame = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
s = torch.cuda.Stream()
sptr = s.cuda_stream
fov = float(sc.a["cam_fov"][0])
cams = [N.CameraDesc(N.Vec3(*[float(v) for v in loc]), (N.C.c_float * 9)(*[float(v) for v in rot]), W, H, fov)
        for loc, rot in orbit_poses(sc.a, 60)]
for _ in range(30):
    g.render_device(st, frame.data_ptr(), sptr)
torch.cuda.synchronize()
if "--counts" in sys.argv:   # bench.py: work counters of one frame, then the per-wave counts
    g.count_work(st)
if "--waves" in sys.argv:
    g.wave_counts()
if "--bins-ms" in sys.argv:   # bench.py: the binning alone, 50 times
    print("bins_ms", g.bins_ms(50), flush=True)
if "--toggles" in sys.argv:   # bench.py: bins_reuse 0 / bins 0 frames, then back
    for opt, v in (("bins_reuse", 0), ("bins_reuse", 1), ("bins", 0), ("bins", 1)):
        g.set_option(opt, v)
        for _ in range(5):
            g.render_device(st, frame.data_ptr(), sptr)
    torch.cuda.synchronize()
blocking = "--no-blocking" not in sys.argv
if blocking:
    g.render(st)
out = {}
for name, n in [("orbit_warm", 10), ("orbit", 30)]:
    ts = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(n):
        a = time.perf_counter()
        g.set_camera_desc(cams[k % len(cams)])
        g.render_device(st, frame.data_ptr(), sptr)
        ts.append((time.perf_counter() - a) * 1e3)
    torch.cuda.synchronize()
    out[name] = {"ms_per_frame": round((time.perf_counter() - t0) / n * 1e3, 3),
                 "host_call_ms_median": round(float(np.median(ts)), 3), "host_call_ms_max": round(max(ts), 3)}
print(json.dumps({"argv": sys.argv[1:], **out}))
