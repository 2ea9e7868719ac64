#!/usr/bin/env python3
"""Diagnostic: the render kernel of an orbit pose (bench --camera-orbit) when
the pose was set on the home scene (the bins sized by the home camera's
sizing pass) against a scene created with that pose (sized by its own), and
the BVH walk of the pose: whether the orbit's slower frames come from the pose
or from the home camera's sizing."""
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.camera import orbit_poses  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

sc = load_npz(ROOT / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz")
st = N.RendererSettings.default()
fov = float(sc.a["cam_fov"][0])
out = torch.empty(1920 * 1080 * 3, dtype=torch.float32, device="cuda")
stream = torch.cuda.Stream()   # a stream of its own (the null stream's handle 0 means the scene's stream)
sptr = stream.cuda_stream


def render_ms(g, n=30):
    for _ in range(3):
        g.render_device(st, out.data_ptr(), sptr)
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        g.render_device(st, out.data_ptr(), sptr)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


home = N.HipScene(sc)
poses = orbit_poses(sc.a, 60)
for k in [0, 5, 10, 15, 20, 30, 40, 45, 50, 55]:
    loc, rot = poses[k]
    home.set_camera(loc, rot, fov_degrees=fov)
    t_home = render_ms(home)
    own = N.HipScene(sc.set_camera(location=loc, rotation=rot, fov_degrees=fov))
    t_own = render_ms(own)
    own.set_option("bins", 0)
    t_bvh = render_ms(own)
    print(f"pose {k:2d}: home-sized bins {t_home:.4f} ms  own-sized bins {t_own:.4f} ms  BVH walk {t_bvh:.4f} ms",
          flush=True)
    del own
