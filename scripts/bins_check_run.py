"""Diagnostic: the camera-bins kernels of a CRT_BINS_CHECK build (every index
checked, scripts/make_variant.sh chk BINS_FLAGS=-DCRT_BINS_CHECK) over the
bins scenes: device lists vs the host checker, frames vs the oracle, several
frames back to back.  A violation raises CrtError("bins check: ...")."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
PKG = Path(os.environ.get("CRT_PKG", ROOT / "abtest" / "chk")).resolve()
sys.path.insert(0, str(PKG))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402
from oracle import pyoracle  # noqa: E402

print("lib", N.LIB_PATH, N.build_id(), flush=True)
cases = [("14-01-acceleration-tree__scene1", None), ("14-01-acceleration-tree__scene1", (333, 177)),
         ("12-01-textures__scene4", (640, 360)), ("09-02-diffuse-smooth-shading__scene3", (480, 270)),
         ("13-01-optimizations__scene0", (640, 360))]
from test_gpu_bins import floor_scene, wall_scene  # noqa: E402

cases += [("14-01-acceleration-tree__scene1", (3840, 2160)), ("wall", (640, 360)), ("wall", (1920, 1080)), ("floor", (400, 240))]
st = N.RendererSettings.default()
for name, size in cases:
    if name == "wall":
        sc = wall_scene(N, *size)
    elif name == "floor":
        sc = floor_scene(N, *size)
    else:
        sc = load_npz(ROOT / "tests" / "golden" / "scenes" / f"{name}.npz")
        if size:
            sc.set_resolution(*size)
    hl, hr = N.HostScene(sc).camera_bins()
    g = N.HipScene(sc)
    for _ in range(3):
        dl, dr = g.camera_bins()
        assert np.array_equal(hl, dl) and hr.tobytes() == dr.tobytes(), name
    want = pyoracle.OracleScene(sc).render(st) if size and size[0] <= 640 else None
    for _ in range(3):
        img = g.render(st)
        if want is not None:
            assert np.array_equal(img.view(np.uint32), want.view(np.uint32)), name
    g.count_work(st)
    g.camera_bins()   # reports any violation of the frames above
    print("ok", name, size, len(dr), flush=True)
print("all ok", flush=True)
