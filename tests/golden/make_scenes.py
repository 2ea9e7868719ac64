"""Regenerate tests/golden/scenes/*.npz from the reference's .crtscene files.

Runs only where /root/reference exists.  Each .npz is the flat scene
description (include/crt_hip.h crt_scene_desc) our loader produces from the
scene file — input data for GPU tests and bench.py on machines without the
reference checkout.  tests/test_loader.py checks the loader reproduces them.
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import save_npz  # noqa: E402

REF = Path("/root/reference/scenes")
OUT = Path(__file__).resolve().parent / "scenes"

SCENES = [
    "09-01-barycentric-coordinates/scene1",
    "09-02-diffuse-smooth-shading/scene2", "09-02-diffuse-smooth-shading/scene3",
    "09-03-reflective/scene4", "09-03-reflective/scene5",
    "11-01-refractive/scene0", "11-01-refractive/scene1", "11-01-refractive/scene2",
    "11-01-refractive/scene3", "11-01-refractive/scene4", "11-01-refractive/scene5",
    "11-01-refractive/scene6", "11-01-refractive/scene7", "11-01-refractive/scene8",
    "12-01-textures/scene3", "12-01-textures/scene4",
    "13-01-optimizations/scene0",
    "14-01-acceleration-tree/scene0", "14-01-acceleration-tree/scene1",
    "15-01-conclusion/scene0", "15-01-conclusion/scene1", "15-01-conclusion/scene2",
]


def name_of(s: str) -> str:
    return s.replace("/", "__")


def main():
    OUT.mkdir(exist_ok=True)
    for s in SCENES:
        sf = N.SceneFile(path=REF / f"{s}.crtscene")
        save_npz(sf, OUT / f"{name_of(s)}.npz")
        print("wrote", name_of(s))


if __name__ == "__main__":
    main()
