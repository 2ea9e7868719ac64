#!/usr/bin/env python3
"""Diagnostic: wall time of the multi-GPU create probe (crt_scene_info.
multi_probe_ms: a 64x36 frame through the replicas and through device 0
alone, plus the two view rebuilds) for each config's scene, forced over
repeated devices (create flag SCENE_PROBE_FORCE; the box has one GPU), against the
same create without it."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
sys.path.insert(0, str(ROOT / "tests"))
from crt_amd import native as N  # noqa: E402
from conftest import scene_npz  # noqa: E402

cases = [("c2", scene_npz("14-01-acceleration-tree__scene1")),
         ("c3", scene_npz("11-01-refractive__scene8")),
         ("c4", scene_npz("15-01-conclusion__scene2").set_resolution(3840, 2160))]
for name, sc in cases:
    for mode in ("0", "force"):
        t0 = time.perf_counter()
        g = N.HipScene(sc, devices=[0, 0], create_flags=N.SCENE_PROBE_OFF if mode == "0" else N.SCENE_PROBE_FORCE)
        wall = (time.perf_counter() - t0) * 1e3
        i = g.info()
        print(f"{name} probe={mode:5s} create {wall:8.1f} ms  multi_probe {i['multi_probe']}  "
              f"multi_probe_ms {i['multi_probe_ms']:.2f}", flush=True)
        del g
