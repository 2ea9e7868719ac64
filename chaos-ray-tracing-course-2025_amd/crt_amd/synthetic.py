"""Synthetic scenes of the BASELINE configs.

C5: N random triangles — centres uniform in [-1,1]^3, each vertex the centre
plus uniform(-s,s)^3 with s = 2/cbrt(N) (0.02 at N = 1e6), float32, numpy
default_rng(1234); 3N unshared vertices; one diffuse material (0.8, 0.8, 0.8),
one light (I = 1000 at (2, 2, 3)), background (0, 0.5, 0), camera at
(0, 0, 1.5), identity rotation, fov 90.
"""
from __future__ import annotations

import numpy as np

from .native import SyntheticScene


def c5_mesh(n: int = 1_000_000, seed: int = 1234):
    rng = np.random.default_rng(seed)
    s = 2.0 / np.cbrt(n)
    centres = rng.uniform(-1.0, 1.0, (n, 3)).astype(np.float32)
    offsets = rng.uniform(-s, s, (n, 3, 3)).astype(np.float32)
    verts = (centres[:, None, :] + offsets).astype(np.float32).reshape(-1, 3)
    idx = np.arange(3 * n, dtype=np.int32)
    return verts, idx


def c5_scene(n: int = 1_000_000, width: int = 3840, height: int = 2160, seed: int = 1234) -> SyntheticScene:
    verts, idx = c5_mesh(n, seed)
    return SyntheticScene(verts, idx, width=width, height=height, camera_location=(0.0, 0.0, 1.5),
                          fov_degrees=90.0, background=(0.0, 0.5, 0.0), albedo=(0.8, 0.8, 0.8),
                          lights=((1000.0, (2.0, 2.0, 3.0)),))
