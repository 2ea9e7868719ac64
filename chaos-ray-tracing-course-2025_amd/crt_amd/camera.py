"""Camera poses for moving-camera frames (tests, bench.py --camera-orbit).

The reference's camera (crt_camera.cpp:7-35) maps v = (dx, dy, -1) to the ray
direction v * R (row vector times the row-major rotation, crt_matrix.h:66-74),
so R's rows are the camera's right, up and back axes in world space.  An orbit
turns the camera about a pivot: a world-space rotation M (acting on row
vectors) moves the location to pivot + (loc - pivot) M and the axes to R M,
so the pivot stays where it was on screen.
"""
from __future__ import annotations

import numpy as np


def rotation(axis, degrees: float) -> np.ndarray:
    """3x3 rotation (row-vector convention: w = v @ M) about `axis` by `degrees`."""
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    t = np.deg2rad(degrees)
    c, s = np.cos(t), np.sin(t)
    x, y, z = a
    # column-vector matrix, transposed for row vectors
    m = np.array([[c + x * x * (1 - c), x * y * (1 - c) - z * s, x * z * (1 - c) + y * s],
                  [y * x * (1 - c) + z * s, c + y * y * (1 - c), y * z * (1 - c) - x * s],
                  [z * x * (1 - c) - y * s, z * y * (1 - c) + x * s, c + z * z * (1 - c)]])
    return m.T


def orbit(location, rot, pivot, yaw_deg: float, pitch_deg: float = 0.0):
    """The pose `yaw_deg` about the world y axis and `pitch_deg` about the
    camera's right axis around `pivot`: (location[3], rotation[9]) as float32."""
    loc = np.asarray(location, np.float64)
    R = np.asarray(rot, np.float64).reshape(3, 3)
    M = rotation(R[0], pitch_deg) @ rotation((0.0, 1.0, 0.0), yaw_deg)
    p = np.asarray(pivot, np.float64)
    new_loc = p + (loc - p) @ M
    new_R = R @ M
    return new_loc.astype(np.float32), new_R.astype(np.float32).ravel()


def scene_pivot(arrays: dict) -> np.ndarray:
    """Centre of the bounding box of every mesh of an ArrayScene's arrays."""
    pts = [arrays[k].reshape(-1, 3) for k in arrays if k.endswith("_pos")]
    p = np.concatenate(pts, 0)
    return (p.min(0) + p.max(0)) * 0.5


def orbit_poses(arrays: dict, n: int, yaw_amp: float = 20.0, pitch_amp: float = 6.0):
    """n poses of a camera swinging around the scene's centre from its own
    pose: yaw yaw_amp * sin, pitch pitch_amp * cos over one period."""
    loc0 = np.asarray(arrays["cam_loc"], np.float32)
    rot0 = np.asarray(arrays["cam_rot"], np.float32)
    pivot = scene_pivot(arrays)
    out = []
    for k in range(n):
        ph = 2.0 * np.pi * k / max(n, 1)
        out.append(orbit(loc0, rot0, pivot, yaw_amp * np.sin(ph), pitch_amp * (np.cos(ph) - 1.0)))
    return out
