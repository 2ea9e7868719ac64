import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "chaos-ray-tracing-course-2025_amd"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"
SCENES = GOLDEN / "scenes"
REFERENCE = Path(os.environ.get("CRT_REFERENCE", "/root/reference"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def has_reference() -> bool:
    return (REFERENCE / "src" / "core" / "crt_intersection.cpp").exists()


def scene_npz(name: str):
    from crt_amd.scene_npz import load_npz
    return load_npz(SCENES / f"{name}.npz")


@pytest.fixture(scope="session")
def native_lib():
    from crt_amd import native
    return native.lib()


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    return pyoracle


def bits(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def hits_equal(a: np.ndarray, b: np.ndarray, with_tri: bool = True):
    """Field-wise bit equality of two HIT_DTYPE arrays; returns (ok, first bad index)."""
    bad = np.zeros(len(a), bool)
    for f in a.dtype.names:
        if f == "triangle_index" and not with_tri:
            continue
        x, y = np.ascontiguousarray(a[f]), np.ascontiguousarray(b[f])
        xb = x.view(np.uint32) if x.dtype == np.float32 else x
        yb = y.view(np.uint32) if y.dtype == np.float32 else y
        d = xb != yb
        bad |= d.reshape(len(a), -1).any(axis=1)
    idx = np.flatnonzero(bad)
    return len(idx) == 0, (int(idx[0]) if len(idx) else -1), int(bad.sum())
