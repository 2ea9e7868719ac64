import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = Path(os.environ["CRT_PKG"]).resolve() if os.environ.get("CRT_PKG") else ROOT / "chaos-ray-tracing-course-2025_amd"   # CRT_PKG: a variant build
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


class DeviceBuffers:
    """hipMalloc'd scratch through the HIP runtime libcrt_hip.so already loaded
    (same SONAME), freed on close; for tests of the device-pointer entry points."""

    def __init__(self):
        import ctypes as C
        self.C = C
        self.hip = C.CDLL("libamdhip64.so.7")
        self.hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        self.hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self.hip.hipFree.argtypes = [C.c_void_p]
        self.hip.hipDeviceSynchronize.argtypes = []
        self.hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
        self.hip.hipStreamDestroy.argtypes = [C.c_void_p]
        self.ptrs = []
        self.streams = []

    def stream(self) -> int:
        """A non-blocking HIP stream (hipStreamNonBlocking), destroyed on close."""
        s = self.C.c_void_p()
        assert self.hip.hipStreamCreateWithFlags(self.C.byref(s), 1) == 0
        self.streams.append(s)
        return s.value

    def alloc(self, nbytes: int) -> int:
        p = self.C.c_void_p()
        assert self.hip.hipMalloc(self.C.byref(p), max(int(nbytes), 1)) == 0
        self.ptrs.append(p)
        return p.value

    def upload(self, a: np.ndarray) -> int:
        a = np.ascontiguousarray(a)
        p = self.alloc(a.nbytes)
        assert self.hip.hipMemcpy(p, a.ctypes.data, a.nbytes, 1) == 0
        return p

    def download(self, p: int, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype)
        assert self.hip.hipDeviceSynchronize() == 0
        assert self.hip.hipMemcpy(out.ctypes.data, p, out.nbytes, 2) == 0
        return out

    def sync(self):
        assert self.hip.hipDeviceSynchronize() == 0

    def close(self):
        if self.ptrs or self.streams:
            self.hip.hipDeviceSynchronize()
        for p in self.ptrs:
            self.hip.hipFree(p)
        self.ptrs = []
        for s in self.streams:
            self.hip.hipStreamDestroy(s)
        self.streams = []


@pytest.fixture
def devbuf():
    b = DeviceBuffers()
    yield b
    b.close()


def ppm_quantize(rgb: np.ndarray, maxc: int = 255) -> np.ndarray:
    """write_ppm's conversion (crt_image_ppm.cpp:15-18) in numpy:
    clamp(static_cast<int>(c * max), 0, max) with x86 cvttss2si semantics."""
    x = np.asarray(rgb, np.float32) * np.float32(maxc)
    ok = (x >= np.float32(-2147483648.0)) & (x < np.float32(2147483648.0))
    v = np.where(ok, np.trunc(np.where(ok, x, 0)).astype(np.int64), -2147483648)
    return np.clip(v, 0, maxc).astype(np.uint8)


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
