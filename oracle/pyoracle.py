"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path never does.

  OracleScene  → oracle/_build/liboracle.so  (from-scratch CPU restatement, crt_oracle.cpp)
  RefScene     → oracle/_ref/libref.so       (the reference's own src/core TUs, built in
                                               this container only; absent on the GPU box)
Both take a crt_scene_desc* (crt_amd.native.SceneFile / SyntheticScene / SceneDesc).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
ORACLE_LIB = ORACLE_DIR / "_build" / "liboracle.so"
REF_LIB = ORACLE_DIR / "_ref" / "libref.so"
REFERENCE = Path(os.environ.get("CRT_REFERENCE", "/root/reference"))

_P = C.c_void_p
_oracle = None
_ref = None


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def build_ref() -> bool:
    """Compile the reference's TUs in place (only where /root/reference exists)."""
    if not (REFERENCE / "src" / "core" / "crt_intersection.cpp").exists():
        return REF_LIB.exists()
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR), "ref", f"REF={REFERENCE}"], check=True)
    return True


def oracle_lib() -> C.CDLL:
    global _oracle
    if _oracle is None:
        if not ORACLE_LIB.exists():
            build_oracle()
        L = C.CDLL(str(ORACLE_LIB))
        L.oracle_scene_create.restype = _P
        L.oracle_scene_create.argtypes = [_P]
        L.oracle_scene_destroy.argtypes = [_P]
        L.oracle_set_shadows.argtypes = [_P, C.c_int]
        L.oracle_render.argtypes = [_P, _P, _P, C.c_int, _P]
        L.oracle_render_pixels.argtypes = [_P, _P, C.c_int64, C.c_int64, _P, _P]
        L.oracle_trace.argtypes = [_P, _P, C.c_int64, _P, _P, _P]
        L.oracle_camera_rays.argtypes = [_P, _P, C.c_int64, _P]
        for n in ("oracle_node_count", "oracle_triangle_count", "oracle_vertex_count"):
            getattr(L, n).restype = C.c_int64
            getattr(L, n).argtypes = [_P]
        L.oracle_tree_dump.argtypes = [_P, _P, _P, _P, _P]
        L.oracle_vertex_normals.argtypes = [_P, _P]
        L.oracle_face_normals.argtypes = [_P, _P]
        _oracle = L
    return _oracle


def ref_available() -> bool:
    return REF_LIB.exists() or build_ref()


def ref_lib() -> C.CDLL:
    global _ref
    if _ref is None:
        if not REF_LIB.exists() and not build_ref():
            raise FileNotFoundError("oracle/_ref/libref.so unavailable (needs /root/reference)")
        L = C.CDLL(str(REF_LIB))
        L.ref_scene_create.restype = _P
        L.ref_scene_create.argtypes = [_P]
        L.ref_scene_destroy.argtypes = [_P]
        L.ref_node_count.restype = C.c_int64
        L.ref_node_count.argtypes = [_P]
        L.ref_tree_dump.argtypes = [_P, _P, _P, _P, _P]
        L.ref_trace.argtypes = [_P, _P, C.c_int64, _P]
        L.ref_camera_rays.argtypes = [_P, _P, C.c_int64, _P]
        L.ref_vertex_normals.argtypes = [_P, _P]
        L.ref_face_normals.argtypes = [_P, _P]
        L.ref_write_ppm.argtypes = [_P, C.c_int32, C.c_int32, C.c_char_p]
        _ref = L
    return _ref


def _addr(desc_src) -> int:
    p = desc_src.desc_ptr() if hasattr(desc_src, "desc_ptr") else desc_src
    return C.cast(p, C.c_void_p).value


def _hit_dtype():
    from crt_amd.native import HIT_DTYPE  # noqa: WPS433 (shared record layout)
    return HIT_DTYPE


class OracleScene:
    def __init__(self, desc_src):
        self._L = oracle_lib()
        self._h = self._L.oracle_scene_create(_addr(desc_src))
        self._keep = desc_src
        self.width = desc_src.desc().camera.width
        self.height = desc_src.desc().camera.height

    def set_shadows(self, on: bool = True) -> "OracleScene":
        """Trace the shadow rays (the course's earlier renderer; dead code at
        HEAD, crt_renderer.cpp:29-44,90-92): a light counts only when the shadow
        ray's closest hit is absent or farther than the light."""
        self._L.oracle_set_shadows(self._h, int(bool(on)))
        return self

    def render(self, settings, nthreads: int = 0, counts=None) -> np.ndarray:
        out = np.zeros((self.height, self.width, 3), np.float32)
        self._L.oracle_render(self._h, C.addressof(settings), out.ctypes.data, nthreads,
                              C.addressof(counts) if counts is not None else None)
        return out

    def render_pixels(self, settings, first: int, count: int, counts=None) -> np.ndarray:
        out = np.zeros((count, 3), np.float32)
        self._L.oracle_render_pixels(self._h, C.addressof(settings), first, count, out.ctypes.data,
                                     C.addressof(counts) if counts is not None else None)
        return out

    def trace(self, rays: np.ndarray):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        hits = np.zeros(len(rays), _hit_dtype())
        nodes = np.zeros(len(rays), np.int64)
        tris = np.zeros(len(rays), np.int64)
        self._L.oracle_trace(self._h, rays.ctypes.data, len(rays), hits.ctypes.data, nodes.ctypes.data,
                             tris.ctypes.data)
        return hits, nodes, tris

    def camera_rays(self, xy: np.ndarray) -> np.ndarray:
        xy = np.ascontiguousarray(xy, np.int32).reshape(-1, 2)
        out = np.zeros((len(xy), 6), np.float32)
        self._L.oracle_camera_rays(self._h, xy.ctypes.data, len(xy), out.ctypes.data)
        return out

    def tree(self):
        n = self._L.oracle_node_count(self._h)
        off = np.zeros(n + 1, np.int64)
        self._L.oracle_tree_dump(self._h, None, None, off.ctypes.data, None)
        b = np.zeros((n, 6), np.float32)
        c = np.zeros((n, 2), np.int32)
        t = np.zeros(max(int(off[-1]), 1), np.int32)
        self._L.oracle_tree_dump(self._h, b.ctypes.data, c.ctypes.data, off.ctypes.data, t.ctypes.data)
        return b, c, off, t[: int(off[-1])]

    def vertex_normals(self) -> np.ndarray:
        out = np.zeros((self._L.oracle_vertex_count(self._h), 3), np.float32)
        self._L.oracle_vertex_normals(self._h, out.ctypes.data)
        return out

    def face_normals(self) -> np.ndarray:
        out = np.zeros((self._L.oracle_triangle_count(self._h), 3), np.float32)
        self._L.oracle_face_normals(self._h, out.ctypes.data)
        return out

    def __del__(self):
        try:
            self._L.oracle_scene_destroy(self._h)
        except Exception:
            pass


class RefScene:
    """The reference's own compiled hot path (oracle/_ref/libref.so)."""

    def __init__(self, desc_src):
        self._L = ref_lib()
        self._h = self._L.ref_scene_create(_addr(desc_src))
        self._keep = desc_src

    def trace(self, rays: np.ndarray):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        hits = np.zeros(len(rays), _hit_dtype())
        self._L.ref_trace(self._h, rays.ctypes.data, len(rays), hits.ctypes.data)
        return hits

    def camera_rays(self, xy: np.ndarray) -> np.ndarray:
        xy = np.ascontiguousarray(xy, np.int32).reshape(-1, 2)
        out = np.zeros((len(xy), 6), np.float32)
        self._L.ref_camera_rays(self._h, xy.ctypes.data, len(xy), out.ctypes.data)
        return out

    def tree(self):
        n = self._L.ref_node_count(self._h)
        off = np.zeros(n + 1, np.int64)
        self._L.ref_tree_dump(self._h, None, None, off.ctypes.data, None)
        b = np.zeros((n, 6), np.float32)
        c = np.zeros((n, 2), np.int32)
        t = np.zeros(max(int(off[-1]), 1), np.int32)
        self._L.ref_tree_dump(self._h, b.ctypes.data, c.ctypes.data, off.ctypes.data, t.ctypes.data)
        return b, c, off, t[: int(off[-1])]

    def vertex_normals(self, n: int) -> np.ndarray:
        out = np.zeros((n, 3), np.float32)
        self._L.ref_vertex_normals(self._h, out.ctypes.data)
        return out

    def face_normals(self, n: int) -> np.ndarray:
        out = np.zeros((n, 3), np.float32)
        self._L.ref_face_normals(self._h, out.ctypes.data)
        return out

    def write_ppm(self, path: str, rgb: np.ndarray) -> None:
        rgb = np.ascontiguousarray(rgb, np.float32)
        self._L.ref_write_ppm(rgb.ctypes.data, rgb.shape[1], rgb.shape[0], str(path).encode())

    def __del__(self):
        try:
            self._L.ref_scene_destroy(self._h)
        except Exception:
            pass
