"""tests/golden/reftree_<scene>.npz: the reference's own built crt::Scene
geometry — its vertex array after vertex_array_extend (crt_mesh.cpp:32-73) and
its acceleration tree after acceleration_tree::build (crt_acceleration_tree.cpp:
87-106), dumped by oracle/_ref/libref.so (the reference's TUs compiled in
place, oracle/ref_driver.cpp).  Input of crt_hip_scene_from_tree in the tests:
rendering from it must equal rendering from the flat scene description.
Runs only where /root/reference exists; commits only data."""
from __future__ import annotations

import ctypes as C
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
sys.path.insert(0, str(ROOT))

from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

SCENES = ["14-01-acceleration-tree__scene1", "11-01-refractive__scene8", "15-01-conclusion__scene2",
          "12-01-textures__scene4"]


def dump(name: str) -> dict:
    sc = load_npz(HERE / "scenes" / f"{name}.npz")
    ref = O.RefScene(sc)
    L = O.ref_lib()
    L.ref_vertex_count.restype = C.c_int64
    L.ref_vertex_count.argtypes = [C.c_void_p]
    L.ref_vertex_dump.argtypes = [C.c_void_p, C.c_void_p]
    L.ref_leaf_triangles.argtypes = [C.c_void_p, C.c_void_p]
    b, c, off, _ = ref.tree()
    nv = L.ref_vertex_count(ref._h)
    verts = np.zeros((nv, 9), np.float32)
    L.ref_vertex_dump(ref._h, verts.ctypes.data)
    tris = np.zeros(int(off[-1]), N.TREE_TRI_DTYPE)
    L.ref_leaf_triangles(ref._h, tris.ctypes.data)
    return {"vertices": verts, "bounds": b, "children": c, "leaf_offsets": off,
            "leaf_triangles": tris.view(np.uint8).reshape(len(tris), -1)}


def main():
    for name in SCENES:
        out = HERE / f"reftree_{name}.npz"
        np.savez_compressed(out, **dump(name))
        print(out, out.stat().st_size)


if __name__ == "__main__":
    main()
