"""crt_hip_scene_from_tree: the drop-in path for a caller that already holds
the reference's built crt::Scene (vertex array after vertex_array_extend,
crt_mesh.cpp:32-73; tree after acceleration_tree::build,
crt_acceleration_tree.cpp:87-106).  The fixtures tests/golden/reftree_*.npz
are that data as the reference's own compiled TUs produced it
(tests/golden/make_reftree.py, oracle/ref_driver.cpp).

CPU: the flattened host scene equals the one built from the flat scene
description (same tree, bounds, leaf order, normals).  GPU: images and
per-ray hits from it are bit-equal to those from crt_hip_scene_create; the
compiled crt::render_image shim (csrc/shim/, built against the reference's
own headers into oracle/_ref/libshim_check.so) renders the same bits.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import GOLDEN, bits, hits_equal, scene_npz

SCENES = sorted(p.stem[len("reftree_"):] for p in GOLDEN.glob("reftree_*.npz"))


def tree_scene(name, w=None, h=None):
    from crt_amd.native import TreeScene
    sc = scene_npz(name)
    if w:
        sc.set_resolution(w, h)
    z = np.load(GOLDEN / f"reftree_{name}.npz")
    return sc, TreeScene(sc, z["vertices"], z["bounds"], z["children"], z["leaf_offsets"], z["leaf_triangles"])


@pytest.mark.parametrize("name", SCENES)
def test_host_scene_from_tree_equals_built(name):
    from crt_amd.native import HostScene
    sc, ts = tree_scene(name)
    a, b = HostScene(ts), HostScene(sc)
    ia, ib = a.info(), b.info()
    for k in ("node_count", "leaf_count", "leaf_ref_count", "max_depth", "max_leaf_size", "vertex_count",
              "triangle_count"):
        assert ia[k] == ib[k], k
    ta, tb = a.tree(), b.tree()
    for x, y in zip(ta[:3], tb[:3]):
        assert np.array_equal(bits(x), bits(y))
    # same triangle copy in every leaf slot (global ids may be numbered differently)
    fa, fb = a.face_normals(), b.face_normals()
    assert np.array_equal(bits(fa[ta[3]]), bits(fb[tb[3]]))
    assert np.array_equal(bits(a.vertex_normals()), bits(b.vertex_normals()))


def test_from_tree_rejects_malformed():
    from crt_amd.native import CrtError, HostScene, TreeScene
    sc = scene_npz("14-01-acceleration-tree__scene1")
    z = np.load(GOLDEN / "reftree_14-01-acceleration-tree__scene1.npz")
    bad = z["children"].copy()
    bad[0, 0] = 0                                  # a node as its own child
    with pytest.raises(CrtError):
        HostScene(TreeScene(sc, z["vertices"], z["bounds"], bad, z["leaf_offsets"], z["leaf_triangles"]))
    tris = z["leaf_triangles"].copy().view(np.int32).reshape(len(z["leaf_triangles"]), -1)
    tris[0, 0] = 10 ** 8                           # vertex index out of range
    with pytest.raises(CrtError):
        HostScene(TreeScene(sc, z["vertices"], z["bounds"], z["children"], z["leaf_offsets"], tris.view(np.uint8)))


@pytest.mark.gpu
@pytest.mark.parametrize("name", SCENES)
def test_render_from_tree_bit_equal(name):
    from crt_amd import native as N
    w, h = 240, 135
    sc, ts = tree_scene(name, w, h)
    over = {"max_ray_depth": 8} if "refractive" in name else {}
    st = N.RendererSettings.default(**over)
    want = N.HipScene(sc).render(st)
    got = N.HipScene(ts).render(st)
    assert np.array_equal(bits(got), bits(want))
    ys, xs = np.mgrid[0:h:5, 0:w:5]
    from oracle import pyoracle
    rays = pyoracle.OracleScene(sc).camera_rays(np.stack([xs.ravel(), ys.ravel()], 1))
    ok, first, nbad = hits_equal(N.HipScene(ts).trace(rays), N.HipScene(sc).trace(rays), with_tri=False)
    assert ok, f"{nbad} rays differ (first {first})"


@pytest.mark.gpu
def test_render_image_shim(tmp_path):
    """crt::render_image (csrc/shim/crt_render_image_hip.cpp, compiled against
    the reference's crt_renderer.h / crt_scene.h) called on a crt::Scene that
    the reference's own TUs built (vertex_array_extend, acceleration_tree::build,
    Camera) returns the image crt_hip_render gives for the flat description."""
    from crt_amd import native as N
    from oracle.pyoracle import ORACLE_DIR
    path = ORACLE_DIR / "_ref" / "libshim_check.so"
    if not path.exists():
        pytest.skip("oracle/_ref/libshim_check.so not built (needs /root/reference at build time)")
    N.lib()
    L = C.CDLL(str(path))
    L.shim_check_render.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.shim_check_render.restype = C.c_int
    for name, over in [("14-01-acceleration-tree__scene1", {}), ("11-01-refractive__scene8", {"max_ray_depth": 8}),
                       ("15-01-conclusion__scene2", {}), ("12-01-textures__scene4", {})]:
        sc = scene_npz(name).set_resolution(200, 120)
        st = N.RendererSettings.default(**over)
        want = N.HipScene(sc).render(st)
        got = np.zeros_like(want)
        assert L.shim_check_render(C.addressof(sc.desc()), C.addressof(st), got.ctypes.data) == 0, name
        assert np.array_equal(bits(got), bits(want)), name


@pytest.mark.gpu
def test_render_image_tree_core(oracle):
    """The shim's body (csrc/shim/crt_shim_core.cpp, in lib/libcrt_hip.so):
    crt::render_image on the reference's built Scenes (tests/golden/reftree_*)
    renders the oracle's bits; the same Scene again reuses its cached device
    scene; the Scene with only its camera moved moves the cached scene's
    camera (no new device scene) and renders the moved camera's bits; two
    other scenes fill the two-entry cache and evict the first."""
    from crt_amd import native as N
    from crt_amd.camera import orbit_poses
    lib = N.lib()
    lib.crt_hip_render_image_tree_reset()
    name = "14-01-acceleration-tree__scene1"
    st = N.RendererSettings.default()
    sc, ts = tree_scene(name, 240, 135)
    want = bits(oracle.OracleScene(sc).render(st))
    s0 = N.render_image_tree_stats()
    assert np.array_equal(bits(N.render_image_tree(ts, st)), want)
    assert np.array_equal(bits(N.render_image_tree(ts, st)), want)
    s1 = N.render_image_tree_stats()
    assert s1["creates"] - s0["creates"] == 1 and s1["reuses"] - s0["reuses"] == 1
    fov = np.float32(np.float32(sc.desc().camera.fov_degrees) * np.float32(np.pi)) / np.float32(180.0)
    for loc, rot in orbit_poses(sc.a, 5)[1:]:
        sc.set_camera(location=loc, rotation=rot)
        ts.set_camera(location=loc, rotation=rot, fov_radians=fov)
        assert np.array_equal(bits(N.render_image_tree(ts, st)), bits(oracle.OracleScene(sc).render(st)))
    ts.set_resolution(200, 160)
    sc.set_resolution(200, 160)
    assert np.array_equal(bits(N.render_image_tree(ts, st)), bits(oracle.OracleScene(sc).render(st)))
    s2 = N.render_image_tree_stats()
    assert s2["creates"] == s1["creates"] and s2["camera_moves"] - s1["camera_moves"] == 5
    for other in [n for n in SCENES if n != name][:2]:
        sc2, ts2 = tree_scene(other, 160, 90)
        st2 = N.RendererSettings.default(**({"max_ray_depth": 8} if "refractive" in other else {}))
        assert np.array_equal(bits(N.render_image_tree(ts2, st2)), bits(oracle.OracleScene(sc2).render(st2)))
    assert np.array_equal(bits(N.render_image_tree(ts, st)), bits(oracle.OracleScene(sc).render(st)))
    assert N.render_image_tree_stats()["creates"] - s2["creates"] == 3   # the first scene was evicted
    lib.crt_hip_render_image_tree_reset()


@pytest.mark.gpu
def test_render_image_tree_same_shape_other_content():
    """A Scene with the cached one's shape (counts, materials, lights) but other
    content in one of its large arrays: the cached scene is rendered while the
    arrays are compared on the copy's host threads (crt_shim_core.cpp
    slice_same); the difference must be found in any slice (first and last
    float of the vertices, a leaf triangle's normal in the middle, a node
    bound) and the new content rendered from a new device scene."""
    from crt_amd import native as N
    lib = N.lib()
    lib.crt_hip_render_image_tree_reset()
    name = "14-01-acceleration-tree__scene1"
    st = N.RendererSettings.default()
    z = np.load(GOLDEN / f"reftree_{name}.npz")
    sc = scene_npz(name).set_resolution(320, 180)

    def ts_of(vertices=None, bounds=None, tris=None):
        return N.TreeScene(sc, z["vertices"] if vertices is None else vertices, z["bounds"] if bounds is None else bounds,
                           z["children"], z["leaf_offsets"], z["leaf_triangles"] if tris is None else tris)

    base = ts_of()
    N.render_image_tree(base, st)
    v0 = z["vertices"].copy().reshape(-1)
    v0[0] = np.float32(v0[0] + 0.5)                   # first slice: vertex 0's x
    v1 = z["vertices"].copy().reshape(-1)
    v1[-3 - 2] = np.float32(-v1[-3 - 2])              # last slice: a vertex normal component
    tr = z["leaf_triangles"].copy()
    raw = tr.view(np.uint8).reshape(len(tr), -1)
    mid = len(tr) // 2
    fn = raw[mid, 12:16].view(np.float32)
    fn[0] = np.float32(-fn[0])                        # a face normal in the middle
    b = z["bounds"].copy()
    b.reshape(-1)[-1] = np.float32(b.reshape(-1)[-1] + 1.0)
    for k, ts in enumerate([ts_of(vertices=v0), ts_of(vertices=v1), ts_of(tris=tr), ts_of(bounds=b)]):
        s0 = N.render_image_tree_stats()
        got = N.render_image_tree(ts, st)
        s1 = N.render_image_tree_stats()
        assert s1["creates"] - s0["creates"] == 1, f"case {k}: the changed content was not found"
        want = N.HipScene(ts).render(st)
        assert np.array_equal(bits(got), bits(want)), f"case {k}"
        assert np.array_equal(bits(N.render_image_tree(ts, st)), bits(want)), f"case {k} repeat"
        assert N.render_image_tree_stats()["reuses"] - s1["reuses"] == 1
    lib.crt_hip_render_image_tree_reset()


def test_render_image_shim_builds_against_reference_headers():
    """The shim compiles against the reference's crt_renderer.h / crt_scene.h
    and links with its TUs (oracle/Makefile `shim`, run by build())."""
    from conftest import has_reference
    from oracle.pyoracle import ORACLE_DIR
    path = ORACLE_DIR / "_ref" / "libshim_check.so"
    if not has_reference():
        pytest.skip("needs /root/reference")
    assert path.exists()
    import subprocess
    syms = subprocess.run(["nm", "-DC", str(path)], capture_output=True, text=True, check=True).stdout
    assert "crt::render_image(crt::Scene const&, crt::RendererSettings const&)" in syms
    assert "crt_hip_render_image_tree" in syms and "shim_check_render" in syms
