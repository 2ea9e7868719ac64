"""The device-built BVH (crt_lbvh.hip) of scenes above 2^18 triangles: its
records hold the host build's contract (crt_bvh_build.cpp: every triangle
once, leaves of at most two, skip links of a preorder, each box holding its
children's boxes and its triangles), and the walks over it return the
reference's hits — C5's 1M-triangle mesh rendered bit for bit against the
oracle (test_gpu_configs.py::test_c5_1m_triangles) and scattered rays traced
through it equal to the reference-order walk's hits (crt_intersection.cpp:
109-136)."""
import numpy as np
import pytest

from conftest import hits_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    from crt_amd import native
    native.lib()
    return native


@pytest.fixture(scope="module")
def c5_small():
    from crt_amd.synthetic import c5_scene
    return c5_scene(1_000_000, 64, 36)


@pytest.fixture(scope="module")
def c5_gpu(N, c5_small):
    return N.HipScene(c5_small)


def test_lbvh_records(N, c5_gpu):
    from crt_amd.synthetic import c5_mesh
    info = c5_gpu.info()
    assert info["bvh_on_device"] == 1 and info["bvh_depth"] > 0
    nodes, ids = c5_gpu.bvh()
    nt = info["triangle_count"]
    tri = ids & 0x7FFFFFFF
    assert np.array_equal(np.sort(tri), np.arange(nt)), "leaf order is not a permutation of the triangles"
    verts, _ = c5_mesh(1_000_000)
    v = verts.reshape(-1, 3, 3)[tri]                     # triangles in leaf order
    vlo, vhi = v.min(axis=1), v.max(axis=1)
    n = nodes.shape[1] - 1
    leaf_sets = []
    for o in range(8):
        a = nodes[o]
        assert a[n]["skip"] == 0 and a[n]["leaf"] == 0     # the zero record after the order
        a = a[:n]
        k = np.arange(n)
        skip, leaf = a["skip"], a["leaf"]
        inner = leaf == 0
        assert np.all(skip > k) and np.all(skip <= n) and skip[0] == n
        assert np.all(skip[~inner] == k[~inner] + 1), "a leaf's skip is its successor"
        c1 = k[inner] + 1                                   # first child
        c2 = skip[c1]                                       # second child
        assert np.all(c2 < skip[inner]) and np.all(skip[c2] == skip[inner]), "children do not tile the subtree"
        for c in (c1, c2):
            for ax in "xyz":
                assert np.all(a[f"lo_{ax}"][c] >= a[f"lo_{ax}"][inner]), f"order {o}: child box outside ({ax})"
                assert np.all(a[f"hi_{ax}"][c] <= a[f"hi_{ax}"][inner]), f"order {o}: child box outside ({ax})"
        first, cnt = leaf[~inner] >> 4, leaf[~inner] & 15
        assert np.all((cnt >= 1) & (cnt <= 2))
        order = np.argsort(first)
        f, c = first[order], cnt[order]
        assert f[0] == 0 and np.all(f[1:] == f[:-1] + c[:-1]) and f[-1] + c[-1] == nt, "leaves do not cover once"
        # every leaf box holds its triangles' vertices (the hulls are wider still)
        lk = k[~inner]
        for j in range(2):
            m = cnt > j
            t = first[m] + j
            for q, ax in enumerate("xyz"):
                assert np.all(a[f"lo_{ax}"][lk[m]] <= vlo[t, q]) and np.all(a[f"hi_{ax}"][lk[m]] >= vhi[t, q])
        leaf_sets.append(np.sort(leaf[~inner]))
    for s in leaf_sets[1:]:
        assert np.array_equal(s, leaf_sets[0]), "the octant orders hold different leaves"


def test_lbvh_scattered_rays_equal_reference_walk(N, c5_small):
    """Rays from inside and around the cloud in every direction, traced
    through the device BVH + proof (trace_walk 2) and through the reference's
    own node order (trace_walk 0): same hits, bit for bit."""
    rng = np.random.default_rng(7)
    n = 4096
    o = rng.uniform(-1.3, 1.3, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], axis=1).astype(np.float32)
    got = N.HipScene(c5_small, trace_walk=2).trace(rays)
    want = N.HipScene(c5_small, trace_walk=0).trace(rays)
    ok, first, nbad = hits_equal(got, want)
    assert ok, f"{nbad} rays differ (first {first}: bvh={got[first]} ref={want[first]})"
    assert int(got["hit"].sum()) > n // 4


def test_lbvh_off_keeps_kd_walk(N, c5_small):
    """Create flag CRT_SCENE_NO_DEVICE_BVH: no device BVH (the pruned kd walks,
    as before); the frame is the same bits either way."""
    g0 = N.HipScene(c5_small, create_flags=N.SCENE_NO_DEVICE_BVH)
    assert g0.info()["bvh_on_device"] == 0 and g0.bvh() is None
    st = N.RendererSettings.default()
    a = g0.render(st)
    b = N.HipScene(c5_small).render(st)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))

