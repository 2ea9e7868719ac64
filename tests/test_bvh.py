"""The secondary-ray BVH walk (crt_bvh.h), checked on the CPU.

tests/tools/prune_sim.cpp runs the product's trace_bvh_exact — closest hit
over all triangles through the BVH, then the proof on the reference's tree
that the reference reaches a copy of that triangle, else the exact pruned kd
walk — next to the reference-order walk (crt_intersection.cpp:109-136), from
the same sources the HIP library compiles.  The bar is exact: the same
triangle and the same t bits for every ray (the copy the two walks report may
differ; copies of a triangle give the same Intersection record).
"""
import ctypes as C

import numpy as np
import pytest

from conftest import scene_npz
from test_prune import SCENES, sim, stress_rays  # noqa: F401  (fixture)

_P = C.c_void_p


def bvh_run(sim, sc, rays):  # noqa: F811
    from crt_amd.native import _desc_ptr
    sim.bvh_sim_trace.argtypes = [_P, _P, C.c_int64, _P, _P, _P, _P, _P]
    sim.bvh_sim_trace.restype = C.c_int
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    n = len(rays)
    rs, rt = np.zeros(n, np.int32), np.zeros(n, np.float32)
    bs, bt = np.zeros(n, np.int32), np.zeros(n, np.float32)
    cnt = np.zeros(5, np.uint64)
    rc = sim.bvh_sim_trace(C.cast(_desc_ptr(sc), _P), rays.ctypes.data, n, rs.ctypes.data, rt.ctypes.data,
                           bs.ctypes.data, bt.ctypes.data, cnt.ctypes.data)
    assert rc == 0
    return rs, rt, bs, bt, cnt


def assert_same_tri(rs, rt, bs, bt, label):
    bad = np.flatnonzero((rs != bs) | (rt.view(np.uint32) != bt.view(np.uint32)))
    assert len(bad) == 0, f"{label}: {len(bad)} rays differ, first {bad[0]}: ref ({rs[bad[0]]}, {rt[bad[0]]!r}) " \
                          f"bvh ({bs[bad[0]]}, {bt[bad[0]]!r})"


def bounce_rays(sim, sc, rays, seed, per_hit=2):  # noqa: F811
    """Secondary rays as GI makes them: from each hit point p + n * 1e-2 in a
    random direction of the normal's hemisphere."""
    from crt_amd.native import HostScene
    rs, rt, _, _, _ = bvh_run(sim, sc, rays)
    hit = rs >= 0
    o, d, t = rays[hit, :3], rays[hit, 3:], rt[hit]
    fn = HostScene(sc).face_normals().reshape(-1, 3)[rs[hit]]
    p = o + d * t[:, None]
    n = np.where((np.einsum("ij,ij->i", fn, d) > 0)[:, None], -fn, fn).astype(np.float32)
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(per_hit):
        r = rng.normal(size=p.shape).astype(np.float32)
        r /= np.linalg.norm(r, axis=1, keepdims=True)
        r = np.where((np.einsum("ij,ij->i", r, n) < 0)[:, None], -r, r)
        out.append(np.concatenate([p + n * np.float32(1e-2), r], 1))
    return np.concatenate(out, 0).astype(np.float32)


@pytest.mark.parametrize("name,w,h", SCENES)
def test_bvh_walk_exact(sim, oracle, name, w, h):  # noqa: F811
    from crt_amd.native import _desc_ptr
    sc = scene_npz(name).set_resolution(w, h)
    sim.bvh_sim_check.argtypes = [_P]
    sim.bvh_sim_check.restype = C.c_int64
    assert sim.bvh_sim_check(C.cast(_desc_ptr(sc), _P)) == 0
    orc = oracle.OracleScene(sc)
    ys, xs = np.mgrid[0:h, 0:w]
    cam = orc.camera_rays(np.stack([xs.ravel(), ys.ravel()], 1))
    rng = np.random.default_rng(3)
    o = rng.uniform(-10, 10, (4000, 3)).astype(np.float32)
    d = rng.normal(size=(4000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    b1 = bounce_rays(sim, sc, cam, 1)
    b2 = bounce_rays(sim, sc, b1, 2, per_hit=1)
    rays = np.concatenate([cam, np.concatenate([o, d], 1), stress_rays(sc, 6000, 11), b1, b2], 0)
    rs, rt, bs, bt, cnt = bvh_run(sim, sc, rays)
    assert_same_tri(rs, rt, bs, bt, name)
    assert (rs >= 0).sum() > 0
    # on camera rays and bounces the fallback is the exception (ties between
    # triangles: rays through shared edges; the stress rays aim at edges and
    # vertices on purpose), and the BVH tests far fewer triangles
    _, _, _, _, cb = bvh_run(sim, sc, np.concatenate([cam, b1, b2], 0))
    assert cb[4] < 0.01 * (len(cam) + len(b1) + len(b2)), cb
    assert cb[3] * 2 < cb[1], cb


def test_bvh_walk_exact_synthetic(sim):  # noqa: F811
    from crt_amd.synthetic import c5_scene
    sc = c5_scene(20_000, 64, 36)
    rays = stress_rays(sc, 4000, 5)
    rays = np.concatenate([rays, bounce_rays(sim, sc, rays, 4)], 0)
    rs, rt, bs, bt, cnt = bvh_run(sim, sc, rays)
    assert_same_tri(rs, rt, bs, bt, "c5-20k")


def test_bvh_far_and_nan_rays(sim):  # noqa: F811
    """Far origins (no pruning: the hull margins are only proven below 4x the
    scene's coordinate range) and rays with NaN components (the reference
    misses: every face test reads a NaN) stay exact."""
    from crt_amd.synthetic import c5_scene
    sc = c5_scene(2_000, 16, 16)
    rng = np.random.default_rng(9)
    o = np.tile(np.array([[0.0, 0.0, 50.0]], np.float32), (500, 1))
    d = (rng.uniform(-0.01, 0.01, (500, 3)) + [0, 0, -1]).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    far = np.concatenate([o, d], 1)
    nan = far[:6].copy()
    for k in range(6):
        nan[k, k] = np.nan
    rs, rt, bs, bt, _ = bvh_run(sim, sc, np.concatenate([far, nan], 0))
    assert_same_tri(rs, rt, bs, bt, "far+nan")
    assert (rs[-6:] == -1).all()


@pytest.mark.parametrize("name,w,h", SCENES)
def test_topology_proof_equals_descent(sim, oracle, name, w, h):  # noqa: F811
    """verify_topo (8-B topology records, child cells as the parent's halves
    computed in registers) proves exactly what verify_kd (the 32-B node
    descent) proves: same slot or -1 and the same node tests, ray for ray."""
    from crt_amd.native import _desc_ptr
    sc = scene_npz(name).set_resolution(w, h)
    ys, xs = np.mgrid[0:h, 0:w]
    cam = oracle.OracleScene(sc).camera_rays(np.stack([xs.ravel(), ys.ravel()], 1))
    b1 = bounce_rays(sim, sc, cam, 1)
    rays = np.ascontiguousarray(np.concatenate([cam, b1, stress_rays(sc, 4000, 13)], 0), np.float32)
    sim.bvh_sim_proof_check.argtypes = [_P, _P, C.c_int64, _P]
    sim.bvh_sim_proof_check.restype = C.c_int
    out = np.zeros(3, np.uint64)
    assert sim.bvh_sim_proof_check(C.cast(_desc_ptr(sc), _P), rays.ctypes.data, len(rays), out.ctypes.data) == 0
    assert out[0] > 0 and out[1] == 0, out
    assert out[2] > 0.95 * out[0], out


BINS_CASES = [("14-01-acceleration-tree__scene1", None), ("14-01-acceleration-tree__scene0", None),
              ("12-01-textures__scene4", None), ("09-02-diffuse-smooth-shading__scene3", None),
              ("11-01-refractive__scene0", None), ("11-01-refractive__scene8", None),
              ("15-01-conclusion__scene2", None), ("14-01-acceleration-tree__scene1", (333, 177)),
              ("15-01-conclusion__scene2", (1001, 643))]


@pytest.mark.parametrize("name,size", BINS_CASES)
def test_camera_bins_equal_bvh_walk(sim, name, size):  # noqa: F811
    """Camera bins (crt_bvh_build.cpp build_camera_bins, crt_bvh.h walk_bins):
    every camera ray of the frame gets the BVH walk's t bits and tie flag, and
    its triangle where there is no tie — so the proof and the fallback, shared
    with the BVH walk (resolve_closest), see the same inputs."""
    from crt_amd.native import _desc_ptr
    sc = scene_npz(name)
    if size:
        sc = sc.set_resolution(*size)
    sim.bins_sim_check.argtypes = [_P, _P]
    sim.bins_sim_check.restype = C.c_int
    out = np.zeros(7, np.uint64)
    assert sim.bins_sim_check(C.cast(_desc_ptr(sc), _P), out.ctypes.data) == 0
    rays, diff, tested, _, _, cands, built = (int(x) for x in out)
    assert built == 1
    assert rays > 0 and diff == 0, f"{name}: {diff} of {rays} camera rays differ"
    assert tested < 8 * rays   # the lists are short: a few candidates per ray


@pytest.mark.parametrize("name,size", BINS_CASES)
def test_camera_bins_lanes_equal_serial_walk(sim, name, size):  # noqa: F811
    """K lanes per pixel on one cell's list (crt_walks.h trace_bins_lanes, the
    split 4x4 waves of camera-bins frames), restated on the host with the
    device's schedule (positions j = lane mod K, one record per lane per
    round, the bound shared after every round, then the merge): the same hit,
    t bits and tie flag as the serial walk_bins on every camera ray, and the
    same triangle where there is no tie."""
    from crt_amd.native import _desc_ptr
    sc = scene_npz(name)
    if size:
        sc = sc.set_resolution(*size)
    sim.bins_sim_lanes_check.argtypes = [_P, C.c_int, _P]
    sim.bins_sim_lanes_check.restype = C.c_int
    for k in (4, 2):
        out = np.zeros(3, np.uint64)
        assert sim.bins_sim_lanes_check(C.cast(_desc_ptr(sc), _P), k, out.ctypes.data) == 0
        rays, diff, _shared = (int(x) for x in out)
        assert rays > 0 and diff == 0, f"{name} K={k}: {diff} of {rays} camera rays differ"
