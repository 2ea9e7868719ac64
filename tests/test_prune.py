"""The pruned walks' correctness argument, checked on the CPU.

tests/tools/prune_sim.cpp runs the product's per-ray pruned walk
(crt_device.h walk_pruned over the octant-ordered PNode arrays that
crt_scene_build.cpp builds) next to the reference-order walk
(crt_intersection.cpp:109-136), from the same sources the HIP library is
compiled from.  The bar is exact: the same winning slot (reference visit-order
numbering) and the same t bits for every ray, including rays built to stress
the hull margins (grazing rays nearly in a triangle's plane, rays through
vertices and edges, origins on surfaces as secondary rays have).
"""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import ROOT, scene_npz

TOOLS = ROOT / "tests" / "tools"
SIM = TOOLS / "_build" / "libprune_sim.so"
_P = C.c_void_p


@pytest.fixture(scope="module")
def sim():
    subprocess.run(["make", "-s", "-C", str(TOOLS)], check=True)
    L = C.CDLL(str(SIM))
    L.prune_sim_trace.argtypes = [_P, _P, C.c_int64, _P, _P, _P, _P, _P]
    L.prune_sim_trace.restype = C.c_int
    L.prune_sim_check_hulls.argtypes = [_P]
    L.prune_sim_check_hulls.restype = C.c_int64
    return L


def run(sim, sc, rays):
    from crt_amd.native import _desc_ptr
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    n = len(rays)
    rs, rt = np.zeros(n, np.int32), np.zeros(n, np.float32)
    ps, pt = np.zeros(n, np.int32), np.zeros(n, np.float32)
    cnt = np.zeros(4, np.uint64)
    rc = sim.prune_sim_trace(C.cast(_desc_ptr(sc), _P), rays.ctypes.data, n, rs.ctypes.data, rt.ctypes.data,
                             ps.ctypes.data, pt.ctypes.data, cnt.ctypes.data)
    assert rc == 0
    return rs, rt, ps, pt, cnt


def assert_same(rs, rt, ps, pt, label):
    bad = np.flatnonzero((rs != ps) | (rt.view(np.uint32) != pt.view(np.uint32)))
    assert len(bad) == 0, f"{label}: {len(bad)} rays differ, first {bad[0]}: ref ({rs[bad[0]]}, {rt[bad[0]]}) " \
                          f"pruned ({ps[bad[0]]}, {pt[bad[0]]})"


def stress_rays(sc, n, seed):
    """Rays aimed at points on triangles (interior, edges, vertices), from
    near-grazing to head-on directions, plus origins on the surfaces."""
    from crt_amd.native import HostScene
    hs = HostScene(sc)
    fnorm = hs.face_normals().reshape(-1, 3)
    d = sc.desc()
    pos, idx = [], []
    base = 0
    for m in range(d.mesh_count):
        md = d.meshes[m]
        p = np.ctypeslib.as_array(md.positions, (md.vertex_count * 3,)).reshape(-1, 3).astype(np.float32)
        ii = np.ctypeslib.as_array(md.indices, (md.index_count,)).reshape(-1, 3)
        pos.append(p)
        idx.append(ii + base)
        base += len(p)
    P = np.concatenate(pos)
    I = np.concatenate(idx)
    rng = np.random.default_rng(seed)
    tri = rng.integers(0, len(I), n)
    bary = rng.dirichlet((1.0, 1.0, 1.0), n).astype(np.float32)
    # a third on edges / vertices exactly
    k = n // 3
    bary[:k // 2, rng.integers(0, 3)] = 0.0
    bary[k // 2:k] = np.eye(3, dtype=np.float32)[rng.integers(0, 3, k - k // 2)]
    bary /= bary.sum(1, keepdims=True)
    v = P[I[tri]]                                  # n, 3, 3
    target = np.einsum("nk,nkc->nc", bary, v).astype(np.float32)
    N = fnorm[tri]
    e = v[:, 1] - v[:, 0]
    e /= np.maximum(np.linalg.norm(e, axis=1, keepdims=True), 1e-30)
    eps = np.float32(10.0) ** rng.uniform(-7, 0, n).astype(np.float32)
    sgn = np.where(rng.random(n) < 0.5, -1.0, 1.0).astype(np.float32)
    dirs = e + (sgn * eps)[:, None] * N
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    dist = np.float32(10.0) ** rng.uniform(-3, 1, n).astype(np.float32)
    o = target - dirs * dist[:, None]
    grazing = np.concatenate([o, dirs], 1)
    # secondary-like: origin on a surface point, random direction
    rd = rng.normal(size=(n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    surface = np.concatenate([target, rd], 1)
    return np.concatenate([grazing, surface], 0).astype(np.float32)


SCENES = [
    ("14-01-acceleration-tree__scene1", 160, 90),
    ("11-01-refractive__scene8", 120, 68),
    ("15-01-conclusion__scene2", 96, 96),
    ("09-02-diffuse-smooth-shading__scene2", 96, 54),
    ("13-01-optimizations__scene0", 96, 54),
]


@pytest.mark.parametrize("name,w,h", SCENES)
def test_pruned_walk_exact(sim, oracle, name, w, h):
    sc = scene_npz(name).set_resolution(w, h)
    assert sim.prune_sim_check_hulls(C.cast(sc.desc_ptr(), _P)) == 0
    orc = oracle.OracleScene(sc)
    ys, xs = np.mgrid[0:h, 0:w]
    cam = orc.camera_rays(np.stack([xs.ravel(), ys.ravel()], 1))
    rng = np.random.default_rng(3)
    o = rng.uniform(-10, 10, (4000, 3)).astype(np.float32)
    d = rng.normal(size=(4000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([cam, np.concatenate([o, d], 1), stress_rays(sc, 6000, 11)], 0)
    rs, rt, ps, pt, cnt = run(sim, sc, rays)
    assert_same(rs, rt, ps, pt, name)
    assert (rs >= 0).sum() > 0
    # the reference-order walk here agrees with the oracle's own trace
    ref_hits, _, _ = orc.trace(rays[:2000])
    assert np.array_equal(ref_hits["hit"].astype(bool), rs[:2000] >= 0)
    assert cnt[2] <= cnt[0] and cnt[3] <= cnt[1]


def test_pruned_walk_exact_synthetic(sim, oracle):
    from crt_amd.synthetic import c5_scene
    sc = c5_scene(20_000, 64, 36)
    orc = oracle.OracleScene(sc)
    ys, xs = np.mgrid[0:36, 0:64]
    cam = orc.camera_rays(np.stack([xs.ravel(), ys.ravel()], 1))
    rays = np.concatenate([cam, stress_rays(sc, 4000, 5)], 0)
    rs, rt, ps, pt, cnt = run(sim, sc, rays)
    assert_same(rs, rt, ps, pt, "c5-20k")
    n = len(cam)
    _, _, _, _, c_cam = run(sim, sc, cam)
    # deep random mesh: most of the reference's tests are behind the first hit
    assert c_cam[2] * 2 < c_cam[0] and c_cam[3] * 2 < c_cam[1], c_cam / n


def test_far_origin_disables_pruning(sim):
    """Rays from beyond 4x the scene's coordinate range get no pruning (the hull
    margins are only proven below it) and stay exact."""
    from crt_amd.synthetic import c5_scene
    sc = c5_scene(2_000, 16, 16)
    rng = np.random.default_rng(9)
    o = np.tile(np.array([[0.0, 0.0, 50.0]], np.float32), (500, 1))
    d = (rng.uniform(-0.01, 0.01, (500, 3)) + [0, 0, -1]).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rs, rt, ps, pt, cnt = run(sim, sc, np.concatenate([o, d], 1))
    assert_same(rs, rt, ps, pt, "far")
    assert cnt[2] == cnt[0] and cnt[3] == cnt[1]
