"""Light bins (crt_light_bins.cpp, crt_bvh.h occluded_lbins), checked on the CPU.

tests/tools/prune_sim.cpp lbins_sim_check builds the product's light bins
for every light of a scene and answers shadow rays with them — occluded (the
first hit within the light, proved on the reference's tree), lit, or
undecided (the BVH then decides) — next to the reference-order closest hit
(crt_intersection.cpp:109-136; a light is occluded when that hit has
fl(t * t) <= |light - p|^2, crt_renderer.cpp:90-92).  The bar: every decided
answer equals the reference's; rays the bins are built for (bias within
e_max) are decided almost always.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import scene_npz
from test_bvh import bvh_run
from test_prune import sim, stress_rays  # noqa: F401  (fixture)

_P = C.c_void_p


def lbins_run(sim, sc, rays, e_max=0.02, n=64):  # noqa: F811
    from crt_amd.native import _desc_ptr
    sim.lbins_sim_check.argtypes = [_P, _P, C.c_int64, C.c_double, C.c_int, _P, _P, _P]
    sim.lbins_sim_check.restype = C.c_int
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    k = len(rays)
    ref, lb = np.zeros(k, np.int8), np.zeros(k, np.int8)
    info = np.zeros(4, np.int64)
    rc = sim.lbins_sim_check(C.cast(_desc_ptr(sc), _P), rays.ctypes.data, k, e_max, n, ref.ctypes.data,
                             lb.ctypes.data, info.ctypes.data)
    assert rc == 0
    return ref, lb, info


def shadow_rays(points, normals, lights, bias, rng):
    """Per point and light: o = p + n bias, d = normalize(L - p), r2 = |L - p|^2
    in fp32 as the renderer forms them (crt_shade.h diffuse_finish)."""
    out = []
    for li, L in enumerate(lights):
        ld = (L[None, :] - points).astype(np.float32)
        r2 = np.einsum("ij,ij->i", ld, ld).astype(np.float32)
        d = (ld / np.sqrt(r2)[:, None]).astype(np.float32)
        b = bias if np.ndim(bias) else np.full(len(points), bias, np.float32)
        o = (points + normals * b[:, None]).astype(np.float32)
        out.append(np.concatenate([o, d, r2[:, None], np.full((len(points), 1), li, np.float32)], 1))
    return np.concatenate(out, 0).astype(np.float32)


def scene_lights(sc):
    if not hasattr(sc, "a"):   # crt_amd.synthetic scenes: one light at (2, 2, 3)
        return np.array([[2.0, 2.0, 3.0]], np.float32)
    return np.asarray(sc.a["lights"], np.float32).reshape(-1, 4)[:, 1:4]


def camera_hits(sim, sc, oracle, w, h):  # noqa: F811
    from crt_amd.native import HostScene
    orc = oracle.OracleScene(sc)
    ys, xs = np.mgrid[0:h, 0:w]
    cam = orc.camera_rays(np.stack([xs.ravel(), ys.ravel()], 1))
    rs, rt, _, _, _ = bvh_run(sim, sc, cam)
    hit = rs >= 0
    p = (cam[hit, :3] + cam[hit, 3:] * rt[hit, None]).astype(np.float32)
    fn = HostScene(sc).face_normals().reshape(-1, 3)[rs[hit]]
    return p, fn.astype(np.float32)


SCENES = [
    ("14-01-acceleration-tree__scene1", 160, 90),
    ("09-02-diffuse-smooth-shading__scene2", 96, 54),
    ("13-01-optimizations__scene0", 96, 54),
    ("15-01-conclusion__scene2", 96, 96),
    ("11-01-refractive__scene8", 120, 68),
]


@pytest.mark.parametrize("name,w,h", SCENES)
def test_light_bins_shadow_rays(sim, oracle, name, w, h):  # noqa: F811
    """Shadow rays of the camera's hit points (bias 1e-2 along the face normal
    either way, and random biases up to past e_max) plus rays from random
    points on triangles: decided answers equal the reference's."""
    sc = scene_npz(name).set_resolution(w, h)
    lights = scene_lights(sc)
    if len(lights) == 0:
        pytest.skip("no lights")
    rng = np.random.default_rng(5)
    p, fn = camera_hits(sim, sc, oracle, w, h)
    sgn = np.where(rng.random(len(p)) < 0.8, 1.0, -1.0).astype(np.float32)[:, None]
    main = shadow_rays(p, fn * sgn, lights, np.float32(1e-2), rng)
    sr = stress_rays(sc, 2000, 17)[2000:]          # origins on triangles (interior, edges, vertices)
    q = sr[:, :3]
    nq = rng.normal(size=q.shape).astype(np.float32)
    nq /= np.linalg.norm(nq, axis=1, keepdims=True)
    odd = shadow_rays(q, nq, lights, rng.uniform(0, 0.03, len(q)).astype(np.float32), rng)
    rays = np.concatenate([main, odd], 0)
    ref, lb, info = lbins_run(sim, sc, rays)
    dec = lb >= 0
    bad = np.flatnonzero(dec & (lb != ref))
    assert len(bad) == 0, f"{name}: {len(bad)} shadow rays differ, first {rays[bad[0]]} ref {ref[bad[0]]}"
    assert info[1] > 0, "no light took bins"
    nm = len(main)
    assert dec[:nm].mean() > 0.97, dec[:nm].mean()
    assert ref[dec].min() == 0 or ref.mean() > 0.99   # both answers occur (or the scene is all dark)


def test_light_bins_near_light(sim):  # noqa: F811
    """Rays from points close to a light (within and around R0: the near list,
    origins nearer than R0, ends past the light) and rays aimed past it."""
    from crt_amd.synthetic import c5_scene
    sc = scene_npz("14-01-acceleration-tree__scene1")
    lights = scene_lights(sc)
    rng = np.random.default_rng(9)
    rows = []
    for li, L in enumerate(lights):
        for scale in (0.05, 0.3, 1.0, 1.5, 3.0, 8.0):
            dirs = rng.normal(size=(3000, 3)).astype(np.float32)
            dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
            p = (L[None, :] + dirs * np.float32(scale) * rng.uniform(0.5, 1.5, (3000, 1))).astype(np.float32)
            n = rng.normal(size=p.shape).astype(np.float32)
            n /= np.linalg.norm(n, axis=1, keepdims=True)
            r = shadow_rays(p, n, L[None, :], rng.uniform(0, 0.025, len(p)).astype(np.float32), rng)
            r[:, 7] = li
            rows.append(r)
    rays = np.concatenate(rows, 0)
    ref, lb, info = lbins_run(sim, sc, rays)
    bad = np.flatnonzero((lb >= 0) & (lb != ref))
    assert len(bad) == 0, f"{len(bad)} differ, first {rays[bad[0]]}"
    assert (lb >= 0).mean() > 0.8
    # a coarse cube map and a small e_max: more undecided rays, never a wrong one
    ref2, lb2, _ = lbins_run(sim, sc, rays, e_max=0.005, n=8)
    assert not np.any((lb2 >= 0) & (lb2 != ref2))
    # a synthetic scene with many small triangles
    sc5 = c5_scene(20_000, 64, 36)
    l5 = scene_lights(sc5)
    if len(l5):
        pts = stress_rays(sc5, 3000, 21)[3000:, :3]
        nn = rng.normal(size=pts.shape).astype(np.float32)
        nn /= np.linalg.norm(nn, axis=1, keepdims=True)
        r5 = shadow_rays(pts, nn, l5, np.float32(1e-2), rng)
        ref5, lb5, _ = lbins_run(sim, sc5, r5)
        assert not np.any((lb5 >= 0) & (lb5 != ref5))


def test_light_bins_margin_edge_cases(sim):  # noqa: F811
    """Small triangles on a shell just past R0 around a light and rays whose
    lines pass the light at up to e_max, aimed at the triangles' edges and
    corners: hit directions seen from the light differ from the origin's by
    up to asin(e_max / R0), the angular margin the cells are widened by."""
    from crt_amd.native import SyntheticScene
    rng = np.random.default_rng(13)
    n = 4000
    L = np.zeros(3, np.float32)
    dirs = rng.normal(size=(n, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    c = dirs * rng.uniform(1.3, 1.8, (n, 1))
    verts = (c[:, None, :] + rng.uniform(-0.04, 0.04, (n, 3, 3))).astype(np.float32).reshape(-1, 3)
    sc = SyntheticScene(verts, np.arange(3 * n, dtype=np.int32), width=64, height=36,
                        camera_location=(0.0, 0.0, 5.0), fov_degrees=90.0, background=(0.0, 0.0, 0.0),
                        albedo=(0.8, 0.8, 0.8), lights=((100.0, (0.0, 0.0, 0.0)),))
    v = verts.reshape(n, 3, 3)
    k = 6 * n
    tri = rng.integers(0, n, k)
    bary = rng.dirichlet((1.0, 1.0, 1.0), k)
    bary[: k // 2, 0] = rng.uniform(-1e-6, 1e-6, k // 2)       # on an edge
    bary[k // 2: 3 * k // 4] = np.eye(3)[rng.integers(0, 3, k // 4)]   # at a corner
    bary /= bary.sum(1, keepdims=True)
    q = np.einsum("nk,nkc->nc", bary, v[tri])
    w = q - L
    perp = np.cross(w, rng.normal(size=(k, 3)))
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    lp = L + perp * rng.uniform(0.0, 0.0199, (k, 1))             # the line passes within e of L
    d = (lp - q) / np.linalg.norm(lp - q, axis=1, keepdims=True)
    o = q - d * rng.uniform(0.002, 2.5, (k, 1))
    r2 = np.einsum("ij,ij->i", lp - o, lp - o)
    rays = np.concatenate([o, d, r2[:, None], np.zeros((k, 1))], 1).astype(np.float32)
    ref, lb, info = lbins_run(sim, sc, rays)
    assert info[1] == 1 and info[2] == 0
    bad = np.flatnonzero((lb >= 0) & (lb != ref))
    assert len(bad) == 0, f"{len(bad)} differ, first {rays[bad[0]]}"
    assert (lb >= 0).mean() > 0.95 and ref.mean() > 0.2
