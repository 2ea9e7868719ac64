"""Pin the CPU oracle (oracle/crt_oracle.cpp) to the reference's own compiled
translation units (oracle/_ref, built from /root/reference/src/core) — runs only
where the reference checkout exists; tests/test_golden.py pins the same oracle
against committed fixtures everywhere else."""
import numpy as np
import pytest

from conftest import bits, has_reference, hits_equal, scene_npz

pytestmark = pytest.mark.skipif(not has_reference(), reason="needs /root/reference")

SCENES = ["14-01-acceleration-tree__scene1", "14-01-acceleration-tree__scene0", "11-01-refractive__scene8",
          "15-01-conclusion__scene2", "09-02-diffuse-smooth-shading__scene3", "09-03-reflective__scene5",
          "11-01-refractive__scene5"]


@pytest.fixture(scope="module")
def ref_mod(oracle):
    assert oracle.ref_available()
    return oracle


@pytest.mark.parametrize("name", SCENES)
def test_tree_and_normals_equal_reference(ref_mod, name):
    sc = scene_npz(name)
    o, r = ref_mod.OracleScene(sc), ref_mod.RefScene(sc)
    for a, b in zip(o.tree(), r.tree()):
        assert np.array_equal(bits(a), bits(b))
    nv = len(o.vertex_normals())
    assert np.array_equal(bits(o.vertex_normals()), bits(r.vertex_normals(nv)))
    nt = len(o.face_normals())
    assert np.array_equal(bits(o.face_normals()), bits(r.face_normals(nt)))


@pytest.mark.parametrize("name,w,h", [("14-01-acceleration-tree__scene1", 320, 180),
                                      ("11-01-refractive__scene8", 160, 90),
                                      ("15-01-conclusion__scene2", 96, 96),
                                      ("09-02-diffuse-smooth-shading__scene3", 160, 90)])
def test_camera_rays_and_hits_equal_reference(ref_mod, name, w, h):
    sc = scene_npz(name).set_resolution(w, h)
    o, r = ref_mod.OracleScene(sc), ref_mod.RefScene(sc)
    ys, xs = np.mgrid[0:h, 0:w]
    xy = np.stack([xs.ravel(), ys.ravel()], 1)
    ro, rr = o.camera_rays(xy), r.camera_rays(xy)
    assert np.array_equal(bits(ro), bits(rr))
    rng = np.random.default_rng(3)
    extra = np.concatenate([rng.uniform(-10, 10, (512, 3)), rng.normal(size=(512, 3))], 1).astype(np.float32)
    rays = np.concatenate([rr, extra]).astype(np.float32)
    ho, _, _ = o.trace(rays)
    hr = r.trace(rays)
    ok, first, nbad = hits_equal(ho, hr, with_tri=False)
    assert ok, f"{nbad} rays differ, first {first}"


def test_product_host_prep_equals_reference(ref_mod):
    from crt_amd.native import HostScene
    for name in SCENES:
        sc = scene_npz(name)
        hs, r = HostScene(sc), ref_mod.RefScene(sc)
        for a, b in zip(hs.tree(), r.tree()):
            assert np.array_equal(bits(a), bits(b)), name
        nv = hs.info()["vertex_count"]
        assert np.array_equal(bits(hs.vertex_normals()), bits(r.vertex_normals(nv))), name


def test_ppm_bytes_equal_reference(ref_mod, tmp_path):
    from crt_amd.native import write_ppm
    rng = np.random.default_rng(11)
    img = rng.uniform(-1, 2, (13, 17, 3)).astype(np.float32)
    img[0, 0] = [np.nan, np.inf, -np.inf]
    img[3, 4] = [3e9, -3e9, 1.0]
    sc = scene_npz("14-01-acceleration-tree__scene0")
    ref_mod.RefScene(sc).write_ppm(str(tmp_path / "ref.ppm"), img)
    write_ppm(tmp_path / "ours.ppm", img)
    assert (tmp_path / "ours.ppm").read_bytes() == (tmp_path / "ref.ppm").read_bytes()
