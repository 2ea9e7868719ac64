"""The oracle and the product's host prep against the committed fixtures
(tests/golden/, produced from the reference by tests/golden/make_golden.py).
Runs everywhere, including machines without /root/reference."""
import hashlib
import json

import numpy as np
import pytest

from conftest import GOLDEN, bits, hits_equal, scene_npz

TREES = json.loads((GOLDEN / "trees.json").read_text())
HASHES = json.loads((GOLDEN / "image_hashes.json").read_text())


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("name", sorted(TREES))
def test_oracle_tree_signature(oracle, name):
    b, c, off, t = oracle.OracleScene(scene_npz(name)).tree()
    want = TREES[name]
    assert len(c) == want["nodes"] and int(off[-1]) == want["leaf_refs"]
    assert sha(b, c, off, t) == want["sha256"]


@pytest.mark.parametrize("name", sorted(TREES))
def test_product_tree_signature(name):
    from crt_amd.native import HostScene
    hs = HostScene(scene_npz(name))
    info = hs.info()
    want = TREES[name]
    assert (info["node_count"], info["leaf_count"], info["leaf_ref_count"]) == \
        (want["nodes"], want["leaves"], want["leaf_refs"])
    assert sha(*hs.tree()) == want["sha256"]
    # scene-create cost is reported for host builds too (crt_scene_info)
    assert info["tree_build_ms"] > 0.0 and info["prep_ms"] >= info["tree_build_ms"]


@pytest.mark.parametrize("name", sorted(p.stem[4:] for p in GOLDEN.glob("kat_*.npz")))
def test_oracle_per_ray_known_answers(oracle, name):
    from crt_amd.native import HIT_DTYPE
    z = np.load(GOLDEN / f"kat_{name}.npz")
    orc = oracle.OracleScene(scene_npz(name))
    cam = orc.camera_rays(z["xy"])
    assert np.array_equal(bits(cam), bits(z["rays"][: len(cam)]))
    got, _, _ = orc.trace(z["rays"])
    want = np.ascontiguousarray(z["hits"]).view(HIT_DTYPE).reshape(-1)
    ok, first, nbad = hits_equal(got, want, with_tri=False)
    assert ok, f"{name}: {nbad} rays differ (first {first})"


IMAGES = [("c2_small", "14-01-acceleration-tree__scene1", 160, 90, {}),
          ("s0_small", "14-01-acceleration-tree__scene0", 96, 54, {}),
          ("c3_small", "11-01-refractive__scene8", 160, 90, {"max_ray_depth": 8}),
          ("c4_small", "15-01-conclusion__scene2", 64, 64, {}),
          ("refl_small", "15-01-conclusion__scene1", 160, 90, {}),
          ("smooth_small", "09-02-diffuse-smooth-shading__scene3", 160, 90, {}),
          ("refr3_small", "11-01-refractive__scene3", 160, 90, {})]


@pytest.mark.parametrize("key,name,w,h,over", IMAGES)
def test_oracle_images(oracle, key, name, w, h, over):
    from crt_amd.native import RendererSettings
    want = np.load(GOLDEN / "images.npz")[key]
    got = oracle.OracleScene(scene_npz(name).set_resolution(w, h)).render(RendererSettings.default(**over))
    assert np.array_equal(bits(got), bits(want))


def test_oracle_c1_full_hash_and_counts(oracle):
    """Config C1: 14-01/scene1 at 640x480 on the CPU path."""
    from crt_amd.native import RendererSettings, WorkCounts
    h = HASHES["C1"]
    wc = WorkCounts()
    img = oracle.OracleScene(scene_npz(h["scene"]).set_resolution(640, 480)).render(RendererSettings.default(),
                                                                                 counts=wc)
    assert sha(img) == h["fp32_sha256"]
    assert wc.as_dict() == {k: h[k] for k in ("traversals", "node_tests", "triangle_tests", "hits")}


def test_oracle_c2_full_hash_and_ppm(oracle, tmp_path):
    """Config C2 (the bench workload) at full 1920x1080 + its PPM bytes."""
    from crt_amd.native import RendererSettings, write_ppm
    h = HASHES["C2"]
    img = oracle.OracleScene(scene_npz(h["scene"])).render(RendererSettings.default())
    assert sha(img) == h["fp32_sha256"]
    write_ppm(tmp_path / "c2.ppm", img)
    assert hashlib.sha256((tmp_path / "c2.ppm").read_bytes()).hexdigest() == h["ppm_sha256"]


MASKS = [("14-01-scene1", "14-01-acceleration-tree__scene1"), ("14-01-scene0", "14-01-acceleration-tree__scene0"),
         ("13-01", "13-01-optimizations__scene0"), ("09-02-scene2", "09-02-diffuse-smooth-shading__scene2"),
         ("09-02-scene3", "09-02-diffuse-smooth-shading__scene3")]


@pytest.mark.parametrize("key,name", MASKS)
def test_oracle_coverage_matches_reference_png(oracle, key, name):
    """Hit/miss coverage of primary rays equals the foreground of the reference's
    committed render (results/png, rendered at older tags — coverage is the part
    of them HEAD still reproduces)."""
    z = np.load(GOLDEN / "masks.npz")
    shape = tuple(z[key + "_shape"])
    want = np.unpackbits(z[key])[: shape[0] * shape[1]].reshape(shape).astype(bool)
    sc = scene_npz(name)
    orc = oracle.OracleScene(sc)
    h, w = shape
    ys, xs = np.mgrid[0:h, 0:w]
    hits, _, _ = orc.trace(orc.camera_rays(np.stack([xs.ravel(), ys.ravel()], 1)))
    got = hits["hit"].reshape(h, w).astype(bool)
    assert int((got != want).sum()) == 0


def test_ppm_known_answer():
    """crt_write_ppm reproduces the bytes of the reference's crt::write_ppm."""
    import tempfile
    from pathlib import Path
    from crt_amd.native import write_ppm
    z = np.load(GOLDEN / "ppm_kat.npz")
    with tempfile.TemporaryDirectory() as d:
        p = Path(d) / "x.ppm"
        write_ppm(p, z["image"])
        assert p.read_bytes() == z["ppm"].tobytes()
