"""Full-image shading pins against the reference's own committed renders.

The course's committed renders (results/png, frozen in tests/golden/png_pins.npz
by make_png_pins.py) were made by earlier versions of crt_renderer.cpp:

* before HEAD divided every diffuse colour by diffuse_reflection_ray_count + 1
  (crt_renderer.cpp:98) — with GI off that count enters nothing else, so HEAD
  with diffuse_reflection_ray_count = 0 is that renderer, through the
  reference's own settings;
* the 09-xx scenes while shadow rays were still traced (dead code at HEAD,
  :29-44): the "shadows" variant restates :90-92.

Each pinned render equals write_ppm's bytes of the chosen variant at every one
of its 2,073,600 pixels: C2's scene (14-01/scene1) and C1's (14-01/scene0),
13-01, a reflective + refractive scene (11-01/scene0, Fresnel and both
recursions), two smooth-shaded diffuse scenes and a reflective one with shadow
rays.  So the shading arithmetic of the oracle (CPU) and of the HIP path (GPU)
is pinned to the reference's output, not only to its restatement.
"""
import json

import numpy as np
import pytest

from conftest import GOLDEN, bits, scene_npz

PINS = json.loads((GOLDEN / "png_pins.json").read_text())
SHADOW_PINS = [k for k, v in PINS.items() if v["shadows"]]


@pytest.fixture(scope="module")
def pngs():
    with np.load(GOLDEN / "png_pins.npz") as z:
        return {k: z[k] for k in z.files}


def quantise(img: np.ndarray) -> np.ndarray:
    """write_ppm (crt_image_ppm.cpp:15-18), max component 255."""
    return np.clip((img * np.float32(255.0)).astype(np.int64), 0, 255).astype(np.uint8)


def undivided_settings():
    from crt_amd import native as N
    st = N.RendererSettings.default()
    st.diffuse_reflection_ray_count = 0   # GI off: only the final / (count + 1) uses it
    return st


def test_fixture_covers_the_headline_scene():
    assert "14-01-acceleration-tree__scene1" in PINS and len(SHADOW_PINS) >= 2


@pytest.mark.parametrize("name", list(PINS))
def test_oracle_reproduces_committed_png(oracle, pngs, name):
    sc = scene_npz(name)
    assert not sc.desc().gi_on
    img = oracle.OracleScene(sc).set_shadows(PINS[name]["shadows"]).render(undivided_settings())
    got = quantise(img)
    bad = int(np.any(got != pngs[name], axis=2).sum())
    assert bad == 0, f"{name}: {bad} pixels differ from {PINS[name]['png']}"


@pytest.mark.parametrize("name", SHADOW_PINS)
def test_shadow_pin_resolves_shadow_rays(oracle, pngs, name):
    """Without the shadow rays the same render misses the committed image."""
    img = oracle.OracleScene(scene_npz(name)).render(undivided_settings())
    bad = int(np.any(quantise(img) != pngs[name], axis=2).sum())
    assert bad == PINS[name]["pixels_differing_other_variant"] > 0


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", list(PINS))
def test_gpu_reproduces_committed_png(oracle, pngs, name):
    from crt_amd import native as N
    sc = scene_npz(name)
    shadows = PINS[name]["shadows"]
    gpu = N.HipScene(sc, shadows=int(shadows))
    got = gpu.render(undivided_settings())
    bad = int(np.any(quantise(got) != pngs[name], axis=2).sum())
    assert bad == 0, f"{name}: {bad} pixels differ from {PINS[name]['png']}"
    if shadows:   # the shadow-ray kernels, bit for bit against the oracle too
        want = oracle.OracleScene(sc).set_shadows(True).render(undivided_settings())
        nbad = int((bits(got) != bits(want)).sum())
        assert nbad == 0, f"{name}: {nbad} floats differ from the oracle"


SHADOW_CASES = [
    # name, w, h, settings overrides: every shading path with shadow rays
    ("14-01-acceleration-tree__scene1", 1920, 1080, {}),          # C2 with shadow rays
    ("11-01-refractive__scene8", 160, 90, {"max_ray_depth": 8}),  # reflect / refract recursion
    ("15-01-conclusion__scene2", 64, 64, {}),                      # GI fan-out
    ("12-01-textures__scene4", 96, 54, {}),                        # textures
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h,over", SHADOW_CASES)
def test_gpu_shadow_rays_match_oracle(oracle, name, w, h, over):
    from crt_amd import native as N
    sc = scene_npz(name).set_resolution(w, h)
    st = N.RendererSettings.default(**over)
    want = oracle.OracleScene(sc).set_shadows(True).render(st)
    gpu = N.HipScene(sc, shadows=1)
    got = gpu.render(st)
    nbad = int((bits(got) != bits(want)).sum())
    assert nbad == 0, f"{name}: {nbad} floats differ"
    if name.startswith("14-01"):
        head = N.HipScene(sc).render(st)
        assert (bits(head) != bits(got)).any()   # the scene has occluded lights
        # rays traced = camera rays + one shadow ray per (diffuse hit, light)
        wc = N.WorkCounts()
        oracle.OracleScene(sc).set_shadows(True).render(st, counts=wc)
        gc = gpu.count_work(st)
        assert gc["traversals"] == wc.traversals > w * h   # shadow rays stop at their first occluder, so
                                                            # hits are not compared


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [{}, {"bins": 0}, {"traversal": 8}, {"bins_reuse": 0}, {"light_bins": 0},
                                  {"shadow_defer": 0}, {"shadow_defer": 0, "light_bins": 0}, {"bins": 0, "light_bins": 0}])
def test_gpu_shadow_walks_agree(oracle, opts):
    """Shadow rays through every camera walk: camera bins (the default), the
    BVH walk (bins off), the kd packet walk; each frame's shadow rays go
    through the BVH to their first hit within the light (crt_bvh.h
    occluded_bvh) — all equal to the oracle's closest-hit shadow test, frame
    after frame, and at three camera poses (bins rebuilt per pose)."""
    from crt_amd import native as N
    from crt_amd.camera import orbit_poses
    name = "14-01-acceleration-tree__scene1"
    st = N.RendererSettings.default()
    gpu = N.HipScene(scene_npz(name).set_resolution(640, 360), shadows=1, **opts)
    for k, (loc, rot) in enumerate(orbit_poses(scene_npz(name).a, 3, yaw_amp=25.0)):
        sc = scene_npz(name).set_resolution(640, 360).set_camera(location=loc, rotation=rot)
        want = bits(oracle.OracleScene(sc).set_shadows(True).render(st))
        gpu.set_camera(location=loc, rotation=rot)
        for f in range(2):
            got = bits(gpu.render(st))
            assert int((got != want).sum()) == 0, f"pose {k} frame {f} {opts}"


@pytest.mark.gpu
def test_gpu_light_bins(oracle):
    """Shadow rays over the light bins (crt_light_bins.cpp, built at the first
    shadow-ray frame, kept across camera moves): equal to the oracle with the
    bins on and off, and with a larger shadow bias than the bins were built
    for (its rays pass the light farther than e_max: the BVH decides them)."""
    from crt_amd import native as N
    from crt_amd.camera import orbit_poses
    name = "14-01-acceleration-tree__scene1"
    gpu = N.HipScene(scene_npz(name).set_resolution(480, 270), shadows=1)
    st = N.RendererSettings.default()
    for k, (loc, rot) in enumerate(orbit_poses(scene_npz(name).a, 3, yaw_amp=30.0)):
        sc = scene_npz(name).set_resolution(480, 270).set_camera(location=loc, rotation=rot)
        want = bits(oracle.OracleScene(sc).set_shadows(True).render(st))
        gpu.set_camera(location=loc, rotation=rot)
        for lb in (1, 0, 1):
            gpu.set_option("light_bins", lb)
            assert np.array_equal(bits(gpu.render(st)), want), f"pose {k} light_bins {lb}"
    info = gpu.info()
    assert info["light_bin_records"] > 0 and info["light_bins_ms"] > 0
    big = N.RendererSettings.default(shadow_bias=0.08)
    want = bits(oracle.OracleScene(scene_npz(name).set_resolution(480, 270)).set_shadows(True).render(big))
    gpu.set_camera(location=scene_npz(name).a["cam_loc"], rotation=scene_npz(name).a["cam_rot"])
    assert np.array_equal(bits(gpu.render(big)), want)
    # a scene whose lights sit among its triangles (near lists), GI off
    name = "11-01-refractive__scene8"
    sc = scene_npz(name).set_resolution(200, 112)
    st1 = N.RendererSettings.default(max_ray_depth=1)
    g2 = N.HipScene(sc, shadows=1, light_bins=1)
    assert np.array_equal(bits(g2.render(st1)), bits(oracle.OracleScene(sc).set_shadows(True).render(st1)))


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [3, 8])
def test_gpu_shadow_shards_reassemble(devbuf, shards):
    """Shadow-ray frames sharded by the reference's bucket grid (compact shards,
    as bench.py --gpus N --shadows would run them) reassemble into the
    single-GPU shadow frame bit for bit."""
    from crt_amd import native as N
    sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(640, 360)
    st = N.RendererSettings.default()
    gpu = N.HipScene(sc, shadows=1)
    full = gpu.render(st)
    stride = gpu.compact_stride(shards)
    gathered = devbuf.alloc(4 * stride * shards)
    frame = devbuf.alloc(full.nbytes)
    for s in range(shards):
        gpu.render_shard_compact(st, s, shards, gathered + 4 * s * stride)
        devbuf.sync()
    gpu.unpack_compact(shards, gathered, frame)
    out = devbuf.download(frame, full.shape, np.float32)
    assert np.array_equal(bits(out), bits(full))
