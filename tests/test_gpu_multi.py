"""Several GPUs behind one scene handle (crt_hip_scene_create_on / _mask,
csrc/crt_multi.hip): the scene replicated per device, the bucket grid dealt
to the replicas (compact shards), peer copies into the first device and the
unpack there.  A device listed twice holds two replicas, so the one-GPU box
runs the whole split; the image must equal the single-device render bit for
bit (pixels are independent: per-pixel PCG seed, read-only scene)."""
import numpy as np
import pytest

from conftest import bits, scene_npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    from crt_amd import native
    native.lib()
    return native

CASES = [
    ("14-01-acceleration-tree__scene1", 480, 270, {}),
    ("11-01-refractive__scene8", 240, 135, {"max_ray_depth": 8}),
    ("15-01-conclusion__scene2", 96, 96, {}),
    ("12-01-textures__scene4", 200, 120, {}),
    ("09-03-reflective__scene5", 96, 54, {"max_ray_depth": 5}),
]


@pytest.mark.parametrize("name,w,h,over", CASES)
@pytest.mark.parametrize("replicas", [2, 3, 8])
def test_replicas_render_identically(N, name, w, h, over, replicas):
    sc = scene_npz(name).set_resolution(w, h)
    st = N.RendererSettings.default(**over)
    want = N.HipScene(sc).render(st)
    multi = N.HipScene(sc, devices=[0] * replicas)
    assert multi.devices() == [0] * replicas
    for _ in range(3):   # recorded wavefront sizes / captured graphs on every replica
        got = multi.render(st)
        assert np.array_equal(bits(got), bits(want)), name
    ms = multi.replica_ms()
    assert len(ms) == replicas and all(m >= 0.0 for m in ms)


def test_mask_and_single_replica(N):
    sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(160, 90)
    st = N.RendererSettings.default()
    want = N.HipScene(sc).render(st)
    one = N.HipScene(sc, devices=[0])
    assert one.devices() == [0]
    assert np.array_equal(bits(one.render(st)), bits(want))
    import ctypes as C
    h = C.c_void_p()
    lib = N.lib()
    N._check(lib.crt_hip_scene_create_mask(N._desc_ptr(sc), 0, 0, C.byref(h)))   # every visible device
    n = lib.crt_hip_scene_devices(h, None, 0)
    assert n == lib.crt_hip_device_count() >= 1
    out = np.zeros(3 * 160 * 90, np.float32)
    N._check(lib.crt_hip_render(h, C.byref(st), out.ctypes.data, None))
    lib.crt_hip_scene_destroy(h)
    assert np.array_equal(bits(out.reshape(want.shape)), bits(want))


def test_replicas_from_tree(N):
    """The shim's entry (crt_hip_scene_from_tree_on) with two replicas."""
    from test_from_tree import tree_scene
    sc, ts = tree_scene("14-01-acceleration-tree__scene1", 320, 180)
    st = N.RendererSettings.default()
    want = N.HipScene(sc).render(st)
    got = N.HipScene(ts, devices=[0, 0]).render(st)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("opts,over", [({"shadows": 1}, {}), ({"traversal": 8}, {}), ({"bins": 0}, {}),
                                       ({"bins_split": 1, "bins_quad": 0}, {}),
                                       ({"secondary": 10}, {"max_ray_depth": 5})])
def test_options_reach_every_replica(N, opts, over):
    """An option set on a multi-GPU handle applies to every replica: the image
    equals the single-device render with the same option (shadows change it)."""
    name = "09-03-reflective__scene5" if "secondary" in opts else "14-01-acceleration-tree__scene1"
    sc = scene_npz(name).set_resolution(200, 112)
    st = N.RendererSettings.default(**over)
    want = N.HipScene(sc, **opts).render(st)
    multi = N.HipScene(sc, devices=[0, 0, 0])
    for k, v in opts.items():
        multi.set_option(k, v)
    assert np.array_equal(bits(multi.render(st)), bits(want))


def test_concurrent_renders_into_pageable_memory(N):
    """Two host threads rendering two scenes into pageable buffers at once: the
    staged copies (one host copy pool) keep each image whole."""
    import threading
    a = scene_npz("14-01-acceleration-tree__scene1").set_resolution(640, 360)
    b = scene_npz("12-01-textures__scene4").set_resolution(512, 288)
    st = N.RendererSettings.default()
    ga, gb = N.HipScene(a), N.HipScene(b)
    wa, wb = ga.render(st), gb.render(st)
    errs = []

    def run(g, want):
        try:
            for _ in range(20):
                if not np.array_equal(bits(g.render(st)), bits(want)):
                    errs.append("differs")
        except Exception as e:   # noqa: BLE001
            errs.append(repr(e))

    ts = [threading.Thread(target=run, args=(ga, wa)), threading.Thread(target=run, args=(gb, wb))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts), "a render did not return"
    assert errs == []


@pytest.mark.parametrize("inject", [0, 1])
def test_multi_probe_keeps_or_drops_replicas(N, oracle, inject):
    """The create's multi-GPU probe (forced over repeated devices here: the
    box has one GPU): a 64x36 frame through the replicas against device 0
    alone.  Matching bits keep the replicas; an injected differing bit drops
    them (crt_scene_info.multi_probe -1, the reason in crt_hip_last_error())
    and the handle renders on one GPU — the same image either way."""
    sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(320, 180)
    st = N.RendererSettings.default()
    g = N.HipScene(sc, devices=[0, 0, 0],
                   create_flags=N.SCENE_PROBE_FORCE | (N.SCENE_PROBE_TEST_MISMATCH if inject else 0))
    info = g.info()
    assert info["multi_probe"] == (-1 if inject else 1), info["multi_probe"]
    assert len(g.devices()) == (1 if inject else 3)
    if inject:
        assert "differs" in N.last_error()
    assert np.array_equal(bits(g.render(st)), bits(oracle.OracleScene(sc).render(st)))
