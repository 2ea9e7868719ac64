"""How many GPUs a frame is spread over when the caller leaves the choice
(crt_auto_gpus, used by the CLI, _crt and the crt::render_image shim; DESIGN
§5).  CPU only: the policy reads the scene description and the settings.

The reference's render_image spans every hardware thread
(crt_renderer.cpp:176-196); spreading a frame over GPUs pays only when the
frame is long: the measured 8-shard speed-ups are 1.04x (C2) and 1.12x (C3)
against 6.1x (C4) and 7.5x (C5), so C2 / C3 stay on one GPU and C4 / C5 take
them all."""
import ctypes as C

import pytest

from conftest import scene_npz


@pytest.fixture(scope="module")
def N():
    from crt_amd import native
    native.lib()
    return native


def gpus(N, sc, visible, **st):
    s = N.RendererSettings.default(**st)
    return N.lib().crt_auto_gpus(N._desc_ptr(sc), C.byref(s), visible)


def test_baseline_configs(N, monkeypatch):
    monkeypatch.delenv("CRT_HIP_GPUS", raising=False)
    from crt_amd.synthetic import c5_scene
    c2 = scene_npz("14-01-acceleration-tree__scene1").set_resolution(1920, 1080)
    c3 = scene_npz("11-01-refractive__scene8").set_resolution(1920, 1080)
    c4 = scene_npz("15-01-conclusion__scene2").set_resolution(3840, 2160)
    c5 = c5_scene(1_000_000)
    assert gpus(N, c2, 8) == 1
    assert gpus(N, c3, 8, max_ray_depth=8) == 1
    assert gpus(N, c4, 8) == 8
    assert gpus(N, c5, 8) == 8
    assert gpus(N, c4, 1) == 1 and gpus(N, c4, 4) == 4
    # camera rays alone stay short even at 4K (C2's scene)
    assert gpus(N, scene_npz("14-01-acceleration-tree__scene1").set_resolution(3840, 2160), 8) == 1
    # the CLI default scene at its native size still spreads (GI fan-out)
    assert gpus(N, scene_npz("15-01-conclusion__scene2"), 8) > 1


def test_env_override(N, monkeypatch):
    c2 = scene_npz("14-01-acceleration-tree__scene1")
    monkeypatch.setenv("CRT_HIP_GPUS", "3")
    assert gpus(N, c2, 8) == 3
    assert gpus(N, c2, 2) == 2
    monkeypatch.setenv("CRT_HIP_GPUS", "0")
    assert gpus(N, c2, 8) == 1


def test_tree_desc_policy(N, monkeypatch):
    monkeypatch.delenv("CRT_HIP_GPUS", raising=False)
    from test_from_tree import tree_scene
    _, ts = tree_scene("15-01-conclusion__scene2", 3840, 2160)
    s = N.RendererSettings.default()
    assert N.lib().crt_auto_gpus_tree(ts.tree_desc_ptr(), C.byref(s), 8) == 8
    _, ts2 = tree_scene("14-01-acceleration-tree__scene1", 1920, 1080)
    assert N.lib().crt_auto_gpus_tree(ts2.tree_desc_ptr(), C.byref(s), 8) == 1


def test_multi_probe_verdict(N):
    """The multi-GPU probe's decision (crt_multi.hip, run by the create of a
    handle over >= 2 distinct devices): identical probe frames keep the
    replicas; one differing bit or a failed probe render falls back to one GPU."""
    import numpy as np
    a = np.random.default_rng(1).random(64 * 36 * 3).astype(np.float32)
    b = a.copy()
    f = N.lib().crt_multi_probe_verdict
    assert f(a.ctypes.data, b.ctypes.data, a.size, 0) == 0
    b.view(np.uint32)[1234] ^= 1
    assert f(a.ctypes.data, b.ctypes.data, a.size, 0) == 1
    assert f(a.ctypes.data, a.ctypes.data, a.size, -4) == 2
    assert f(a.ctypes.data, a.ctypes.data, 0, 0) == 0
