"""A device scene whose camera moves (crt_hip_scene_set_camera): every pose and
resolution renders the bits the oracle renders for a scene file holding that
camera, through the blocking entry point and through device frames issued back
to back with a new pose each (frames in flight keep the camera they were
issued with).  The reference re-renders whatever camera its Scene holds
(crt_renderer.cpp:157-199; per Blender frame, bl_crt_engine.py:12-31)."""
import numpy as np
import pytest

from conftest import bits, scene_npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    from crt_amd import native
    native.lib()
    return native


def posed(name, loc, rot, fov=None, size=None):
    sc = scene_npz(name)
    if size:
        sc = sc.set_resolution(*size)
    return sc.set_camera(location=loc, rotation=rot, fov_degrees=fov)


def poses(name, n, **kw):
    from crt_amd.camera import orbit_poses
    return orbit_poses(scene_npz(name).a, n, **kw)


def test_camera_poses_c2_bins(N, oracle, devbuf):
    """C2's scene (camera bins rebuilt every frame): 10 poses and two
    resolutions; each pose blocking, then all poses again as device frames
    back to back (no host wait), every frame against the oracle."""
    name = "14-01-acceleration-tree__scene1"
    st = N.RendererSettings.default()
    for size in [(640, 360), (480, 480)]:
        g = N.HipScene(scene_npz(name).set_resolution(640, 360))
        ps = poses(name, 10)
        fovs = [None] * 8 + [60.0, 100.0]
        wants = []
        for (loc, rot), fov in zip(ps, fovs):
            want = bits(oracle.OracleScene(posed(name, loc, rot, fov, size)).render(st))
            wants.append(want)
            g.set_camera(loc, rot, fov_degrees=fov if fov else float(scene_npz(name).a["cam_fov"][0]),
                         width=size[0], height=size[1])
            assert np.array_equal(bits(g.render(st)), want)
        nb = size[0] * size[1] * 3 * 4
        d = [devbuf.alloc(nb) for _ in ps]
        for k, ((loc, rot), fov) in enumerate(zip(ps, fovs)):
            g.set_camera(loc, rot, fov_degrees=fov if fov else float(scene_npz(name).a["cam_fov"][0]))
            g.render_device(st, d[k])
        bad = [k for k in range(len(ps))
               if not np.array_equal(bits(devbuf.download(d[k], (size[1], size[0], 3), np.float32)), wants[k])]
        assert not bad, f"device frames {bad} differ"
        info = g.info()
        assert info["camera_moves"] >= 18
        assert info["view_rebuilds"] <= (1 if size != (640, 360) else 0) + 1, info["view_rebuilds"]


def test_camera_bins_grid_outgrown(N, oracle):
    """A pose far closer to the dragon than the scene's sizing pass saw: more
    cells list more candidates than the grid has slots, so grid slots take
    several work-list entries (crt_render.hip bins_tile rep) — same bits."""
    name = "14-01-acceleration-tree__scene1"
    st = N.RendererSettings.default()
    a = scene_npz(name).a
    from crt_amd.camera import scene_pivot
    loc0 = np.asarray(a["cam_loc"], np.float64)
    piv = scene_pivot(a)
    g = N.HipScene(scene_npz(name).set_resolution(960, 540))
    for f in (0.55, 0.35, 1.6):
        loc = (piv + (loc0 - piv) * f).astype(np.float32)
        want = bits(oracle.OracleScene(posed(name, loc, a["cam_rot"], None, (960, 540))).render(st))
        g.set_camera(loc)
        assert np.array_equal(bits(g.render(st)), want), f"scale {f}"


def test_camera_out_of_bins_bound_and_back(N, oracle):
    """A camera outside the hull margins' origin bound takes no camera bins
    (the view is rebuilt without them, BVH walk), and bins again once it
    returns."""
    name = "14-01-acceleration-tree__scene1"
    st = N.RendererSettings.default()
    a = scene_npz(name).a
    g = N.HipScene(scene_npz(name).set_resolution(320, 180))
    far = (np.asarray(a["cam_loc"], np.float64) * 1e4).astype(np.float32)
    for loc in (far, np.asarray(a["cam_loc"], np.float32)):
        want = bits(oracle.OracleScene(posed(name, loc, a["cam_rot"], None, (320, 180))).render(st))
        g.set_camera(loc)
        assert np.array_equal(bits(g.render(st)), want)
    assert g.info()["view_rebuilds"] == 2


def test_camera_poses_c3_wavefront(N, oracle, devbuf):
    """C3's scene (reflect / refract levels, recorded level sizes and graphs):
    a new camera drops the recorded sizes; poses blocking and back to back."""
    name = "11-01-refractive__scene8"
    st = N.RendererSettings.default(max_ray_depth=8)
    g = N.HipScene(scene_npz(name).set_resolution(320, 180))
    ps = poses(name, 6, yaw_amp=15.0)
    wants = []
    for loc, rot in ps:
        want = bits(oracle.OracleScene(posed(name, loc, rot, None, (320, 180))).render(st))
        wants.append(want)
        g.set_camera(loc, rot)
        for _ in range(2):   # the read-back frame, then a recorded-size frame
            assert np.array_equal(bits(g.render(st)), want)
    d = [devbuf.alloc(320 * 180 * 12) for _ in ps]
    for k, (loc, rot) in enumerate(ps):
        g.set_camera(loc, rot)
        g.render_device(st, d[k])
    bad = [k for k in range(len(ps)) if not np.array_equal(bits(devbuf.download(d[k], (180, 320, 3), np.float32)), wants[k])]
    assert not bad, f"device frames {bad} differ"


def test_c3_device_sized_frames(N, oracle, devbuf):
    """Wavefront frames with no recorded level sizes (every frame after a
    camera move) size their levels on the device instead of reading them back
    (option wf_dynamic): 8 poses issued back to back as device frames run
    side by side on the buffer sets and each equals the oracle's render of
    its pose; a blocking frame of the last pose records its sizes, and the
    frame after it replays them.  A device-sized frame whose levels outgrow
    their capacities (wf_dyn_ids 1: no room for any child's id) is rendered
    again with read-backs by crt_hip_render and reported by the next device
    frame's call."""
    name = "11-01-refractive__scene8"
    st = N.RendererSettings.default(max_ray_depth=8)
    size = (240, 135)
    ps = poses(name, 8, yaw_amp=18.0)
    wants = [bits(oracle.OracleScene(posed(name, loc, rot, None, size)).render(st)) for loc, rot in ps]
    g = N.HipScene(scene_npz(name).set_resolution(*size))
    d = [devbuf.alloc(size[0] * size[1] * 12) for _ in ps]
    for k, (loc, rot) in enumerate(ps):
        g.set_camera(loc, rot)
        g.render_device(st, d[k])
    bad = [k for k in range(len(ps))
           if not np.array_equal(bits(devbuf.download(d[k], (size[1], size[0], 3), np.float32)), wants[k])]
    assert not bad, f"device-sized frames {bad} differ"
    for _ in range(3):   # device-sized (its sizes recorded behind it), then recorded-size frames
        assert np.array_equal(bits(g.render(st)), wants[-1])
    assert g.info()["wf_sets"] >= 2
    h = N.HipScene(scene_npz(name).set_resolution(*size), wf_dyn_ids=1)
    h.set_camera(*ps[2])
    assert np.array_equal(bits(h.render(st)), wants[2])   # overflowed, rendered again with read-backs
    h = N.HipScene(scene_npz(name).set_resolution(*size), wf_dyn_ids=1)   # (h's read-back frame grew its ids)
    h.set_camera(*ps[3])
    h.render_device(st, d[0])                              # overflows: reported on the next call
    devbuf.sync()
    with pytest.raises(N.CrtError):
        h.render_device(st, d[1])
    assert np.array_equal(bits(h.render(st)), wants[3])   # read-back frame


def test_c3_overflow_over_stale_queues(N, oracle, devbuf):
    """An overflowing device-sized frame (wf_dyn_ids 2: the ids run out a few
    levels down) over queues and nodes full of another pose's rays: the
    overflowing waves fill their reserved slots with rays the next level skips
    and final black activations, so no level reads a stale ray (no fault); the
    frame is reported and every frame rendered afterwards is exact."""
    name = "11-01-refractive__scene8"
    st = N.RendererSettings.default(max_ray_depth=8)
    size = (240, 135)
    ps = poses(name, 4, yaw_amp=25.0)
    g = N.HipScene(scene_npz(name).set_resolution(*size))
    d = [devbuf.alloc(size[0] * size[1] * 12) for _ in range(3)]
    for loc, rot in ps[:2]:   # queues, nodes and colours hold these poses' rays
        g.set_camera(loc, rot)
        g.render_device(st, d[0])
        g.render_device(st, d[1])
    devbuf.sync()
    g.set_option("wf_dyn_ids", 2)
    g.set_camera(*ps[2])
    g.render_device(st, d[2])
    devbuf.sync()
    try:
        g.render_device(st, d[2])   # reports the previous frame's overflow (if its ids ran out)
    except N.CrtError:
        pass
    devbuf.sync()
    want = bits(oracle.OracleScene(posed(name, *ps[2], None, size)).render(st))
    assert np.array_equal(bits(g.render(st)), want)
    g.set_option("wf_dyn_ids", 4)
    g.set_camera(*ps[3])
    assert np.array_equal(bits(g.render(st)), bits(oracle.OracleScene(posed(name, *ps[3], None, size)).render(st)))


def test_c3_moving_camera_three_streams(N, oracle, devbuf):
    """Frames with a new pose each, issued back to back on three caller streams
    in turn (the device scene record ring: a slot is rewritten only after every
    wavefront set that read it is done, WfSet::rec_slots), each equal to the
    oracle's render of its pose."""
    name = "11-01-refractive__scene8"
    st = N.RendererSettings.default(max_ray_depth=8)
    size = (200, 112)
    ps = poses(name, 24, yaw_amp=20.0)
    g = N.HipScene(scene_npz(name).set_resolution(*size))
    streams = [devbuf.stream() for _ in range(3)]
    d = [devbuf.alloc(size[0] * size[1] * 12) for _ in ps]
    for k, (loc, rot) in enumerate(ps):
        g.set_camera(loc, rot)
        g.render_device(st, d[k], streams[k % 3])
    devbuf.sync()
    for k in (0, 5, 11, 17, 23):
        want = bits(oracle.OracleScene(posed(name, *ps[k], None, size)).render(st))
        assert np.array_equal(bits(devbuf.download(d[k], (size[1], size[0], 3), np.float32)), want), f"pose {k}"


def test_camera_poses_gi(N, oracle):
    """C4's GI scene at 96x96: new poses through the GI state machine."""
    name = "15-01-conclusion__scene2"
    st = N.RendererSettings.default()
    g = N.HipScene(scene_npz(name).set_resolution(96, 96))
    for loc, rot in poses(name, 3, yaw_amp=10.0)[1:]:
        want = bits(oracle.OracleScene(posed(name, loc, rot, None, (96, 96))).render(st))
        g.set_camera(loc, rot)
        assert np.array_equal(bits(g.render(st)), want)


def test_camera_multi_replica(N, oracle):
    """A handle over three replicas (device 0 listed three times): every
    replica takes the camera, the compact shards follow the new live mask."""
    name = "14-01-acceleration-tree__scene1"
    st = N.RendererSettings.default()
    g = N.HipScene(scene_npz(name).set_resolution(480, 270), devices=[0, 0, 0])
    for loc, rot in poses(name, 4)[1:]:
        want = bits(oracle.OracleScene(posed(name, loc, rot, None, (480, 270))).render(st))
        g.set_camera(loc, rot)
        assert np.array_equal(bits(g.render(st)), want)
    g.set_camera(width=320, height=200)
    loc, rot = poses(name, 4)[3]
    want = bits(oracle.OracleScene(posed(name, loc, rot, None, (320, 200))).render(st))
    assert np.array_equal(bits(g.render(st)), want)
