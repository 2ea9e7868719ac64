"""Camera bins built on the device inside every camera frame (crt_bins.hip):
the lists equal the host checker's (crt_bvh_build.cpp build_camera_bins, the
restatement the CPU walk checks in test_bvh.py run on) record for record —
per 8x8 cell the same length (-1: over the cell cap, the BVH walk), and the
same records in the same order: hull box, dmin bits, id, geometry, pixel mask
and `rest` — and frames rendered through them stay bit-identical to the BVH
walk and to the oracle, frame after frame (the per-frame counters reset)."""
import numpy as np
import pytest

from conftest import bits, scene_npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    from crt_amd import native
    native.lib()
    return native


def floor_scene(N, w, h, n=600, seed=5, cam=(0.0, 0.3, 0.0), rot=None, fov=70.0):
    """A random triangle cloud in front of the camera above a large floor that
    reaches behind it: the floor's two hulls are not in front of the camera,
    so every cell lists them (the everywhere path)."""
    rng = np.random.default_rng(seed)
    c = rng.uniform([-2.0, -0.5, -6.0], [2.0, 1.5, -2.0], (n, 3)).astype(np.float32)
    v = (c[:, None, :] + rng.uniform(-0.15, 0.15, (n, 3, 3))).astype(np.float32).reshape(-1, 3)
    floor = np.array([[-40, -1, 40], [40, -1, 40], [40, -1, -40], [-40, -1, -40]], np.float32)
    pos = np.concatenate([v, floor], 0)
    b = len(v)
    idx = np.concatenate([np.arange(len(v), dtype=np.int32), np.array([b, b + 1, b + 2, b, b + 2, b + 3], np.int32)])
    return N.SyntheticScene(pos, idx, width=w, height=h, camera_location=cam, camera_rotation=rot, fov_degrees=fov)


def wall_scene(N, w, h, n=400, seed=9):
    """A triangle cloud in front of two large walls, wholly in front of the
    camera: each wall triangle covers thousands of cells, so its group has more
    pairs than k_bins_project scatters itself and queues the rest for
    k_bins_pairs."""
    rng = np.random.default_rng(seed)
    c = rng.uniform([-2.0, -1.0, -6.0], [2.0, 1.0, -3.0], (n, 3)).astype(np.float32)
    v = (c[:, None, :] + rng.uniform(-0.2, 0.2, (n, 3, 3))).astype(np.float32).reshape(-1, 3)
    wall = np.array([[-30, -20, -9], [30, -20, -9], [30, 20, -9], [-30, 20, -9]], np.float32)
    b = len(v)
    idx = np.concatenate([np.arange(b, dtype=np.int32), np.array([b, b + 1, b + 2, b, b + 2, b + 3], np.int32)])
    return N.SyntheticScene(np.concatenate([v, wall], 0), idx, width=w, height=h, fov_degrees=80.0)


CASES = [("14-01-acceleration-tree__scene1", None), ("14-01-acceleration-tree__scene1", (333, 177)),
         ("14-01-acceleration-tree__scene1", (3840, 2160)), ("14-01-acceleration-tree__scene0", None),
         ("12-01-textures__scene4", None), ("12-01-textures__scene3", (517, 301)),
         ("09-02-diffuse-smooth-shading__scene3", None), ("09-01-barycentric-coordinates__scene1", (1001, 643)),
         ("13-01-optimizations__scene0", (640, 360))]


def _compare(N, sc, **opts):
    hl, hr = N.HostScene(sc).camera_bins()
    g = N.HipScene(sc, **opts)
    dl, dr = g.camera_bins()
    assert len(hr) > 0, "the host built no bins"
    assert len(dr) > 0, "the device built no bins"
    assert np.array_equal(hl, dl), f"list lengths differ in {int((hl != dl).sum())} cells"
    assert hr.tobytes() == dr.tobytes(), "records differ"
    dl2, dr2 = g.camera_bins()   # a second frame: counters were reset
    assert np.array_equal(dl2, dl) and dr2.tobytes() == dr.tobytes()
    return hl


@pytest.mark.parametrize("name,size", CASES)
def test_device_bins_equal_host(N, name, size):
    sc = scene_npz(name)
    if size:
        sc = sc.set_resolution(*size)
    _compare(N, sc)


def test_device_bins_everywhere_and_overflow(N):
    sc = floor_scene(N, 400, 240)
    ln = _compare(N, sc)
    assert (ln >= 2).all() or (ln < 0).any()   # the floor is in every cell's list


@pytest.mark.parametrize("size", [(640, 360), (1920, 1080)])
def test_device_bins_queued_groups(N, oracle, size):
    """Groups with more pairs than the projection block scatters (the walls)."""
    sc = wall_scene(N, *size)
    _compare(N, sc)
    if size[0] <= 640:
        st = N.RendererSettings.default()
        assert np.array_equal(bits(N.HipScene(sc).render(st)), bits(oracle.OracleScene(sc).render(st)))


@pytest.mark.parametrize("qmax", [1, 2])
def test_device_bins_groups_past_the_queue(N, oracle, qmax):
    """More queued groups than k_bins_pairs takes: the queue's capacity
    (kMaxGroups = 8192, 2^18 triangles) lowered to qmax for the test
    (option "bins_qmax").  Five large triangles 32 apart each make their group
    queue its pairs past kExpand; the groups past qmax scatter their own pairs,
    kExpand a round.  The lists equal the host checker's record for record and
    the frame the oracle's."""
    rng = np.random.default_rng(17)
    n = 160
    c = rng.uniform([-2.0, -1.0, -6.0], [2.0, 1.0, -3.0], (n, 3)).astype(np.float32)
    v = (c[:, None, :] + rng.uniform(-0.2, 0.2, (n, 3, 3))).astype(np.float32)
    for k in range(5):   # triangle 32 k: a large slanted panel behind the cloud
        z = -8.0 - k
        v[32 * k] = np.array([[-12 + 2 * k, -9, z], [12, -9 + k, z - 1], [0, 9, z + 0.5]], np.float32)
    sc = N.SyntheticScene(v.reshape(-1, 3), np.arange(3 * n, dtype=np.int32), width=640, height=360, fov_degrees=80.0)
    _compare(N, sc, bins_qmax=qmax)
    st = N.RendererSettings.default()
    assert np.array_equal(bits(N.HipScene(sc, bins_qmax=qmax).render(st)), bits(oracle.OracleScene(sc).render(st)))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_device_bins_random_cameras(N, oracle, seed):
    rng = np.random.default_rng(seed)
    a, b = rng.uniform(-0.4, 0.4, 2)
    ca, sa, cb, sb = np.cos(a), np.sin(a), np.cos(b), np.sin(b)
    rot = (np.array([[cb, 0, -sb], [0, 1, 0], [sb, 0, cb]]) @ np.array([[1, 0, 0], [0, ca, sa], [0, -sa, ca]]))
    w, h = [(257, 129), (96, 311), (400, 225)][seed - 1]
    sc = floor_scene(N, w, h, seed=seed, rot=tuple(float(x) for x in rot.ravel()), fov=float(rng.uniform(20, 150)))
    _compare(N, sc)
    st = N.RendererSettings.default()
    g = N.HipScene(sc)
    ref = oracle.OracleScene(sc).render(st)
    for _ in range(2):
        assert np.array_equal(bits(g.render(st)), bits(ref))


def test_bins_frames_repeat_bit_exact(N, oracle, devbuf):
    """C2's scene through the camera bins, several frames back to back into
    device memory (the binning, the priority lists and the counters of every
    frame) and through the host entry point: every frame equals the oracle."""
    sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(640, 360)
    st = N.RendererSettings.default()
    want = bits(oracle.OracleScene(sc).render(st))
    g = N.HipScene(sc)
    d = devbuf.alloc(640 * 360 * 3 * 4)
    for _ in range(3):
        g.render_device(st, d)
    for _ in range(3):
        g.render_device(st, d)
        assert np.array_equal(bits(devbuf.download(d, (360, 640, 3), np.float32)), want)
    assert np.array_equal(bits(g.render(st)), want)
    assert np.array_equal(bits(N.HipScene(sc, bins_split=1000).render(st)), want)   # no heavy cells split


def test_bins_frames_pipelined_bit_exact(N, oracle, devbuf):
    """Frames issued back to back without a host wait: the next frames'
    binnings run on the binning stream while frame k renders (crt_bins.hip
    bins_enqueue), on kBinSets (3) sets of lists taken in turn.  Forty frames
    into three rotating buffers, then a host frame: all equal the oracle."""
    sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(960, 540)
    st = N.RendererSettings.default()
    want = bits(oracle.OracleScene(sc).render(st))
    g = N.HipScene(sc)
    d = [devbuf.alloc(960 * 540 * 3 * 4) for _ in range(3)]
    for k in range(40):
        g.render_device(st, d[k % 3])
    for k in range(3):
        assert np.array_equal(bits(devbuf.download(d[k], (540, 960, 3), np.float32)), want)
    assert np.array_equal(bits(g.render(st)), want)


@pytest.mark.parametrize("reuse", [1, 0])
def test_bins_frames_pipelined_full_size_every_frame(N, oracle, devbuf, reuse):
    """The bench's own C2 mode at the benched size: 1920x1080 frames issued back
    to back with no host wait, each into a buffer of its own, and every one of
    the 24 frames compared with the oracle's frame.  reuse 1 (the default): the
    camera does not move, so the frames render the first binning's lists;
    reuse 0: every frame bins (the next frames' binnings overlap frame k's
    render, kBinSets sets of lists in turn)."""
    sc = scene_npz("14-01-acceleration-tree__scene1")
    st = N.RendererSettings.default()
    want = bits(oracle.OracleScene(sc).render(st))
    g = N.HipScene(sc, bins_reuse=reuse)
    nb = 1920 * 1080 * 3 * 4
    d = [devbuf.alloc(nb) for _ in range(24)]
    for k in range(24):
        g.render_device(st, d[k])
    bad = [k for k in range(24) if not np.array_equal(bits(devbuf.download(d[k], (1080, 1920, 3), np.float32)), want)]
    assert not bad, f"frames {bad} differ from the oracle"
    info = g.info()
    if reuse:
        assert info["bins_reuses"] >= 23, info
    else:
        assert info["bins_reuses"] == 0 and info["bins_binnings"] >= 24, info


@pytest.mark.parametrize("reuse", [1, 0])
def test_bins_frames_on_alternating_streams(N, oracle, devbuf, reuse):
    """Frames issued on two caller streams in turn, no host wait: a binning
    waits for the render kBinSets frames back and for the previous binning
    whichever stream they ran on (crt_bins.hip bins_enqueue), so the shared
    binning scratch is never rewritten under a render; frames that take the
    last binning's lists again (reuse 1) chain their set's render events
    across the streams.  30 frames, each into a buffer of its own, every one
    equal to the oracle."""
    sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(960, 540)
    st = N.RendererSettings.default()
    want = bits(oracle.OracleScene(sc).render(st))
    g = N.HipScene(sc, bins_reuse=reuse)
    streams = [devbuf.stream(), devbuf.stream()]
    d = [devbuf.alloc(960 * 540 * 3 * 4) for _ in range(30)]
    for k in range(30):
        g.render_device(st, d[k], streams[k % 2])
    bad = [k for k in range(30) if not np.array_equal(bits(devbuf.download(d[k], (540, 960, 3), np.float32)), want)]
    assert not bad, f"frames {bad} differ from the oracle"


def test_bins_reuse_across_camera_moves_and_streams(N, oracle, devbuf):
    """Two poses, three frames each in turn, issued on two caller streams with
    no host wait: a pose's first frame bins (a new set), the next two render
    those lists again; a binning after reused frames waits for every render of
    the set it clears, whichever stream.  24 frames, each against the oracle's
    frame for its pose."""
    from crt_amd.camera import orbit_poses
    name = "14-01-acceleration-tree__scene1"
    w, h = 960, 540
    base = scene_npz(name).set_resolution(w, h)
    st = N.RendererSettings.default()
    ps = orbit_poses(scene_npz(name).a, 4)[:2]
    fov = float(scene_npz(name).a["cam_fov"][0])
    wants = [bits(oracle.OracleScene(base.set_camera(location=l, rotation=r, fov_degrees=fov)).render(st))
             for l, r in ps]
    g = N.HipScene(base)
    streams = [devbuf.stream(), devbuf.stream()]
    d = [devbuf.alloc(w * h * 3 * 4) for _ in range(24)]
    pose = []
    for k in range(24):
        i = (k // 3) % 2
        if k % 3 == 0:
            g.set_camera(*ps[i], fov_degrees=fov)
        pose.append(i)
        g.render_device(st, d[k], streams[k % 2])
    bad = [k for k in range(24)
           if not np.array_equal(bits(devbuf.download(d[k], (h, w, 3), np.float32)), wants[pose[k]])]
    assert not bad, f"frames {bad} differ from the oracle"
    info = g.info()
    assert info["bins_binnings"] >= 8 and info["bins_reuses"] >= 16, info
