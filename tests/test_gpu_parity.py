"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar (north_star): pixel RMSE < 1e-4 vs the reference, written below; every
case is also asserted bit-exact (the Fresnel term reads a table of the host
libm's powf, so refractive scenes are exact too).
"""
import numpy as np
import pytest

from conftest import bits, hits_equal, scene_npz

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-4   # north_star: pixel RMSE < 1e-4 vs reference (fp32 RGB)


@pytest.fixture(scope="module")
def N():
    from crt_amd import native
    native.lib()
    return native


def camera_and_random_rays(orc, w, h, n_random=4096, seed=7):
    ys, xs = np.mgrid[0:h, 0:w]
    xy = np.stack([xs.ravel(), ys.ravel()], 1)
    cam = orc.camera_rays(xy)
    rng = np.random.default_rng(seed)
    o = rng.uniform(-20, 20, (n_random, 3)).astype(np.float32)
    d = rng.normal(size=(n_random, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    rnd = np.concatenate([o, d], 1).astype(np.float32)
    # axis-aligned and near-parallel directions stress the 1e-6 guards
    ax = np.zeros((6, 6), np.float32)
    ax[:, :3] = cam[len(cam) // 2, :3]
    for k in range(3):
        ax[2 * k, 3 + k] = 1.0
        ax[2 * k + 1, 3 + k] = -1.0
    return np.concatenate([cam, rnd, ax], 0)


TRACE_SCENES = [
    ("14-01-acceleration-tree__scene1", 320, 180),
    ("11-01-refractive__scene8", 160, 90),
    ("15-01-conclusion__scene2", 128, 128),
    ("09-02-diffuse-smooth-shading__scene2", 160, 90),
    ("14-01-acceleration-tree__scene0", 64, 36),
]


@pytest.mark.parametrize("walk", [0, 1], ids=["reference-order", "pruned"])
@pytest.mark.parametrize("name,w,h", TRACE_SCENES)
def test_trace_batch_bit_exact(N, oracle, name, w, h, walk):
    sc = scene_npz(name).set_resolution(w, h)
    orc = oracle.OracleScene(sc)
    rays = camera_and_random_rays(orc, w, h)
    ref_hits, _, _ = orc.trace(rays)
    gpu = N.HipScene(sc, trace_walk=walk)
    got = gpu.trace(rays)
    ok, first, nbad = hits_equal(got, ref_hits)
    assert ok, f"{name}: {nbad} rays differ, first {first}: gpu={got[first]} oracle={ref_hits[first]}"
    assert got["hit"].sum() > 0


RENDER_CASES = [
    # name, w, h, settings overrides, exact?
    ("14-01-acceleration-tree__scene1", 320, 180, {}, True),
    ("14-01-acceleration-tree__scene0", 96, 54, {}, True),
    ("13-01-optimizations__scene0", 160, 90, {}, True),
    ("09-02-diffuse-smooth-shading__scene3", 160, 90, {}, True),
    ("09-03-reflective__scene5", 160, 90, {}, True),
    ("15-01-conclusion__scene1", 160, 90, {}, True),
    ("12-01-textures__scene3", 192, 108, {}, True),     # JPEG bitmap texture
    ("12-01-textures__scene4", 192, 108, {}, True),     # albedo / edges / checker / bitmap
    ("11-01-refractive__scene8", 160, 90, {"max_ray_depth": 8}, True),
    ("11-01-refractive__scene3", 160, 90, {}, True),
    ("15-01-conclusion__scene2", 48, 48, {}, True),
]


@pytest.mark.parametrize("name,w,h,over,exact", RENDER_CASES)
def test_render_matches_oracle(N, oracle, name, w, h, over, exact):
    sc = scene_npz(name).set_resolution(w, h)
    st = N.RendererSettings.default(**over)
    want = oracle.OracleScene(sc).render(st)
    got = N.HipScene(sc).render(st)
    rmse = float(np.sqrt(np.mean((got.astype(np.float64) - want) ** 2)))
    nbad = int((bits(got) != bits(want)).sum())
    assert rmse < RMSE_TOL, f"{name}: rmse {rmse} ({nbad} differing floats)"
    if exact:
        assert nbad == 0, f"{name}: {nbad} floats differ (rmse {rmse})"


def test_c2_full_frame_bit_exact(N, oracle):
    """Config C2: 14-01/scene1 at 1920x1080, default settings."""
    sc = scene_npz("14-01-acceleration-tree__scene1")
    st = N.RendererSettings.default()
    want = oracle.OracleScene(sc).render(st)
    gpu = N.HipScene(sc)
    got = gpu.render(st)
    assert got.shape == (1080, 1920, 3)
    assert np.array_equal(bits(got), bits(want))
    counts = gpu.count_work(st)
    assert counts["traversals"] == 1920 * 1080


def test_work_counts_match_oracle(N, oracle):
    """The reference-order walks (traversal 7: packet camera rays, range sharing
    for secondaries) test exactly the reference's nodes and triangles."""
    from crt_amd.native import WorkCounts
    sc = scene_npz("11-01-refractive__scene8").set_resolution(160, 90)
    st = N.RendererSettings.default(max_ray_depth=8)
    wc = WorkCounts()
    oracle.OracleScene(sc).render(st, counts=wc)
    got = N.HipScene(sc, traversal=7).count_work(st)
    assert got == wc.as_dict()


@pytest.mark.parametrize("name,w,h,over", [
    ("14-01-acceleration-tree__scene1", 480, 270, {}),
    ("11-01-refractive__scene8", 240, 135, {"max_ray_depth": 8}),
    ("15-01-conclusion__scene2", 64, 64, {}),
])
def test_pruned_walks_equal_reference_walks(N, oracle, name, w, h, over):
    """Pruned walks (default) vs reference-order walks: same image bits, same
    traversal and hit counts, fewer node and triangle tests."""
    from crt_amd.native import WorkCounts
    sc = scene_npz(name).set_resolution(w, h)
    st = N.RendererSettings.default(**over)
    fast = N.HipScene(sc, traversal=8, secondary=10)   # GI frames default to walk 4; force the pruned one
    ref = N.HipScene(sc, traversal=7)
    a, b = fast.render(st), ref.render(st)
    assert np.array_equal(bits(a), bits(b))
    ca, cb = fast.count_work(st), ref.count_work(st)
    wc = WorkCounts()
    oracle.OracleScene(sc).render(st, counts=wc)
    assert cb == wc.as_dict()
    assert ca["traversals"] == cb["traversals"] and ca["hits"] == cb["hits"]
    assert ca["node_tests"] < cb["node_tests"] and ca["triangle_tests"] < cb["triangle_tests"]


def test_pruned_synthetic_bit_exact(N, oracle):
    """C5-style random mesh (deep tree): pruned render equals the oracle."""
    from crt_amd.synthetic import c5_scene
    sc = c5_scene(50_000, 160, 90)
    st = N.RendererSettings.default()
    want = oracle.OracleScene(sc).render(st)
    gpu = N.HipScene(sc, traversal=8)
    got = gpu.render(st)
    assert np.array_equal(bits(got), bits(want))
    c = gpu.count_work(st)
    r = N.HipScene(sc, traversal=7).count_work(st)
    assert c["hits"] == r["hits"] and c["node_tests"] * 2 < r["node_tests"]
    # camera rays through the BVH (the default for scenes with one) + their proof
    bvh = N.HipScene(sc, traversal=14)
    assert np.array_equal(bits(bvh.render(st)), bits(want))
    cb = bvh.count_work(st)
    assert cb["hits"] == r["hits"] and cb["triangle_tests"] * 4 < r["triangle_tests"]


SHARD_CASES = [
    ("14-01-acceleration-tree__scene1", 333, 200, {}, [1, 2, 3, 8]),
    ("15-01-conclusion__scene2", 70, 45, {}, [2, 3]),                       # GI: refill kernel per shard
    ("11-01-refractive__scene8", 150, 100, {"max_ray_depth": 8}, [2, 3]),   # wavefront levels per shard
]


@pytest.mark.parametrize("name,w,h,over,shards",
                         [(n, w, h, o, k) for n, w, h, o, ks in SHARD_CASES for k in ks])
def test_shard_render_and_unpack(N, name, w, h, over, shards):
    """Bucket shards (multi-GPU tiles mode) rendered packed and unpacked equal
    the full-frame render bit for bit, for primary-only, GI and depth-8
    reflect/refract frames."""
    import ctypes as C
    from crt_amd import native
    sc = scene_npz(name).set_resolution(w, h)
    gpu = N.HipScene(sc)
    st = N.RendererSettings.default(**over)
    full = gpu.render(st)
    stride = gpu.shard_stride(shards)
    # device buffers through the HIP runtime the library already uses
    hip = C.CDLL("libamdhip64.so.7")   # the runtime libcrt_hip.so already loaded (same SONAME)
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []
    gathered, frame = C.c_void_p(), C.c_void_p()
    assert hip.hipMalloc(C.byref(gathered), stride * shards * 4) == 0
    assert hip.hipMalloc(C.byref(frame), full.size * 4) == 0
    try:
        for s in range(shards):
            assert gpu.shard_floats(s, shards) <= stride
            gpu.render_shard(st, s, shards, gathered.value + 4 * s * stride)
        gpu.unpack_shards(shards, gathered.value, frame.value)
        assert hip.hipDeviceSynchronize() == 0
        out = np.empty_like(full)
        assert hip.hipMemcpy(out.ctypes.data, frame, full.size * 4, 2) == 0
        assert np.array_equal(bits(out), bits(full))
    finally:
        hip.hipFree(gathered)
        hip.hipFree(frame)
    del native


@pytest.mark.parametrize("calib_k", [4000, 1500])
def test_window_walk_equals_packet_walk(N, oracle, calib_k):
    """Walk 13 (window walk for the plan's split tiles) against
    walk 12 and the oracle on the C2 frame; a low split threshold puts many
    4x4 (16 rays x 4 nodes) and 2x2 (4 rays x 16 nodes) tiles through it."""
    sc = scene_npz("14-01-acceleration-tree__scene1")
    st = N.RendererSettings.default()
    win = N.HipScene(sc, traversal=8, calib_k_milli=calib_k)
    xywh, _ = win.plan_tiles(st)
    sizes = {(int(w), int(h)) for w, h in xywh[:, 2:4]}
    assert (2, 2) in sizes or (4, 4) in sizes
    a = win.render(st)
    b = N.HipScene(sc, traversal=8, window=0).render(st)
    want = oracle.OracleScene(sc).render(st)
    assert np.array_equal(bits(a), bits(want))
    assert np.array_equal(bits(b), bits(want))
    ca, cb = win.count_work(st), N.HipScene(sc, traversal=8, window=0).count_work(st)
    assert ca["traversals"] == cb["traversals"] == 1920 * 1080 and ca["hits"] == cb["hits"]


@pytest.mark.parametrize("opt,values", [("wf_rpw", [64, 32, 5, 1]), ("secondary", [4, 10, 14])])
def test_wavefront_level_layouts_bit_identical(N, oracle, opt, values):
    """Wavefront levels >= 1 (reflect/refract recursion, C3 scene at depth 8):
    rays per wave (idle lanes take donated pieces) and the secondary walk
    (cooperative, pruned or not) change only the schedule, never the image
    bits; the work counts keep the traversal and hit totals."""
    sc = scene_npz("11-01-refractive__scene8").set_resolution(240, 135)
    st = N.RendererSettings.default(max_ray_depth=8)
    base = N.HipScene(sc)
    want = base.render(st)
    ref = oracle.OracleScene(sc).render(st)
    assert float(np.sqrt(np.mean((want.astype(np.float64) - ref) ** 2))) < RMSE_TOL
    assert np.array_equal(bits(want), bits(ref))
    cw = base.count_work(st)
    for v in values:
        g = N.HipScene(sc).set_option(opt, v)
        assert np.array_equal(bits(g.render(st)), bits(want)), f"{opt}={v}"
        c = g.count_work(st)
        assert c["traversals"] == cw["traversals"] and c["hits"] == cw["hits"], f"{opt}={v}"
    with pytest.raises(Exception):
        N.HipScene(sc).set_option(opt, 99)


@pytest.mark.parametrize("name,w,h,over", [
    ("11-01-refractive__scene8", 240, 135, {"max_ray_depth": 8}),
    ("15-01-conclusion__scene2", 64, 64, {}),
    ("15-01-conclusion__scene1", 64, 64, {}),
    ("09-03-reflective__scene5", 96, 54, {"max_ray_depth": 5}),
])
def test_bvh_walk_equals_reference_walks(N, oracle, name, w, h, over):
    """Scattered rays through the BVH with its proof on the reference's tree
    (secondary walk 14, crt_bvh.h, the default) vs the reference-order walks:
    same image bits and the same traversal and hit counts as the oracle's,
    far fewer triangle tests."""
    from crt_amd.native import WorkCounts
    sc = scene_npz(name).set_resolution(w, h)
    st = N.RendererSettings.default(**over)
    fast = N.HipScene(sc, secondary=14)
    ref = N.HipScene(sc, traversal=7)
    a, b = fast.render(st), ref.render(st)
    assert np.array_equal(bits(a), bits(b))
    assert np.array_equal(bits(a), bits(oracle.OracleScene(sc).render(st)))
    ca, cb = fast.count_work(st), ref.count_work(st)
    wc = WorkCounts()
    oracle.OracleScene(sc).render(st, counts=wc)
    assert cb == wc.as_dict()
    assert ca["traversals"] == cb["traversals"] and ca["hits"] == cb["hits"]
    assert ca["triangle_tests"] < cb["triangle_tests"]


@pytest.mark.parametrize("w,h", [(70, 45), (96, 96)])
def test_gi_pixel_refill_bit_identical(N, oracle, w, h):
    """GI frames (15-01/scene2): persistent waves refilling finished lanes with
    the next pixel give the same bits as one wave per 8x8 tile, including
    partial tiles (70x45: the bucket grid's last row/column absorbs the rest),
    and match the oracle within the tolerance this scene is held to."""
    sc = scene_npz("15-01-conclusion__scene2").set_resolution(w, h)
    st = N.RendererSettings.default()
    got = N.HipScene(sc).set_option("gi_refill", 1).render(st)
    tiles = N.HipScene(sc).set_option("gi_refill", 0).render(st)
    assert np.array_equal(bits(got), bits(tiles))
    want = oracle.OracleScene(sc).render(st)
    assert float(np.sqrt(np.mean((got.astype(np.float64) - want) ** 2))) < RMSE_TOL   # as test_render_matches_oracle
    assert np.array_equal(bits(got), bits(want))
    ca = N.HipScene(sc).set_option("gi_refill", 1).count_work(st)
    cb = N.HipScene(sc).set_option("gi_refill", 0).count_work(st)
    # the tile kernel takes the cooperative walk, refill the BVH walk: same rays
    assert ca["traversals"] == cb["traversals"] and ca["hits"] == cb["hits"]
    for walk in (4, 10, 14):
        g = N.HipScene(sc, secondary=walk)
        assert g.count_work(st) == g.count_work(st)
        assert np.array_equal(bits(g.render(st)), bits(want)), walk


BINS_FRAMES = [("14-01-acceleration-tree__scene1", 1920, 1080), ("14-01-acceleration-tree__scene0", 480, 270),
               ("12-01-textures__scene4", 480, 270), ("09-02-diffuse-smooth-shading__scene3", 480, 270),
               ("13-01-optimizations__scene0", 640, 360), ("14-01-acceleration-tree__scene1", 333, 177)]


@pytest.mark.parametrize("name,w,h", BINS_FRAMES)
def test_camera_bins_frames_bit_exact(N, oracle, name, w, h):
    """Camera frames through the camera bins (walk 15, the default for scenes
    without recursion): bit-identical to the per-lane BVH walk (option bins 0)
    and to the oracle, same traversal and hit counts; odd sizes leave partial
    tiles at the right and bottom edges."""
    sc = scene_npz(name).set_resolution(w, h)
    st = N.RendererSettings.default()
    g = N.HipScene(sc)
    assert g.plan_info()["calib_k"] == 0.0   # no probes: one wave per 8x8 cell
    a = g.render(st)
    b = N.HipScene(sc, bins=0).render(st)
    gq = N.HipScene(sc, bins_split=1)   # every cell with a candidate as four 4x4 waves, four lanes per pixel
    q = gq.render(st)
    q1 = N.HipScene(sc, bins_split=1, bins_quad=0).render(st)   # ... one lane per pixel
    want = oracle.OracleScene(sc).render(st)
    assert np.array_equal(bits(a), bits(want))
    assert np.array_equal(bits(b), bits(want))
    assert np.array_equal(bits(q), bits(want))
    assert np.array_equal(bits(q1), bits(want))
    ca, cb = g.count_work(st), N.HipScene(sc, bins=0).count_work(st)
    assert ca["traversals"] == cb["traversals"] == w * h and ca["hits"] == cb["hits"]
    cq = gq.count_work(st)
    assert cq["traversals"] == w * h and cq["hits"] == ca["hits"]
