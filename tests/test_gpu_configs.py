"""GPU parity at the BASELINE configs' own sizes, and against the reference's
own per-ray records.

  C3  11-01/scene8, 1920x1080, depth 8  — full frame against the oracle and the
      committed full-resolution hash (tests/golden/image_hashes.json "C3")
  C4  15-01/scene2 at its native 1080x1080 — work counts of the reference-order
      walks equal the reference's (85,480,935 traversals, "C4_native"), the GI
      frame's fp32 hash, and a 256x256 GI frame against the oracle
  C5  the synthetic 1M-triangle mesh rendered at 64x36 and
      160x90 against the oracle (device-built tree, pruned walks)
  KAT the HIP trace hook against tests/golden/kat_*.npz — the Intersection
      records the reference's own compiled ray_intersect_acceleration_tree
      produced (crt_intersection.cpp:109-136), no oracle in between
"""
import hashlib
import json

import numpy as np
import pytest

from conftest import GOLDEN, bits, hits_equal, ppm_quantize, scene_npz

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-4   # north_star: pixel RMSE < 1e-4 vs reference (fp32 RGB)
HASHES = json.loads((GOLDEN / "image_hashes.json").read_text())


@pytest.fixture(scope="module")
def N():
    from crt_amd import native
    native.lib()
    return native


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def compare(got, want):
    rmse = float(np.sqrt(np.mean((got.astype(np.float64) - want) ** 2)))
    nbad = int((bits(got) != bits(want)).sum())
    return rmse, nbad


def test_c3_full_frame(N, oracle):
    """C3 at its own size: 1920x1080, max_ray_depth 8 (wavefront levels; levels
    >= 1 through the per-lane BVH walk)."""
    h = HASHES["C3"]
    sc = scene_npz(h["scene"])
    st = N.RendererSettings.default(**h["settings"])
    gpu = N.HipScene(sc)
    got = gpu.render(st)
    assert got.shape == (1080, 1920, 3)
    want = oracle.OracleScene(sc).render(st)
    rmse, nbad = compare(got, want)
    print(f"C3 1920x1080 depth 8: rmse {rmse:.3g}, {nbad} of {got.size} floats differ")
    assert rmse < RMSE_TOL
    assert nbad == 0, f"{nbad} floats differ (rmse {rmse})"
    assert sha(got) == h["fp32_sha256"]
    c = gpu.count_work(st)
    assert c["traversals"] == h["traversals"] and c["hits"] == h["hits"]
    r = N.HipScene(sc, traversal=7).count_work(st)
    assert r == {k: h[k] for k in ("traversals", "node_tests", "triangle_tests", "hits")}


def test_c4_native_counts_and_hash(N):
    """C4's scene at its native 1080x1080 (GI on): the reference-order walks
    execute exactly the reference's traversals / node / triangle tests, the
    pruned default the same traversals and hits, and the frame's fp32 bits
    equal the committed hash of the oracle's frame."""
    h = HASHES["C4_native"]
    sc = scene_npz(h["scene"]).set_resolution(h["width"], h["height"])
    st = N.RendererSettings.default(**h["settings"])
    ref = N.HipScene(sc, traversal=7).count_work(st)
    assert ref == {k: h[k] for k in ("traversals", "node_tests", "triangle_tests", "hits")}
    gpu = N.HipScene(sc)
    c = gpu.count_work(st)
    assert c["traversals"] == h["traversals"] and c["hits"] == h["hits"]
    img = gpu.render(st)
    assert sha(img) == h["fp32_sha256"]


def test_c4_gi_256(N, oracle):
    """A 256x256 GI frame of C4's scene against the oracle."""
    sc = scene_npz("15-01-conclusion__scene2").set_resolution(256, 256)
    st = N.RendererSettings.default()
    got = N.HipScene(sc).render(st)
    want = oracle.OracleScene(sc).render(st)
    rmse, nbad = compare(got, want)
    print(f"C4 scene 256x256 GI: rmse {rmse:.3g}, {nbad} floats differ")
    assert rmse < RMSE_TOL and nbad == 0


@pytest.fixture(scope="module")
def c5_1m():
    from crt_amd.synthetic import c5_scene
    return c5_scene(1_000_000, 160, 90)


@pytest.mark.parametrize("w,h", [(64, 36), (160, 90)])
def test_c5_1m_triangles(N, oracle, c5_1m, w, h):
    """C5's 1M-triangle mesh (880,933 nodes, device-built tree) rendered
    through the device-built BVH (crt_lbvh.hip) and the proof on the
    device-built tree, bit for bit against the oracle."""
    sc = c5_1m
    sc.desc().camera.width, sc.desc().camera.height = w, h
    st = N.RendererSettings.default()
    gpu = N.HipScene(sc)
    info = gpu.info()
    assert info["tree_on_device"] == 1 and info["node_count"] == 880_933
    assert info["bvh_on_device"] == 1
    got = gpu.render(st)
    want = oracle.OracleScene(sc).render(st)
    rmse, nbad = compare(got, want)
    assert nbad == 0, f"{nbad} floats differ (rmse {rmse})"
    c = gpu.count_work(st)
    assert c["traversals"] == w * h


@pytest.mark.parametrize("walk", [0, 1, 2], ids=["reference-order", "pruned", "bvh"])
@pytest.mark.parametrize("name", sorted(p.stem[4:] for p in GOLDEN.glob("kat_*.npz")))
def test_trace_matches_reference_records(N, name, walk):
    """The HIP trace hook returns, for every ray, the Intersection the
    reference's own ray_intersect_acceleration_tree returned (distance, point,
    normal, uv, barycentrics, material; misses as misses), bit for bit."""
    z = np.load(GOLDEN / f"kat_{name}.npz")
    want = np.ascontiguousarray(z["hits"]).view(N.HIT_DTYPE).reshape(-1)
    got = N.HipScene(scene_npz(name), trace_walk=walk).trace(z["rays"])
    ok, first, nbad = hits_equal(got, want, with_tri=False)
    assert ok, f"{name}: {nbad} rays differ (first {first}: gpu={got[first]} ref={want[first]})"
    assert int(got["hit"].sum()) == int(want["hit"].sum()) > 0


def test_deep_recursion_wavefront(N, oracle):
    """max_ray_depth beyond the old fixed level cap (66) on a mirror scene:
    the wavefront path traces every level up to the depth (no silent cut)."""
    sc = scene_npz("09-03-reflective__scene5").set_resolution(48, 27)
    st = N.RendererSettings.default(max_ray_depth=70)
    got = N.HipScene(sc).render(st)
    want = oracle.OracleScene(sc).render(st)
    rmse, nbad = compare(got, want)
    assert nbad == 0, f"{nbad} floats differ (rmse {rmse})"
    with pytest.raises(N.CrtError):
        N.HipScene(sc).render(N.RendererSettings.default(max_ray_depth=5000))


def test_quantize_rgb8(N, devbuf):
    """Device write_ppm conversion (crt_image_ppm.cpp:15-18) on ordinary and
    special values, odd lengths and unaligned starts."""
    rng = np.random.default_rng(3)
    x = rng.uniform(-0.5, 1.5, 4099).astype(np.float32)
    x[:12] = [np.nan, np.inf, -np.inf, -0.0, 0.0, 1.0, 255.0 / 255.0, 0.99999994, 1e30, -1e30, 8.5e6, 2.0 ** 31]
    d_in = devbuf.upload(x)
    d_out = devbuf.alloc(x.size + 8)
    for off, n in [(0, x.size), (1, 4097), (3, 5), (0, 1)]:
        N.quantize_rgb8(d_in + 4 * off, n, d_out + off, 255)
        got = devbuf.download(d_out + off, n, np.uint8)
        assert np.array_equal(got, ppm_quantize(x[off:off + n]))
    N.quantize_rgb8(d_in, x.size, d_out, 7)
    assert np.array_equal(devbuf.download(d_out, x.size, np.uint8), ppm_quantize(x, 7))
    with pytest.raises(N.CrtError):
        N.quantize_rgb8(d_in, x.size, d_out, 256)


@pytest.mark.parametrize("shards", [1, 3, 8])
def test_shard_rgb8_pack_and_unpack(N, devbuf, shards):
    """tiles mode with the 8-bit payload: each packed shard quantised on the
    device, gathered (here: side by side) and unpacked equals the quantised
    full frame, i.e. the PPM components the reference writes."""
    sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(333, 200)
    gpu = N.HipScene(sc)
    st = N.RendererSettings.default()
    full = gpu.render(st)
    stride = gpu.shard_stride(shards)
    f32 = devbuf.alloc(4 * stride)
    gathered = devbuf.alloc(stride * shards)
    frame8 = devbuf.alloc(full.size)
    for s in range(shards):
        gpu.render_shard(st, s, shards, f32)
        devbuf.sync()
        N.quantize_rgb8(f32, stride, gathered + s * stride, 255)
        devbuf.sync()
    gpu.unpack_shards_rgb8(shards, gathered, frame8)
    out = devbuf.download(frame8, full.shape, np.uint8)
    assert np.array_equal(out, ppm_quantize(full))


COMPACT_CASES = [
    ("14-01-acceleration-tree__scene1", 1920, 1080, {}, None, [1, 2, 8]),
    ("14-01-acceleration-tree__scene1", 333, 200, {}, 20, [3]),        # bucket grid off the 8x8 grid
    ("11-01-refractive__scene8", 240, 135, {"max_ray_depth": 8}, None, [2, 3]),
    ("15-01-conclusion__scene2", 70, 45, {}, None, [2]),                # GI, camera inside the root cell
]


@pytest.mark.parametrize("name,w,h,over,bucket,shards",
                         [(n, w, h, o, b, k) for n, w, h, o, b, ks in COMPACT_CASES for k in ks])
def test_compact_shards_lossless(N, devbuf, name, w, h, over, bucket, shards):
    """Compact shards (only live tiles rendered and gathered; unpack writes the
    background elsewhere) reproduce the full frame bit for bit, in fp32 and as
    write_ppm bytes; the live mask only drops pixels whose ray misses."""
    sc = scene_npz(name).set_resolution(w, h)
    if bucket:
        sc.set_settings(bucket_size=bucket)
    gpu = N.HipScene(sc)
    st = N.RendererSettings.default(**over)
    full = gpu.render(st)
    mask = gpu.live_mask()
    stride = gpu.compact_stride(shards)
    assert stride <= gpu.shard_stride(shards) + 64
    gathered = devbuf.alloc(4 * stride * shards)
    g8 = devbuf.alloc(stride * shards)
    frame = devbuf.alloc(full.nbytes)
    frame8 = devbuf.alloc(full.size)
    for s in range(shards):
        assert gpu.compact_floats(s, shards) <= stride
        gpu.render_shard_compact(st, s, shards, gathered + 4 * s * stride)
        devbuf.sync()
        N.quantize_rgb8(gathered + 4 * s * stride, stride, g8 + s * stride, 255)
        devbuf.sync()
    gpu.unpack_compact(shards, gathered, frame)
    gpu.unpack_compact_rgb8(shards, g8, frame8)
    out = devbuf.download(frame, full.shape, np.float32)
    assert np.array_equal(bits(out), bits(full))
    assert np.array_equal(devbuf.download(frame8, full.shape, np.uint8), ppm_quantize(full))
    # dead pixels are misses: exactly the background colour
    bg = np.array([sc.desc().background_color.x, sc.desc().background_color.y, sc.desc().background_color.z],
                  np.float32)
    assert np.array_equal(bits(full[mask == 0]), bits(np.broadcast_to(bg, full[mask == 0].shape)))
    if name.startswith("14-01") and w == 1920:
        frac = float(mask.mean())
        assert 0.15 < frac < 0.4, frac     # the dragon's root cell covers ~28% of the C2 frame


@pytest.mark.parametrize("graph", [1, 0], ids=["graph", "no-graph"])
def test_c3_recorded_level_sizes(N, devbuf, graph):
    """Wavefront frames after the first launch every level with the recorded
    level sizes and no host read-back (as a captured HIP graph, or launch by
    launch): the same bits as the read-back frame, through the host and the
    device entry points, and for a second tile list (a shard) next to the
    full frame's."""
    sc = scene_npz("11-01-refractive__scene8").set_resolution(320, 180)
    st = N.RendererSettings.default(max_ray_depth=8)
    ref = N.HipScene(sc, wf_replay=0).render(st)
    g = N.HipScene(sc, wf_graph=graph)
    for _ in range(3):
        assert np.array_equal(bits(g.render(st)), bits(ref))
    d = devbuf.alloc(ref.nbytes)
    for _ in range(2):
        g.render_device(st, d)
        devbuf.sync()
        assert np.array_equal(bits(devbuf.download(d, ref.shape, np.float32)), bits(ref))
    stride = g.shard_stride(2)
    packed = devbuf.alloc(4 * stride)
    outs = []
    for _ in range(2):
        g.render_shard(st, 1, 2, packed)
        devbuf.sync()
        outs.append(devbuf.download(packed, (stride,), np.float32))
        assert np.array_equal(bits(g.render(st)), bits(ref))
    assert np.array_equal(bits(outs[0]), bits(outs[1]))


def test_c3_recorded_sizes_overflow(N, devbuf):
    """A frame whose levels outgrow the recorded sizes (forced: wf_replay 2
    records every size one short) is detected: crt_hip_render renders it again
    with read-backs, a device-side render reports it on the next call."""
    sc = scene_npz("11-01-refractive__scene8").set_resolution(160, 90)
    st = N.RendererSettings.default(max_ray_depth=8)
    ref = N.HipScene(sc, wf_replay=0).render(st)
    g = N.HipScene(sc, wf_replay=2)
    assert np.array_equal(bits(g.render(st)), bits(ref))      # read-back frame, sizes recorded one short
    assert np.array_equal(bits(g.render(st)), bits(ref))      # replay overflows: rendered again (and re-recorded)
    d = devbuf.alloc(ref.nbytes)
    g.render_device(st, d)                                    # replay overflows (reported on the next call)
    devbuf.sync()
    with pytest.raises(N.CrtError):
        g.render_device(st, d)


def test_c3_frames_pipelined(N, devbuf):
    """Recorded-size wavefront frames issued back to back take the free buffer
    sets (up to 12, each set's levels on a stream of its own), so frame k + 1's
    levels run beside frame k's (crt_host_render.hip render_wavefront; each set
    replays a graph captured on its own buffers); the pixels stay in the
    caller's stream order.  Twelve frames into four rotating buffers, then a
    host frame: all equal the read-back frame."""
    sc = scene_npz("11-01-refractive__scene8").set_resolution(480, 270)
    st = N.RendererSettings.default(max_ray_depth=8)
    ref = N.HipScene(sc, wf_replay=0).render(st)
    g = N.HipScene(sc)
    assert np.array_equal(bits(g.render(st)), bits(ref))   # records the level sizes
    d = [devbuf.alloc(ref.nbytes) for _ in range(4)]
    for k in range(12):
        g.render_device(st, d[k % 4])
    for k in range(4):
        assert np.array_equal(bits(devbuf.download(d[k], ref.shape, np.float32)), bits(ref))
    assert np.array_equal(bits(g.render(st)), bits(ref))


def test_c3_frames_pipelined_full_size_every_frame(N, oracle, devbuf):
    """The bench's own C3 mode at the benched size: 1920x1080 depth-8 frames
    issued back to back (levels of up to 12 frames side by side on the sets'
    streams), each into a buffer of its own; every one of the 24 frames equal
    to the oracle's frame."""
    h = HASHES["C3"]
    sc = scene_npz(h["scene"])
    st = N.RendererSettings.default(**h["settings"])
    want = bits(oracle.OracleScene(sc).render(st))
    g = N.HipScene(sc)
    assert np.array_equal(bits(g.render(st)), want)   # records the level sizes
    nb = 1920 * 1080 * 3 * 4
    d = [devbuf.alloc(nb) for _ in range(24)]
    for k in range(24):
        g.render_device(st, d[k])
    bad = [k for k in range(24) if not np.array_equal(bits(devbuf.download(d[k], (1080, 1920, 3), np.float32)), want)]
    assert not bad, f"frames {bad} differ from the oracle"
    assert g.info()["wf_sets"] >= 2   # the frames did run on several sets


def test_c3_blocking_frames_stay_on_one_set(N):
    """A caller that waits for every frame (the CLI, _crt, the shim: the
    reference's blocking render_image) finds set 0 free each time and never
    allocates another set's buffers or captures another graph."""
    sc = scene_npz("11-01-refractive__scene8").set_resolution(480, 270)
    st = N.RendererSettings.default(max_ray_depth=8)
    g = N.HipScene(sc)
    first = g.render(st)
    for _ in range(20):
        assert np.array_equal(bits(g.render(st)), bits(first))
    assert g.info()["wf_sets"] <= 2, g.info()["wf_sets"]
