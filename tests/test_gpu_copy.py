"""crt_hip_render's compact image copy (crt_api.hip image_to_host): only each
row's span of non-background pixels crosses PCIe, the host writes the rest.
The reference's render_image returns the whole host image (crt_image.h:11-27,
crt_renderer.cpp:157-199), so every frame here must equal the oracle's, or
the whole-image copy of the same frame, bit for bit — into pageable and pinned
memory, with and without the previous frame's spans as the prediction, and
when the prediction is wrong (camera moves, resolutions, scenes with no
background or nothing but background)."""
import ctypes as C

import numpy as np
import pytest

from conftest import bits, scene_npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    from crt_amd import native
    native.lib()
    return native


class Pinned:
    """hipHostMalloc'd float32 image (the runtime libcrt_hip.so loaded)."""

    def __init__(self, h, w):
        self.hip = C.CDLL("libamdhip64.so.7")
        self.hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
        self.hip.hipHostFree.argtypes = [C.c_void_p]
        self.p = C.c_void_p()
        n = h * w * 3
        assert self.hip.hipHostMalloc(C.byref(self.p), n * 4, 0) == 0
        self.a = np.ctypeslib.as_array((C.c_float * n).from_address(self.p.value)).reshape(h, w, 3)

    def close(self):
        self.a = None
        self.hip.hipHostFree(self.p)


def render_into(gpu, st, out):
    gpu.render_host(st, out.ctypes.data)
    return out


def test_compact_copy_c2_full_size(N, oracle):
    """C2 at 1920x1080: the first frame (no prediction) and the next frames
    (the prediction holds) into pageable memory, then into pinned memory,
    each against the oracle; garbage in the caller's buffer beforehand."""
    sc = scene_npz("14-01-acceleration-tree__scene1")
    st = N.RendererSettings.default()
    want = bits(oracle.OracleScene(sc).render(st))
    gpu = N.HipScene(sc)
    page = np.empty((1080, 1920, 3), np.float32)
    for k in range(3):
        page.view(np.uint32)[...] = 0x7fc00000 + k   # NaN garbage
        assert np.array_equal(bits(render_into(gpu, st, page)), want), f"pageable frame {k}"
    pin = Pinned(1080, 1920)
    try:
        for k in range(3):
            pin.a.view(np.uint32)[...] = 0xdeadbeef
            gpu.render_host(st, pin.p.value)
            assert np.array_equal(bits(pin.a), want), f"pinned frame {k}"
    finally:
        pin.close()
    gpu.set_option("compact_copy", 0)
    assert np.array_equal(bits(gpu.render(st)), want)


def test_compact_copy_camera_moves(N):
    """Poses in turn (each frame's prediction is the previous pose's spans:
    bands that match and bands that do not), then the same pose twice, each
    frame against the whole-image copy of that pose."""
    from crt_amd.camera import orbit_poses
    name = "14-01-acceleration-tree__scene1"
    sc = scene_npz(name).set_resolution(960, 540)
    st = N.RendererSettings.default()
    gpu = N.HipScene(sc)
    ref = N.HipScene(sc, compact_copy=0)
    fov = float(sc.a["cam_fov"][0])
    poses = orbit_poses(scene_npz(name).a, 6, yaw_amp=35.0, pitch_amp=15.0)
    for k, (loc, rot) in enumerate(poses + poses[::-1] + [poses[2], poses[2]]):
        for g in (gpu, ref):
            g.set_camera(location=loc, rotation=rot, fov_degrees=fov)
        out = np.full((540, 960, 3), 3.0, np.float32)
        render_into(gpu, st, out)
        assert np.array_equal(bits(out), bits(ref.render(st))), f"pose {k}"


@pytest.mark.parametrize("name,size,over", [
    ("11-01-refractive__scene8", (1920, 1080), {"max_ray_depth": 8}),   # C3: 63 % of the pixels hit
    ("15-01-conclusion__scene2", (96, 96), {}),                          # GI, a frame of no background
    ("14-01-acceleration-tree__scene1", (161, 97), {}),                  # rows of 3 W % 4 != 0 floats
    ("14-01-acceleration-tree__scene1", (7, 1), {}),
])
def test_compact_copy_frames_equal_oracle(N, oracle, name, size, over):
    sc = scene_npz(name).set_resolution(*size)
    st = N.RendererSettings.default(**over)
    want = bits(oracle.OracleScene(sc).render(st))
    gpu = N.HipScene(sc)
    for k in range(2):
        out = np.full((size[1], size[0], 3), -1.0, np.float32)
        assert np.array_equal(bits(render_into(gpu, st, out)), want), f"frame {k}"


def test_compact_copy_all_background_and_resizes(N):
    """A camera that sees nothing (every row's span empty), then back, then
    new resolutions (the copy's buffers follow the frame size)."""
    name = "14-01-acceleration-tree__scene1"
    sc = scene_npz(name).set_resolution(320, 180)
    st = N.RendererSettings.default()
    gpu = N.HipScene(sc)
    ref = N.HipScene(sc, compact_copy=0)
    loc = np.asarray(sc.a["cam_loc"], np.float32)
    rot = np.asarray(sc.a["cam_rot"], np.float32)
    away = (loc, (-rot.reshape(3, 3)).ravel())   # turned around: axes negated (right, up, back)
    for pose, size in [(away, (320, 180)), ((loc, rot), (320, 180)), (away, (320, 180)),
                       ((loc, rot), (200, 120)), ((loc, rot), (640, 360)), (away, (64, 48))]:
        for g in (gpu, ref):
            g.set_camera(location=pose[0], rotation=pose[1], width=size[0], height=size[1])
        for _ in range(2):
            out = np.full((size[1], size[0], 3), 9.0, np.float32)
            render_into(gpu, st, out)
            assert np.array_equal(bits(out), bits(ref.render(st)))
    bg = np.asarray(sc.a["background"], np.float32)
    gpu.set_camera(location=away[0], rotation=away[1], width=64, height=48)
    out = gpu.render(st)
    assert np.array_equal(bits(out), bits(np.broadcast_to(bg, out.shape))), "nothing in view: all background"
