"""ctypes binding of the C-ABI in include/crt_hip.h (lib/libcrt_hip.so).

Host-side plumbing only: every computation runs in the native library (host
C++ for loading / tree build, HIP kernels for rendering).  There is no Python
or CPU fallback for the render path: if the library or a GPU is missing the
calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent          # chaos-ray-tracing-course-2025_amd/
LIB_PATH = PKG_DIR / "lib" / "libcrt_hip.so"

CRT_OK = 0
CRT_E_INVALID, CRT_E_PARSE, CRT_E_UNSUPPORTED, CRT_E_HIP, CRT_E_NOMEM, CRT_E_IO, CRT_E_STATE = -1, -2, -3, -4, -5, -6, -7

MATERIAL_DIFFUSE, MATERIAL_REFLECTIVE, MATERIAL_REFRACTIVE, MATERIAL_CONSTANT = 0, 1, 2, 3
TEXTURE_ALBEDO, TEXTURE_EDGES, TEXTURE_CHECKER, TEXTURE_BITMAP = 0, 1, 2, 3


class CrtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class ParseError(CrtError):
    pass


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class TextureDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("color0", Vec3), ("color1", Vec3), ("scalar", C.c_float),
                ("bitmap_width", C.c_int32), ("bitmap_height", C.c_int32),
                ("bitmap_rgb", C.POINTER(C.c_float))]


class MaterialDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("albedo_texture_index", C.c_int32), ("ior", C.c_float),
                ("smooth_shading", C.c_int32), ("back_face_culling", C.c_int32)]


class MeshDesc(C.Structure):
    _fields_ = [("positions", C.POINTER(C.c_float)), ("uvs", C.POINTER(C.c_float)),
                ("vertex_count", C.c_int64), ("indices", C.POINTER(C.c_int32)),
                ("index_count", C.c_int64), ("material_index", C.c_int32)]


class LightDesc(C.Structure):
    _fields_ = [("intensity", C.c_float), ("position", Vec3)]


class CameraDesc(C.Structure):
    _fields_ = [("location", Vec3), ("rotation", C.c_float * 9), ("width", C.c_int32),
                ("height", C.c_int32), ("fov_degrees", C.c_float)]


class SceneDesc(C.Structure):
    _fields_ = [("background_color", Vec3), ("camera", CameraDesc), ("bucket_size", C.c_int32),
                ("gi_on", C.c_int32), ("reflections_on", C.c_int32), ("refractions_on", C.c_int32),
                ("meshes", C.POINTER(MeshDesc)), ("mesh_count", C.c_int32),
                ("materials", C.POINTER(MaterialDesc)), ("material_count", C.c_int32),
                ("textures", C.POINTER(TextureDesc)), ("texture_count", C.c_int32),
                ("lights", C.POINTER(LightDesc)), ("light_count", C.c_int32)]


class TreeTriangle(C.Structure):
    """crt_tree_triangle: one Triangle copy of a leaf (crt_triangle.h:19-23)."""
    _fields_ = [("v", C.c_int32 * 3), ("face_normal", C.c_float * 3), ("material_index", C.c_int32),
                ("flags", C.c_int32)]


TREE_TRI_DTYPE = np.dtype([("v", "<i4", 3), ("face_normal", "<f4", 3), ("material_index", "<i4"), ("flags", "<i4")])
assert TREE_TRI_DTYPE.itemsize == C.sizeof(TreeTriangle)


class TreeSceneDesc(C.Structure):
    """crt_tree_scene_desc: the reference's built crt::Scene (crt_scene.h:18-30)."""
    _fields_ = [("background_color", Vec3), ("camera_location", Vec3), ("camera_rotation", C.c_float * 9),
                ("width", C.c_int32), ("height", C.c_int32), ("fov_radians", C.c_float), ("bucket_size", C.c_int32),
                ("gi_on", C.c_int32), ("reflections_on", C.c_int32), ("refractions_on", C.c_int32),
                ("vertices", C.POINTER(C.c_float)), ("vertex_count", C.c_int64),
                ("node_bounds", C.POINTER(C.c_float)), ("node_children", C.POINTER(C.c_int32)),
                ("leaf_offsets", C.POINTER(C.c_int64)), ("leaf_triangles", C.POINTER(TreeTriangle)),
                ("node_count", C.c_int64),
                ("materials", C.POINTER(MaterialDesc)), ("material_count", C.c_int32),
                ("textures", C.POINTER(TextureDesc)), ("texture_count", C.c_int32),
                ("lights", C.POINTER(LightDesc)), ("light_count", C.c_int32)]


class RendererSettings(C.Structure):
    """crt_renderer.h:18-25; defaults = crt_renderer.h:10-16."""
    _fields_ = [("max_ray_depth", C.c_uint32), ("diffuse_reflection_ray_count", C.c_uint32),
                ("shadow_bias", C.c_float), ("reflection_bias", C.c_float),
                ("diffuse_reflection_bias", C.c_float), ("refraction_bias", C.c_float)]

    @classmethod
    def default(cls, **over) -> "RendererSettings":
        s = cls(3, 4, 1e-2, 1e-2, 1e-2, 1e-2)
        for k, v in over.items():
            setattr(s, k, v)
        return s


class Hit(C.Structure):
    _fields_ = [("distance", C.c_float), ("point", C.c_float * 3), ("normal", C.c_float * 3),
                ("uv", C.c_float * 3), ("bary_u", C.c_float), ("bary_v", C.c_float),
                ("material_index", C.c_int32), ("hit", C.c_int32), ("triangle_index", C.c_int32)]


HIT_DTYPE = np.dtype([("distance", "<f4"), ("point", "<f4", 3), ("normal", "<f4", 3), ("uv", "<f4", 3),
                      ("bary_u", "<f4"), ("bary_v", "<f4"), ("material_index", "<i4"), ("hit", "<i4"),
                      ("triangle_index", "<i4")])
assert HIT_DTYPE.itemsize == C.sizeof(Hit)


class SceneInfo(C.Structure):
    _fields_ = [("triangle_count", C.c_int64), ("vertex_count", C.c_int64), ("node_count", C.c_int64),
                ("leaf_count", C.c_int64), ("leaf_ref_count", C.c_int64), ("max_depth", C.c_int32),
                ("max_leaf_size", C.c_int32), ("device_bytes", C.c_int64), ("width", C.c_int32),
                ("height", C.c_int32), ("bucket_size", C.c_int32), ("gi_on", C.c_int32),
                ("reflections_on", C.c_int32), ("refractions_on", C.c_int32), ("tree_on_device", C.c_int32),
                ("tree_build_ms", C.c_double), ("prep_ms", C.c_double), ("bvh_ms", C.c_double),
                ("bins_ms", C.c_double), ("upload_ms", C.c_double), ("create_ms", C.c_double),
                ("wf_sets", C.c_int32), ("pad0", C.c_int32), ("camera_moves", C.c_int64),
                ("view_rebuilds", C.c_int64), ("records_written", C.c_int64), ("multi_probe", C.c_int32),
                ("pad1", C.c_int32), ("multi_probe_ms", C.c_double), ("bins_binnings", C.c_int64),
                ("bins_reuses", C.c_int64), ("bvh_on_device", C.c_int32), ("bvh_depth", C.c_int32),
                ("light_bin_records", C.c_int64), ("light_bins_ms", C.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


TREE_AUTO, TREE_HOST, TREE_DEVICE = 0, 1, 2   # crt_hip_scene_create_ex flags
# further create flag bits (include/crt_hip.h)
SCENE_NO_DEVICE_BVH, SCENE_PROBE_OFF, SCENE_PROBE_FORCE, SCENE_PROBE_TEST_MISMATCH = 1 << 4, 1 << 5, 1 << 6, 1 << 7


class RenderStats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("total_ms", C.c_double), ("width", C.c_int32), ("height", C.c_int32)]


class WorkCounts(C.Structure):
    _fields_ = [("traversals", C.c_uint64), ("node_tests", C.c_uint64), ("triangle_tests", C.c_uint64),
                ("hits", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class WaveCounts(C.Structure):
    _fields_ = [("node_steps", C.c_uint64), ("triangle_steps", C.c_uint64), ("edge_steps", C.c_uint64),
                ("waves", C.c_uint64), ("box_steps", C.c_uint64), ("pass_steps", C.c_uint64),
                ("window_waves", C.c_uint64), ("window_steps", C.c_uint64), ("window_slots", C.c_uint64),
                ("window_reached", C.c_uint64), ("window_tri_rounds", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


# Every symbol include/crt_hip.h declares: (name, restype, argtypes)
_P = C.c_void_p
EXPORTS = [
    ("crt_scene_file_parse", C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(_P)]),
    ("crt_scene_file_load", C.c_int, [C.c_char_p, C.POINTER(_P)]),
    ("crt_scene_file_desc", C.POINTER(SceneDesc), [_P]),
    ("crt_scene_file_set_resolution", C.c_int, [_P, C.c_int32, C.c_int32]),
    ("crt_scene_file_destroy", None, [_P]),
    ("crt_image_decode_rgb8", C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), _P, C.c_size_t]),
    ("crt_host_scene_create", C.c_int, [C.POINTER(SceneDesc), C.POINTER(_P)]),
    ("crt_host_scene_info", C.c_int, [_P, C.POINTER(SceneInfo)]),
    ("crt_host_scene_tree", C.c_int, [_P, _P, _P, _P, _P]),
    ("crt_host_scene_vertex_normals", C.c_int, [_P, _P]),
    ("crt_host_scene_face_normals", C.c_int, [_P, _P]),
    ("crt_host_scene_destroy", None, [_P]),
    ("crt_hip_scene_create", C.c_int, [C.POINTER(SceneDesc), C.c_int, C.POINTER(_P)]),
    ("crt_hip_scene_create_ex", C.c_int, [C.POINTER(SceneDesc), C.c_int, C.c_int, C.POINTER(_P)]),
    ("crt_hip_device_count", C.c_int, []),
    ("crt_hip_scene_create_on", C.c_int, [C.POINTER(SceneDesc), _P, C.c_int32, C.c_int, C.POINTER(_P)]),
    ("crt_hip_scene_from_tree_on", C.c_int, [C.POINTER(TreeSceneDesc), _P, C.c_int32, C.POINTER(_P)]),
    ("crt_hip_scene_create_mask", C.c_int, [C.POINTER(SceneDesc), C.c_uint64, C.c_int, C.POINTER(_P)]),
    ("crt_hip_scene_from_tree_mask", C.c_int, [C.POINTER(TreeSceneDesc), C.c_uint64, C.POINTER(_P)]),
    ("crt_hip_scene_devices", C.c_int, [_P, _P, C.c_int32]),
    ("crt_multi_probe_verdict", C.c_int, [_P, _P, C.c_int64, C.c_int]),
    ("crt_auto_gpus", C.c_int, [C.POINTER(SceneDesc), C.POINTER(RendererSettings), C.c_int]),
    ("crt_auto_gpus_tree", C.c_int, [C.POINTER(TreeSceneDesc), C.POINTER(RendererSettings), C.c_int]),
    ("crt_hip_scene_create_auto", C.c_int, [C.POINTER(SceneDesc), C.POINTER(RendererSettings), C.c_int, C.POINTER(_P)]),
    ("crt_hip_scene_from_tree_auto", C.c_int, [C.POINTER(TreeSceneDesc), C.POINTER(RendererSettings),
                                               C.POINTER(_P)]),
    ("crt_hip_last_replica_ms", C.c_int, [_P, _P, C.c_int32]),
    ("crt_hip_scene_from_tree", C.c_int, [C.POINTER(TreeSceneDesc), C.c_int, C.POINTER(_P)]),
    ("crt_hip_render_image_tree", C.c_int, [C.POINTER(TreeSceneDesc), C.POINTER(RendererSettings), _P]),
    ("crt_hip_render_image_tree_stats", C.c_int, [C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    ("crt_hip_render_image_tree_reset", None, []),
    ("crt_host_scene_from_tree", C.c_int, [C.POINTER(TreeSceneDesc), C.POINTER(_P)]),
    ("crt_hip_scene_tree", C.c_int, [_P, _P, _P, _P, _P]),
    ("crt_hip_scene_bvh", C.c_int64, [_P, _P, _P]),
    ("crt_hip_scene_upload", C.c_int, [_P, C.c_int, C.POINTER(_P)]),
    ("crt_hip_scene_info", C.c_int, [_P, C.POINTER(SceneInfo)]),
    ("crt_hip_scene_destroy", None, [_P]),
    ("crt_hip_render", C.c_int, [_P, C.POINTER(RendererSettings), _P, C.POINTER(RenderStats)]),
    ("crt_hip_render_device", C.c_int, [_P, C.POINTER(RendererSettings), _P, _P]),
    ("crt_hip_shard_floats", C.c_int64, [_P, C.c_int, C.c_int]),
    ("crt_hip_shard_stride", C.c_int64, [_P, C.c_int]),
    ("crt_hip_render_shard", C.c_int, [_P, C.POINTER(RendererSettings), C.c_int, C.c_int, _P, _P]),
    ("crt_hip_unpack_shards", C.c_int, [_P, C.c_int, _P, _P, _P]),
    ("crt_hip_unpack_shards_rgb8", C.c_int, [_P, C.c_int, _P, _P, _P]),
    ("crt_hip_quantize_rgb8", C.c_int, [_P, C.c_int64, C.c_int32, _P, _P]),
    ("crt_hip_live_mask", C.c_int, [_P, _P]),
    ("crt_hip_compact_floats", C.c_int64, [_P, C.c_int, C.c_int]),
    ("crt_hip_compact_stride", C.c_int64, [_P, C.c_int]),
    ("crt_hip_render_shard_compact", C.c_int, [_P, C.POINTER(RendererSettings), C.c_int, C.c_int, _P, _P]),
    ("crt_hip_unpack_compact", C.c_int, [_P, C.c_int, _P, _P, _P]),
    ("crt_hip_unpack_compact_rgb8", C.c_int, [_P, C.c_int, _P, _P, _P]),
    ("crt_shard_compact_plan", C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_int, C.c_int, _P, _P, C.c_int64]),
    ("crt_shard_plan", C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_int, C.c_int, _P, C.c_int64]),
    ("crt_hip_trace_batch", C.c_int, [_P, _P, C.c_int64, _P]),
    ("crt_hip_camera_bins", C.c_int64, [_P, _P, _P, C.c_int64]),
    ("crt_host_camera_bins", C.c_int64, [_P, _P, _P, C.c_int64]),
    ("crt_hip_bins_time", C.c_int, [_P, C.c_int32, C.POINTER(C.c_double)]),
    ("crt_hip_count_work", C.c_int, [_P, C.POINTER(RendererSettings), C.POINTER(WorkCounts)]),
    ("crt_hip_last_kernel_ms", C.c_int, [_P, C.POINTER(C.c_double)]),
    ("crt_hip_plan_info", C.c_int, [_P, _P]),
    ("crt_hip_wave_counts", C.c_int, [_P, C.POINTER(WaveCounts)]),
    ("crt_hip_scene_set_option", C.c_int, [_P, C.c_char_p, C.c_int]),
    ("crt_hip_scene_set_camera", C.c_int, [_P, C.POINTER(CameraDesc)]),
    ("crt_hip_scene_set_camera_rad", C.c_int, [_P, C.POINTER(Vec3), C.POINTER(C.c_float), C.c_float, C.c_int32,
                                               C.c_int32]),
    ("crt_hip_scene_camera", C.c_int, [_P, C.POINTER(CameraDesc), C.POINTER(C.c_float)]),
    ("crt_hip_profile_waves", C.c_int, [_P, C.POINTER(RendererSettings), _P, C.c_int64, _P]),
    ("crt_hip_plan_tiles", C.c_int, [_P, C.POINTER(RendererSettings), _P, _P, C.c_int64]),
    ("crt_renderer_settings_default", None, [C.POINTER(RendererSettings)]),
    ("crt_write_ppm", C.c_int, [C.c_char_p, _P, C.c_int32, C.c_int32, C.c_int32]),
    ("crt_hip_last_error", C.c_char_p, []),
    ("crt_hip_abi_version", C.c_int, []),
    ("crt_hip_build_id", C.c_char_p, []),
]

_lib = None


def lib() -> C.CDLL:
    """Load lib/libcrt_hip.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise CrtError(CRT_E_UNSUPPORTED,
                           f"{LIB_PATH} is missing: build it with `make -C {PKG_DIR}` "
                           "(or __graft_entry__.build())")
        L = C.CDLL(str(LIB_PATH))
        for name, res, args in EXPORTS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    m = lib().crt_hip_last_error()
    return m.decode() if m else ""


def build_id() -> str:
    """Hash of the loaded library's sources and build flags (crt_hip_build_id)."""
    return lib().crt_hip_build_id().decode()


def _check(rc: int, exc=CrtError) -> None:
    if rc != CRT_OK:
        raise exc(rc, last_error())


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def decode_image(data: bytes) -> np.ndarray:
    """read_stb's pixel bytes (crt_image_stbi.cpp:16-40) for an image file's
    contents: uint8 (h, w, 3), top row first.  Raises CrtError where read_stb
    would fail (undecodable file, component count != 3)."""
    w, h, n = C.c_int32(), C.c_int32(), C.c_int32()
    _check(lib().crt_image_decode_rgb8(data, len(data), C.byref(w), C.byref(h), C.byref(n), None, 0))
    out = np.empty((h.value, w.value, 3), np.uint8)
    _check(lib().crt_image_decode_rgb8(data, len(data), C.byref(w), C.byref(h), C.byref(n),
                                       out.ctypes.data, out.nbytes))
    return out


# --------------------------------------------------------------------------
#  scene descriptions
# --------------------------------------------------------------------------
class SceneFile:
    """A parsed .crtscene (crt_json.cpp:541-647 semantics), owned by the C library."""

    def __init__(self, path: str | os.PathLike | None = None, text: str | bytes | None = None,
                 asset_root: str = ""):
        h = C.c_void_p()
        if path is not None:
            _check(lib().crt_scene_file_load(str(path).encode(), C.byref(h)), ParseError)
        else:
            data = text.encode() if isinstance(text, str) else text
            _check(lib().crt_scene_file_parse(data, len(data), asset_root.encode(), C.byref(h)), ParseError)
        self._h = h

    @property
    def handle(self):
        return self._h

    def desc(self) -> SceneDesc:
        d = lib().crt_scene_file_desc(self._h).contents
        d._owner = self          # the struct views memory this object owns
        return d

    def desc_ptr(self):
        return lib().crt_scene_file_desc(self._h)

    def set_resolution(self, width: int, height: int) -> "SceneFile":
        _check(lib().crt_scene_file_set_resolution(self._h, width, height))
        return self

    def close(self):
        if getattr(self, "_h", None):
            lib().crt_scene_file_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SyntheticScene:
    """A scene description built from numpy arrays (keeps them alive)."""

    def __init__(self, positions: np.ndarray, indices: np.ndarray, *, width: int, height: int,
                 camera_location=(0.0, 0.0, 0.0), camera_rotation=None, fov_degrees: float = 90.0,
                 background=(0.0, 0.5, 0.0), albedo=(0.8, 0.8, 0.8), lights=((1000.0, (2.0, 2.0, 3.0)),),
                 bucket_size: int = 24, smooth_shading: bool = False, gi_on: bool = False):
        self.positions = np.ascontiguousarray(positions, dtype=np.float32).reshape(-1)
        self.indices = np.ascontiguousarray(indices, dtype=np.int32).reshape(-1)
        self._mesh = (MeshDesc * 1)()
        self._mesh[0] = MeshDesc(_fptr(self.positions), None, self.positions.size // 3,
                                 self.indices.ctypes.data_as(C.POINTER(C.c_int32)), self.indices.size, 0)
        self._tex = (TextureDesc * 1)()
        self._tex[0].type = TEXTURE_ALBEDO
        self._tex[0].color0 = Vec3(*albedo)
        self._mat = (MaterialDesc * 1)()
        self._mat[0] = MaterialDesc(MATERIAL_DIFFUSE, 0, 1.0, int(smooth_shading), 0)
        self._lights = (LightDesc * len(lights))()
        for i, (inten, pos) in enumerate(lights):
            self._lights[i] = LightDesc(inten, Vec3(*pos))
        rot = camera_rotation if camera_rotation is not None else (1, 0, 0, 0, 1, 0, 0, 0, 1)
        cam = CameraDesc(Vec3(*camera_location), (C.c_float * 9)(*rot), width, height, fov_degrees)
        self._desc = SceneDesc(Vec3(*background), cam, bucket_size, int(gi_on), 1, 1,
                               self._mesh, 1, self._mat, 1, self._tex, 1, self._lights, len(lights))

    def desc(self) -> SceneDesc:
        return self._desc

    def desc_ptr(self):
        return C.pointer(self._desc)


class TreeScene:
    """A crt_tree_scene_desc over numpy arrays: the reference's vertex array
    (9 floats per vertex) and its built tree (bounds, children, leaf offsets,
    leaf Triangle copies), plus materials / textures / lights / camera / flags
    taken from a scene description (`shading`, e.g. an ArrayScene)."""

    def __init__(self, shading, vertices, bounds, children, leaf_offsets, leaf_triangles):
        d = shading.desc()
        self._shading = shading
        self.vertices = np.ascontiguousarray(vertices, np.float32).reshape(-1)
        self.bounds = np.ascontiguousarray(bounds, np.float32).reshape(-1)
        self.children = np.ascontiguousarray(children, np.int32).reshape(-1)
        self.offsets = np.ascontiguousarray(leaf_offsets, np.int64).reshape(-1)
        self.tris = np.ascontiguousarray(leaf_triangles).view(TREE_TRI_DTYPE).reshape(-1)
        n = self.offsets.size - 1
        # crt_camera.h:20: m_fov_radians = fov_degrees * pi_v<float> / 180.0f (float ops)
        fov = np.float32(np.float32(d.camera.fov_degrees) * np.float32(np.pi)) / np.float32(180.0)
        self._desc = TreeSceneDesc(
            d.background_color, d.camera.location, d.camera.rotation, d.camera.width, d.camera.height,
            float(fov), d.bucket_size, d.gi_on, d.reflections_on, d.refractions_on,
            _fptr(self.vertices), self.vertices.size // 9, _fptr(self.bounds),
            self.children.ctypes.data_as(C.POINTER(C.c_int32)), self.offsets.ctypes.data_as(C.POINTER(C.c_int64)),
            self.tris.ctypes.data_as(C.POINTER(TreeTriangle)), n,
            d.materials, d.material_count, d.textures, d.texture_count, d.lights, d.light_count)

    def set_resolution(self, width: int, height: int) -> "TreeScene":
        self._desc.width, self._desc.height = width, height
        return self

    def set_camera(self, location=None, rotation=None, fov_radians=None) -> "TreeScene":
        """The reference Camera's transform and stored m_fov_radians."""
        if location is not None:
            self._desc.camera_location = Vec3(*(float(x) for x in location))
        if rotation is not None:
            self._desc.camera_rotation = (C.c_float * 9)(*(float(x) for x in np.ravel(rotation)))
        if fov_radians is not None:
            self._desc.fov_radians = float(fov_radians)
        return self

    def tree_desc_ptr(self):
        return C.pointer(self._desc)


def _desc_ptr(src):
    if hasattr(src, "desc_ptr"):
        return src.desc_ptr()
    if isinstance(src, SceneDesc):
        return C.pointer(src)
    return src


# crt_layout.h CamCand (96 B): one camera-bins candidate
CAMCAND_DTYPE = np.dtype([("lo_x", "<f4"), ("hi_x", "<f4"), ("lo_y", "<f4"), ("hi_y", "<f4"), ("lo_z", "<f4"),
                          ("hi_z", "<f4"), ("dmin", "<f4"), ("id", "<i4"), ("g", "<f4", (12,)), ("mask", "<u8"),
                          ("rest", "<u8")])
assert CAMCAND_DTYPE.itemsize == 96


def _camera_bins(fn, handle, width: int, height: int):
    """(len[cells], records) of a camera-bins hook (crt_hip_camera_bins /
    crt_host_camera_bins): per 8x8 cell its list length (-1: over the cell cap)
    and the lists back to back in cell order."""
    ncell = ((width + 7) // 8) * ((height + 7) // 8)
    ln = np.zeros(ncell, np.int32)
    n = fn(handle, ln.ctypes.data, None, 0)
    if n < 0:
        _check(int(n))
    recs = np.zeros(max(int(n), 1), CAMCAND_DTYPE)
    m = fn(handle, ln.ctypes.data, recs.ctypes.data, max(int(n), 1))
    if m < 0:
        _check(int(m))
    return ln, recs[:int(m)]


# --------------------------------------------------------------------------
#  host scene (mesh prep + tree build, no GPU)
# --------------------------------------------------------------------------
class HostScene:
    def __init__(self, src):
        h = C.c_void_p()
        if hasattr(src, "tree_desc_ptr"):
            _check(lib().crt_host_scene_from_tree(src.tree_desc_ptr(), C.byref(h)))
        else:
            _check(lib().crt_host_scene_create(_desc_ptr(src), C.byref(h)))
        self._h = h
        self._src = src

    def info(self) -> dict:
        i = SceneInfo()
        _check(lib().crt_host_scene_info(self._h, C.byref(i)))
        return i.as_dict()

    def tree(self):
        """(bounds[n,6], children[n,2], leaf_offsets[n+1], leaf_tris[m]) in reference numbering."""
        info = self.info()
        n, m = info["node_count"], info["leaf_ref_count"]
        b = np.zeros((n, 6), np.float32)
        c = np.zeros((n, 2), np.int32)
        o = np.zeros(n + 1, np.int64)
        t = np.zeros(max(m, 1), np.int32)
        _check(lib().crt_host_scene_tree(self._h, b.ctypes.data, c.ctypes.data, o.ctypes.data, t.ctypes.data))
        return b, c, o, t[:m]

    def vertex_normals(self) -> np.ndarray:
        out = np.zeros((self.info()["vertex_count"], 3), np.float32)
        _check(lib().crt_host_scene_vertex_normals(self._h, out.ctypes.data))
        return out

    def camera_bins(self):
        """The host checker's camera bins (build_camera_bins): (len[cells], records)."""
        i = self.info()
        return _camera_bins(lib().crt_host_camera_bins, self._h, i["width"], i["height"])

    def face_normals(self) -> np.ndarray:
        out = np.zeros((self.info()["triangle_count"], 3), np.float32)
        _check(lib().crt_host_scene_face_normals(self._h, out.ctypes.data))
        return out

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            lib().crt_host_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --------------------------------------------------------------------------
#  device scene (HBM-resident) and rendering
# --------------------------------------------------------------------------
class PlanInfo(C.Structure):
    _fields_ = [("calib_k", C.c_double), ("tiles", C.c_int32), ("small_tiles", C.c_int32)]


class HipScene:
    def __init__(self, src, device: int = 0, tree_build: str = "auto", devices=None, create_flags: int = 0,
                 **options):
        """tree_build: "auto" | "host" | "device" — where the acceleration tree is
        built (crt_hip_scene_create_ex; both builds give identical bits).
        devices: a list of HIP devices (repeats allowed) — the scene replicated
        on each, frames split over them (crt_hip_scene_create_on).
        create_flags: further SCENE_* flag bits of the create call."""
        h = C.c_void_p()
        flag = {"auto": TREE_AUTO, "host": TREE_HOST, "device": TREE_DEVICE}[tree_build] | int(create_flags)
        if devices is not None:
            devs = np.ascontiguousarray(devices, np.int32)
            if hasattr(src, "tree_desc_ptr"):
                _check(lib().crt_hip_scene_from_tree_on(src.tree_desc_ptr(), devs.ctypes.data, len(devs), C.byref(h)))
            else:
                _check(lib().crt_hip_scene_create_on(_desc_ptr(src), devs.ctypes.data, len(devs), flag, C.byref(h)))
            device = int(devs[0])
        elif isinstance(src, HostScene):
            _check(lib().crt_hip_scene_upload(src.handle, device, C.byref(h)))
        elif hasattr(src, "tree_desc_ptr"):
            _check(lib().crt_hip_scene_from_tree(src.tree_desc_ptr(), device, C.byref(h)))
        else:
            _check(lib().crt_hip_scene_create_ex(_desc_ptr(src), device, flag, C.byref(h)))
        self._h = h
        self.device = device
        for k, v in options.items():
            self.set_option(k, v)

    def devices(self) -> list:
        """HIP devices of the scene's replicas (crt_hip_scene_devices)."""
        n = lib().crt_hip_scene_devices(self._h, None, 0)
        _check(min(int(n), 0))
        out = np.zeros(n, np.int32)
        _check(min(int(lib().crt_hip_scene_devices(self._h, out.ctypes.data, n)), 0))
        return [int(d) for d in out]

    def replica_ms(self) -> list:
        """Kernel ms of each replica's shard in the last render (crt_hip_last_replica_ms)."""
        n = len(self.devices())
        out = np.zeros(n, np.float64)
        _check(min(int(lib().crt_hip_last_replica_ms(self._h, out.ctypes.data, n)), 0))
        return [float(x) for x in out]

    def set_camera(self, location=None, rotation=None, fov_degrees=None, width=None, height=None) -> "HipScene":
        """A new camera for the next frames (crt_hip_scene_set_camera); omitted
        fields keep the current camera's."""
        cur = CameraDesc()
        _check(lib().crt_hip_scene_camera(self._h, C.byref(cur), None))
        loc = location if location is not None else (cur.location.x, cur.location.y, cur.location.z)
        rot = rotation if rotation is not None else tuple(cur.rotation)
        cam = CameraDesc(Vec3(*[float(v) for v in loc]), (C.c_float * 9)(*[float(v) for v in np.ravel(rot)]),
                         int(width if width is not None else cur.width), int(height if height is not None else cur.height),
                         float(fov_degrees if fov_degrees is not None else cur.fov_degrees))
        _check(lib().crt_hip_scene_set_camera(self._h, C.byref(cam)))
        return self

    def set_camera_desc(self, cam: CameraDesc) -> None:
        """crt_hip_scene_set_camera with a prepared CameraDesc (no read-back of the current camera)."""
        _check(lib().crt_hip_scene_set_camera(self._h, C.byref(cam)))

    def set_camera_rad(self, location, rotation, fov_radians: float, width: int, height: int) -> "HipScene":
        """Same with the reference Camera's stored m_fov_radians (crt_hip_scene_set_camera_rad)."""
        rot = (C.c_float * 9)(*[float(v) for v in np.ravel(rotation)])
        _check(lib().crt_hip_scene_set_camera_rad(self._h, C.byref(Vec3(*[float(v) for v in location])), rot,
                                                  float(fov_radians), int(width), int(height)))
        return self

    def camera(self) -> dict:
        cur = CameraDesc()
        fov = C.c_float()
        _check(lib().crt_hip_scene_camera(self._h, C.byref(cur), C.byref(fov)))
        return {"location": (cur.location.x, cur.location.y, cur.location.z), "rotation": tuple(cur.rotation),
                "width": cur.width, "height": cur.height, "fov_radians": fov.value}

    def set_option(self, name: str, value: int) -> "HipScene":
        """Walk selection (crt_hip_scene_set_option): traversal / secondary / wavefront / trace_walk."""
        _check(lib().crt_hip_scene_set_option(self._h, name.encode(), int(value)))
        return self

    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        i = SceneInfo()
        _check(lib().crt_hip_scene_info(self._h, C.byref(i)))
        return i.as_dict()

    def tree(self):
        """(bounds[n,6], children[n,2], leaf_offsets[n+1], leaf_tris[m]) in reference numbering."""
        info = self.info()
        n, m = info["node_count"], info["leaf_ref_count"]
        b = np.zeros((n, 6), np.float32)
        c = np.zeros((n, 2), np.int32)
        o = np.zeros(n + 1, np.int64)
        t = np.zeros(max(m, 1), np.int32)
        _check(lib().crt_hip_scene_tree(self._h, b.ctypes.data, c.ctypes.data, o.ctypes.data, t.ctypes.data))
        return b, c, o, t[:m]

    def bvh(self):
        """The secondary-ray BVH (crt_hip_scene_bvh): (nodes, tri_ids) with
        nodes an (8, N + 1) structured array of BNode records, or None."""
        n = lib().crt_hip_scene_bvh(self._h, None, None)
        if n < 0:
            _check(int(n))
        if n == 0:
            return None
        dt = np.dtype([("lo_x", "<f4"), ("hi_x", "<f4"), ("lo_y", "<f4"), ("hi_y", "<f4"), ("lo_z", "<f4"),
                       ("hi_z", "<f4"), ("skip", "<i4"), ("leaf", "<i4")])
        nodes = np.zeros((8, n + 1), dt)
        ids = np.zeros(self.info()["triangle_count"], np.int32)
        r = lib().crt_hip_scene_bvh(self._h, nodes.ctypes.data, ids.ctypes.data)
        if r < 0:
            _check(int(r))
        return nodes, ids
    def render(self, settings: RendererSettings | None = None, with_stats: bool = False):
        """Blocking render_image: returns float32 [H, W, 3], top row first."""
        st = settings or RendererSettings.default()
        info = self.info()
        out = np.empty((info["height"], info["width"], 3), np.float32)
        stats = RenderStats()
        _check(lib().crt_hip_render(self._h, C.byref(st), out.ctypes.data, C.byref(stats)))
        if with_stats:
            return out, {"kernel_ms": stats.kernel_ms, "total_ms": stats.total_ms}
        return out

    def render_host(self, settings: RendererSettings, host_ptr: int) -> dict:
        """Blocking render_image into caller memory at host_ptr (W*H*3 fp32; pinned
        memory makes the D2H a direct DMA).  Returns the call's stats."""
        stats = RenderStats()
        _check(lib().crt_hip_render(self._h, C.byref(settings), C.c_void_p(host_ptr), C.byref(stats)))
        return {"kernel_ms": stats.kernel_ms, "total_ms": stats.total_ms}

    def render_device(self, settings: RendererSettings, d_rgb: int, stream: int | None = None) -> None:
        _check(lib().crt_hip_render_device(self._h, C.byref(settings), C.c_void_p(d_rgb),
                                           C.c_void_p(stream or 0)))

    def shard_floats(self, shard: int, count: int) -> int:
        v = lib().crt_hip_shard_floats(self._h, shard, count)
        if v < 0:
            _check(int(v))
        return int(v)

    def shard_stride(self, count: int) -> int:
        v = lib().crt_hip_shard_stride(self._h, count)
        if v < 0:
            _check(int(v))
        return int(v)

    def render_shard(self, settings: RendererSettings, shard: int, count: int, d_packed: int,
                     stream: int | None = None) -> None:
        _check(lib().crt_hip_render_shard(self._h, C.byref(settings), shard, count, C.c_void_p(d_packed),
                                          C.c_void_p(stream or 0)))

    def unpack_shards(self, count: int, d_gathered: int, d_rgb: int, stream: int | None = None) -> None:
        _check(lib().crt_hip_unpack_shards(self._h, count, C.c_void_p(d_gathered), C.c_void_p(d_rgb),
                                           C.c_void_p(stream or 0)))

    # compact shards: only live tiles (camera ray passes the root-cell test) are
    # rendered / packed; unpacking writes the background into the others
    def live_mask(self) -> np.ndarray:
        info = self.info()
        out = np.zeros((info["height"], info["width"]), np.uint8)
        _check(lib().crt_hip_live_mask(self._h, out.ctypes.data))
        return out

    def compact_floats(self, shard: int, count: int) -> int:
        v = lib().crt_hip_compact_floats(self._h, shard, count)
        if v < 0:
            _check(int(v))
        return int(v)

    def compact_stride(self, count: int) -> int:
        v = lib().crt_hip_compact_stride(self._h, count)
        if v < 0:
            _check(int(v))
        return int(v)

    def render_shard_compact(self, settings: RendererSettings, shard: int, count: int, d_packed: int,
                             stream: int | None = None) -> None:
        _check(lib().crt_hip_render_shard_compact(self._h, C.byref(settings), shard, count, C.c_void_p(d_packed),
                                                  C.c_void_p(stream or 0)))

    def unpack_compact(self, count: int, d_gathered: int, d_rgb: int, stream: int | None = None) -> None:
        _check(lib().crt_hip_unpack_compact(self._h, count, C.c_void_p(d_gathered), C.c_void_p(d_rgb),
                                            C.c_void_p(stream or 0)))

    def unpack_compact_rgb8(self, count: int, d_gathered: int, d_rgb8: int, stream: int | None = None) -> None:
        _check(lib().crt_hip_unpack_compact_rgb8(self._h, count, C.c_void_p(d_gathered), C.c_void_p(d_rgb8),
                                                 C.c_void_p(stream or 0)))

    def unpack_shards_rgb8(self, count: int, d_gathered: int, d_rgb8: int, stream: int | None = None) -> None:
        _check(lib().crt_hip_unpack_shards_rgb8(self._h, count, C.c_void_p(d_gathered), C.c_void_p(d_rgb8),
                                                C.c_void_p(stream or 0)))

    def plan_info(self) -> dict:
        """The full-frame plan in use (crt_hip_plan_info): calib_k, tiles, small_tiles."""
        out = PlanInfo()
        _check(lib().crt_hip_plan_info(self._h, C.byref(out)))
        return {f: getattr(out, f) for f, _ in PlanInfo._fields_}

    def last_kernel_ms(self) -> float:
        v = C.c_double()
        _check(lib().crt_hip_last_kernel_ms(self._h, C.byref(v)))
        return v.value

    def bins_ms(self, frames: int = 50) -> float:
        """Device ms of one frame's camera binning alone (0 without camera bins)."""
        v = C.c_double()
        _check(lib().crt_hip_bins_time(self._h, frames, C.byref(v)))
        return v.value

    def camera_bins(self):
        """One frame's device camera bins (crt_bins.hip): (len[cells], records)."""
        i = self.info()
        return _camera_bins(lib().crt_hip_camera_bins, self._h, i["width"], i["height"])

    def trace(self, rays: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        out = np.zeros(len(rays), HIT_DTYPE)
        _check(lib().crt_hip_trace_batch(self._h, rays.ctypes.data, len(rays), out.ctypes.data))
        return out

    def profile_waves(self, settings: RendererSettings | None = None):
        """Diagnostic frame: (stamps[ntiles, 2] in 10-ns ticks, tile_xy[ntiles, 2]) in dispatch order."""
        st = settings or RendererSettings.default()
        n = lib().crt_hip_profile_waves(self._h, C.byref(st), None, 0, None)
        if n < 0:
            _check(n)
        stamps = np.zeros((n, 2), np.uint64)
        xy = np.zeros((n, 2), np.int32)
        rc = lib().crt_hip_profile_waves(self._h, C.byref(st), stamps.ctypes.data, n, xy.ctypes.data)
        if rc < 0:
            _check(rc)
        return stamps, xy

    def plan_tiles(self, settings: RendererSettings | None = None):
        """Diagnostic: full-frame tile plan (dispatch order) → (xywh[n, 4], measured cost[n])."""
        st = settings or RendererSettings.default()
        n = lib().crt_hip_plan_tiles(self._h, C.byref(st), None, None, 0)
        if n < 0:
            _check(n)
        xywh = np.zeros((n, 4), np.int32)
        cost = np.zeros(n, np.float32)
        rc = lib().crt_hip_plan_tiles(self._h, C.byref(st), xywh.ctypes.data, cost.ctypes.data, n)
        if rc < 0:
            _check(rc)
        return xywh, cost

    def count_work(self, settings: RendererSettings | None = None) -> dict:
        st = settings or RendererSettings.default()
        w = WorkCounts()
        _check(lib().crt_hip_count_work(self._h, C.byref(st), C.byref(w)))
        return w.as_dict()

    def wave_counts(self) -> dict:
        """Wave-level steps of the last count_work frame (packet walks only)."""
        w = WaveCounts()
        _check(lib().crt_hip_wave_counts(self._h, C.byref(w)))
        return w.as_dict()

    def close(self):
        if getattr(self, "_h", None):
            lib().crt_hip_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_image_tree(tree_scene: "TreeScene", settings: RendererSettings | None = None) -> np.ndarray:
    """crt::render_image's body for the reference's built Scene
    (crt_hip_render_image_tree: cached device scenes, camera moves in place):
    float32 [H, W, 3], top row first."""
    st = settings or RendererSettings.default()
    d = tree_scene.tree_desc_ptr().contents
    out = np.empty((d.height, d.width, 3), np.float32)
    _check(lib().crt_hip_render_image_tree(tree_scene.tree_desc_ptr(), C.byref(st), out.ctypes.data))
    return out


def render_image_tree_stats() -> dict:
    c, m, r = C.c_int64(), C.c_int64(), C.c_int64()
    _check(lib().crt_hip_render_image_tree_stats(C.byref(c), C.byref(m), C.byref(r)))
    return {"creates": c.value, "camera_moves": m.value, "reuses": r.value}


def shard_plan(width: int, height: int, bucket_size: int, shard: int, shard_count: int) -> np.ndarray:
    """Buckets of one shard: int64 [k, 6] = (x, y, w, h, packed_pixel_offset, bucket_index)."""
    n = lib().crt_shard_plan(width, height, bucket_size, shard, shard_count, None, 0)
    if n < 0:
        _check(int(n))
    out = np.zeros((n, 6), np.int64)
    if n:
        lib().crt_shard_plan(width, height, bucket_size, shard, shard_count, out.ctypes.data, n)
    return out


def quantize_rgb8(d_rgb: int, n: int, d_out: int, max_color_component: int = 255, stream: int | None = None) -> None:
    """Device write_ppm conversion of n floats at d_rgb into n bytes at d_out
    (crt_hip_quantize_rgb8, current device, `stream` or the null stream)."""
    _check(lib().crt_hip_quantize_rgb8(C.c_void_p(d_rgb), n, max_color_component, C.c_void_p(d_out),
                                       C.c_void_p(stream or 0)))


def shard_compact_plan(width: int, height: int, bucket_size: int, shard: int, shard_count: int,
                       live_mask: np.ndarray | None) -> np.ndarray:
    """Live tiles of one shard for a live-pixel mask (H x W bytes; None = all
    live): int64 [k, 5] = (x, y, w, h, packed_pixel_offset)."""
    m = None
    if live_mask is not None:
        live_mask = np.ascontiguousarray(live_mask, np.uint8)
        assert live_mask.shape == (height, width)
        m = live_mask.ctypes.data
    n = lib().crt_shard_compact_plan(width, height, bucket_size, shard, shard_count, m, None, 0)
    if n < 0:
        _check(int(n))
    out = np.zeros((n, 5), np.int64)
    if n:
        n2 = lib().crt_shard_compact_plan(width, height, bucket_size, shard, shard_count, m, out.ctypes.data, n)
        if n2 < 0:
            _check(int(n2))
        if n2 != n:
            raise RuntimeError(f"crt_shard_compact_plan: {n2} tiles on the second call, {n} on the first")
    return out


def write_ppm(path: str | os.PathLike, rgb: np.ndarray, max_color_component: int = 255) -> None:
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    _check(lib().crt_write_ppm(str(path).encode(), rgb.ctypes.data, w, h, max_color_component))
