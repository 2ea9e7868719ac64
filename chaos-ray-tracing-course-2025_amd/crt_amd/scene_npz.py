"""Flat scene description <-> .npz (a data format next to the path).

A crt_scene_desc (include/crt_hip.h) is serialised as numpy arrays so a parsed
.crtscene travels to machines without the scene files (the GPU box never sees
/root/reference).  The arrays are exactly what the loader produced (fp32 after
rapidjson-style GetFloat narrowing), so a round trip is bit-exact.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from .native import (CameraDesc, LightDesc, MaterialDesc, MeshDesc, SceneDesc, TextureDesc, Vec3)


def _texels(b8: np.ndarray) -> np.ndarray:
    """read_stb's conversion of decoded bytes: byte / 255.0f in fp32 (crt_image_stbi.cpp:29-37)."""
    return (b8.astype(np.float32) / np.float32(255.0)).astype(np.float32)


def desc_to_arrays(d: SceneDesc) -> dict:
    out = {
        "background": np.array([d.background_color.x, d.background_color.y, d.background_color.z], np.float32),
        "cam_loc": np.array([d.camera.location.x, d.camera.location.y, d.camera.location.z], np.float32),
        "cam_rot": np.array(list(d.camera.rotation), np.float32),
        "cam_size": np.array([d.camera.width, d.camera.height], np.int32),
        "cam_fov": np.array([d.camera.fov_degrees], np.float32),
        "flags": np.array([d.bucket_size, d.gi_on, d.reflections_on, d.refractions_on], np.int32),
    }
    mats = [(m.type, m.albedo_texture_index, m.ior, m.smooth_shading, m.back_face_culling)
            for m in (d.materials[i] for i in range(d.material_count))]
    out["mat_i"] = np.array([[t, a, s, b] for t, a, _, s, b in mats], np.int32).reshape(-1, 4)
    out["mat_ior"] = np.array([m[2] for m in mats], np.float32)
    tex_f, tex_i = [], []
    for i in range(d.texture_count):
        t = d.textures[i]
        if t.type == 3:   # decoded texels (fp32 = byte / 255.0f, crt_image_stbi.cpp:29-37), top row first
            n = t.bitmap_width * t.bitmap_height * 3
            rgb = np.ctypeslib.as_array(t.bitmap_rgb, (n,)).copy().reshape(t.bitmap_height, t.bitmap_width, 3)
            b8 = np.clip(np.rint(rgb * 255.0), 0, 255).astype(np.uint8)
            if np.array_equal(_texels(b8).view(np.uint32), rgb.view(np.uint32)):
                out[f"tex{i}_rgb8"] = b8          # lossless: the bytes read_stb produced
            else:
                out[f"tex{i}_rgb"] = rgb
        tex_i.append(t.type)
        tex_f.append([t.color0.x, t.color0.y, t.color0.z, t.color1.x, t.color1.y, t.color1.z, t.scalar])
    out["tex_i"] = np.array(tex_i, np.int32)
    out["tex_f"] = np.array(tex_f, np.float32).reshape(-1, 7)
    out["lights"] = np.array([[d.lights[i].intensity, d.lights[i].position.x, d.lights[i].position.y,
                               d.lights[i].position.z] for i in range(d.light_count)], np.float32).reshape(-1, 4)
    out["mesh_count"] = np.array([d.mesh_count], np.int32)
    for i in range(d.mesh_count):
        m = d.meshes[i]
        nv, ni = m.vertex_count, m.index_count
        out[f"m{i}_pos"] = np.ctypeslib.as_array(m.positions, (nv * 3,)).copy() if nv else np.zeros(0, np.float32)
        out[f"m{i}_idx"] = np.ctypeslib.as_array(m.indices, (ni,)).copy() if ni else np.zeros(0, np.int32)
        if m.uvs:
            out[f"m{i}_uv"] = np.ctypeslib.as_array(m.uvs, (nv * 3,)).copy()
        out[f"m{i}_mat"] = np.array([m.material_index], np.int32)
    return out


class ArrayScene:
    """A crt_scene_desc backed by numpy arrays (from desc_to_arrays / an .npz)."""

    def __init__(self, arrays: dict):
        self.a = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
        a = self.a
        n = int(a["mesh_count"][0])
        self._meshes = (MeshDesc * max(n, 1))()
        for i in range(n):
            pos, idx = a[f"m{i}_pos"].astype(np.float32), a[f"m{i}_idx"].astype(np.int32)
            a[f"m{i}_pos"], a[f"m{i}_idx"] = pos, idx
            uv = a.get(f"m{i}_uv")
            self._meshes[i] = MeshDesc(pos.ctypes.data_as(C.POINTER(C.c_float)),
                                       uv.ctypes.data_as(C.POINTER(C.c_float)) if uv is not None else None,
                                       pos.size // 3, idx.ctypes.data_as(C.POINTER(C.c_int32)), idx.size,
                                       int(a[f"m{i}_mat"][0]))
        nm = len(a["mat_i"])
        self._mats = (MaterialDesc * max(nm, 1))()
        for i in range(nm):
            t, alb, s, b = (int(x) for x in a["mat_i"][i])
            self._mats[i] = MaterialDesc(t, alb, float(a["mat_ior"][i]), s, b)
        nt = len(a["tex_i"])
        self._tex = (TextureDesc * max(nt, 1))()
        for i in range(nt):
            f = a["tex_f"][i]
            self._tex[i].type = int(a["tex_i"][i])
            self._tex[i].color0 = Vec3(*f[0:3])
            self._tex[i].color1 = Vec3(*f[3:6])
            self._tex[i].scalar = float(f[6])
            rgb = a.get(f"tex{i}_rgb")
            if rgb is None and f"tex{i}_rgb8" in a:
                rgb = _texels(a[f"tex{i}_rgb8"])
            if rgb is not None:
                rgb = np.ascontiguousarray(rgb, np.float32)
                a[f"tex{i}_rgb"] = rgb
                self._tex[i].bitmap_height, self._tex[i].bitmap_width = rgb.shape[0], rgb.shape[1]
                self._tex[i].bitmap_rgb = rgb.ctypes.data_as(C.POINTER(C.c_float))
        nl = len(a["lights"])
        self._lights = (LightDesc * max(nl, 1))()
        for i in range(nl):
            self._lights[i] = LightDesc(float(a["lights"][i][0]), Vec3(*a["lights"][i][1:4]))
        w, h = (int(x) for x in a["cam_size"])
        cam = CameraDesc(Vec3(*a["cam_loc"]), (C.c_float * 9)(*a["cam_rot"]), w, h, float(a["cam_fov"][0]))
        bucket, gi, refl, refr = (int(x) for x in a["flags"])
        self._desc = SceneDesc(Vec3(*a["background"]), cam, bucket, gi, refl, refr,
                               self._meshes, n, self._mats, nm, self._tex, nt, self._lights, nl)

    def desc(self) -> SceneDesc:
        return self._desc

    def desc_ptr(self):
        return C.pointer(self._desc)

    def set_resolution(self, width: int, height: int) -> "ArrayScene":
        self._desc.camera.width = width
        self._desc.camera.height = height
        return self

    def set_camera(self, location=None, rotation=None, fov_degrees=None) -> "ArrayScene":
        """Move the camera (crt_camera.h: location, row-major rotation, fov)."""
        if location is not None:
            self._desc.camera.location = Vec3(*(float(x) for x in location))
        if rotation is not None:
            self._desc.camera.rotation = (C.c_float * 9)(*(float(x) for x in np.ravel(rotation)))
        if fov_degrees is not None:
            self._desc.camera.fov_degrees = float(fov_degrees)
        return self

    def set_settings(self, *, gi_on=None, reflections_on=None, refractions_on=None, bucket_size=None):
        if gi_on is not None:
            self._desc.gi_on = int(gi_on)
        if reflections_on is not None:
            self._desc.reflections_on = int(reflections_on)
        if refractions_on is not None:
            self._desc.refractions_on = int(refractions_on)
        if bucket_size is not None:
            self._desc.bucket_size = int(bucket_size)
        return self


def save_npz(desc_src, path: str | Path) -> None:
    d = desc_src.desc() if hasattr(desc_src, "desc") else desc_src
    np.savez_compressed(path, **desc_to_arrays(d))


def load_npz(path: str | Path) -> ArrayScene:
    with np.load(path, allow_pickle=False) as z:
        return ArrayScene({k: z[k] for k in z.files})
