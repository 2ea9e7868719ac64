""".crtscene documents from flat scene arrays (the inverse of the loader).

The GPU box never sees /root/reference, so the CLI and `_crt` surfaces are
exercised there on documents rebuilt from the committed .npz scenes.  The
loader (csrc/crt_json.cpp, restating crt_json.cpp:541-647) must read such a
document back to exactly the same crt_scene_desc:

* every float is written as the shortest decimal of the float32 value widened
  to double (exactly that float32), so parse-to-double + GetFloat narrowing
  gives the same bits;
* textures keep their order and are referenced by name, so material texture
  indices are unchanged (no inline albedo is re-appended);
* refractive materials carry `ior` and no `albedo` (crt_json.cpp:494-516).
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

_MAT_TYPES = {0: "diffuse", 1: "reflective", 2: "refractive", 3: "constant"}
_TEX_TYPES = {0: "albedo", 1: "edges", 2: "checker", 3: "bitmap"}


def _f(x) -> float:
    return float(np.float32(x))


def _vec(v) -> list:
    return [_f(x) for x in v]


def arrays_to_crtscene(a: dict, bitmap_files: dict | None = None) -> dict:
    """crt_amd.scene_npz arrays -> a .crtscene JSON document (Python dict).

    Bitmap textures are files next to the scene: `bitmap_files` maps a texture
    index to its "file_path" (read as asset_root / relative path), whose image
    must decode to the texels the arrays hold."""
    w, h = (int(x) for x in a["cam_size"])
    bucket, gi, refl, refr = (int(x) for x in a["flags"])
    doc: dict = {
        "settings": {
            "background_color": _vec(a["background"]),
            "image_settings": {"width": w, "height": h, "bucket_size": bucket},
            "gi_on": bool(gi), "reflections_on": bool(refl), "refractions_on": bool(refr),
        },
        "camera": {"matrix": _vec(a["cam_rot"]), "position": _vec(a["cam_loc"]),
                   "fov_degrees": _f(a["cam_fov"][0])},
        "lights": [{"intensity": _f(l[0]), "position": _vec(l[1:4])} for l in a["lights"]],
    }
    textures = []
    for i, (t, f) in enumerate(zip(a["tex_i"], a["tex_f"])):
        t = int(t)
        if t not in _TEX_TYPES:
            raise ValueError(f"texture type {t} has no .crtscene form here")
        d = {"name": f"tex{i}", "type": _TEX_TYPES[t]}
        if t == 0:
            d["albedo"] = _vec(f[0:3])
        elif t == 1:
            d.update(edge_color=_vec(f[0:3]), inner_color=_vec(f[3:6]), edge_width=_f(f[6]))
        elif t == 2:
            d.update(color_A=_vec(f[0:3]), color_B=_vec(f[3:6]), square_size=_f(f[6]))
        else:
            if not bitmap_files or i not in bitmap_files:
                raise ValueError(f"bitmap texture {i} needs its image file (bitmap_files)")
            d["file_path"] = bitmap_files[i]
        textures.append(d)
    doc["textures"] = textures
    mats = []
    for (t, alb, smooth, cull), ior in zip(a["mat_i"], a["mat_ior"]):
        m = {"type": _MAT_TYPES[int(t)], "smooth_shading": bool(smooth), "back_face_culling": bool(cull)}
        if int(t) == 2:
            m["ior"] = _f(ior)
        else:
            m["albedo"] = f"tex{int(alb)}"
        mats.append(m)
    doc["materials"] = mats
    objs = []
    for i in range(int(a["mesh_count"][0])):
        o = {"vertices": [_f(x) for x in a[f"m{i}_pos"]],
             "triangles": [int(x) for x in a[f"m{i}_idx"]],
             "material_index": int(a[f"m{i}_mat"][0])}
        if f"m{i}_uv" in a:
            o["uvs"] = [_f(x) for x in a[f"m{i}_uv"]]
        objs.append(o)
    doc["objects"] = objs
    return doc


def write_crtscene(a: dict, path: str | Path, bitmap_files: dict | None = None) -> Path:
    path = Path(path)
    path.write_text(json.dumps(arrays_to_crtscene(a, bitmap_files)))
    return path
