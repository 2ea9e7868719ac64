"""Scene loader (crt_json.cpp:541-647 semantics) — host only, no GPU.

Number parsing follows rapidjson's default (normal-precision) reader, which
is the third-party dependency the reference loader uses (vendor/rapidjson,
an un-checked-out submodule whose pinned commit is unavailable here).  Its
published algorithm (reader.h ParseNumber → internal/strtod.h
StrtodNormalPrecision) is restated in Python below and used as the checker;
for the ≤9-significant-digit decimals the course scenes contain it equals the
correctly rounded double, narrowed by GetFloat() to float32.
"""
import json
import math
import random

import numpy as np
import pytest

from conftest import REFERENCE, SCENES, bits, has_reference


def parse(text: str):
    from crt_amd.native import SceneFile
    return SceneFile(text=text)


def minimal(**over):
    doc = {
        "settings": {"background_color": [0, 0.5, 0], "image_settings": {"width": 64, "height": 48}},
        "camera": {"matrix": [1, 0, 0, 0, 1, 0, 0, 0, 1], "position": [0, 0, 0]},
        "lights": [{"intensity": 100, "position": [1, 2, 3]}],
        "materials": [{"type": "diffuse", "albedo": [0.5, 0.25, 1], "smooth_shading": False}],
        "objects": [{"material_index": 0, "vertices": [-1, -1, -3, 1, -1, -3, 0, 1, -3], "triangles": [0, 1, 2]}],
    }
    for k, v in over.items():
        doc[k] = v
    return doc


# ---------------------------------------------------------------- scene files
@pytest.mark.skipif(not has_reference(), reason="needs /root/reference scene files")
def test_scene_files_match_committed_fixtures():
    from crt_amd.native import SceneFile
    from crt_amd.scene_npz import desc_to_arrays
    for npz in sorted(SCENES.glob("*.npz")):
        rel = npz.stem.replace("__", "/")
        got = desc_to_arrays(SceneFile(path=REFERENCE / "scenes" / f"{rel}.crtscene").desc())
        want = np.load(npz)
        assert set(got) == set(want.files), rel
        for k in want.files:
            assert np.array_equal(bits(got[k]), bits(want[k])), (rel, k)


@pytest.mark.skipif(not has_reference(), reason="needs /root/reference scene files")
@pytest.mark.parametrize("rel", ["07-01-scene/scene0", "07-01-scene/scene4", "08-01-light/scene3",
                                 "09-01-barycentric-coordinates/scene0"])
def test_scene_files_the_reference_rejects(rel):
    """No "materials" (07-01, 08-01) or no "lights" (09-01/scene0): crt_json.cpp:590-592, 608-610."""
    from crt_amd.native import ParseError, SceneFile
    with pytest.raises(ParseError):
        SceneFile(path=REFERENCE / "scenes" / f"{rel}.crtscene")


@pytest.mark.skipif(not has_reference(), reason="needs /root/reference scene files")
def test_bitmap_scenes_load_with_the_decoder():
    """12-01 textures include a JPEG bitmap (read from the scene's directory,
    crt_json.cpp:358-360, decoded by csrc/crt_image_decode.cpp): the texture
    list survives and materials resolve the bitmap by name."""
    from crt_amd.native import SceneFile
    d = SceneFile(path=REFERENCE / "scenes" / "12-01-textures" / "scene3.crtscene").desc()
    assert d.textures[d.materials[0].albedo_texture_index].type == 3


# ---------------------------------------------------------------- defaults & rules
def test_defaults():
    d = parse(json.dumps(minimal())).desc()
    assert d.bucket_size == 24                        # crt_scene.h:16
    assert d.camera.fov_degrees == 90.0               # crt_camera.h:13-15
    assert (d.gi_on, d.reflections_on, d.refractions_on) == (0, 1, 1)   # crt_json.cpp:616
    assert d.material_count == 1 and d.texture_count == 1               # inline albedo → texture
    assert d.materials[0].albedo_texture_index == 0
    assert d.materials[0].back_face_culling == 0
    t = d.textures[0]
    assert (t.color0.x, t.color0.y, t.color0.z) == (0.5, 0.25, 1.0)


def test_settings_and_camera_fields():
    doc = minimal()
    doc["settings"].update({"gi_on": True, "reflections_on": False, "refractions_on": False})
    doc["settings"]["image_settings"]["bucket_size"] = 16
    doc["camera"]["fov_degrees"] = 45
    d = parse(json.dumps(doc)).desc()
    assert (d.gi_on, d.reflections_on, d.refractions_on, d.bucket_size) == (1, 0, 0, 16)
    assert d.camera.fov_degrees == 45.0 and (d.camera.width, d.camera.height) == (64, 48)


def test_textures_and_material_lookup():
    doc = minimal(textures=[{"name": "e", "type": "edges", "edge_color": [0, 1, 0], "inner_color": [1, 0, 0],
                             "edge_width": 0.04},
                            {"name": "c", "type": "checker", "color_A": [0, 0, 0], "color_B": [1, 1, 1],
                             "square_size": 0.125}],
                  materials=[{"type": "diffuse", "albedo": "c", "smooth_shading": True, "back_face_culling": True},
                             {"type": "refractive", "ior": 1.5, "smooth_shading": False},
                             {"type": "constant", "albedo": [1, 2, 3], "smooth_shading": False}])
    d = parse(json.dumps(doc)).desc()
    assert d.texture_count == 3
    assert d.materials[0].albedo_texture_index == 1 and d.materials[0].back_face_culling == 1
    assert d.materials[1].type == 2 and d.materials[1].albedo_texture_index == -1
    assert d.materials[1].ior == np.float32(1.5)
    assert d.materials[2].albedo_texture_index == 2
    assert d.textures[0].type == 1 and d.textures[0].scalar == np.float32(0.04)
    assert d.textures[1].type == 2 and d.textures[1].scalar == 0.125


@pytest.mark.parametrize("mutate", [
    lambda d: d.pop("materials"),
    lambda d: d.pop("lights"),
    lambda d: d.pop("objects"),
    lambda d: d.pop("camera"),
    lambda d: d["settings"].pop("background_color"),
    lambda d: d["settings"]["image_settings"].__setitem__("width", 64.0),     # IsInt() false
    lambda d: d["settings"]["image_settings"].__setitem__("bucket_size", "24"),
    lambda d: d.__setitem__("materials", []),                                 # Empty() rejected
    lambda d: d["materials"][0].pop("smooth_shading"),
    lambda d: d["materials"][0].__setitem__("albedo", "nope"),                # unknown texture name
    lambda d: d["materials"][0].__setitem__("type", "glossy"),
    lambda d: d["objects"][0].__setitem__("triangles", [0, 1]),               # % 3
    lambda d: d["objects"][0].__setitem__("vertices", [0, 1, 2, 3]),
    lambda d: d["objects"][0].__setitem__("triangles", [0, 1, 2.0]),          # not IsInt
    lambda d: d["objects"][0].__setitem__("uvs", [0, 0, 0]),                  # size mismatch
    lambda d: d["camera"].__setitem__("matrix", [1, 0, 0]),
    lambda d: d["settings"].__setitem__("gi_on", 1),
    lambda d: d["lights"][0].__setitem__("intensity", "x"),
])
def test_rejections(mutate):
    from crt_amd.native import ParseError
    doc = minimal()
    mutate(doc)
    with pytest.raises(ParseError):
        parse(json.dumps(doc))


@pytest.mark.parametrize("text", ['{', '{"a":1,}', '[1,2]x', '{"a":01}', '{"a":-}', '{"a":1.}', '{"a":NaN}',
                                  '{"a":"\\x"}', '{"a":1e400}'])
def test_syntax_errors(text):
    from crt_amd.native import ParseError
    with pytest.raises(ParseError):
        parse(text)


def test_first_duplicate_key_wins():
    text = json.dumps(minimal())
    text = text.replace('"lights":', '"lights": [], "lights":', 1)
    d = parse(text).desc()
    assert d.light_count == 0


def test_unicode_escapes_in_names():
    doc = minimal(textures=[{"name": "téx\U0001F600", "type": "albedo", "albedo": [1, 0, 0]}])
    doc["materials"][0]["albedo"] = "téx\U0001F600"
    d = parse(json.dumps(doc, ensure_ascii=True)).desc()
    assert d.materials[0].albedo_texture_index == 0


def test_texture_failure_drops_the_whole_list():
    """A bitmap texture fails like a failed read_stb: textures = {} (crt_json.cpp:582-588);
    a material with an inline albedo still loads (its texture index restarts at 0)."""
    doc = minimal(textures=[{"name": "a", "type": "albedo", "albedo": [1, 0, 0]},
                            {"name": "b", "type": "bitmap", "file_path": "/x.jpg"}])
    d = parse(json.dumps(doc)).desc()
    assert d.texture_count == 1 and d.materials[0].albedo_texture_index == 0


# ---------------------------------------------------------------- numbers
POW10 = [float(f"1e{i}") for i in range(309)]


def rapidjson_double(s: str):
    """rapidjson reader.h ParseNumber (default flags, 64-bit) + StrtodNormalPrecision."""
    i = 0
    minus = s[0] == "-"
    if minus:
        i = 1
    j = i
    while j < len(s) and s[j].isdigit():
        j += 1
    intpart = s[i:j]
    frac = ""
    exp = 0
    if j < len(s) and s[j] == ".":
        k = j + 1
        while k < len(s) and s[k].isdigit():
            k += 1
        frac = s[j + 1:k]
        j = k
    if j < len(s) and s[j] in "eE":
        exp = int(s[j + 1:])
    if not frac and exp == 0 and j == len(s) and "e" not in s.lower():
        return None  # integer path
    # significand accumulation as in reader.h: uint64 until > 2^53-1, then double
    i64 = 0
    d = None
    exp_frac = 0
    sig = 0
    digits = intpart.lstrip("0") or "0"
    if len(digits) > 19 or int(digits) >= 2 ** 64:
        raise ValueError("test generator keeps integer parts small")
    i64 = int(intpart)
    sig = max(len(intpart) - 1, 0)
    if frac:
        for ch in frac:
            if d is None:
                if i64 > 0x1FFFFFFFFFFFFF:
                    d = float(i64)
                else:
                    i64 = i64 * 10 + int(ch)
                    exp_frac -= 1
                    if i64 != 0:
                        sig += 1
                    continue
            if sig < 17:
                d = d * 10.0 + int(ch)
                exp_frac -= 1
                if d > 0.0:
                    sig += 1
        if d is None:
            d = float(i64)
    else:
        d = float(i64)
    p = exp + exp_frac

    def fast(x, e):
        if e < -308:
            return 0.0
        return x * POW10[e] if e >= 0 else x / POW10[-e]
    if p < -308:
        d = fast(fast(d, -308), p + 308)
    else:
        d = fast(d, p)
    return -d if minus else d


def light_intensity(text_number: str) -> float:
    doc = json.dumps(minimal()).replace('"intensity": 100', f'"intensity": {text_number}')
    return parse(doc).desc().lights[0].intensity


def test_scene_style_numbers_are_correctly_rounded():
    rng = random.Random(42)
    for _ in range(400):
        digits = rng.randint(1, 9)
        mant = rng.randint(1, 10 ** digits - 1)
        point = rng.randint(0, digits)
        s = str(mant).rjust(point + 1, "0")
        s = s[: len(s) - point] + ("." + s[len(s) - point:] if point else "")
        if rng.random() < 0.3:
            s += f"e{rng.randint(-12, 5)}"
        if rng.random() < 0.5:
            s = "-" + s
        want = np.float32(float(s))
        got = np.float32(light_intensity(s))
        assert got.view(np.uint32) == want.view(np.uint32), s


def test_long_mantissas_follow_rapidjson_normal_precision():
    rng = random.Random(7)
    for _ in range(300):
        nd = rng.randint(16, 24)
        frac = "".join(rng.choice("0123456789") for _ in range(nd))
        s = f"{rng.randint(0, 999)}.{frac}"
        if rng.random() < 0.5:
            s += f"e{rng.randint(-30, 10)}"
        want = np.float32(rapidjson_double(s))
        got = np.float32(light_intensity(s))
        assert got.view(np.uint32) == want.view(np.uint32), s


def test_integer_typing():
    # "-0" is an Int(0): GetFloat() gives +0.0, while "-0.0" is a double -0.0
    assert math.copysign(1.0, light_intensity("-0")) == 1.0
    assert math.copysign(1.0, light_intensity("-0.0")) == -1.0
    assert light_intensity("4294967295") == np.float32(4294967295.0)
    assert light_intensity("123456789012345678901") == np.float32(123456789012345678901.0)


# ---------------------------------------------------------------- writer round trip
@pytest.mark.parametrize("npz", sorted(SCENES.glob("*.npz")), ids=lambda p: p.stem)
def test_crtscene_writer_round_trip(npz):
    """crt_amd.scene_json writes a document the loader reads back to the same
    description, bit for bit (what the CLI / _crt GPU tests rely on)."""
    from crt_amd.native import SceneFile
    from crt_amd.scene_json import arrays_to_crtscene
    from crt_amd.scene_npz import desc_to_arrays
    want = dict(np.load(npz))
    bitmaps = {i: "/textures/dragon.jpg" for i, t in enumerate(want["tex_i"]) if t == 3}   # tests/golden/textures
    sf = SceneFile(text=json.dumps(arrays_to_crtscene(want, bitmaps)), asset_root=str(SCENES.parent))
    got = desc_to_arrays(sf.desc())
    assert set(got) == set(want)
    for k in want:
        assert np.array_equal(bits(got[k]), bits(want[k])), k
