"""The C-ABI library loads and exports every symbol include/crt_hip.h declares
(no compute calls: this runs without a GPU)."""
import ctypes as C
import re

from conftest import ROOT


def header_functions():
    text = (ROOT / "include" / "crt_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(crt_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = header_functions()
    for required in ("crt_hip_render", "crt_hip_scene_create", "crt_hip_scene_destroy",
                     "crt_hip_trace_batch", "crt_hip_last_error", "crt_scene_file_parse",
                     "crt_hip_render_shard", "crt_hip_unpack_shards"):
        assert required in names


def test_library_exports_every_declared_symbol(native_lib):
    missing = [n for n in header_functions() if not hasattr(native_lib, n)]
    assert not missing, f"declared in include/crt_hip.h but not exported: {missing}"


def test_python_binding_covers_every_symbol():
    from crt_amd.native import EXPORTS
    bound = {n for n, _, _ in EXPORTS}
    assert set(header_functions()) == bound


def test_abi_version_and_defaults(native_lib):
    from crt_amd.native import RendererSettings
    assert native_lib.crt_hip_abi_version() == 1
    s = RendererSettings()
    native_lib.crt_renderer_settings_default(C.byref(s))
    # crt_renderer.h:10-16
    assert (s.max_ray_depth, s.diffuse_reflection_ray_count) == (3, 4)
    for f in ("shadow_bias", "reflection_bias", "diffuse_reflection_bias", "refraction_bias"):
        assert getattr(s, f) == C.c_float(1e-2).value


def test_struct_sizes_match_c_layout():
    from crt_amd import native as N
    # crt_hit: 12 floats + 3 int32
    assert C.sizeof(N.Hit) == 60
    assert C.sizeof(N.RendererSettings) == 24
    assert C.sizeof(N.Vec3) == 12


def test_no_gpu_means_loud_failure_not_fallback():
    """Without a HIP device the render path must raise, never fall back to CPU."""
    import pytest
    from crt_amd import native as N
    from conftest import scene_npz
    try:
        import torch  # noqa: F401
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(N.CrtError) as e:
        N.HipScene(scene_npz("14-01-acceleration-tree__scene0"))
    assert e.value.code == N.CRT_E_HIP


def test_blender_extension_package(tmp_path):
    """scripts/package_blender.py: the add-on's files + _crt + lib/libcrt_hip.so;
    the packaged _crt imports from the extracted directory (rpath $ORIGIN/lib)
    and exposes the reference module's API (py_crt_module.cpp:16-169)."""
    import subprocess
    import sys
    import zipfile
    import pytest
    from conftest import REFERENCE, has_reference
    if not has_reference():
        pytest.skip("needs the reference's src/blender add-on files")
    out = tmp_path / "ext.zip"
    subprocess.run([sys.executable, str(ROOT / "scripts" / "package_blender.py"), "--addon-src",
                    str(REFERENCE / "src" / "blender"), "--out", str(out)], check=True, capture_output=True)
    names = zipfile.ZipFile(out).namelist()
    assert {"__init__.py", "bl_crt_engine.py", "blender_manifest.toml", "lib/libcrt_hip.so"} <= set(names)
    assert any(n.startswith("_crt") and n.endswith(".so") for n in names)
    zipfile.ZipFile(out).extractall(tmp_path / "x")
    code = ("import sys; sys.path.insert(0, sys.argv[1]); import _crt; "
            "s = _crt.RendererSettings((3, 4, 0.01, 0.01, 0.01, 0.01)); "
            "print(_crt.DEFAULT_MAX_RAY_DEPTH, s.max_ray_depth, hasattr(_crt, 'render_scene_from_dict'))")
    r = subprocess.run([sys.executable, "-c", code, str(tmp_path / "x")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["3", "3", "True"]


def test_library_resolves_every_kernel():
    """Every kernel the host layer launches is compiled into the library: no
    crt_amd symbol is left undefined (each kernel family is instantiated in
    one translation unit, crt_kernels.h; the link also uses --no-undefined)."""
    import subprocess
    lib = ROOT / "chaos-ray-tracing-course-2025_amd" / "lib" / "libcrt_hip.so"
    out = subprocess.run(["nm", "-DC", "--undefined-only", str(lib)], capture_output=True, text=True,
                         check=True).stdout
    assert "crt_amd::" not in out, [ln for ln in out.splitlines() if "crt_amd::" in ln][:5]
