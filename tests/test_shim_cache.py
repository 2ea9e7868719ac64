"""The crt::render_image shim's device-scene cache is bounded:
a host that renders a new crt::Scene per call (the Python module, the
Blender add-on) keeps at most two device scenes alive; evicted entries are
destroyed.  The cache logic (csrc/shim/crt_scene_lru.h) is checked on the
CPU by tests/tools/lru_check.cpp."""
import subprocess

from conftest import ROOT


def test_shim_scene_cache_bounded(tmp_path):
    exe = tmp_path / "lru_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-o", str(exe), str(ROOT / "tests" / "tools" / "lru_check.cpp")],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout
