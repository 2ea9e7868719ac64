#!/usr/bin/env python3
"""Blender extension package with the MI355X render path.

Same layout as the reference's `crt_blender_extension` target
(CMakeLists.txt:65-85: src/blender/* + the _crt module, zipped): the add-on's
own Python files and manifest come from the user's checkout of the reference
(--addon-src, unchanged: bl_crt_engine.py does `from . import _crt`), the _crt
module is this repo's drop-in (csrc/python/py_crt_module.cpp), and its C-ABI
library travels next to it as lib/libcrt_hip.so (found through _crt's
$ORIGIN/lib rpath).  Blender 4.2+ embeds Python 3.11: build _crt for it with
`make -C chaos-ray-tracing-course-2025_amd py PYTHON=python3.11` first.

  python scripts/package_blender.py --addon-src /path/to/reference/src/blender --out crt_blender_extension.zip
"""
import argparse
import sys
import zipfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "chaos-ray-tracing-course-2025_amd"


def package(addon_src: Path, out: Path) -> list:
    addon_src = Path(addon_src)
    if not (addon_src / "blender_manifest.toml").exists():
        raise SystemExit(f"{addon_src}: not the reference's src/blender (no blender_manifest.toml)")
    mods = sorted(PKG.glob("_crt*.so"))
    lib = PKG / "lib" / "libcrt_hip.so"
    if not mods or not lib.exists():
        raise SystemExit("build the _crt module and lib/libcrt_hip.so first (make -C chaos-ray-tracing-course-2025_amd)")
    members = []
    with zipfile.ZipFile(out, "w", zipfile.ZIP_DEFLATED) as z:
        for f in sorted(addon_src.iterdir()):
            if f.is_file() and (f.suffix in (".py", ".toml")):
                z.write(f, f.name)
                members.append(f.name)
        for m in mods:
            z.write(m, m.name)
            members.append(m.name)
        z.write(lib, "lib/libcrt_hip.so")
        members.append("lib/libcrt_hip.so")
    return members


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--addon-src", default="/root/reference/src/blender")
    p.add_argument("--out", default=str(PKG / "build" / "crt_blender_extension.zip"))
    a = p.parse_args()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    for m in package(Path(a.addon_src), Path(a.out)):
        print(" ", m)
    print("wrote", a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
