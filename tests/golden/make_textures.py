"""Regenerate the bitmap-texture fixtures from the reference.

Runs only where /root/reference exists; commits only data:

  textures/dragon.jpg   the course's JPEG texture (scenes/12-01-textures/textures/,
                        an input data file of the reference's scenes)
  textures.json         size + sha256 of the bytes our decoder
                        (csrc/crt_image_decode.cpp, read_stb's replacement)
                        produces for it — frozen so later changes are noticed
  png_12_01.npz         the reference's committed renders results/png/12-01-textures-scene{0..4}.png
                        as uint8 arrays.  They were rendered before HEAD divided
                        every diffuse colour by diffuse_reflection_ray_count + 1
                        (crt_renderer.cpp:98): HEAD's image x 5
                        (fp32) quantised like write_ppm reproduces them at every
                        pixel — including the bitmap-textured scenes 3 and 4, which
                        pins the decoded texels (tests/test_image_decode.py)
  scenes/12-01-textures__scene{3,4}.npz   the loader's flat description (texels as bytes)
"""
import hashlib
import json
import shutil
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))

from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import save_npz  # noqa: E402

REF = Path("/root/reference")


def main():
    from PIL import Image
    src = REF / "scenes" / "12-01-textures" / "textures" / "dragon.jpg"
    dst = HERE / "textures" / "dragon.jpg"
    dst.parent.mkdir(exist_ok=True)
    shutil.copyfile(src, dst)
    rgb = N.decode_image(dst.read_bytes())
    meta = {"dragon.jpg": {"width": int(rgb.shape[1]), "height": int(rgb.shape[0]),
                           "rgb_sha256": hashlib.sha256(rgb.tobytes()).hexdigest()}}
    (HERE / "textures.json").write_text(json.dumps(meta, indent=1))
    pngs = {f"scene{k}": np.asarray(Image.open(REF / "results" / "png" / f"12-01-textures-scene{k}.png")
                                    .convert("RGB")) for k in range(5)}
    np.savez_compressed(HERE / "png_12_01.npz", **pngs)
    for k in (3, 4):
        save_npz(N.SceneFile(path=REF / "scenes" / "12-01-textures" / f"scene{k}.crtscene"),
                 HERE / "scenes" / f"12-01-textures__scene{k}.npz")
    print("wrote", meta)


if __name__ == "__main__":
    main()
