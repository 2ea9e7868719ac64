"""crt_amd — MI355X-native drop-in for the render path of bvpav/chaos-ray-tracing-course-2025.

Python host mirror of the reference's interface for this path:
    render_image(scene, settings)       -> crt::render_image  (src/core/crt_renderer.h:27)
    load_scene(path)                    -> crt::json::read_scene_from_istream (src/core/crt_json.h:11)
    RendererSettings                    -> crt::RendererSettings (src/core/crt_renderer.h:18-25)
    write_ppm(path, image)              -> crt::write_ppm (src/core/crt_image_ppm.h:9)
The computation lives in lib/libcrt_hip.so (HIP kernels for gfx950 + host C++).
"""
from .native import (  # noqa: F401
    CrtError, ParseError, RendererSettings, SceneFile, SyntheticScene, HostScene, HipScene,
    write_ppm, lib, last_error, HIT_DTYPE,
)


def load_scene(path, width: int | None = None, height: int | None = None) -> SceneFile:
    """Parse a .crtscene file (optionally overriding the image size)."""
    sf = SceneFile(path=path)
    if width is not None or height is not None:
        d = sf.desc()
        sf.set_resolution(width or d.camera.width, height or d.camera.height)
    return sf


def render_image(scene, settings: RendererSettings | None = None, device: int = 0):
    """Drop-in for crt::render_image: float32 [H, W, 3], top row first, unclamped."""
    hs = scene if isinstance(scene, HipScene) else HipScene(scene, device)
    return hs.render(settings)
