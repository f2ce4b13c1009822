"""rray_amd — MI355X (gfx950) render path for davelpz/rray.

Replaces Camera::render -> Scene::color_at -> intersect -> prepare_computations -> lighting
(with shadows and reflect/refract recursion) by hand-written HIP kernels behind the C ABI in
include/rray/rray.h; scenes come from the reference's YAML format (C++ front-end) or from the
programmatic SceneBuilder.  There is no CPU fallback.
"""
from ._lib import LIB_PATH, RRError, lib  # noqa: F401
from .render import (  # noqa: F401
    Renderer,
    SceneBuilder,
    balance_bands,
    YamlScene,
    camera,
    device_count,
    part_rows,
    quantize,
    rccl_unique_id,
    render_scene_from_file,
    render_scene_from_str,
    stage_row_offset,
    unshuffle,
    write_png,
)

__all__ = ["Renderer", "SceneBuilder", "YamlScene", "camera", "part_rows", "quantize", "write_png",
           "render_scene_from_str", "render_scene_from_file", "device_count", "rccl_unique_id", "stage_row_offset", "unshuffle", "balance_bands", "RRError",
           "lib"]
